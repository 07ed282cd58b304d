"""Searches from several host threads at once (each thread has its own search
stream and timing events per device, kfmi_search.hip ThreadRes): every
thread's results stay those of the oracle, on one shared index, with small
batches (whose kernels overlap on the device) and a large one mixed in."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup(kfmi_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    rng = np.random.default_rng(31)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=2_000_003)]
    return t, K.Index.build(t.tobytes(), k=2, d=64, gpu=True)


@pytest.mark.parametrize("backend", ["task-mid", "coop-mid", "task-ac-mid"])
def test_threads_search_one_index(kfmi_mod, oracle_mod, setup, backend):
    K = kfmi_mod
    t, idx = setup
    K.set_backend(backend)
    K.transfer_to_gpu(idx, None, None)
    ref_img = idx.alt_counters()[0].image() if backend == "task-ac-mid" else idx.image()
    batches = []
    for j in range(8):
        rng = np.random.default_rng(100 + j)
        n = 200_000 if j == 0 else 1_000 * (j + 1)
        st = rng.integers(0, t.size - 100, size=n)
        q = np.ascontiguousarray(t[st[:, None] + np.arange(100)[None, :]])
        batches.append((q, oracle_mod.search(ref_img, q)[0]))
    errs = []

    def worker(j):
        try:
            K.set_device(0)
            K.set_backend(backend)         # the backend choice is per thread
            q, want = batches[j]
            qq = K.Queries.from_array(q)
            r = K.Results.alloc(q.shape[0])
            K.transfer_to_gpu(idx, qq, r)      # the index is already there for this backend
            for _ in range(25):
                K.search(idx, qq, r)
                K.transfer_to_cpu(r)
                if not np.array_equal(r.array(), want):
                    errs.append((j, "mismatch"))
                    break
            qq.close()
            r.close()
        except Exception as e:             # reported below
            errs.append((j, repr(e)))

    th = [threading.Thread(target=worker, args=(j,)) for j in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs


def test_reupload_while_another_thread_searches(kfmi_mod, oracle_mod, setup):
    """One thread searches handle A without pause while another replaces the
    device copies of A (another plain-semantics layout: an exclusive upload;
    the reader's searches run on whichever layout is there) and of an
    unrelated handle B, then frees B's: every search result stays the
    oracle's, and the writer finishes all its uploads while the reader keeps
    searching -- the per-handle lock prefers writers (kfmi_fmi_t::rw), and B's
    uploads never wait on A's searches (the old lock stripes were
    shared by unrelated handles and preferred readers)."""
    import time
    K = kfmi_mod
    t, idx = setup
    rng = np.random.default_rng(77)
    b_text = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=300_001)].tobytes()
    idx_b = K.Index.build(b_text, k=2, d=64, gpu=True)
    st = rng.integers(0, t.size - 100, size=50_000)
    q = np.ascontiguousarray(t[st[:, None] + np.arange(100)[None, :]])
    want = oracle_mod.search(idx.image(), q)[0]
    stop = threading.Event()
    errs, n_search = [], [0]

    def reader():
        try:
            K.set_device(0)
            K.set_backend("task-mid")
            qq = K.Queries.from_array(q)
            r = K.Results.alloc(q.shape[0])
            K.transfer_to_gpu(idx, qq, r)
            while not stop.is_set():
                K.search(idx, qq, r)
                K.transfer_to_cpu(r)
                if not np.array_equal(r.array(), want):
                    errs.append("mismatch")
                    break
                n_search[0] += 1
            qq.close()
            r.close()
        except Exception as e:
            errs.append(repr(e))

    th = threading.Thread(target=reader)
    th.start()
    time.sleep(0.5)
    K.set_device(0)
    t0 = time.perf_counter()
    for i in range(6):
        K.set_backend("coop-mid" if i % 2 else "task-mid")
        K.transfer_to_gpu(idx_b, None, None)       # unrelated handle
        idx_b.free_gpu()
        K.set_backend("task" if i % 2 else "task-mid")   # plain semantics: the reader's results stay
        K.transfer_to_gpu(idx, None, None)         # replaces A's device copy under the reader
    writer_s = time.perf_counter() - t0
    stop.set()
    th.join()
    idx_b.close()
    assert not errs, errs
    assert n_search[0] > 0
    assert writer_s < 60, writer_s
