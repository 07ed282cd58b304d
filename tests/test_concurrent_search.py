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
