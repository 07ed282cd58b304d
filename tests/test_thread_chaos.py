"""Seeded multi-thread chaos on one index handle: host threads each run a
random sequence of searches (any backend the geometry takes, which re-uploads
the handle's device copy under its writer lock while others search), jump-start
tables (thread-local), streamed searches, locate and the reference trio, every
result checked against the oracle or brute force.  The reference is
single-threaded (SURVEY 8(b) threading); this is the serving-side contract of
the library (kfmi_search.hip: per-thread streams and events, per-handle
writer-preferring lock, kfmi_internal.h)."""
import threading

import numpy as np
import pytest

import util

pytestmark = pytest.mark.gpu

# the K = 2 backends: a grouped one would derive a K = 4 device copy, and a
# batch packed for one K meets a copy of the other as a refusal (code 33), by
# design, not a result
BACKENDS = ("task", "coop", "task-mid", "coop-mid", "task-ac", "coop-ac",
            "task-ac-mid", "coop-ac-mid")


@pytest.fixture(scope="module")
def world(kfmi_mod, oracle_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    rng = np.random.default_rng(4711)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=400_003)].copy()
    for _ in range(30):
        a, b = rng.integers(0, t.size - 400, size=2)
        t[b:b + 300] = t[a:a + 300]
    text = t.tobytes()
    idx = K.Index.build(text, k=2, d=64, gpu=True, sa_rate=8)
    sa = util.suffix_array(text + b"$")
    batches = []
    for j in range(24):
        m = int(rng.choice([12, 40, 100, 150, 256, 300]))
        n = int(rng.integers(1, 5000))
        st = rng.integers(0, t.size - m, size=n)
        q = np.ascontiguousarray(np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                                                 rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(n // 6, m))]))
        batches.append((q, oracle_mod.search(idx.image(), q)[0]))
    yield K, idx, sa, batches
    idx.close()


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_thread_chaos(world, seed):
    K, idx, sa, batches = world
    errs = []

    def worker(w):
        rng = np.random.default_rng(seed * 100 + w)
        try:
            for op in range(60):
                q, want = batches[int(rng.integers(0, len(batches)))]
                kind = rng.choice(["search", "search", "search", "ftab", "stream", "locate", "handles"])
                b = str(rng.choice(BACKENDS))
                K.set_backend(b)
                if kind == "ftab":
                    K.set_ftab(int(rng.choice([2, 4, 8])))
                    got = K.search_array(idx, q, b)
                    K.set_ftab(0)
                elif kind == "stream":
                    K.transfer_to_gpu(idx, None, None)
                    got = K.search_stream(idx, q, chunk=int(rng.choice([7, 64, 1000])))
                elif kind == "locate":
                    got, off, pos = K.locate_array(idx, q, str(rng.choice(["task-mid", "coop-mid", "task", "task-ac"])))
                    exp = np.concatenate([sa[int(got[2 * i]):int(got[2 * i + 1])] for i in range(q.shape[0])] +
                                         [sa[:0]]).astype(np.uint32)
                    if not np.array_equal(pos, exp):
                        errs.append((w, op, "locate positions"))
                elif kind == "handles":   # the reference trio on this thread's own handles
                    qq = K.Queries.from_array(q)
                    rr = K.Results.alloc(q.shape[0])
                    K.transfer_to_gpu(idx, qq, rr)
                    K.search(idx, qq, rr)
                    K.transfer_to_cpu(rr)
                    got = rr.array().copy()
                    qq.close()
                    rr.close()
                else:
                    got = K.search_array(idx, q, b)
                if not np.array_equal(got, want):
                    errs.append((w, op, kind, b, int(np.sum(got != want))))
        except Exception as e:   # noqa: BLE001 -- reported below, the test fails on it
            errs.append((w, "exception", repr(e)))

    th = [threading.Thread(target=worker, args=(w,)) for w in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    assert not any(x.is_alive() for x in th), "a worker hung"
    assert not errs, errs[:10]
