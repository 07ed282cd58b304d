"""kfmi_probe_replay (diagnostic): the search's own MID128 line
requests replayed without the LF dependence.  It must fetch exactly the lines
the task kernel fetches (count_blocks) at every unroll, and refuse the
layouts it does not model."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_replay_probe_counts_and_rejects(kfmi_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    rng = np.random.default_rng(12)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=1_000_001)]
    idx = K.Index.build(t.tobytes(), k=2, d=64, gpu=True)
    st = rng.integers(0, t.size - 100, size=200_003)
    reads = np.ascontiguousarray(t[st[:, None] + np.arange(100)[None, :]])
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    for backend in ("task-mid", "coop-mid"):
        K.set_backend(backend)
        K.transfer_to_gpu(idx, q, r)
        blocks = K.count_blocks(idx, q)
        for u, g in ((0, 1), (0, 2), (1, 1), (1, 2), (2, 2), (4, 1), (8, 2)):
            p = K.probe_replay(idx, q, unroll=u, groups=g, reps=2)
            assert p["lines"] == blocks and p["ms"] > 0, (backend, u, g, p)
            assert p["trace_bytes"] == 8 * 50 * ((reads.shape[0] + 63) // 64 * 64), p
        K.search(idx, q, r)                          # the index and reads are untouched by the probe
        K.transfer_to_cpu(r)
        assert np.array_equal(r.array(), K.search_array(idx, reads, "task"))
    for backend in ("task", "task-ac-mid"):
        K.set_backend(backend)
        K.transfer_to_gpu(idx, q, r)
        with pytest.raises(K.KfmiError) as e:
            K.probe_replay(idx, q)
        assert e.value.code == 33
    for u, g in ((3, 1), (1, 3)):
        with pytest.raises(K.KfmiError):
            K.probe_replay(idx, q, unroll=u, groups=g)
    for h in (q, r, idx):
        h.close()
