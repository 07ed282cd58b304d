"""Seeded random query files through the three readers: the mapped parallel
loadQueries, its line-by-line loop (KFMI_LOAD_MMAP=0, the restatement of
common/common.c:132-199 for well-formed files) and the device parser
(kfmi_load_queries_gpu, GPU suite).  Files mix headers of 0-400 bytes (runs of
several), reads with 0-3 trailing '\\r', a missing final newline, and -- in
some worlds -- one defect (a short, long or empty read line) before or after
the read limit; sizes cross the 64 KiB device tiles and the host ranges.
The readers must agree: the same reads, or the same error
(KFMI_E_READING_MFASTA_FILE = 12)."""
import numpy as np
import pytest

from test_ingest import both, search_loaded

WORLDS = 80


def world(i):
    rng = np.random.default_rng(31_000 + i)
    m = int(rng.choice([1, 2, 3, 4, 17, 64, 99, 100, 150, 255, 300]))
    nreads = int(rng.integers(1, 6000))
    reads = np.frombuffer(b"ACGTNacgt", np.uint8)[rng.integers(0, 9, size=(nreads, m))]
    lines = []
    want_ok = True
    limit = int(rng.integers(1, nreads + 1))
    defect_at = int(rng.integers(0, nreads)) if rng.random() < 0.4 else -1
    for j in range(nreads):
        for _ in range(int(rng.choice([0, 1, 1, 1, 2]))):
            lines.append(b">" + b"h" * int(rng.integers(0, 400)))
        r = reads[j].tobytes()
        if j == defect_at:
            kind = int(rng.integers(0, 3))
            r = r[:-1] if kind == 0 and m > 1 else (r + b"A" if kind == 1 else b"")
            if j < limit:
                want_ok = False
        lines.append(r + b"\r" * int(rng.choice([0, 0, 0, 1, 3])))
    body = b"\n".join(lines) + (b"\n" if rng.random() < 0.8 else b"")
    return m, limit, body, reads[:limit], want_ok


@pytest.mark.parametrize("i", range(WORLDS))
def test_ingest_world_host(kfmi_mod, tmp_path, monkeypatch, i):
    m, limit, body, want, ok = world(i)
    path = tmp_path / "q.fa"
    path.write_bytes(body)
    a, b = both(kfmi_mod, path, m, limit, monkeypatch)
    if ok:
        assert isinstance(a, np.ndarray) and np.array_equal(a, want), (i, m, limit)
        assert isinstance(b, np.ndarray) and np.array_equal(b, want), (i, m, limit)
    else:
        assert a == b == 12, (i, m, limit, a if isinstance(a, int) else "data", b if isinstance(b, int) else "data")


@pytest.fixture(scope="module")
def gpu_text_idx(kfmi_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    rng = np.random.default_rng(17)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=100_001).tobytes()
    return K.Index.build(text, k=2, d=64, gpu=True)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(WORLDS))
def test_ingest_world_device(kfmi_mod, gpu_text_idx, tmp_path, i):
    K = kfmi_mod
    m, limit, body, want, ok = world(i)
    path = tmp_path / "q.fa"
    path.write_bytes(body)
    try:
        dev = K.Queries.load_gpu(path, m, limit)
    except K.KfmiError as e:
        dev = e.code
    if not ok:
        assert dev == 12, (i, m, limit)
        return
    assert not isinstance(dev, int), (i, m, limit, dev)
    assert dev.num() == limit
    got = search_loaded(K, gpu_text_idx, dev)
    dev.close()
    assert np.array_equal(got, K.search_array(gpu_text_idx, want, "task-mid")), (i, m, limit)
