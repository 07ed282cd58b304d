"""Query ingest: the multi-threaded mapped loadQueries against
the line-by-line loop it replaces (reference common/common.c:132-199
semantics, kept as the KFMI_LOAD_MMAP=0 path) on the golden query files, a
1M-read file and the malformed-input cases."""
import os

import numpy as np
import pytest

import util


def load(K, path, m, n):
    q = K.Queries.load(path, m, n)
    L = K.load()
    import ctypes

    class Q(ctypes.Structure):
        _fields_ = [("num", ctypes.c_uint64), ("size", ctypes.c_uint32), ("h", ctypes.c_void_p)]
    qs = Q.from_address(q.ptr.value)
    out = np.ctypeslib.as_array((ctypes.c_uint8 * (qs.num * qs.size)).from_address(qs.h)).reshape(qs.num, qs.size)
    out = out.copy()
    q.close()
    del L
    return out


def both(K, path, m, n, monkeypatch):
    """(mapped parallel result or error code, line-loop result or error code)"""
    res = []
    for mm in ("1", "0"):
        monkeypatch.setenv("KFMI_LOAD_MMAP", mm)
        try:
            res.append(load(K, path, m, n))
        except K.KfmiError as e:
            res.append(e.code)
    monkeypatch.delenv("KFMI_LOAD_MMAP")
    return res


def test_golden_query_files_equal(kfmi_mod, monkeypatch):
    seen = 0
    for case, c in sorted(util.manifest().items()):
        for m, qd in sorted(c["queries"].items()):
            m = int(m)
            path = util.GOLDEN / case / qd["file"]
            a, b = both(kfmi_mod, path, m, qd["num"], monkeypatch)
            assert isinstance(a, np.ndarray) and np.array_equal(a, b), (case, m)
            assert np.array_equal(a, util.read_qry(path, m))
            seen += 1
    assert seen


@pytest.mark.parametrize("threads", ["1", "3", "8"])
def test_million_reads_file(kfmi_mod, tmp_path, monkeypatch, threads):
    """1M x 100 bp reads with ragged headers and CRLF lines, parsed over several
    byte ranges (a range boundary falls inside headers and reads)."""
    rng = np.random.default_rng(int(threads))
    n, m = 1_000_000, 100
    reads = rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(n, m))
    path = tmp_path / "q.fa"
    with open(path, "wb") as f:
        for i in range(0, n, 100_000):
            blk = reads[i:i + 100_000]
            f.write(b"".join(b">r%d%s\n%s%s\n" % (i + j, b" x" * (j % 7), blk[j].tobytes(), b"\r" * (j % 3 == 0))
                             for j in range(blk.shape[0])))
    monkeypatch.setenv("KFMI_HOST_THREADS", threads)
    a, b = both(kfmi_mod, path, m, n, monkeypatch)
    assert np.array_equal(a, reads) and np.array_equal(b, reads)
    # the first 777 reads only: everything after them is ignored
    a, b = both(kfmi_mod, path, m, 777, monkeypatch)
    assert np.array_equal(a, reads[:777]) and np.array_equal(b, reads[:777])


@pytest.mark.parametrize("body,n,ok", [
    (b">a\nACGT\n>b\nTTTT\n", 2, True),
    (b">a\nACGT\n>b\nTTTT", 2, True),                 # no final newline
    (b"ACGT\nTTTT\nGGGG\n", 3, True),                  # no headers at all
    (b">a\nACGT\n>b\nTTTT\n", 3, False),              # too few reads
    (b">a\nACGT\n>b\nTTT\n", 2, False),               # short read before the limit
    (b">a\nACGT\n>b\nTTTT\n>c\nTT\n", 2, True),        # malformed read after the limit: ignored
    (b">a\nACGT\n\n>b\nTTTT\n", 2, False),             # empty line counts as a (bad) read
    (b">a\r\nACGT\r\n>b\r\nTTTT\r\n", 2, True),        # CRLF
    (b">\n>\nACGT\n", 1, True),                        # bare headers
])
def test_edge_cases_equal(kfmi_mod, tmp_path, monkeypatch, body, n, ok):
    for pad in (0, 5_000_000):       # small files parse on one thread, large ones in ranges
        path = tmp_path / "e.fa"
        path.write_bytes(b">pad\n" * (pad // 5) + body if pad else body)
        a, b = both(kfmi_mod, path, 4, n, monkeypatch)
        if ok:
            assert isinstance(a, np.ndarray) and np.array_equal(a, b), (body, pad)
        else:
            assert a == b == 12, (body, pad, a, b)     # KFMI_E_READING_MFASTA_FILE


# ---- device parse (kfmi_load_queries_gpu) -----------------------------------

@pytest.fixture(scope="module")
def gpu_idx(kfmi_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    rng = np.random.default_rng(9)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=200_001).tobytes()
    return K.Index.build(text, k=2, d=64, gpu=True), text


def search_loaded(K, idx, q):
    K.set_backend("task-mid")
    r = K.Results.alloc(q.num())
    K.transfer_to_gpu(idx, q, r)
    K.search(idx, q, r)
    K.transfer_to_cpu(r)
    out = r.array().copy()
    r.close()
    return out


@pytest.mark.gpu
def test_gpu_parse_golden_and_large(kfmi_mod, gpu_idx, tmp_path):
    K = kfmi_mod
    idx, text = gpu_idx
    for case, c in sorted(util.manifest().items()):
        for m, qd in sorted(c["queries"].items()):
            m = int(m)                    # odd m included: remainder table (test_remainder.py)
            path = util.GOLDEN / case / qd["file"]
            q = K.Queries.load_gpu(path, m, qd["num"])
            assert q.num() == qd["num"]
            want = K.search_array(idx, util.read_qry(path, m), "task-mid")
            assert np.array_equal(search_loaded(K, idx, q), want), (case, m)
            q.close()
    # 300K reads, ragged headers and CRLF, several 64 KiB tiles; all reads (num 0) and a prefix
    rng = np.random.default_rng(4)
    t = np.frombuffer(text, np.uint8)
    reads = np.concatenate([t[rng.integers(0, len(t) - 150, size=250_000)[:, None] + np.arange(150)],
                            rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(50_000, 150))])
    path = tmp_path / "q.fa"
    with open(path, "wb") as f:
        f.write(b"".join(b">r%d%s\n%s%s\n" % (j, b" x" * (j % 7), reads[j].tobytes(), b"\r" * (j % 3 == 0))
                         for j in range(reads.shape[0])))
    want = K.search_array(idx, reads, "task-mid")
    q = K.Queries.load_gpu(path, 150)
    assert q.num() == reads.shape[0]
    assert np.array_equal(search_loaded(K, idx, q), want)
    q.close()
    q = K.Queries.load_gpu(path, 150, 12_345)
    assert np.array_equal(search_loaded(K, idx, q), want[:2 * 12_345])
    q.close()
    # long reads (several pack-kernel word chunks; odd length -> remainder table)
    long = np.concatenate([t[rng.integers(0, len(t) - 5001, size=300)[:, None] + np.arange(5001)],
                           rng.choice(np.frombuffer(b"ACGT", np.uint8), size=(20, 5001))])
    path = tmp_path / "long.fa"
    path.write_bytes(b"".join(b">l%d\n%s\n" % (j, long[j].tobytes()) for j in range(long.shape[0])))
    q = K.Queries.load_gpu(path, 5001)
    assert np.array_equal(search_loaded(K, idx, q), K.search_array(idx, long, "task-mid"))
    q.close()


@pytest.mark.gpu
@pytest.mark.parametrize("body,n,ok", [
    (b">a\nACGT\n>b\nTTTT\n", 2, True),
    (b">a\nACGT\n>b\nTTTT", 2, True),
    (b"ACGT\nTTTT\nGGGG\n", 3, True),
    (b">a\nACGT\n>b\nTTTT\n", 3, False),
    (b">a\nACGT\n>b\nTTT\n", 2, False),
    (b">a\nACGT\n>b\nTTTT\n>c\nTT\n", 2, True),
    (b">a\nACGT\n\n>b\nTTTT\n", 2, False),
    (b">a\r\nACGT\r\n>b\r\nTTTT\r\n", 2, True),
    (b">\n>\nACGT\n", 1, True),
    (b">a\nACGTA\n>b\nTTTT\n", 2, False),              # long line
    (b">a\nAC\rT\n", 1, True),                         # '\r' inside the read is a base, as on the host
    (b">a\nACG\r\n>b\nTTTT\n", 2, False),             # ... but a trailing one is not: a 3-base read
    (b">a\nACG\r\r\n", 1, False),
])
def test_gpu_parse_edge_cases_match_host(kfmi_mod, gpu_idx, tmp_path, body, n, ok):
    K = kfmi_mod
    idx, _ = gpu_idx
    for pad in (0, 300_000):    # the read lines in the first tile, or after several
        path = tmp_path / "e.fa"
        path.write_bytes(b">pad\n" * (pad // 5) + body if pad else body)
        try:
            host = K.Queries.load(path, 4, n)
        except K.KfmiError as e:
            host = e.code
        try:
            dev = K.Queries.load_gpu(path, 4, n)
        except K.KfmiError as e:
            dev = e.code
        if ok:
            assert not isinstance(host, int) and not isinstance(dev, int), (body, pad, host, dev)
            want = search_loaded(K, idx, host)
            assert np.array_equal(search_loaded(K, idx, dev), want), (body, pad)
        else:
            assert host == dev == 12, (body, pad, host, dev)
