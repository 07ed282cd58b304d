"""Host query packing (kfmi_pack_queries, csrc/host/qpack.c): the 2-bit code
words kfmi_search_stream sends instead of ASCII.  Checked on the CPU against a
restatement of the device pack kernel's order (fmIndexCPUBaseline.c:200-226:
step t consumes bases m-1-K*t-i, i < K) built from util.code_of, for K = 1 and
K = 2 (one bit string serves both), every read length class and every byte."""
import numpy as np
import pytest

import util


def words_ref(reads: np.ndarray, k: int) -> np.ndarray:
    n, m = reads.shape
    steps, spw = m // k, 16 // k
    nw = (steps + spw - 1) // spw
    out = np.zeros((nw, n), dtype=np.uint32)
    for q in range(n):
        for st in range(steps):
            c = 0
            for i in range(k):
                c |= util.code_of(int(reads[q, m - 1 - k * st - i])) << (2 * i)
            out[st // spw, q] |= np.uint32(c << (2 * k * (st % spw)))
    return out


@pytest.mark.parametrize("isa", ["scalar", "avx2", "avx512"])
@pytest.mark.parametrize("m", [2, 4, 16, 30, 32, 34, 63, 64, 65, 96, 100, 126, 128, 150, 160, 250, 256, 300])
def test_pack_matches_step_order(kfmi_mod, m, isa, monkeypatch):
    K = kfmi_mod
    monkeypatch.setenv("KFMI_QPACK_ISA", isa)
    rng = np.random.default_rng(m)
    reads = rng.choice(np.frombuffer(b"ACGTNacgtn", np.uint8), size=(37, m))
    got = K.pack_queries(reads)
    for k in (1, 2):
        if m % k == 0:          # odd m is K=1 only
            assert np.array_equal(got, words_ref(reads, k)), k


@pytest.mark.parametrize("isa", ["scalar", "avx2", "avx512"])
def test_pack_every_byte_value(kfmi_mod, isa, monkeypatch):
    K = kfmi_mod
    monkeypatch.setenv("KFMI_QPACK_ISA", isa)
    reads = np.arange(256, dtype=np.uint8).reshape(4, 64)   # codes of all 256 bytes, both SIMD lanes
    assert np.array_equal(K.pack_queries(reads), words_ref(reads, 2))
    reads = np.arange(256, dtype=np.uint8).reshape(2, 128)
    assert np.array_equal(K.pack_queries(reads), words_ref(reads, 2))


def test_pack_large_batch_and_errors(kfmi_mod):
    K = kfmi_mod
    rng = np.random.default_rng(3)
    reads = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=(20_000, 100))
    got = K.pack_queries(reads)
    # vectorised restatement: reversed codes, 16 per word
    codes = (((reads >> 1) & 3) ^ ((reads >> 2) & 1)).astype(np.uint64)[:, ::-1]
    codes = np.pad(codes, ((0, 0), (0, 112 - 100)))
    w = (codes.reshape(-1, 7, 16) << (2 * np.arange(16, dtype=np.uint64))).sum(axis=2).astype(np.uint32)
    assert np.array_equal(got, w.T)
    assert K.pack_queries(reads[:0]).shape == (7, 0)
    assert K.load().kfmi_pack_queries(None, 5, 100, None) == 33


def words_rem_ref(reads: np.ndarray, k: int) -> np.ndarray:
    """Remainder layout: the K-step stream of bases 0 .. m-r-1
    (as if the read were m - r long), then one row: code of base m-1 at bits
    0-1, m-2 at 2-3, ... (the remainder-table index)."""
    n, m = reads.shape
    r = m % k
    head = words_ref(np.ascontiguousarray(reads[:, :m - r]), 1) if m - r else np.zeros((0, n), np.uint32)
    if not r:
        return head
    rc = np.zeros(n, dtype=np.uint32)
    for u in range(r):
        rc |= np.array([util.code_of(int(x)) for x in reads[:, m - 1 - u]], dtype=np.uint32) << np.uint32(2 * u)
    return np.vstack([head, rc[None, :]])


@pytest.mark.parametrize("isa", ["scalar", "avx2", "avx512"])
@pytest.mark.parametrize("k", [1, 2, 4])
@pytest.mark.parametrize("m", [1, 3, 5, 17, 33, 63, 65, 99, 101, 150, 151, 257])
def test_pack_remainder_rows(kfmi_mod, isa, k, m, monkeypatch):
    """Host packing of reads with m % K != 0 for the streamed search: the
    stream stops r = m % K bases early and a row of remainder codes follows,
    the rows the device pack kernel writes (every ISA path, every length class)."""
    K = kfmi_mod
    monkeypatch.setenv("KFMI_QPACK_ISA", isa)
    rng = np.random.default_rng(m * 10 + k)
    reads = rng.choice(np.frombuffer(b"ACGTNacgtn", np.uint8), size=(29, m))
    got = K.pack_queries_k(reads, k)
    assert np.array_equal(got, words_rem_ref(reads, k))
    if m % k == 0:
        assert np.array_equal(got, K.pack_queries(reads))
    assert K.load().kfmi_pack_queries_k(reads.ctypes.data, 29, m, 3, got.ctypes.data) == 33   # K = 3 streams ASCII
