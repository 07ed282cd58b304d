"""Shared helpers for the test-suite (fixtures, FASTA readers, brute force)."""
from __future__ import annotations

import bisect
import json
import sys
from functools import lru_cache
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
PKG = REPO / "k-step_fm-index_amd"

for p in (str(REPO), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


@lru_cache(maxsize=None)
def manifest() -> dict:
    return json.loads((GOLDEN / "manifest.json").read_text())


def read_fasta_text(path) -> str:
    lines = Path(path).read_text().splitlines()
    return "".join(line for line in lines[1:])


def read_qry(path, m: int) -> np.ndarray:
    """Multi-FASTA query file -> uint8 [N, m] (common.c:167-173 semantics)."""
    data = Path(path).read_bytes()
    rows = [ln for ln in data.split(b"\n") if ln and not ln.startswith(b">")]
    for r in rows:
        assert len(r) == m, (len(r), m)
    if not rows:
        return np.zeros((0, m), dtype=np.uint8)
    return np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(-1, m).copy()


def golden_cases():
    """Yield (case, key, k, d, tag, m, index_path, qry_path, res_path)."""
    for case, c in sorted(manifest().items()):
        for key, ent in sorted(c["indexes"].items()):
            for rk, r in sorted(ent["results"].items()):
                m, base_tag = (int(x) for x in rk.split("."))
                for tag in ((100, 101) if base_tag == 100 else (200, 201)):
                    yield (case, key, ent["k"], ent["d"], tag, m,
                           GOLDEN / case / ent["files"][str(tag)]["file"],
                           GOLDEN / case / c["queries"][str(m)]["file"],
                           GOLDEN / case / r["file"])


def results_md5(kfmi, res: np.ndarray, tmpdir) -> str:
    """md5 of the reference results file for res = [L0,R0,...], written by the
    library's writeResults (common.c:201-220 format, byte-identical to the
    reference's per tests/test_dropin.py) -- fast at 10M queries."""
    import ctypes
    import hashlib
    res = np.ascontiguousarray(res, dtype=np.uint32)
    fn = Path(tmpdir) / "res.txt"
    err = kfmi.load().writeResults(str(fn).encode(), res.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                   res.size // 2)
    assert err == 0, err
    h = hashlib.md5()
    with open(fn, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    fn.unlink()
    return h.hexdigest()


def code_of(x: int) -> int:
    """base2index (genFMindex.c:71-84)."""
    b1 = x & 4
    f2 = x & 2
    b0 = (f2 ^ 2) if b1 else f2
    return (b1 | b0) >> 1


def suffix_array(t: bytes) -> np.ndarray:
    """Suffix array of t (bytes) by prefix doubling, O(n log^2 n) with numpy."""
    n = len(t)
    rank = np.frombuffer(t, dtype=np.uint8).astype(np.int64)
    sa = np.arange(n)
    k = 1
    while True:
        r2 = np.full(n, -1, dtype=np.int64)
        r2[:n - k] = rank[k:] if k < n else r2[:0]
        order = np.lexsort((r2, rank))
        key1, key2 = rank[order], r2[order]
        diff = np.ones(n, dtype=np.int64)
        diff[1:] = (key1[1:] != key1[:-1]) | (key2[1:] != key2[:-1])
        newrank = np.empty(n, dtype=np.int64)
        newrank[order] = np.cumsum(diff) - 1
        rank = newrank
        sa = order
        if rank.max() == n - 1:
            return sa
        k *= 2


class BruteForce:
    """[L, R) = suffix-rank interval of a pattern over T$ ('$' sorts lowest)."""

    def __init__(self, text: str):
        self.t = text.encode() + b"$"
        self.sa = suffix_array(self.t)

    def interval(self, pattern: bytes):
        p = bytes(b"ACGT"[code_of(c)] for c in pattern)
        t, sa, m = self.t, self.sa, len(p)
        key = lambda i: t[i:i + m]  # noqa: E731
        lo = bisect.bisect_left(sa, p, key=key)
        hi = bisect.bisect_right(sa, p, key=key)
        return lo, hi
