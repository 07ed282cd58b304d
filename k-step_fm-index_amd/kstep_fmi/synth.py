"""Seeded synthetic references and reads (SURVEY.md Appendix C recipe).

The reference's read generator (resources/genreads.py:50-76) is Python 2
only; its behaviour -- uniform start in [0, L-m], exact substring -- is
restated here with Python 3's random.Random, so every file is reproducible
and md5-pinned:
  text_64m()  -> ref64.fa sequence, md5 of the FASTA 3b2187508abd0701281aa92b257571a5
  text_3g()   -> ref3g.fa sequence, md5 of the FASTA 98050b607461cfb198278ccbc7fe9fef
  reads_3g(10_000_000, seed=10) -> q10M.qry reads (md5 6a87831e1e7fade3e64b4dca4d400148)
"""
from __future__ import annotations

import hashlib
import random

import numpy as np

TBL = bytes(ord("ACGT"[i & 3]) for i in range(256))

MD5 = {
    "ref64.fa": "3b2187508abd0701281aa92b257571a5",
    "q64.qry": "91a016200b8850733eb060e2a65916a2",
    "ref64.k2d64.fmi": "d738b1d4bd0a3ae9231b511ed4cb68f9",
    "ref64.k1d64.fmi": "de095b820b898920173c76bb7d2a17cc",
    "res64": "0366ea2278af9e4c3beb29e4717beb12",
    "ref3g.fa": "98050b607461cfb198278ccbc7fe9fef",
    "q10M.qry": "6a87831e1e7fade3e64b4dca4d400148",
    "q1M.qry": "973c43bb5741630c636bb826551b92fc",
    "ref3g.k2d64.fmi": "38f85a87df616bdc7f0bae518bd537b3",
    "ref3g.k2d64.fmi.interleaving": "9430112b17949807805fa580043a272f",
    "ref3g.k2d64.fmi.ac": "15daefb7de0addd47dcd5afcdd390d70",
    "ref3g.k2d64.fmi.interleaving.ac": "ef15da2cabf5b83f85427bbf1af76435",
    "res3g.q10M": "cfa6bc65658c6f789e3bb92c9eb6fe67",
    "res3g.q1M": "96148f994f28f308f34a1e5263e6799d",
}


def text_64m() -> tuple[bytes, random.Random]:
    """2^26 uniform ACGT bases (seed 20261015); returns the rng for the reads."""
    rng = random.Random(20261015)
    return rng.randbytes(1 << 26).translate(TBL), rng


def reads_64m(text: bytes, rng: random.Random, num: int = 1 << 20, m: int = 100) -> np.ndarray:
    st = np.fromiter((rng.randint(0, len(text) - m) for _ in range(num)), dtype=np.int64, count=num)
    return gather_reads(text, st, m)


def text_3g(n: int = 3_000_000_000) -> bytes:
    """3 Gbase uniform ACGT (seed 3000000000), generated in 70 Mbase chunks."""
    return b"".join(text_chunks(n))


def text_chunks(n: int):
    """The bench texts as a stream of chunks (peak memory one chunk): the 3 Gbase
    recipe (seed 3000000000, 70 Mbase chunks) for n = 3e9, otherwise
    random.Random(n) in 2^27-base chunks (bench.py's other sizes)."""
    if n == 3_000_000_000:
        rng, ch = random.Random(3000000000), 70 * 1000000
    else:
        rng, ch = random.Random(n), 1 << 27      # getrandbits takes < 2^31 bits per call
    for off in range(0, n, ch):
        yield rng.randbytes(min(ch, n - off)).translate(TBL)


def read_starts(n_text: int, num: int, m: int, seed: int) -> np.ndarray:
    rng = random.Random(seed)
    hi = n_text - m
    return np.fromiter((rng.randint(0, hi) for _ in range(num)), dtype=np.int64, count=num)


def gather_reads(text: bytes, starts: np.ndarray, m: int, chunk: int = 1 << 20) -> np.ndarray:
    """uint8 [num, m] exact substrings text[s:s+m]."""
    t = np.frombuffer(text, dtype=np.uint8)
    out = np.empty((starts.size, m), dtype=np.uint8)
    ar = np.arange(m, dtype=np.int64)
    for i in range(0, starts.size, chunk):
        s = starts[i:i + chunk]
        out[i:i + s.size] = t[s[:, None] + ar[None, :]]
    return out


def fasta_md5(text: bytes, header: bytes) -> str:
    h = hashlib.md5()
    h.update(header)
    ch = 70 * 1000000
    for off in range(0, len(text), ch):
        s = text[off:off + ch]
        h.update(b"\n".join(s[i:i + 70] for i in range(0, len(s), 70)) + b"\n")
    return h.hexdigest()


def qry_md5(reads: np.ndarray, prefix: bytes = b"r") -> str:
    """md5 of the multi-FASTA file the survey generated (">r<i>\\n<read>\\n")."""
    h = hashlib.md5()
    for i in range(reads.shape[0]):
        h.update(b">%s%d\n" % (prefix, i) + reads[i].tobytes() + b"\n")
    return h.hexdigest()


def results_md5(res: np.ndarray) -> str:
    """md5 of the reference results file (common.c:201-220) for res = [L0,R0,...]."""
    n = res.size // 2
    h = hashlib.md5()
    h.update(b"%d\n" % n)
    r = res.reshape(-1, 2)
    step = 1 << 20
    for i in range(0, n, step):
        blk = r[i:i + step]
        h.update(b"".join(b"%d %d\n" % (a, b) for a, b in blk.tolist()))
    return h.hexdigest()
