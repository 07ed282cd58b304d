"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper around oracle/_build/liboracle.so (fmi_oracle.c, the C
restatement of /root/reference/src/fmIndexCPUBaseline.c:157-292 and
fmIndexCPUBaseline-AltCounters.c:145-310).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the
product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liboracle.so"
REF_DIR = HERE / "_ref"

_lib = None


def build() -> None:
    subprocess.run(["make", "-C", str(HERE), "oracle"], check=True,
                   stdout=subprocess.DEVNULL)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        L.oracle_search.restype = ctypes.c_int32
        L.oracle_search.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                    ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_header.restype = ctypes.c_int32
        L.oracle_header.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_max_threads.restype = ctypes.c_int32
        _lib = L
    return _lib


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    return np.frombuffer(buf, dtype=np.uint8)


def header(image) -> dict:
    img = _as_u8(image)
    out = np.zeros(14, dtype=np.uint32)
    err = lib().oracle_header(img.ctypes.data, img.nbytes, out.ctypes.data)
    if err:
        raise ValueError(f"bad index image (error {err})")
    k = int(out[1])
    return dict(tag=int(out[0]), steps=k, bwtsize=int(out[2]), ncounters=int(out[3]),
                nentries=int(out[4]), chunk=int(out[5]),
                dollar_pos=[int(x) for x in out[6:6 + k]],
                dollar_base=[int(x) for x in out[10:10 + k]])


def search(image, queries: np.ndarray, nthreads: int = 0):
    """Backward search of every row of `queries` (uint8 [N, m] ASCII).

    Returns (results uint32[2N] = [L0,R0,L1,R1,...], distinct_blocks)."""
    img = _as_u8(image)
    q = np.ascontiguousarray(queries, dtype=np.uint8)
    if q.ndim != 2:
        raise ValueError("queries must be [N, m]")
    n, m = q.shape
    res = np.zeros(2 * n, dtype=np.uint32)
    blocks = ctypes.c_uint64(0)
    err = lib().oracle_search(img.ctypes.data, img.nbytes, q.ctypes.data, n, m,
                              res.ctypes.data, int(nthreads), ctypes.byref(blocks))
    if err == 98:
        raise ValueError("oracle_search: a step reads past the index, where the reference's result "
                         "is undefined (SURVEY B5); compare with brute-force suffix ranks instead")
    if err:
        raise ValueError(f"oracle_search failed (error {err})")
    return res, int(blocks.value)


def max_threads() -> int:
    return int(lib().oracle_max_threads())


def ref_binary(tool: str, k: int, d: int) -> Path:
    """Path of a reference tool compiled by oracle/Makefile (gfmi, tfmiBMP,
    tfmiAC, cpu, cpuac) for (K, d)."""
    return REF_DIR / f"{tool}_{k}_{d}"


def have_ref() -> bool:
    return REF_DIR.exists() and any(REF_DIR.iterdir())


def read_results_file(path) -> np.ndarray:
    """Parse a reference results file (common.c:201-220): "N\\n" then "L R\\n"."""
    with open(path, "rb") as f:
        n = int(f.readline())
        arr = np.loadtxt(f, dtype=np.uint64, ndmin=2) if n else np.zeros((0, 2))
    arr = np.asarray(arr, dtype=np.uint32).reshape(-1)
    assert arr.size == 2 * n, (arr.size, n)
    return arr


def env_threads() -> int:
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
