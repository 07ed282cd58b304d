"""kstep_fmi -- Python host binding of libkstepfmi.so (include/kstep_fmi.h).

This is the ctypes form of the reference's link-time plugin interface
(/root/reference/common/interface.h:27-41): the same entry points, argument
meaning and error codes, over opaque handles.  It is plumbing for the test
suite, bench.py and multi-GPU runs; the engine itself is the C ABI library
(HIP kernels for gfx950 + C host code) and there is no Python or CPU fallback
for the search: if the library or a GPU is missing, calls fail loudly.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent          # k-step_fm-index_amd/
LIB_PATH = PKG_DIR / "lib" / "libkstepfmi.so"
BIN_DIR = PKG_DIR / "bin"

# (the packed and ac128 layouts were retired in round 6)
BACKENDS = ("task", "coop", "task-ac", "coop-ac", "task-mid", "coop-mid", "task-ac-mid", "coop-ac-mid",
            "task-grp", "coop-grp")
BACKEND_TAG = {"task": 101, "coop": 101, "task-ac": 201, "coop-ac": 201, "task-mid": 101, "coop-mid": 101,
               "task-ac-mid": 201, "coop-ac-mid": 201, "task-grp": 101, "coop-grp": 101}

_lib = None


class KfmiError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _lib.errorCommon(code).decode() if _lib is not None else f"error {code}"
        super().__init__(f"{what}: {msg} (code {code})" if what else f"{msg} (code {code})")


def build(jobs: int = 8) -> None:
    """Compile the HIP + C library and tools in-tree (hipcc --offload-arch=gfx950)."""
    subprocess.run(["make", "-C", str(PKG_DIR), f"-j{jobs}"], check=True)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise FileNotFoundError(f"{LIB_PATH} not built -- run kstep_fmi.build() / make -C {PKG_DIR}")
    L = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    pvp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "loadIndex": (i32, [ctypes.c_char_p, pvp]),
        "saveIndex": (i32, [ctypes.c_char_p, vp]),
        "initResults": (i32, [u32, pvp]),
        "searchIndexGPU": (None, [vp, vp, vp]),
        "freeIndex": (i32, [pvp]),
        "freeReference": (i32, [pvp, pvp]),
        "buildIndex": (i32, [vp, pvp]),
        "freeQueriesGPU": (i32, [pvp]),
        "freeResultsGPU": (i32, [pvp]),
        "freeIndexGPU": (i32, [pvp]),
        "transferGPUtoCPU": (i32, [vp]),
        "transferCPUtoGPU": (i32, [vp, vp, vp]),
        "sampleTime": (ctypes.c_double, []),
        "base2index": (u32, [u32]),
        "loadRef": (i32, [ctypes.c_char_p, u32, pvp]),
        "saveRef": (i32, [ctypes.c_char_p, vp]),
        "loadQueries": (i32, [ctypes.c_char_p, u32, u32, pvp]),
        "writeResults": (i32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32), u32]),
        "loadResults": (i32, [ctypes.c_char_p, pvp]),
        "freeQueries": (i32, [pvp]),
        "freeResults": (i32, [pvp]),
        "saveResults": (i32, [ctypes.c_char_p, vp, vp]),
        "errorCommon": (ctypes.c_char_p, [i32]),
        "kfmi_set_backend": (i32, [ctypes.c_char_p]),
        "kfmi_get_backend": (ctypes.c_char_p, []),
        "kfmi_set_device": (i32, [i32]),
        "kfmi_device_count": (i32, []),
        "kfmi_device_pci_bus_id": (i32, [i32, ctypes.c_char_p, i32]),
        "kfmi_last_error": (i32, []),
        "kfmi_search": (i32, [vp, vp, vp]),
        "searchIndexCPU": (None, [vp, vp, vp]),
        "kfmi_search_cpu": (i32, [vp, vp, vp, i32]),
        "kfmi_last_timing": (i32, [ctypes.POINTER(ctypes.c_double)] * 3),
        "kfmi_load_index_tag": (i32, [ctypes.c_char_p, u32, pvp]),
        "kfmi_index_from_image": (i32, [vp, u64, pvp]),
        "kfmi_index_image": (i32, [vp, pvp, ctypes.POINTER(ctypes.c_uint64)]),
        "kfmi_index_header": (i32, [vp, vp]),
        "kfmi_transform_interleave": (i32, [vp, pvp]),
        "kfmi_transform_ac": (i32, [vp, pvp, pvp]),
        "kfmi_transform_plain": (i32, [vp, pvp]),
        "kfmi_queries_from_buffer": (i32, [vp, u64, u32, pvp]),
        "kfmi_load_queries_gpu": (i32, [ctypes.c_char_p, u32, u64, pvp]),
        "kfmi_results_alloc": (i32, [u64, pvp]),
        "kfmi_results_host": (ctypes.POINTER(ctypes.c_uint32), [vp]),
        "kfmi_results_num": (u64, [vp]),
        "kfmi_build_index_cpu": (i32, [vp, u64, u32, u32, pvp]),
        "kfmi_build_index_gpu": (i32, [vp, u64, u32, u32, i32, pvp]),
        "kfmi_derive_index_gpu": (i32, [vp, u32, i32, pvp]),
        "kfmi_build_stats": (i32, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]),
        "kfmi_count_blocks": (i32, [vp, vp, ctypes.POINTER(ctypes.c_uint64)]),
        "kfmi_count_lines": (i32, [vp, vp, ctypes.POINTER(ctypes.c_uint64)]),
        "kfmi_probe_replay": (i32, [vp, vp, i32, i32, i32, ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "kfmi_device_index_bytes": (u64, [vp]),
        "kfmi_search_stream": (i32, [vp, vp, u64, u32, vp, u64]),
        "kfmi_host_alloc": (i32, [u64, pvp]),
        "kfmi_host_threads": (i32, []),
        "kfmi_host_free": (i32, [vp]),
        "kfmi_stream_release": (i32, []),
        "kfmi_stream_hostpacked_fraction": (ctypes.c_double, []),
        "kfmi_pack_queries": (i32, [vp, u64, u32, vp]),
        "kfmi_pack_queries_k": (i32, [vp, u64, u32, u32, vp]),
        "kfmi_queries_upload_form": (i32, [vp]),
        "kfmi_set_devices": (i32, [ctypes.POINTER(ctypes.c_int32), i32]),
        "kfmi_get_devices": (i32, [ctypes.POINTER(ctypes.c_int32), i32]),
        "kfmi_build_index_ex": (i32, [vp, u64, u32, u32, u32, i32, pvp]),
        "kfmi_set_ftab": (i32, [u32]),
        "kfmi_set_split_class": (i32, [u32]),
        "kfmi_set_fused": (i32, [i32]),
        "kfmi_set_walk_check": (i32, [u32]),
        "kfmi_walk_check_last": (i32, []),
        "kfmi_set_alphabet": (i32, [ctypes.c_char_p]),
        "kfmi_index_sa": (i32, [vp, pvp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]),
        "kfmi_save_sa": (i32, [ctypes.c_char_p, vp]),
        "kfmi_load_sa": (i32, [ctypes.c_char_p, vp]),
        "kfmi_locate": (i32, [vp, vp, u32, pvp]),
        "kfmi_locations_total": (u64, [vp]),
        "kfmi_locations_offsets": (vp, [vp]),
        "kfmi_locations_positions": (vp, [vp]),
        "kfmi_locations_free": (i32, [pvp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def exported_symbols():
    """Names every C-ABI entry point the header declares (for the load test)."""
    load()
    return [n for n in _lib.__dict__ if not n.startswith("_")]


def _check(code: int, what: str) -> None:
    if code:
        raise KfmiError(code, what)


def set_backend(name: str) -> None:
    _check(load().kfmi_set_backend(name.encode()), f"set_backend({name})")


def get_backend() -> str:
    return load().kfmi_get_backend().decode()


def set_ftab(bases: int) -> None:
    """Bowtie-style jump-start table of `bases` bases for the task backends (0 = off)."""
    _check(load().kfmi_set_ftab(int(bases)), f"set_ftab({bases})")


def set_split_class(cls: int) -> None:
    """Fetch form of the task kernels by table-size class (0 = by the uploaded
    table's size, 1 / 2 / 4 = that class); process-wide test knob (KFMI_SPLIT)."""
    _check(load().kfmi_set_split_class(int(cls)), f"set_split_class({cls})")


def set_fused(on: bool) -> None:
    """In-kernel query packing where it fits (True, default) or always the
    separate pack launch (False); process-wide test knob (KFMI_FUSED)."""
    _check(load().kfmi_set_fused(1 if on else 0), f"set_fused({on})")


def set_walk_check(mode: int) -> None:
    """Walk check of locate / derivation: 0 = by size (default), 1 = full
    pointer jumping, 2 = the sampled check; process-wide test knob."""
    _check(load().kfmi_set_walk_check(int(mode)), f"set_walk_check({mode})")


def walk_check_last() -> int:
    """How the last walk check decided: 0 none yet, 1 full, 2 sampled, 3 sampled then full."""
    return int(load().kfmi_walk_check_last())


def set_alphabet(mode: str | None) -> None:
    """Builders' alphabet: "acgt" (default), "map" (base2index every byte) or
    "ref" (byte-compatible with the reference builder); None = KFMI_ALPHABET."""
    _check(load().kfmi_set_alphabet(mode.encode() if mode else None), f"set_alphabet({mode})")


def set_device(dev: int) -> None:
    _check(load().kfmi_set_device(int(dev)), f"set_device({dev})")


def set_devices(devs) -> None:
    """Device group for the transfer/search/transfer trio (kfmi_set_devices):
    index replicated, queries sliced; [] returns to single-device mode."""
    devs = [int(d) for d in devs]
    arr = (ctypes.c_int32 * max(len(devs), 1))(*devs)
    _check(load().kfmi_set_devices(arr, len(devs)), f"set_devices({devs})")


def get_devices() -> list:
    arr = (ctypes.c_int32 * 16)()
    n = load().kfmi_get_devices(arr, 16)
    return [arr[i] for i in range(n)]


def build_stats() -> dict:
    """Tie diagnostics of the last GPU index build (kfmi_build_stats)."""
    t, r = ctypes.c_uint64(), ctypes.c_uint32()
    _check(load().kfmi_build_stats(ctypes.byref(t), ctypes.byref(r)), "build_stats")
    return {"ties": int(t.value), "rounds": int(r.value)}


def device_count() -> int:
    return int(load().kfmi_device_count())


def host_threads() -> int:
    """Threads of the library's parallel host paths (kfmi_host_threads)."""
    return int(load().kfmi_host_threads())


def device_pci_bus_id(dev: int) -> str:
    """PCI bus id of HIP device `dev` (the physical GPU, stable across processes)."""
    buf = ctypes.create_string_buffer(64)
    _check(load().kfmi_device_pci_bus_id(int(dev), buf, 64), f"device_pci_bus_id({dev})")
    return buf.value.decode()


def upload_form(queries) -> str:
    """How transfer_to_gpu left the reads (kfmi_queries_upload_form):
    "none", "ascii" or "packed" (packed to 2-bit words by the host)."""
    return ("none", "ascii", "packed")[load().kfmi_queries_upload_form(queries.ptr)]


def last_timing():
    t = [ctypes.c_double() for _ in range(3)]
    load().kfmi_last_timing(*[ctypes.byref(x) for x in t])
    return {"total_ms": t[0].value, "pack_ms": t[1].value, "lf_ms": t[2].value}


def _owned_view(addr: int, nbytes: int, dtype, owner) -> np.ndarray:
    """numpy view of library-owned memory that keeps `owner` (the handle) alive."""
    buf = (ctypes.c_uint8 * nbytes).from_address(addr)
    buf._kfmi_owner = owner
    return np.frombuffer(buf, dtype=dtype)


class _Handle:
    _free = ""

    def __init__(self, ptr):
        self._p = ctypes.c_void_p(ptr)

    @property
    def ptr(self):
        return self._p

    def close(self):
        if self._p and self._p.value:
            getattr(load(), self._free)(ctypes.byref(self._p))
            self._p = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Index(_Handle):
    """An FM-index (any tag) -- the `fmi_t` handle of fmIndexCPUBaseline.c:54-69."""
    _free = "freeIndex"

    @classmethod
    def load(cls, path, required_tag: int = 0) -> "Index":
        L = load()
        p = ctypes.c_void_p()
        if required_tag:
            _check(L.kfmi_load_index_tag(str(path).encode(), required_tag, ctypes.byref(p)), f"load {path}")
        else:
            _check(L.loadIndex(str(path).encode(), ctypes.byref(p)), f"load {path}")
        return cls(p.value)

    @classmethod
    def from_image(cls, image) -> "Index":
        buf = np.ascontiguousarray(np.frombuffer(image, dtype=np.uint8) if isinstance(image, (bytes, bytearray))
                                   else image).view(np.uint8)
        p = ctypes.c_void_p()
        _check(load().kfmi_index_from_image(buf.ctypes.data, buf.nbytes, ctypes.byref(p)), "index_from_image")
        return cls(p.value)

    @classmethod
    def build(cls, text: bytes, k: int = 2, d: int = 64, gpu: bool = False, host_image: bool = True,
              sa_rate: int = 0) -> "Index":
        """Tag-100 index of `text`; sa_rate > 0 also keeps SA[r] for rows r % sa_rate == 0 (locate)."""
        L = load()
        buf = np.frombuffer(text, dtype=np.uint8)
        p = ctypes.c_void_p()
        if sa_rate:
            err = L.kfmi_build_index_ex(buf.ctypes.data, buf.size, k, d, int(sa_rate), int(bool(gpu)),
                                        ctypes.byref(p))
        elif gpu:
            err = L.kfmi_build_index_gpu(buf.ctypes.data, buf.size, k, d, int(host_image), ctypes.byref(p))
        else:
            err = L.kfmi_build_index_cpu(buf.ctypes.data, buf.size, k, d, ctypes.byref(p))
        _check(err, "build_index")
        return cls(p.value)

    def header(self) -> dict:
        out = np.zeros(14, dtype=np.uint32)
        _check(load().kfmi_index_header(self._p, out.ctypes.data), "header")
        k = int(out[1])
        return dict(tag=int(out[0]), steps=k, bwtsize=int(out[2]), ncounters=int(out[3]),
                    nentries=int(out[4]), chunk=int(out[5]),
                    dollar_pos=[int(x) for x in out[6:6 + k]],
                    dollar_base=[int(x) for x in out[10:10 + k]])

    def image(self) -> np.ndarray:
        """Zero-copy view of the serialised file image (header + entries)."""
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        _check(load().kfmi_index_image(self._p, ctypes.byref(p), ctypes.byref(n)), "image")
        return _owned_view(p.value, n.value, np.uint8, self)

    def save(self, fn) -> None:
        _check(load().saveIndex(str(fn).encode(), self._p), f"saveIndex {fn}")

    def derive(self, k: int, host_image: bool = False) -> "Index":
        """kfmi_derive_index_gpu: the 2K-step index of the same text, derived on
        the current device from this K-step one (K = 1 or 2, k = 2K)."""
        p = ctypes.c_void_p()
        _check(load().kfmi_derive_index_gpu(self._p, int(k), int(bool(host_image)), ctypes.byref(p)), "derive_index")
        return Index(p.value)

    def interleave(self) -> "Index":
        p = ctypes.c_void_p()
        _check(load().kfmi_transform_interleave(self._p, ctypes.byref(p)), "transform_interleave")
        return Index(p.value)

    def alt_counters(self):
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        _check(load().kfmi_transform_ac(self._p, ctypes.byref(a), ctypes.byref(b)), "transform_ac")
        return Index(a.value), Index(b.value)

    def plain(self) -> "Index":
        """The tag-100 index an AltCounters (tag 200/201) index was transformed from."""
        p = ctypes.c_void_p()
        _check(load().kfmi_transform_plain(self._p, ctypes.byref(p)), "transform_plain")
        return Index(p.value)

    def device_bytes(self) -> int:
        return int(load().kfmi_device_index_bytes(self._p))

    def sa(self):
        """(rate, uint32 view of the row-sampled suffix array); (0, empty) when absent."""
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        rate = ctypes.c_uint32()
        _check(load().kfmi_index_sa(self._p, ctypes.byref(p), ctypes.byref(n), ctypes.byref(rate)), "index_sa")
        if not n.value:
            return 0, np.zeros(0, dtype=np.uint32)
        return int(rate.value), _owned_view(p.value, 4 * n.value, np.uint32, self)

    def save_sa(self, fn) -> None:
        _check(load().kfmi_save_sa(str(fn).encode(), self._p), f"save_sa {fn}")

    def load_sa(self, fn) -> None:
        _check(load().kfmi_load_sa(str(fn).encode(), self._p), f"load_sa {fn}")

    def free_gpu(self) -> None:
        load().freeIndexGPU(ctypes.byref(self._p))


class Queries(_Handle):
    """`qrys_t` (common.h:64-69): num reads of `size` ASCII bases, plain layout."""
    _free = "freeQueries"

    @classmethod
    def from_array(cls, q: np.ndarray) -> "Queries":
        q = np.ascontiguousarray(q, dtype=np.uint8)
        n, m = q.shape
        p = ctypes.c_void_p()
        _check(load().kfmi_queries_from_buffer(q.ctypes.data, n, m, ctypes.byref(p)), "queries_from_buffer")
        return cls(p.value)

    @classmethod
    def load(cls, path, size: int, num: int) -> "Queries":
        p = ctypes.c_void_p()
        _check(load().loadQueries(str(path).encode(), size, num, ctypes.byref(p)), f"loadQueries {path}")
        return cls(p.value)

    @classmethod
    def load_gpu(cls, path, size: int, num: int = 0) -> "Queries":
        """FASTA parsed on the device (kfmi_load_queries_gpu); num = 0: every read."""
        p = ctypes.c_void_p()
        _check(load().kfmi_load_queries_gpu(str(path).encode(), size, num, ctypes.byref(p)),
               f"kfmi_load_queries_gpu {path}")
        return cls(p.value)

    def num(self) -> int:
        return int(ctypes.c_uint64.from_address(self._p.value).value)

    def free_gpu(self) -> None:
        load().freeQueriesGPU(ctypes.byref(self._p))


class Results(_Handle):
    """`res_t` (common.h:77-81): 2*num u32 [L0,R0,L1,R1,...]."""
    _free = "freeResults"

    @classmethod
    def alloc(cls, num: int) -> "Results":
        p = ctypes.c_void_p()
        _check(load().kfmi_results_alloc(num, ctypes.byref(p)), "results_alloc")
        return cls(p.value)

    def array(self) -> np.ndarray:
        L = load()
        n = int(L.kfmi_results_num(self._p))
        ptr = L.kfmi_results_host(self._p)
        if not n:
            return np.zeros(0, dtype=np.uint32)
        return _owned_view(ctypes.cast(ptr, ctypes.c_void_p).value, 8 * n, np.uint32, self)

    def save(self, fn) -> None:
        _check(load().saveResults(str(fn).encode(), self._p, None), f"saveResults {fn}")

    def free_gpu(self) -> None:
        load().freeResultsGPU(ctypes.byref(self._p))


def transfer_to_gpu(index: Index | None, queries: Queries | None, results: Results | None) -> None:
    _check(load().transferCPUtoGPU(index.ptr if index else None, queries.ptr if queries else None,
                                   results.ptr if results else None), "transferCPUtoGPU")


def search(index: Index, queries: Queries, results: Results) -> None:
    _check(load().kfmi_search(index.ptr, queries.ptr, results.ptr), "searchIndexGPU")


def transfer_to_cpu(results: Results) -> None:
    _check(load().transferGPUtoCPU(results.ptr), "transferGPUtoCPU")


def count_blocks(index: Index, queries: Queries) -> int:
    n = ctypes.c_uint64()
    _check(load().kfmi_count_blocks(index.ptr, queries.ptr, ctypes.byref(n)), "count_blocks")
    return int(n.value)


def count_lines(index: Index, queries: Queries) -> dict:
    """kfmi_count_lines: the 128-B lines the backend's fetches touch over the batch."""
    out = (ctypes.c_uint64 * 4)()
    _check(load().kfmi_count_lines(index.ptr, queries.ptr, out), "count_lines")
    return {"lines": int(out[0]), "counter_outside_planes_line": int(out[1]), "ends_fetched": int(out[2]),
            "line_local_ends": int(out[3])}


def probe_replay(index: Index, queries: Queries, unroll: int = 1, reps: int = 5, groups: int = 1) -> dict:
    """kfmi_probe_replay: the search's own line requests replayed without the
    LF dependence (MID layouts, K = 2); returns ms per launch, lines per
    launch, trace bytes and the line rate."""
    ms, lines, tb = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
    _check(load().kfmi_probe_replay(index.ptr, queries.ptr, int(unroll), int(groups), int(reps), ctypes.byref(ms),
                                    ctypes.byref(lines), ctypes.byref(tb)), "kfmi_probe_replay")
    return {"unroll": int(unroll), "groups": int(groups), "ms": ms.value, "lines": int(lines.value), "trace_bytes": int(tb.value),
            "G_lines_per_s": lines.value / (ms.value / 1e3) / 1e9 if ms.value > 0 else None}


class Locations(_Handle):
    """Output of kfmi_locate: offsets uint64[num+1], positions uint32[total]."""
    _free = "kfmi_locations_free"

    _num = 0

    def offsets(self) -> np.ndarray:
        return _owned_view(load().kfmi_locations_offsets(self._p), 8 * (self._num + 1), np.uint64, self)

    def positions(self) -> np.ndarray:
        L = load()
        t = self.total()
        if not t:
            return np.zeros(0, dtype=np.uint32)
        return _owned_view(L.kfmi_locations_positions(self._p), 4 * t, np.uint32, self)

    def total(self) -> int:
        return int(load().kfmi_locations_total(self._p))


def locate(index: Index, results: Results, max_occ: int = 0) -> Locations:
    """Text positions of every row of each query's [L, R) (results on the device)."""
    p = ctypes.c_void_p()
    _check(load().kfmi_locate(index.ptr, results.ptr, int(max_occ), ctypes.byref(p)), "kfmi_locate")
    loc = Locations(p.value)
    loc._num = int(load().kfmi_results_num(results.ptr))
    return loc


def locate_array(index: Index, queries: np.ndarray, backend: str | None = None, max_occ: int = 0):
    """Search + locate of uint8 [N, m] reads; returns (results uint32[2N],
    offsets uint64[N+1], positions uint32[total])."""
    if backend:
        set_backend(backend)
    q = Queries.from_array(queries)
    r = Results.alloc(queries.shape[0])
    transfer_to_gpu(index, q, r)
    search(index, q, r)
    loc = locate(index, r, max_occ)
    transfer_to_cpu(r)
    out = (r.array().copy(), loc.offsets().copy(), loc.positions().copy())
    loc.close()
    q.close()
    r.close()
    return out


class _Pinned:
    """Owner of a kfmi_host_alloc block (freed when the last view goes)."""

    def __init__(self, nbytes: int):
        self.ptr = ctypes.c_void_p()
        _check(load().kfmi_host_alloc(int(nbytes), ctypes.byref(self.ptr)), "kfmi_host_alloc")
        self.nbytes = int(nbytes)

    def __del__(self):
        if self.ptr and _lib is not None:
            _lib.kfmi_host_free(self.ptr)
            self.ptr = ctypes.c_void_p()


def pinned_empty(shape, dtype=np.uint8) -> np.ndarray:
    """numpy array in pinned host memory (DMA'd directly by search_stream)."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    owner = _Pinned(max(n, 1))
    return _owned_view(owner.ptr.value, n, dt, owner).reshape(shape)


def pack_queries(reads: np.ndarray) -> np.ndarray:
    """Host 2-bit packing of uint8 [N, m] reads (kfmi_pack_queries): uint32
    [ceil(m/16), N], word-major, the words the search consumes."""
    reads = np.ascontiguousarray(reads, dtype=np.uint8)
    n, m = reads.shape
    out = np.empty(((m + 15) // 16, n), dtype=np.uint32)
    _check(load().kfmi_pack_queries(reads.ctypes.data, n, m, out.ctypes.data), "kfmi_pack_queries")
    return out


def pack_queries_k(reads: np.ndarray, k: int) -> np.ndarray:
    """Host packing for a K-step index and any read length (kfmi_pack_queries_k):
    uint32 [rows, N], the K-step stream of bases 0 .. m-r-1 plus, for r = m % K
    > 0, a row of remainder codes."""
    reads = np.ascontiguousarray(reads, dtype=np.uint8)
    n, m = reads.shape
    r = m % k
    out = np.empty(((m - r + 15) // 16 + (1 if r else 0), n), dtype=np.uint32)
    _check(load().kfmi_pack_queries_k(reads.ctypes.data, n, m, int(k), out.ctypes.data), "kfmi_pack_queries_k")
    return out


def search_stream(index: Index, reads: np.ndarray, out: np.ndarray | None = None, chunk: int = 0) -> np.ndarray:
    """Streamed search of uint8 [N, m] host reads against an index already on the
    device (transfer_to_gpu(index, None, None)); returns uint32[2N]."""
    reads = np.ascontiguousarray(reads, dtype=np.uint8)
    n, m = reads.shape
    if out is None:
        out = np.empty(2 * n, dtype=np.uint32)
    assert out.dtype == np.uint32 and out.flags.c_contiguous and out.size >= 2 * n
    _check(load().kfmi_search_stream(index.ptr, reads.ctypes.data, n, m, out.ctypes.data, int(chunk)),
           "kfmi_search_stream")
    return out


def search_cpu(index: Index, queries: Queries, results: Results, nthreads: int = 0) -> None:
    """searchIndexCPU in its own OpenMP region (kfmi_search_cpu): the host search."""
    _check(load().kfmi_search_cpu(index.ptr, queries.ptr, results.ptr, int(nthreads)), "searchIndexCPU")


def search_cpu_array(index: Index, queries: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """One-shot host search of uint8 [N, m] reads (searchIndexCPU); uint32[2N]."""
    q = Queries.from_array(queries)
    r = Results.alloc(queries.shape[0])
    try:
        search_cpu(index, q, r, nthreads)
        return r.array().copy()
    finally:
        q.close()
        r.close()


def search_array(index: Index, queries: np.ndarray, backend: str | None = None) -> np.ndarray:
    """One-shot GPU search of uint8 [N, m] reads; returns uint32[2N]."""
    if backend:
        set_backend(backend)
    q = Queries.from_array(queries)
    r = Results.alloc(queries.shape[0])
    transfer_to_gpu(index, q, r)
    search(index, q, r)
    transfer_to_cpu(r)
    out = r.array().copy()
    q.close()
    r.close()
    return out


def env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default
