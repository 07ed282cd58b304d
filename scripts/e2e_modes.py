#!/usr/bin/env python3
"""Streamed (host -> host) search: per-chunk transfer mode (KFMI_STREAM_HOSTPACK
0 = ASCII, 1 = host-packed, 2 = adaptive; E2E_ISA, E2E_ROUNDS)
x stream slots (E2E_SLOTS, E2E_MODES comma lists) x host packing ISA, pinned and
pageable input, 3 Gbase / 10M x 100 bp (dev tool; not the bench contract).
One JSON line per measurement on stdout."""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402

K.load()
K.set_device(0)
text = synth.text_3g()
idx = K.Index.build(text, k=2, d=64, gpu=True)
reads = synth.gather_reads(text, synth.read_starts(len(text), 10_000_000, 100, 10), 100)
del text
K.set_backend("task-mid")
want = K.search_array(idx, reads)
K.transfer_to_gpu(idx, None, None)
pin = K.pinned_empty(reads.shape, np.uint8)
pin[:] = reads
pout = K.pinned_empty((2 * reads.shape[0],), np.uint32)
def set_mode(m):
    os.environ["KFMI_STREAM_HOSTPACK"] = m


for isa in os.environ.get("E2E_ISA", "avx2,avx512").split(","):
    os.environ["KFMI_QPACK_ISA"] = isa
    t = time.perf_counter()
    K.pack_queries(reads[:2_000_000])
    p1 = 2_000_000 * 100 / (time.perf_counter() - t) / 1e9
    for kind, src, dst, slots in [(k, s, d, n) for k, s, d in (("pinned", pin, pout), ("pageable", reads, None))
                                  for n in os.environ.get("E2E_SLOTS", "6").split(",")]:
        os.environ["KFMI_STREAM_SLOTS"] = slots
        modes = tuple(os.environ.get("E2E_MODES", "1,2,0").split(","))
        ms = {m: [] for m in modes}
        frac = {}
        ok = {}
        for m in modes:                       # warm-up (and the adaptive model's first measurements)
            set_mode(m)
            K.search_stream(idx, src, out=dst)
        for _ in range(int(os.environ.get("E2E_ROUNDS", "5"))):   # interleaved rounds: drift hits every mode alike
            for m in modes:
                set_mode(m)
                t = time.perf_counter()
                out = K.search_stream(idx, src, out=dst)
                ms[m].append((time.perf_counter() - t) * 1e3)
                frac[m] = K.load().kfmi_stream_hostpacked_fraction()
                ok[m] = bool(np.array_equal(out, want))
        for m in modes:
            med = float(np.median(ms[m]))
            print(json.dumps({"isa": isa, "pack_1thread_GBs": round(p1, 2), "mode": m, "input": kind,
                              "ms": round(med, 3), "ms_all": [round(x, 2) for x in ms[m]],
                              "mqps": round(reads.shape[0] / med * 1e3 / 1e6, 1),
                              "hostpacked_fraction": round(frac[m], 3), "equal": ok[m], "slots": int(slots)}),
                  flush=True)
