#!/usr/bin/env python3
"""Streamed (host -> host) search: chunk-size sweep and the PCIe copy rates
that bound it (dev tool; not the bench contract).

  python scripts/e2e_sweep.py --chunks 262144,524288,1048576,2097152,4194304
prints one JSON line per measurement to stdout.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402


def log(*a):
    print(f"[e2e {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def copy_rates(nbytes: int) -> dict:
    """hipMemcpy H2D / D2H of one pinned buffer (torch), GB/s."""
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        out[name + "_GBs"] = round(5 * nbytes / (time.perf_counter() - t) / 1e9, 1)
    del h, d
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--queries", type=int, default=10_000_000)
    p.add_argument("--chunks", default="262144,524288,1048576,2097152,4194304")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--backend", default="task-mid")
    a = p.parse_args()
    K.load()
    K.set_device(0)
    text = synth.text_3g()
    idx = K.Index.build(text, k=2, d=64, gpu=True)
    reads = synth.gather_reads(text, synth.read_starts(len(text), a.queries, 100, 10), 100)
    del text
    log("inputs ready")
    t = time.perf_counter()
    K.pack_queries(reads[:2_000_000])
    pack1 = 2_000_000 / (time.perf_counter() - t) / 1e6
    print(json.dumps({"copy": copy_rates(reads.nbytes), "pack_1thread_Mq_s": round(pack1, 1)}), flush=True)
    K.set_backend(a.backend)
    K.transfer_to_gpu(idx, None, None)
    pin = K.pinned_empty(reads.shape, np.uint8)
    pin[:] = reads
    pout = K.pinned_empty((2 * reads.shape[0],), np.uint32)
    ref = None
    for c in [int(x) for x in a.chunks.split(",") if x]:
        out = K.search_stream(idx, pin, out=pout, chunk=c)
        ref = out.copy() if ref is None else ref
        t = time.perf_counter()
        for _ in range(a.steps):
            out = K.search_stream(idx, pin, out=pout, chunk=c)
        w = (time.perf_counter() - t) / a.steps
        lt = K.last_timing()
        print(json.dumps({"chunk": c, "ms": round(w * 1e3, 3), "mqps": round(reads.shape[0] / w / 1e6, 1),
                          "host_ms": round(lt["pack_ms"], 3), "wait_ms": round(lt["lf_ms"], 3),
                          "equal": bool(np.array_equal(out, ref))}), flush=True)
        K.load().kfmi_stream_release()


if __name__ == "__main__":
    main()
