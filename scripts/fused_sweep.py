#!/usr/bin/env python3
"""Fused packing against the pack kernel + packed-input LF, per read length
(dev tool; DESIGN.md 4 "fused packing").

  python3 scripts/fused_sweep.py [--lens 100,150] [--reps 10]

The 3 Gbase recipe text and its K = 2 index on the device; per read length m,
10M reads (the bench's seeds: 10 for 100 bp, 20 for config #5's 150 bp) as
ASCII on the device; per KFMI_FUSED in (1, 0) and backend: median pack and LF
times (HIP events) of `reps` searches and results checked equal.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="100,150")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--backends", default="task-mid,coop-mid")
    a = ap.parse_args()
    K.load()
    K.set_device(0)
    text = synth.text_3g()
    idx = K.Index.build(text, k=2, d=64, gpu=True, host_image=False)
    for m in [int(x) for x in a.lens.split(",")]:
        reads = synth.gather_reads(text, synth.read_starts(len(text), 10_000_000, m, seed=10 if m == 100 else 20), m)
        q = K.Queries.from_array(reads)
        r = K.Results.alloc(reads.shape[0])
        first = None
        for backend in a.backends.split(","):
            K.set_backend(backend)
            for fused in ("1", "0"):
                os.environ["KFMI_FUSED"] = fused
                K.transfer_to_gpu(idx, q, r)
                pk, lf, tot = [], [], []
                for i in range(a.reps + 2):
                    K.search(idx, q, r)
                    if i >= 2:
                        t = K.last_timing()
                        pk.append(t["pack_ms"])
                        lf.append(t["lf_ms"])
                        tot.append(t["total_ms"])
                K.transfer_to_cpu(r)
                res = r.array().copy()
                if first is None:
                    first = res
                print(json.dumps({"m": m, "backend": backend, "fused": fused == "1",
                                  "pack_ms": round(statistics.median(pk), 4), "lf_ms": round(statistics.median(lf), 4),
                                  "total_ms": round(statistics.median(tot), 4),
                                  "results_equal": bool(np.array_equal(res, first))}), flush=True)
        os.environ.pop("KFMI_FUSED", None)
        q.close()
        r.close()


if __name__ == "__main__":
    main()
