#!/usr/bin/env python3
"""The transfer/search/transfer trio on the bench batch with either query
upload (dev tool; DESIGN.md 6a "Pageable uploads").

  python3 scripts/upload_probe.py [--reps 5]

The 3 Gbase recipe text, its K = 2 index on the device, the bench's rank-0
reads (10M x 100 bp, pageable numpy memory).  Per upload form (KFMI_UPLOAD =
ascii | packed) and backend (task-mid, coop-mid): wall time of
transfer_to_gpu (queries + zeroed results), of search (with its HIP-event LF
and pack times) and of transfer_to_cpu; medians over `reps`; results checked
equal across forms.  One JSON line per (form, backend).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--queries", type=int, default=10_000_000)
    ap.add_argument("--qlen", type=int, default=100)
    a = ap.parse_args()
    K.load()
    K.set_device(0)
    text = synth.text_3g()
    reads = synth.gather_reads(text, synth.read_starts(len(text), a.queries, a.qlen, seed=10), a.qlen)
    idx = K.Index.build(text, k=2, d=64, gpu=True, host_image=False)
    first = None
    for backend in ("task-mid", "coop-mid"):
        K.set_backend(backend)
        for form in ("ascii", "packed"):
            os.environ["KFMI_UPLOAD"] = form
            q = K.Queries.from_array(reads)
            r = K.Results.alloc(reads.shape[0])
            up, se, lf, pk, dn = [], [], [], [], []
            for i in range(a.reps + 1):
                t0 = time.perf_counter()
                K.transfer_to_gpu(idx, q, r)
                t1 = time.perf_counter()
                K.search(idx, q, r)
                t2 = time.perf_counter()
                K.transfer_to_cpu(r)
                t3 = time.perf_counter()
                if i:                                   # the first round warms up allocations
                    up.append(t1 - t0)
                    se.append(t2 - t1)
                    dn.append(t3 - t2)
                    tm = K.last_timing()
                    lf.append(tm["lf_ms"])
                    pk.append(tm["pack_ms"])
            res = r.array().copy()
            if first is None:
                first = res
            med = lambda x: round(statistics.median(x) * 1e3, 3)  # noqa: E731
            trio = statistics.median(up) + statistics.median(se) + statistics.median(dn)
            print(json.dumps({"backend": backend, "upload": form, "queries": a.queries, "qlen": a.qlen,
                              "transfer_to_gpu_ms": med(up), "search_ms": med(se),
                              "lf_ms": round(statistics.median(lf), 4), "pack_ms": round(statistics.median(pk), 4),
                              "transfer_to_cpu_ms": med(dn), "trio_ms": round(trio * 1e3, 3),
                              "trio_mqps": round(a.queries / trio / 1e6, 1),
                              "results_equal": bool(np.array_equal(res, first))}), flush=True)
            q.close()
            r.close()
    os.environ.pop("KFMI_UPLOAD", None)


if __name__ == "__main__":
    main()
