#!/usr/bin/env python3
"""Kernel-variant sweep on one index build (dev tool; not the bench contract).

Builds the 3 Gbase (or --ref-size) index once on the GPU, then times each
backend x tuning knob and prints one JSON line per variant to stdout:
  python scripts/sweep.py --backends task-mid,task,coop --qpt 1,2 --steps 5
Every variant's results are compared with the first variant's (bit-exact).
"""
from __future__ import annotations

import argparse
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


def log(*a):
    print(f"[sweep {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ref-size", type=int, default=3_000_000_000)
    p.add_argument("--queries", type=int, default=10_000_000)
    p.add_argument("--qlen", type=int, default=100)
    p.add_argument("--k", type=int, default=2)
    p.add_argument("--d", type=int, default=64)
    p.add_argument("--backends", default="task-mid,task,task-ac,coop,coop-ac,coop-mid")
    p.add_argument("--env", default="", help="semicolon list of VAR=v1,v2 knobs swept for every backend")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1, help="untimed searches per variant before its timed steps")
    p.add_argument("--repeat", type=int, default=1,
                   help="time every backend's knob list this many times, in reverse order on odd passes "
                        "(A B B A ...), so an order effect shows as a disagreement between passes")
    p.add_argument("--sort-suffix", default="0",
                   help="experiment: comma list of N; order reads by their last N bases (backward-search "
                        "order, N <= 32), one pass over the backends per N")
    p.add_argument("--xcd-tiles", default="",
                   help="experiment: comma list of bucket counts B; reads grouped by their last 2*ceil(log4 B)... "
                        "bases into B buckets and laid out so that 256-read tile i holds bucket i % B "
                        "(with round-robin workgroup dispatch, XCD x then sees only buckets = x mod 8)")
    a = p.parse_args()

    K.load()
    K.set_device(0)
    t = time.perf_counter()
    text = synth.text_3g(a.ref_size) if a.ref_size == 3_000_000_000 else \
        np.random.default_rng(1).choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=a.ref_size).tobytes()
    log(f"text {time.perf_counter() - t:.1f}s")
    t = time.perf_counter()
    idx = K.Index.build(text, k=a.k, d=a.d, gpu=True)
    log(f"build {time.perf_counter() - t:.1f}s")
    reads0 = synth.gather_reads(text, synth.read_starts(len(text), a.queries, a.qlen, 10), a.qlen)
    log("reads ready")
    knobs = [{}]
    for spec in [s for s in a.env.split(";") if s]:
        var, vals = spec.split("=")
        knobs = [dict(k, **{var: v}) for k in knobs for v in vals.split(",")]
    ref = None
    plans = [("sort", int(x)) for x in a.sort_suffix.split(",")] + \
            [("xcd", int(x)) for x in a.xcd_tiles.split(",") if x]
    for kind, ss in plans:
        inv = None
        reads = reads0
        if kind == "xcd":
            codes = ((reads0[:, -3:] >> 1) & 3).astype(np.int64)       # last 3 bases, a bijection per base
            key = codes[:, 2] * 16 + codes[:, 1] * 4 + codes[:, 0]      # 64 suffix classes
            bucket = key % ss
            per = [np.flatnonzero(bucket == b) for b in range(ss)]
            ntile = max((x.size + 255) // 256 for x in per)
            order = [per[bk][256 * r:256 * (r + 1)] for r in range(ntile) for bk in range(ss)]
            order = np.concatenate(order)
            assert order.size == reads0.shape[0], (order.size, reads0.shape[0])
            reads = np.ascontiguousarray(reads0[order])
            inv = np.empty_like(order)
            inv[order] = np.arange(order.size)
            log(f"reads laid out in 256-read tiles of {ss} suffix buckets")
        elif ss:
            # key: code of base m-1 most significant, then m-2, ... (the order the
            # backward search consumes them), so reads sharing their last j bases
            # are contiguous for every j <= ss
            codes = ((reads0 >> 1) & 3).astype(np.uint64)     # A0 C1 G3 T2: a bijection, fine for grouping
            key = np.zeros(reads0.shape[0], dtype=np.uint64)
            for j in range(ss):
                key = (key << np.uint64(2)) | codes[:, a.qlen - 1 - j]
            order = np.argsort(key, kind="stable")
            reads = np.ascontiguousarray(reads0[order])
            inv = np.empty_like(order)
            inv[order] = np.arange(order.size)
            log(f"reads ordered by their last {ss} bases")
        q = K.Queries.from_array(reads)
        r = K.Results.alloc(reads.shape[0])
        for b in a.backends.split(","):
          for rep in range(a.repeat):
            for kn in (knobs if rep % 2 == 0 else knobs[::-1]):
                for var, v in kn.items():
                    os.environ[var] = v
                try:
                    K.set_backend(b)
                    K.transfer_to_gpu(idx, q, r)
                    for _ in range(max(1, a.warmup)):
                        K.search(idx, q, r)
                    lf, tot = [], []
                    t0 = time.perf_counter()
                    for _ in range(a.steps):
                        K.search(idx, q, r)
                        tm = K.last_timing()
                        lf.append(tm["lf_ms"])
                        tot.append(tm["total_ms"])
                    wall = (time.perf_counter() - t0) / a.steps
                    K.transfer_to_cpu(r)
                    res = r.array().copy()
                    if inv is not None:
                        res = res.reshape(-1, 2)[inv].reshape(-1)
                    if ref is None:
                        ref = res
                    out = {"backend": b, "knobs": kn, "pass": rep, "order": kind, "sort_suffix": ss, "lf_ms": round(float(np.median(lf)), 3),
                           "lf_ms_min": round(float(np.min(lf)), 3), "step_ms": round(float(np.median(tot)), 3),
                           "wall_ms": round(wall * 1e3, 3), "mqps": round(reads.shape[0] / wall / 1e6, 1),
                           "equal": bool(np.array_equal(res, ref)), "dev_bytes": idx.device_bytes(),
                           "res_md5": synth.results_md5(res)}
                except K.KfmiError as e:
                    out = {"backend": b, "knobs": kn, "pass": rep, "order": kind, "sort_suffix": ss, "error": str(e)}
                print(json.dumps(out), flush=True)
                log(out)
                for var in kn:
                    os.environ.pop(var, None)
          idx.free_gpu()
        q.close()
        r.close()


if __name__ == "__main__":
    main()
