#!/usr/bin/env python3
"""Locate throughput vs SA sampling rate on the 3 Gbase index
(dev tool, not the bench contract): one text, one read batch, one index build
per rate; prints one JSON line per (rate, backend)."""
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ref-size", type=int, default=3_000_000_000)
    p.add_argument("--queries", type=int, default=10_000_000)
    p.add_argument("--qlen", type=int, default=100)
    p.add_argument("--rates", default="1,4,16,32,64")
    p.add_argument("--backends", default="task-mid,task-ac")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--coop", default="0,1", help="KFMI_LOCATE_COOP values (MID lines staged through LDS)")
    p.add_argument("--k", type=int, default=2)
    p.add_argument("--env", default="", help="semicolon list of VAR=v1,v2 knobs swept for every backend")
    a = p.parse_args()
    K.load()
    K.set_device(0)
    text = synth.text_3g(a.ref_size) if a.ref_size == 3_000_000_000 else \
        np.random.default_rng(1).choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=a.ref_size).tobytes()
    reads = synth.gather_reads(text, synth.read_starts(len(text), a.queries, a.qlen, 10), a.qlen)
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    t8 = np.frombuffer(text, dtype=np.uint8)
    for rate in [int(x) for x in a.rates.split(",")]:
        t = time.perf_counter()
        idx = K.Index.build(text, k=a.k, d=64, gpu=True, sa_rate=rate, host_image=a.k < 3)
        build_s = time.perf_counter() - t
        knobs = [{}]
        for spec in [x for x in a.env.split(";") if x]:
            var, vals = spec.split("=")
            knobs = [dict(kk, **{var: v}) for kk in knobs for v in vals.split(",")]
        for b, regs, kn in [(b, g, kn) for b in a.backends.split(",") for g in a.coop.split(",") for kn in knobs]:
            os.environ["KFMI_LOCATE_COOP"] = regs
            for var, v in kn.items():
                os.environ[var] = v
            K.set_backend(b)
            K.transfer_to_gpu(idx, q, r)
            K.search(idx, q, r)
            loc = K.locate(idx, r)
            loc.close()
            kms = []
            for _ in range(a.steps):
                loc = K.locate(idx, r)
                kms.append(K.last_timing()["lf_ms"])
                if _ < a.steps - 1:
                    loc.close()
            off, pos = loc.offsets(), loc.positions()
            smp = np.arange(0, reads.shape[0], max(1, reads.shape[0] // 20_000))
            p0 = pos[off[smp].astype(np.int64)].astype(np.int64)
            ok = bool(np.array_equal(t8[p0[:, None] + np.arange(a.qlen)[None, :]], reads[smp]))
            ms = float(np.median(kms))
            import hashlib
            out = {"rate": rate, "backend": b, "coop": int(regs), "knobs": kn, "k": a.k, "pos_md5": hashlib.md5(pos.tobytes()).hexdigest(), "positions": int(loc.total()), "kernel_ms": round(ms, 3),
                   "Mpos_per_s": round(loc.total() / ms / 1e3, 1), "sa_bytes": int(idx.sa()[1].nbytes),
                   "build_s": round(build_s, 2), "positions_start_reads": ok}
            print(json.dumps(out), flush=True)
            loc.close()
            idx.free_gpu()
        idx.close()


if __name__ == "__main__":
    main()
