#!/usr/bin/env python3
"""The LF kernel and the replay probe's kernels on the bench batch, for one
rocprofv3 --pmc pass (dev tool; DESIGN.md 5 "The ceiling the bench states"):

  rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum \
      --kernel-include-regex "task_kernel|replay_lines_kernel|replay_fetch_kernel" \
      -d out -o p --output-format csv -- python3 scripts/pmc_replay.py
  python3 scripts/pmc_replay.py --summarize out/p_counter_collection.csv

The 3 Gbase recipe text and its K = 2 index (task-mid), the bench's rank-0
reads; 5 searches, then kfmi_probe_replay at each (unroll, groups) with 3
timed launches.  --summarize prints, per kernel, the median fabric and L2
requests per launch, the median duration and the request rate.
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))

MODES = ((1, 1), (2, 2), (4, 2), (0, 2))


def run():
    import kstep_fmi as K
    from kstep_fmi import synth
    K.load()
    K.set_device(0)
    text = synth.text_3g()
    reads = synth.gather_reads(text, synth.read_starts(len(text), 10_000_000, 100, seed=10), 100)
    idx = K.Index.build(text, k=2, d=64, gpu=True, host_image=False)
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    K.set_backend("task-mid")
    K.transfer_to_gpu(idx, q, r)
    for _ in range(5):
        K.search(idx, q, r)
    out = {"lf_ms": K.last_timing()["lf_ms"], "replay": []}
    for u, g in MODES:
        out["replay"].append(K.probe_replay(idx, q, unroll=u, groups=g, reps=3))
    print(json.dumps(out), flush=True)


def summarize(fn: str):
    """Per run of consecutive dispatches (the LF kernel's searches, then each
    replay mode's launches in MODES order): medians of the counters, the first
    launch of each run (its warm-up) dropped, and the request rate."""
    sys.path.insert(0, str(ROOT / "scripts"))
    from pmc_summary import runs
    names = ["lf"] + [f"u{u}g{g}" for u, g in MODES]
    for i, run in enumerate(runs(fn)):
        rows = run[1:] if len(run) > 1 else run
        req = statistics.median(x["c"].get("TCC_EA0_RDREQ_sum", 0) for x in rows)
        l2 = statistics.median(x["c"].get("TCC_REQ_sum", 0) for x in rows)
        ms = statistics.median(x["ms"] for x in rows)
        print(json.dumps({"run": names[i] if i < len(names) else i,
                          "kernel": re.sub(r"\(anonymous namespace\)::|kfmi::", "", run[0]["name"]).split("(")[0],
                          "launches": len(rows), "rdreq_per_launch": int(req), "tcc_req_per_launch": int(l2),
                          "ms": round(ms, 4), "G_requests_per_s": round(req / (ms / 1e3) / 1e9, 2)}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarize")
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        run()
