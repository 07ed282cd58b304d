#!/usr/bin/env python3
"""Every backend's LF kernel on the bench batch, for one rocprofv3 --pmc pass
(dev tool; the bench reads the result through scripts/traffic_variants.py ->
profiles/r04/traffic_variants.json).

  rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum --kernel-include-regex "task_kernel|coop_kernel" \
      -d out -o p --output-format csv -- python3 scripts/pmc_variants.py --order out/order.json

The 3 Gbase recipe text, its K = 2 d = 64 index built on the device, the
bench's rank-0 reads (10M x 100 bp, seed 10; --qlen 150 --seed 20: config
#5's shard); each backend: upload, `warmup`
untimed searches, `steps` searches (one LF launch each); then the same reads on
the K = 4 index (coop-grp, task-grp).  The order file lists (backend, K,
launches) in dispatch order, which is how the PMC rows are attributed.
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

K2 = "task-mid,coop-mid,task,coop,task-ac,coop-ac,task-ac-mid,coop-ac-mid"


def log(*a):
    print(f"[pmc_variants {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--order", required=True)
    p.add_argument("--backends", default=K2)
    p.add_argument("--k4-backends", default="coop-grp,task-grp")
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--ref-size", type=int, default=3_000_000_000)
    p.add_argument("--queries", type=int, default=10_000_000)
    p.add_argument("--qlen", type=int, default=100, help="150: config #5's shard shape")
    p.add_argument("--seed", type=int, default=10, help="read seed (bench: 10 + rank main leg, 20 + rank config #5)")
    a = p.parse_args()
    K.load()
    K.set_device(0)
    text = synth.text_3g(a.ref_size) if a.ref_size == 3_000_000_000 else \
        b"".join(synth.text_chunks(a.ref_size))
    reads = synth.gather_reads(text, synth.read_starts(len(text), a.queries, a.qlen, seed=a.seed), a.qlen)
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(a.queries)
    order, first = [], None
    for k, names in ((2, a.backends), (4, a.k4_backends)):
        if not [x for x in names.split(",") if x]:
            continue
        idx = K.Index.build(text, k=k, d=64, gpu=True, host_image=False)
        for b in [x for x in names.split(",") if x]:
            K.set_backend(b)
            K.transfer_to_gpu(idx, q, r)
            lf = []
            for i in range(a.warmup + a.steps):
                K.search(idx, q, r)
                lf.append(K.last_timing()["lf_ms"])
            K.transfer_to_cpu(r)
            res = r.array().copy()
            if first is None:
                first = res
            blocks = K.count_blocks(idx, q)
            # the lines the backend's fetches need (kfmi_count_lines): the
            # structural share of the requests the PMC pass counts
            lines = K.count_lines(idx, q)
            order.append({"backend": b, "k": k, "launches": a.warmup + a.steps, "warmup": a.warmup,
                          "lf_ms_hip_events": round(float(np.mean(lf[a.warmup:])), 4), "distinct_blocks": blocks,
                          "lines_model": lines,
                          "results_equal_first": bool(np.array_equal(res, first))})
            log(order[-1])
            idx.free_gpu()
        idx.close()
    Path(a.order).write_text(json.dumps({"queries": a.queries, "ref_size": a.ref_size, "qlen": a.qlen, "d": 64,
                                         "order": order}, indent=1))


if __name__ == "__main__":
    main()
