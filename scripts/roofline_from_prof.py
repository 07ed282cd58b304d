#!/usr/bin/env python3
"""Roofline of the timed LF launches of one bench.py run, from its rocprofv3
kernel trace and (optionally) a --pmc pass of the SAME command.

  python scripts/roofline_from_prof.py --trace <..._kernel_trace.csv> \
      --bench <bench.json> [--pmc <..._counter_collection.csv>] \
      --warmup 5 --steps 20 > profiles/r02/roofline.json

The LF kernel of the bench's backend is launched first by the main leg:
warmup launches, then exactly `steps` timed launches (later legs -- variants,
config #1, locate -- launch kernels of the same name with other grids or
after them).  So the timed launches are dispatches [warmup, warmup + steps) of
the kernel whose grid covers the rank's queries.  Traffic: TCC_EA0_RDREQ per
launch (every MID128 LF request is one 128-B line; on gfx950 one random line
read of up to 128 B is one RDREQ, scripts/traffic_from_pmc.py), taken over the
same dispatch indices of the PMC pass; x 128 B it bounds the HBM bytes from
above (Infinity-Cache hits are counted too).
"""
import argparse
import csv
import json
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("--trace", required=True)
ap.add_argument("--bench", required=True)
ap.add_argument("--pmc")
ap.add_argument("--kernel", default="task_kernel")
ap.add_argument("--warmup", type=int, required=True)
ap.add_argument("--steps", type=int, required=True)
ap.add_argument("--line-bytes", type=int, default=128)
a = ap.parse_args()

bench = json.loads(open(a.bench).read().strip().splitlines()[-1])
nq = bench["config"]["queries_per_gpu"]
grid = ((nq + 255) // 256) * 256


def lf_rows(rows, grid_key):
    return [r for r in rows if a.kernel in r["Kernel_Name"] and int(r[grid_key]) == grid]


tr = lf_rows(list(csv.DictReader(open(a.trace))), "Grid_Size_X")
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
timed = tr[a.warmup:a.warmup + a.steps]
assert len(timed) == a.steps, (len(tr), a.warmup, a.steps)
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
avg_ms = statistics.mean(durs)
bytes_alg = bench["roofline"]["bytes_per_launch"]
out = {"command": "python3 bench.py --gpus 1 --steps %d --warmup %d" % (a.steps, a.warmup),
       "kernel": timed[0]["Kernel_Name"], "grid": grid, "launches": len(timed),
       "avg_ms": round(avg_ms, 4), "min_ms": round(min(durs), 4), "max_ms": round(max(durs), 4),
       "bench_ms_per_step": bench["ms_per_step"], "bench_lf_ms_hip_events": bench["roofline"]["lf_ms"],
       "algorithmic_bytes_per_launch": bytes_alg,
       "achieved_GBs": round(bytes_alg / (avg_ms / 1e3) / 1e9, 1),
       "frac": round(bytes_alg / (avg_ms / 1e3) / 1e9 / 8000.0, 4),
       "trace": a.trace}
if a.pmc:
    pm = [r for r in csv.DictReader(open(a.pmc))
          if a.kernel in r["Kernel_Name"] and int(r["Grid_Size"]) == grid]
    by_disp = {}
    for r in pm:
        by_disp.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    disp = sorted(by_disp)[a.warmup:a.warmup + a.steps]
    req = statistics.median(by_disp[d]["TCC_EA0_RDREQ_sum"] for d in disp)
    out.update({"pmc": a.pmc, "pmc_launches": len(disp), "rdreq_per_launch": int(req),
                # requests x line bytes counts Infinity-Cache hits too: an upper bound on HBM bytes
                "request_bytes_upper_bound_per_launch": int(req * a.line_bytes),
                "rdreq_per_query": round(req / nq, 2),
                "line_requests_G_per_s": round(req / (avg_ms / 1e3) / 1e9, 2)})
    for c in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_WRREQ_sum"):
        if all(c in by_disp[d] for d in disp):
            out[c] = int(statistics.median(by_disp[d][c] for d in disp))
print(json.dumps(out, indent=1))
