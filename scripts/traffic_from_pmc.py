#!/usr/bin/env python3
"""Per-launch fabric read requests of the LF kernel from a rocprofv3 --pmc CSV.

  python scripts/traffic_from_pmc.py <counter_collection.csv> <kernel-substring> \
      --backend task-mid --line-bytes 128 > profiles/traffic.json

Correction (MI355X_MICROARCH.md §HBM, calibrated here by gather_probe,
profiles/r01/pmc_gather_probe_set1.csv): on gfx950 every random line read of
32, 64 or 128 B is tallied as ONE TCC_EA0_RDREQ (FETCH_SIZE counts it as 64 B,
TCC_BUBBLE stays 0), so the bytes are RDREQ x the bytes of the line the layout
fetches (128 for MID128: every LF touches both 64-B halves of its line).
Infinity-Cache hits are included (the counter is at the L2/fabric boundary), so
RDREQ x line bytes is an upper bound on HBM bytes; hbm_bytes_per_launch_excl_
infinity_cache stays null (no rocprofv3 counter on gfx950 splits them off).
"""
import argparse
import csv
import json
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("kernel")
ap.add_argument("--backend", required=True)
ap.add_argument("--line-bytes", type=int, required=True)
ap.add_argument("--queries", type=int, default=10_000_000)
ap.add_argument("--ref-size", type=int, default=3_000_000_000)
a = ap.parse_args()
vals, durs = [], []
for r in csv.DictReader(open(a.csv)):
    if a.kernel in r["Kernel_Name"] and r["Counter_Name"] == "TCC_EA0_RDREQ_sum":
        vals.append(float(r["Counter_Value"]))
        durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
req = statistics.median(vals)
out = {"backend": a.backend, "queries": a.queries, "ref_size": a.ref_size,
       "rdreq_per_launch": int(req), "bytes_per_request": a.line_bytes,
       "request_bytes_upper_bound": int(req * a.line_bytes),
       "hbm_bytes_per_launch_excl_infinity_cache": None,
       "kernel_ms_under_pmc": round(statistics.median(durs), 3),
       "source": a.csv, "launches": len(vals)}
print(json.dumps(out, indent=1))
