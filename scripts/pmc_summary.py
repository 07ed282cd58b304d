#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --pmc counter_collection.csv (dev tool).

  python3 scripts/pmc_summary.py <counter_collection.csv> [--skip-first]

Consecutive dispatches of the same kernel form a run (gather_probe launches
each kind twice, warm-up then timed; the LF kernel once per search); per run:
the number of dispatches, the median of every counter over them (the first
dropped with --skip-first when the run has more than one) and the median
duration under the PMC pass.  One JSON line per run, in dispatch order.
"""
import argparse
import csv
import json
import re
import statistics


def runs(fn: str) -> list:
    disp = {}
    for row in csv.DictReader(open(fn)):
        d = disp.setdefault(int(row["Dispatch_Id"]), {
            "name": row["Kernel_Name"], "grid": int(row["Grid_Size"]),
            "ms": (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6, "c": {}})
        d["c"][row["Counter_Name"]] = float(row["Counter_Value"])
    out = []
    for k in sorted(disp):
        d = disp[k]
        if out and out[-1][0]["name"] == d["name"] and out[-1][0]["grid"] == d["grid"]:
            out[-1].append(d)
        else:
            out.append([d])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip-first", action="store_true")
    a = ap.parse_args()
    for i, run in enumerate(runs(a.csv)):
        rows = run[1:] if a.skip_first and len(run) > 1 else run
        names = sorted({c for x in rows for c in x["c"]})
        short = re.sub(r"\(anonymous namespace\)::|kfmi::", "", run[0]["name"]).split("(")[0]
        print(json.dumps({"run": i, "kernel": short, "grid": run[0]["grid"], "dispatches": len(rows),
                          "ms": round(statistics.median(x["ms"] for x in rows), 4),
                          **{c: statistics.median(x["c"].get(c, 0.0) for x in rows) for c in names}}))


if __name__ == "__main__":
    main()
