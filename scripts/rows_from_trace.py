#!/usr/bin/env python3
"""Every bench row's LF kernel time from a rocprofv3 kernel trace of the same
bench.py command, and the row's algorithmic-HBM fraction recomputed from it
(each row's `frac` must reproduce from a rocprof summary).

  python scripts/rows_from_trace.py --trace <..._kernel_trace.csv> \
      --detail gpurun_out/bench_detail_n1.json > profiles/r05/rows_<tag>.json

bench.py records, per row, where its timed launches sit (`launches`: kernel
name prefix, the batch size its grid covers, and [first, first + count) among
that kernel's launches over that batch in dispatch order).  Per row this
prints the rocprof mean duration of those launches, the bench's HIP-event LF
time, and bytes_per_launch / rocprof time / 8 TB/s beside the bench's frac.
"""
import argparse
import csv
import json
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("--trace", required=True)
ap.add_argument("--detail", required=True)
a = ap.parse_args()

det = json.load(open(a.detail))
V = det.get("variants") or {}
rows = {}


def add(name, rec, rf=None):
    if not rec or "launches" not in rec:
        return
    rf = rf if rf is not None else (rec.get("roofline") or rec)
    rows[name] = {"launches": rec["launches"], "bytes_per_launch": rf.get("bytes_per_launch"),
                  "lf_ms_hip_events": rf.get("lf_ms", rec.get("lf_ms")), "frac_bench": rf.get("frac")}


add("main:" + det["config"]["backend"], det["roofline"], det["roofline"])
for b, v in V.items():
    if isinstance(v, dict) and "launches" in v and b not in ("config1_64mbase", "config5", "kstep4"):
        add(b, v)
add("config1", V.get("config1_64mbase"), V.get("config1_64mbase"))
if V.get("config5"):
    c5 = V["config5"]
    add("config5", dict(c5.get("roofline") or {}, launches=c5.get("launches")) if c5.get("launches") else None)
k4 = V.get("kstep4") or {}
if k4.get("launches"):
    add("k4:coop-grp", dict(k4.get("roofline") or {}, launches=k4["launches"], lf_ms=k4.get("lf_ms")))
if (k4.get("config5") or {}).get("launches"):
    c = k4["config5"]
    add("k4:config5", dict(c.get("roofline") or {}, launches=c["launches"]))

trace = list(csv.DictReader(open(a.trace)))
gkey = "Grid_Size_X" if "Grid_Size_X" in trace[0] else "Grid_Size"
out = {"trace": a.trace, "detail": a.detail, "rows": {}}
for name, r in rows.items():
    sp = r["launches"]
    sel = [t for t in trace if sp["kernel"] in t["Kernel_Name"] and sp["num"] <= int(t[gkey]) < sp["num"] + 4096]
    sel.sort(key=lambda t: int(t["Start_Timestamp"]))
    timed = sel[sp["first"]:sp["first"] + sp["count"]]
    row = {"kernel": sp["kernel"], "launches_found": len(sel), "timed": len(timed)}
    if len(timed) == sp["count"] and timed:
        ms = statistics.mean((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6 for t in timed)
        row.update({"rocprof_avg_ms": round(ms, 4), "lf_ms_hip_events": r["lf_ms_hip_events"],
                    "bytes_per_launch": r["bytes_per_launch"], "frac_bench": r["frac_bench"]})
        if r["bytes_per_launch"]:
            row["frac_rocprof"] = round(r["bytes_per_launch"] / (ms / 1e3) / 1e9 / 8000.0, 4)
    out["rows"][name] = row
print(json.dumps(out, indent=1))
