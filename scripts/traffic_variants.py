#!/usr/bin/env python3
"""Per-backend fabric read requests of the LF kernels from one rocprofv3 --pmc
pass over scripts/pmc_variants.py (dev tool).

  python scripts/traffic_variants.py <counter_collection.csv> <order.json> \
      --source "<what/where>" > profiles/r04/traffic_variants.json

The LF launches (task_kernel / coop_kernel with a grid covering the batch) are
taken in dispatch order and cut into the order file's (backend, K, launches)
runs; each run's kernel name must carry the backend's kernel family and Geo<K,
NB, layout>.  Per backend: median TCC_EA0_RDREQ_sum and TCC_REQ_sum over its
timed launches (the run's first `warmup` skipped), and the median kernel time
under the PMC pass.  On gfx950 one random line read of up to 128 B is one
TCC_EA0_RDREQ (scripts/traffic_from_pmc.py); Infinity-Cache hits are counted
too, so requests x 128 B bound the HBM bytes from above.
"""
import argparse
import csv
import json
import re
import statistics

# layout ids 2 (packed) and 4 (ac128) name the layouts retired in round 6; kept to read older passes
LAYOUT = {"task": 0, "coop": 0, "task-ac": 1, "coop-ac": 1, "task-packed": 2, "coop-packed": 2, "task-mid": 3,
          "coop-mid": 3, "task-ac128": 4, "coop-ac128": 4, "task-ac-mid": 5, "coop-ac-mid": 5, "task-grp": 6,
          "coop-grp": 6}

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("order")
ap.add_argument("--source", required=True)
a = ap.parse_args()
order = json.load(open(a.order))
nq = order["queries"]
disp = {}
for r in csv.DictReader(open(a.csv)):
    name = r["Kernel_Name"]
    if not re.search(r"kfmi::(task|coop)_kernel<", name):
        continue
    g = int(r["Grid_Size"])
    if not (nq <= g < nq + 64 * 64):
        continue
    d = disp.setdefault(int(r["Dispatch_Id"]), {"name": name, "start": int(r["Start_Timestamp"]),
                                                "end": int(r["End_Timestamp"])})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
rows = [disp[k] for k in sorted(disp)]
out = {"config": {"queries": nq, "ref_size": order["ref_size"], "qlen": order["qlen"], "d": order["d"]},
       "source": a.source, "bytes_per_request": 128, "backends": {}}
i = 0
for o in order["order"]:
    run = rows[i:i + o["launches"]]
    i += o["launches"]
    assert len(run) == o["launches"], (o, len(run))
    fam = "coop" if o["backend"].startswith("coop") else "task"
    m = re.search(r"kfmi::(task|coop)_kernel<kfmi::Geo<(\d+), (\d+), (\d+)>", run[0]["name"])
    assert m and m.group(1) == fam and int(m.group(2)) == o["k"] and int(m.group(4)) == LAYOUT[o["backend"]], \
        (o, run[0]["name"])
    assert all(x["name"] == run[0]["name"] for x in run), o
    timed = run[o["warmup"]:]
    req = statistics.median(x["TCC_EA0_RDREQ_sum"] for x in timed)
    tcc = statistics.median(x["TCC_REQ_sum"] for x in timed) if "TCC_REQ_sum" in timed[0] else None
    ms = statistics.median((x["end"] - x["start"]) / 1e6 for x in timed)
    out["backends"][f"{o['backend']}@k{o['k']}"] = {
        "kernel": run[0]["name"].split("(")[0], "rdreq_per_launch": int(req),
        "line_requests_per_query": round(req / nq, 2), "tcc_req_per_launch": int(tcc) if tcc else None,
        "kernel_ms_under_pmc": round(ms, 3), "lf_ms_hip_events_same_run": o["lf_ms_hip_events"],
        "distinct_blocks": o["distinct_blocks"], "launches_timed": len(timed),
        **({"model_lines_per_query": round(o["lines_model"]["lines"] / nq, 2),
            "model_counter_outside_line_per_end": round(o["lines_model"]["counter_outside_planes_line"]
                                                         / o["lines_model"]["ends_fetched"], 4),
            "model_line_local_per_end": round(o["lines_model"]["line_local_ends"] / o["lines_model"]["ends_fetched"], 4),
            "model_ends_per_query": round(o["lines_model"]["ends_fetched"] / nq, 2)} if "lines_model" in o else {}),
        "request_bytes_upper_bound": int(req * 128)}
assert i == len(rows), (i, len(rows))
print(json.dumps(out, indent=1))
