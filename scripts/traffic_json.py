#!/usr/bin/env python3
"""Refresh profiles/traffic.json -- the headline kernel's counter record that
bench.py attaches to N = 1 lines of the same config -- from this round's PMC
passes (dev tool):

  python scripts/traffic_json.py --variants profiles/r05/traffic_variants.json \
      --fetch profiles/r05/pmc_<tag>_lf_fetch.jsonl --sizes profiles/r05/pmc_<tag>_lf_sizes.jsonl \
      --tag r05 > profiles/traffic.json.new

rdreq_per_launch from the per-backend pass (task-mid@k2); FETCH_SIZE (KB per
launch) from its own pass, doubled per MI355X_MICROARCH.md's gfx950 note;
request sizes from a third pass (every request must be 128 B for the doubling
to be exact).  The replay counts of the previous file are kept (the replay
probe did not change).
"""
import argparse
import json
import statistics
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("--variants", required=True)
ap.add_argument("--fetch", required=True)
ap.add_argument("--sizes", required=True)
ap.add_argument("--old", default="profiles/traffic.json")
ap.add_argument("--tag", required=True)
a = ap.parse_args()


def lf_rows(fn):
    """The LF runs of a pmc_summary.py file (one JSON line per run of launches
    of one kernel and grid): the 10M-read task-mid runs, median counters."""
    rows = [json.loads(x) for x in Path(fn).read_text().splitlines() if x.strip()]
    return [r for r in rows if "task_kernel<Geo<2, 2, 3>" in r["kernel"].replace("kfmi::", "")]


def counter(rows, name):
    vals = []
    for r in rows:
        for k, v in r.items():
            if k == name or k == name + "_sum":
                vals.append(float(v))
    return statistics.median(vals)


tv = json.loads(Path(a.variants).read_text())
row = tv["backends"]["task-mid@k2"]
old = json.loads(Path(a.old).read_text())
fetch = lf_rows(a.fetch)
sizes = lf_rows(a.sizes)
fkb = counter(fetch, "FETCH_SIZE")
sz = {k: int(counter(sizes, k)) for k in ("TCC_EA0_RDREQ_128B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_32B",
                                          "TCC_EA0_RDREQ")}
out = dict(old)
out.update({
    "rdreq_per_launch": row["rdreq_per_launch"], "tcc_req_per_launch": row.get("tcc_req_per_launch"),
    "kernel_ms_under_pmc": row["kernel_ms_under_pmc"], "request_bytes_upper_bound": row["rdreq_per_launch"] * 128,
    "source": f"{tv['source']}; task-mid@k2 row of {a.variants}",
    "fetch_size_kb_per_launch": fkb, "fetch_size_corrected_bytes_per_launch": round(fkb * 2048),
    "request_sizes_per_launch": sz,
    "fetch_size_source": f"{a.fetch} and {a.sizes} (scripts/box/pmc.sh <tag> fetch: rocprofv3 --pmc FETCH_SIZE, "
                         f"then the TCC_EA0_RDREQ size counters, separate passes over scripts/pmc_variants.py "
                         f"--backends task-mid; median over the launches after the first), round {a.tag}",
})
print(json.dumps(out, indent=1))
