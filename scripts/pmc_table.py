#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter_collection CSVs (dev tool).

  python scripts/pmc_table.py profiles/r03/pmc_r3s_tcc.csv profiles/r03/pmc_r3s_sq.csv

One column per LF kernel instantiation (task/coop, layout, template args),
one row per counter: the mean over that kernel's launches, in millions.
Launches with a grid under 1M work-items (ftab / remainder builds) are skipped.
"""
from __future__ import annotations

import csv
import re
import sys
from collections import defaultdict


def main(paths):
    agg = defaultdict(lambda: defaultdict(list))
    order = []
    for p in paths:
        for r in csv.DictReader(open(p)):
            if int(r["Grid_Size"]) < 1_000_000:
                continue
            kn = r["Kernel_Name"]
            m = re.search(r"(\w+_kernel)<kfmi::Geo<(\d+), (\d+), (\d+)>((?:, -?\d+)*)>", kn)
            key = f"{m.group(1).replace('_kernel', '')} K{m.group(2)} nb{m.group(3)} lay{m.group(4)}{m.group(5)}" \
                if m else kn[:40]
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] not in order:
                order.append(r["Counter_Name"])
    keys = sorted(agg)
    w = max(26, max(len(k) for k in keys) + 2)
    print("counter (mean per launch, M)".ljust(34) + "".join(k.rjust(w) for k in keys))
    for c in order:
        cells = []
        for k in keys:
            v = agg[k].get(c)
            cells.append((f"{sum(v) / len(v) / 1e6:.2f}" if v else "-").rjust(w))
        print(c.ljust(34) + "".join(cells))


if __name__ == "__main__":
    main(sys.argv[1:])
