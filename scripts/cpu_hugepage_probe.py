#!/usr/bin/env python3
"""searchIndexCPU on the bench's 3 Gbase index with the host image on 2 MB
pages (default) or 4 KB pages (KFMI_HUGEPAGES=0) -- dev tool, DESIGN.md 2b.

  KFMI_HUGEPAGES=0|1 python3 scripts/cpu_hugepage_probe.py [--reads 2000000] [--threads 16]

The 3 Gbase recipe text, its K = 2 index built on the device with the host
image fetched (kfmi_host_entries: the allocation this probes), 2M of the
bench's reads; one JSON line: Mq/s at the thread count (best of 3), and the
AnonHugePages of the process."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reads", type=int, default=2_000_000)
ap.add_argument("--threads", type=int, default=16)
a = ap.parse_args()
K.load()
K.set_device(0)
text = synth.text_3g()
idx = K.Index.build(text, k=2, d=64, gpu=True, host_image=False)
reads = synth.gather_reads(text, synth.read_starts(len(text), a.reads, 100, seed=10), 100)
del text
K.search_cpu_array(idx, reads[:1000], nthreads=a.threads)      # fetches the host image
best = 0.0
for _ in range(3):
    t = time.perf_counter()
    K.search_cpu_array(idx, reads, nthreads=a.threads)
    best = max(best, a.reads / (time.perf_counter() - t) / 1e6)
huge = [ln.split()[1] for ln in open("/proc/self/smaps_rollup") if ln.startswith("AnonHugePages")]
print(json.dumps({"hugepages_env": os.environ.get("KFMI_HUGEPAGES", "1"), "threads": a.threads, "reads": a.reads,
                  "mqps": round(best, 3), "anon_huge_kb": int(huge[0]) if huge else None}), flush=True)
