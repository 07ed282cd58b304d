"""Walk-check cost (locate's and the derivation's once-per-device-copy check
that every LF_K walk ends at a '$' row, csrc/hip/kfmi_search.hip
check_lf_walks): the first locate call on a fresh device copy, full pointer
jumping (mode 1) against the sampled check (mode 2), on a synthetic index.
  python scripts/walk_check_probe.py [bases=3e9] [out.json]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
import numpy as np
import kstep_fmi as K
from kstep_fmi import synth

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 3_000_000_000
K.set_device(0)
t0 = time.time()
text = b"".join(synth.text_chunks(n))
idx = K.Index.build(text, k=2, d=64, gpu=True, sa_rate=32)
reads = synth.gather_reads(text, synth.read_starts(len(text), 1000, 100, seed=3), 100)
del text
print(f"setup {time.time() - t0:.0f}s", flush=True)
rows = []
for mode in (2, 1, 2):
    K.set_walk_check(mode)
    idx.free_gpu()
    K.set_backend("task-mid")
    K.transfer_to_gpu(idx, None, None)
    K.search_array(idx, reads[:10], "task-mid")             # upload done, check not yet run
    t = time.perf_counter()
    res, off, pos = K.locate_array(idx, reads, "task-mid")
    first = time.perf_counter() - t
    t = time.perf_counter()
    K.locate_array(idx, reads, "task-mid")
    again = time.perf_counter() - t
    row = {"bases": n, "mode": {1: "full", 2: "sampled"}[mode], "decided_by": K.walk_check_last(),
           "first_locate_s": round(first, 3), "next_locate_s": round(again, 4),
           "check_s": round(first - again, 3), "positions": int(off[-1])}
    print(json.dumps(row), flush=True)
    rows.append(row)
K.set_walk_check(0)
if len(sys.argv) > 2:
    Path(sys.argv[2]).write_text(json.dumps(rows, indent=1) + "\n")
