#!/usr/bin/env python3
"""LF kernel time per step right after an idle pause vs under sustained load
(dev tool): does the GPU run the memory-bound search faster when it starts
cool?  Prints one JSON line per phase."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "k-step_fm-index_amd")]
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402

K.load()
K.set_device(0)
text = synth.text_3g()
idx = K.Index.build(text, k=2, d=64, gpu=True)
reads = synth.gather_reads(text, synth.read_starts(len(text), 10_000_000, 100, 10), 100)
del text
q = K.Queries.from_array(reads)
r = K.Results.alloc(reads.shape[0])
K.set_backend("task-mid")
K.transfer_to_gpu(idx, q, r)


def phase(name, steps):
    lf = []
    for _ in range(steps):
        K.search(idx, q, r)
        lf.append(round(K.last_timing()["lf_ms"], 3))
    print(json.dumps({"phase": name, "lf_ms": lf}), flush=True)


phase("right after upload", 10)
phase("sustained", 200)
time.sleep(3)
phase("after 3 s idle", 10)
phase("sustained again", 200)
time.sleep(10)
phase("after 10 s idle", 10)
