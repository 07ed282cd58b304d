#!/usr/bin/env python3
"""Time kfmi_derive_index_gpu on the 3 Gbase bench index (dev tool; run under
rocprofv3 --kernel-trace --stats to see its launches).

  python3 scripts/derive_probe.py [--ref-size N]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "k-step_fm-index_amd")]
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ref-size", type=int, default=3_000_000_000)
ap.add_argument("--host-image", type=int, default=1)
a = ap.parse_args()
K.load()
K.set_device(0)
text = synth.text_3g(a.ref_size) if a.ref_size == 3_000_000_000 else b"".join(synth.text_chunks(a.ref_size))
t = time.perf_counter()
i2 = K.Index.build(text, k=2, d=64, gpu=True, host_image=bool(a.host_image))
out = {"build_k2_s": round(time.perf_counter() - t, 3)}
for rep in range(2):
    t = time.perf_counter()
    i4 = i2.derive(4)
    out[f"derive_s_{rep}"] = round(time.perf_counter() - t, 3)
    i4.close()
t = time.perf_counter()
i4b = K.Index.build(text, k=4, d=64, gpu=True, host_image=False)
out["build_k4_s"] = round(time.perf_counter() - t, 3)
print(json.dumps(out), flush=True)
