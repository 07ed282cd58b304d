#!/usr/bin/env python3
"""Where the K=4 upload time goes (dev tool): 3 Gbase K=4 device-only build,
then transferCPUtoGPU(index) for coop-grp three times (free_gpu between)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402

K.load()
K.set_device(0)
text = synth.text_3g()
t = time.perf_counter()
i4 = K.Index.build(text, k=4, d=64, gpu=True, host_image=False)
print("build_s", round(time.perf_counter() - t, 3), flush=True)
K.set_backend(sys.argv[1] if len(sys.argv) > 1 else "coop-grp")
for i in range(3):
    t = time.perf_counter()
    K.transfer_to_gpu(i4, None, None)
    print("upload_s", round(time.perf_counter() - t, 3), flush=True)
    i4.free_gpu()
