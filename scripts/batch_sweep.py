#!/usr/bin/env python3
"""Per-call cost of searchIndexGPU vs batch size (dev tool): 3 Gbase index,
task-mid / coop-mid / coop-grp (K=4), batches of 1K .. 10M reads already on the
device; wall time per call (Python ctypes call included) and the LF kernel's
HIP-event time."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402

K.load()
K.set_device(0)
text = synth.text_3g()
reads = synth.gather_reads(text, synth.read_starts(len(text), 10_000_000, 100, 10), 100)
idx = {2: K.Index.build(text, k=2, d=64, gpu=True), 4: K.Index.build(text, k=4, d=64, gpu=True, host_image=False)}
for k, backends in ((2, ("task-mid", "coop-mid")), (4, ("coop-grp",))):
    for b in backends:
        K.set_backend(b)
        for n in (1_000, 4_000, 16_000, 64_000, 256_000, 1_000_000, 10_000_000):
            q = K.Queries.from_array(np.ascontiguousarray(reads[:n]))
            r = K.Results.alloc(n)
            K.transfer_to_gpu(idx[k], q, r)
            calls = max(5, min(200, 20_000_000 // n))
            for _ in range(3):
                K.search(idx[k], q, r)
            lf = []
            t0 = time.perf_counter()
            for _ in range(calls):
                K.search(idx[k], q, r)
                lf.append(K.last_timing()["lf_ms"])
            wall = (time.perf_counter() - t0) / calls
            print(json.dumps({"k": k, "backend": b, "reads": n, "calls": calls, "call_us": round(wall * 1e6, 1),
                              "lf_us": round(float(np.median(lf)) * 1e3, 1),
                              "mqps": round(n / wall / 1e6, 1)}), flush=True)
            q.close()
            r.close()
        # several host threads, each its own small batches (per-thread streams)
        import threading
        for n in (1_000, 16_000, 64_000):
            for nt in (1, 2, 4, 8):
                qs = [K.Queries.from_array(np.ascontiguousarray(reads[j * n:(j + 1) * n])) for j in range(nt)]
                rs = [K.Results.alloc(n) for _ in range(nt)]
                for j in range(nt):
                    K.transfer_to_gpu(idx[k], qs[j], rs[j])
                calls = max(20, min(400, 4_000_000 // n))

                def work(j):
                    K.set_device(0)
                    K.set_backend(b)
                    for _ in range(calls):
                        K.search(idx[k], qs[j], rs[j])
                th = [threading.Thread(target=work, args=(j,)) for j in range(nt)]
                t0 = time.perf_counter()
                for x in th:
                    x.start()
                for x in th:
                    x.join()
                wall = time.perf_counter() - t0
                print(json.dumps({"k": k, "backend": b, "reads_per_batch": n, "threads": nt, "calls_per_thread": calls,
                                  "mqps": round(nt * calls * n / wall / 1e6, 1)}), flush=True)
                for x in qs + rs:
                    x.close()
        idx[k].free_gpu()
