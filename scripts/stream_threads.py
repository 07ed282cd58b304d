"""Config #5's host-to-host leg (10M x 150 bp per GPU, 3 Gbase index,
kfmi_search_stream from pageable reads into pageable results) at the host
thread counts an 8-rank node leaves each rank (KFMI_HOST_THREADS=2: the
16-CPU quota over 8 ranks) and at 16, per streaming mode:
  adaptive        KFMI_STREAM_HOSTPACK unset: per-chunk host packing or ASCII
  hostpack        every chunk packed on the host (qpack.c)
  ascii           every chunk as ASCII through pinned staging, packed on the device
  ascii-direct    ASCII DMA'd from the caller's pageable reads (KFMI_STREAM_DIRECT=1)
  adaptive-direct the adaptive chooser with direct ASCII
  pinned-*        the reads in pinned host memory (the results stay pageable)
One child process per row (the host pool and the knobs are read once per
process); the index and reads are made once and shared through files.
  python scripts/stream_threads.py [out.jsonl]
"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))
TMP = Path(os.environ.get("TMPDIR", "/tmp"))
IDX, READS = TMP / "st_idx.fmi", TMP / "st_reads.npy"
ROWS = [
    ("adaptive", {}), ("hostpack", {"KFMI_STREAM_HOSTPACK": "1"}), ("ascii", {"KFMI_STREAM_HOSTPACK": "0"}),
    ("ascii-direct", {"KFMI_STREAM_HOSTPACK": "0", "KFMI_STREAM_DIRECT": "1"}),
    ("adaptive-direct", {"KFMI_STREAM_DIRECT": "1"}),
    ("pinned-adaptive", {"ST_PINNED": "1"}), ("pinned-hostpack", {"ST_PINNED": "1", "KFMI_STREAM_HOSTPACK": "1"}),
    ("pinned-ascii", {"ST_PINNED": "1", "KFMI_STREAM_HOSTPACK": "0"}),
]


def child():
    import numpy as np
    import kstep_fmi as K
    K.set_device(0)
    idx = K.Index.load(IDX)
    reads = np.load(READS, mmap_mode="r")
    if os.environ.get("ST_PINNED") == "1":         # reads already in pinned host memory (kfmi_host_alloc)
        pin = K.pinned_empty(reads.shape, np.uint8)
        pin[:] = reads
        reads = pin
    else:
        reads = np.ascontiguousarray(reads)        # pageable, in RAM
    K.set_backend("task-mid")
    K.transfer_to_gpu(idx, None, None)
    out = np.empty(2 * reads.shape[0], dtype=np.uint32)
    K.search_stream(idx, reads, out=out)           # warm-up: buffers, rates
    want = out.copy()
    walls = []
    for _ in range(3):
        t = time.perf_counter()
        K.search_stream(idx, reads, out=out)
        walls.append(time.perf_counter() - t)
    lt = K.last_timing()
    w = min(walls)
    print(json.dumps({"mqps": round(reads.shape[0] / w / 1e6, 1), "wall_ms": round(w * 1e3, 1),
                      "walls_ms": [round(x * 1e3, 1) for x in walls], "host_ms": round(lt["pack_ms"], 1),
                      "wait_ms": round(lt["lf_ms"], 1), "host_threads": K.host_threads(),
                      "hostpacked_fraction": round(K.load().kfmi_stream_hostpacked_fraction(), 3),
                      "stable": bool(np.array_equal(out, want))}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child()
    outp = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "gpurun_out" / "stream_threads.jsonl"
    import numpy as np
    import kstep_fmi as K
    from kstep_fmi import synth
    t0 = time.time()
    text = b"".join(synth.text_chunks(3_000_000_000))
    K.set_device(0)
    idx = K.Index.build(text, k=2, d=64, gpu=True)
    idx.image().tofile(IDX)
    idx.close()
    reads = synth.gather_reads(text, synth.read_starts(len(text), 10_000_000, 150, seed=20), 150)
    np.save(READS, reads)
    del text, reads
    print(f"setup {time.time() - t0:.0f}s", flush=True)
    with open(outp, "w") as f:
        rows = ROWS
        if os.environ.get("ST_ROWS") == "chunks":   # chunk sizes of the pinned modes
            rows = [(f"pinned-{m}-c{c}", dict({"ST_PINNED": "1", "KFMI_STREAM_CHUNK": str(1 << c)}, **e))
                    for m, e in (("adaptive", {}), ("ascii", {"KFMI_STREAM_HOSTPACK": "0"}),
                                 ("hostpack", {"KFMI_STREAM_HOSTPACK": "1"}))
                    for c in (16, 18, 20, 21)]
        for threads in os.environ.get("ST_THREADS", "2,16").split(","):
            for name, env in rows:
                e = dict(os.environ, KFMI_HOST_THREADS=threads, **env)
                p = subprocess.run([sys.executable, __file__, "--child"], env=e, capture_output=True, text=True,
                                   timeout=240)
                row = {"threads": int(threads), "mode": name}
                try:
                    row.update(json.loads(p.stdout.strip().splitlines()[-1]))
                except (IndexError, json.JSONDecodeError):
                    row["error"] = (p.stdout[-300:] + p.stderr[-300:]).strip()
                print(json.dumps(row), flush=True)
                f.write(json.dumps(row) + "\n")
                if p.returncode:
                    return p.returncode
    IDX.unlink(missing_ok=True)
    READS.unlink(missing_ok=True)


if __name__ == "__main__":
    sys.exit(main() or 0)
