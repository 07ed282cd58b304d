#!/usr/bin/env python3
"""Host contention of the streamed search (kfmi_search_stream) when several
ranks share one host: P worker processes start together (file barrier), each
streams its own 10M x 150 bp reads (config #5's per-GPU shard shape) host
memory -> host results through every transfer mode in turn -- adaptive (the
default per-chunk cost model), always host-packed, always ASCII -- several
rounds, interleaved, with LOCAL_WORLD_SIZE=P as torchrun would set it (the
library then splits the host's CPU share among the ranks, kfmi_host_threads).

  python scripts/stream_contention.py --procs 1 2 --out gpurun_out/stream_contention.jsonl

On a one-GPU box the P processes also share the card and its PCIe link, so
the ASCII mode is charged more than on an 8-GPU node (one link per rank);
the workers say so to the library's cost model (KFMI_LINK_SHARERS=P); the
host-side numbers (packing time, staging) are what this measures.
Summary per (P, input, mode): every rank's median wall over rounds 1.. (round
0 -- first-touch of the output arrays and staging buffers -- excluded), then
the slowest rank.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

WORKER = r"""
import json, os, sys, time
from pathlib import Path
sys.path[:0] = [%(root)r, %(pkg)r]
import numpy as np
import kstep_fmi as K
from kstep_fmi import synth
rank, procs, bdir, rounds, ref_size, nq, m = %(args)s

def barrier(tag):
    Path(bdir, f"{tag}.{rank}").touch()
    while len(list(Path(bdir).glob(f"{tag}.*"))) < procs:
        time.sleep(0.002)

K.load()
K.set_device(0)
rng = np.random.default_rng(5)
text = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=ref_size, dtype=np.uint8)].tobytes()
idx = K.Index.build(text, k=2, d=64, gpu=True)
reads = synth.gather_reads(text, synth.read_starts(len(text), nq, m, seed=20 + rank), m)
K.set_backend("task-mid")
K.transfer_to_gpu(idx, None, None)
want = K.search_array(idx, reads[:200_000])
K.transfer_to_gpu(idx, None, None)
pin = K.pinned_empty(reads.shape, np.uint8)
pin[:] = reads
res = np.zeros(2 * nq, dtype=np.uint32)          # one pageable result buffer, touched once (as bench.py does)
rows = []
for kind, src in (("pageable", reads), ("pinned", pin)):
    for mode in ("2", "1", "0"):
        os.environ["KFMI_STREAM_HOSTPACK"] = mode
        K.search_stream(idx, src[:500_000])                   # warm-up: buffers, cost model
    for r in range(rounds):
        for mode in ("2", "1", "0"):
            os.environ["KFMI_STREAM_HOSTPACK"] = mode
            barrier(f"{kind}.{r}.{mode}")
            t = time.perf_counter()
            out = K.search_stream(idx, src, out=res)
            w = time.perf_counter() - t
            lt = K.last_timing()
            rows.append({"rank": rank, "procs": procs, "input": kind, "round": r,
                         "mode": {"2": "adaptive", "1": "host-packed", "0": "ascii"}[mode],
                         "wall_ms": round(w * 1e3, 2), "mqps": round(nq / w / 1e6, 1),
                         "host_ms": round(lt["pack_ms"], 2), "wait_ms": round(lt["lf_ms"], 2),
                         "hostpacked_fraction": round(K.load().kfmi_stream_hostpacked_fraction(), 3),
                         "host_threads": K.host_threads(),
                         "ok": bool(np.array_equal(out[:400_000], want))})
print(json.dumps(rows))
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--rounds", type=int, default=7, help="rounds per mode; round 0 is a warm-up, not summarised")
    ap.add_argument("--ref-size", type=int, default=1_000_000_000)
    ap.add_argument("--queries", type=int, default=10_000_000)
    ap.add_argument("--qlen", type=int, default=150)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "stream_contention.jsonl"))
    a = ap.parse_args()
    summary = []
    with open(a.out, "w") as fo:
        for P in a.procs:
            with tempfile.TemporaryDirectory() as bdir:
                ps = []
                for rank in range(P):
                    code = WORKER % {"root": str(ROOT), "pkg": str(ROOT / "k-step_fm-index_amd"),
                                     "args": repr((rank, P, bdir, a.rounds, a.ref_size, a.queries, a.qlen))}
                    # the P processes share this one card's PCIe link (KFMI_LINK_SHARERS: the
                    # streamed search's link cost model; on an 8-GPU node each rank has its own)
                    env = dict(os.environ, LOCAL_WORLD_SIZE=str(P), LOCAL_RANK=str(rank), KFMI_LINK_SHARERS=str(P))
                    ps.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                               stderr=subprocess.PIPE, text=True))
                rows = []
                for p in ps:
                    out, err = p.communicate(timeout=900)
                    if p.returncode != 0:
                        print(err[-3000:], file=sys.stderr)
                        return 1
                    rows += json.loads(out.strip().splitlines()[-1])
            for r in rows:
                fo.write(json.dumps(r) + "\n")
            for kind in ("pageable", "pinned"):
                per = {}
                for mode in ("adaptive", "host-packed", "ascii"):
                    sel = [r for r in rows if r["input"] == kind and r["mode"] == mode and r["round"] > 0]
                    # per-rank median over rounds, then the slowest rank (the job's wall)
                    med = []
                    for rank in range(P):
                        w = sorted(x["wall_ms"] for x in sel if x["rank"] == rank)
                        med.append(w[len(w) // 2])
                    per[mode] = {"wall_ms_slowest_rank": max(med),
                                 "mqps_per_rank": round(a.queries / (max(med) / 1e3) / 1e6, 1),
                                 "hostpacked_fraction": round(sum(x["hostpacked_fraction"] for x in sel) / len(sel), 3),
                                 "all_ok": all(x["ok"] for x in sel)}
                best_fixed = min(per["host-packed"]["wall_ms_slowest_rank"], per["ascii"]["wall_ms_slowest_rank"])
                s = {"procs": P, "input": kind, "host_threads_per_rank": rows[0]["host_threads"], "modes": per,
                     "adaptive_vs_best_fixed": round(per["adaptive"]["wall_ms_slowest_rank"] / best_fixed, 3)}
                summary.append(s)
                fo.write(json.dumps({"summary": s}) + "\n")
                print(json.dumps(s), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
