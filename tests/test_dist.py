"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 bench path:
rank/device mapping, per-rank read shards, barrier + max-over-ranks timing and
the whole-job throughput aggregation.  The data path itself has no collective
(each rank holds an index replica and searches its own shard)."""
import json
import os
import socket
import subprocess
import sys
import textwrap

from util import REPO

WORKER = textwrap.dedent(r"""
    import json, os, sys, time
    sys.path.insert(0, %(repo)r); sys.path.insert(0, %(pkg)r)
    import numpy as np
    import bench
    from kstep_fmi import synth
    D = bench.Dist(2)
    text = np.random.default_rng(5).choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=100_000).tobytes()
    st = synth.read_starts(len(text), 1000, 100, seed=10 + D.rank)
    reads = synth.gather_reads(text, st, 100)
    D.barrier()
    t0 = time.perf_counter()
    time.sleep(0.05 * (D.rank + 1))          # rank 1 is the slow one
    D.barrier()
    el = time.perf_counter() - t0
    el_max = D.max(el)
    total = D.sum(float(reads.shape[0]))
    # per-rank rows as bench.py gathers them (rank 1 reports a failed parity sample)
    rows = D.gather({"rank": D.rank, "device": D.local, "queries": int(reads.shape[0]),
                     "lf_ms": 9.0 + D.rank, "step_ms": 9.5 + D.rank, "elapsed_s": el,
                     "parity_ok": D.rank == 0, "parity_sample": 100})
    agg = bench.aggregate_ranks(rows)
    out = json.dumps({"rank": D.rank, "world": D.world, "local": D.local, "el": el, "el_max": el_max,
                      "total": total, "first": reads[0].tobytes().decode(), "start0": int(st[0]), "agg": agg})
    with open("rank%%d.json" %% D.rank, "w") as f:
        f.write(out)
    D.close()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_bench_plumbing(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER % {"repo": str(REPO), "pkg": str(REPO / "k-step_fm-index_amd")})
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script)]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240, cwd=str(tmp_path))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rows = [json.loads((tmp_path / f"rank{i}.json").read_text()) for i in range(2)]
    assert sorted(r["rank"] for r in rows) == [0, 1]
    for r in rows:
        assert r["world"] == 2 and r["local"] == r["rank"]
        assert r["total"] == 2000.0                       # whole-job queries
        assert abs(r["el_max"] - max(x["el"] for x in rows)) < 1e-9
    # disjoint, deterministic shards: rank r uses read seed 10 + r
    assert rows[0]["start0"] != rows[1]["start0"]
    # per-rank aggregation (bench.py "ranks"): same view on every rank
    for r in rows:
        agg = r["agg"]
        assert agg == rows[0]["agg"]
        assert agg["n_ranks"] == 2 and agg["queries"] == 2000
        assert agg["lf_ms_min"] == 9.0 and agg["lf_ms_max"] == 10.0
        assert agg["step_ms_min"] == 9.5 and agg["step_ms_max"] == 10.5
        assert [x["rank"] for x in agg["ranks"]] == [0, 1]
        assert agg["parity_ok_all"] is False                  # one failed rank fails the job


def test_aggregate_ranks_single_and_cpu_threads():
    import bench
    agg = bench.aggregate_ranks([{"rank": 0, "device": 0, "queries": 10, "lf_ms": 1.5, "step_ms": 1.6,
                                  "parity_ok": True}])
    assert agg["parity_ok_all"] is True and agg["lf_ms_min"] == agg["lf_ms_max"] == 1.5
    agg = bench.aggregate_ranks([{"rank": 0, "queries": 1, "lf_ms": 1, "step_ms": 1, "parity_ok": None}])
    assert agg["parity_ok_all"] is None                       # sample skipped: no claim
    assert bench.cpu_threads() == len(os.sched_getaffinity(0))


def test_cpu_thread_counts(monkeypatch):
    import bench
    aff = len(os.sched_getaffinity(0))
    monkeypatch.setattr(bench, "cpu_quota", lambda: None)
    assert bench.baseline_thread_counts() == [aff] and bench.cpu_effective() == aff
    monkeypatch.setattr(bench, "cpu_quota", lambda: 0.5)
    if aff > 1:
        assert bench.baseline_thread_counts() == [aff, 1]
    assert bench.cpu_effective() == 1
