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
    # an auxiliary leg whose local step fails on rank 1 only: both ranks still make
    # the same collective calls (all_ok, then gather), skip the timed part together
    # and report rank 1's error (bench.Steps; ADVICE r2: no hang on a one-rank error)
    S = bench.Steps()
    def boom():
        raise RuntimeError("rank 1 fails")
    S.run(lambda: 1)
    if D.rank == 1:
        S.run(boom)
    S.run(lambda: 2)                      # skipped after the failure
    timed_ran = False
    if D.all_ok(S.ok):
        D.barrier()
        timed_ran = True
    errs = D.gather(S.err)
    # both ranks on one physical GPU (a one-card rehearsal): one distinct device
    dev_same = bench.aggregate_devices(D.gather({"rank": D.rank, "local_rank": D.local, "device": 0,
                                                 "pci_bus_id": "0000:75:00.0", "host": "h"}))
    dev_two = bench.aggregate_devices(D.gather({"rank": D.rank, "local_rank": D.local, "device": D.local,
                                                "pci_bus_id": "0000:%%02x:00.0" %% (0x75 + D.local), "host": "h"}))
    out = json.dumps({"rank": D.rank, "world": D.world, "local": D.local, "el": el, "el_max": el_max,
                      "total": total, "first": reads[0].tobytes().decode(), "start0": int(st[0]), "agg": agg,
                      "timed_ran": timed_ran, "errs": errs, "dev_same": dev_same, "dev_two": dev_two})
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
        # a leg's local failure on one rank: no hang, timed part skipped by both, error reported
        assert r["timed_ran"] is False
        assert r["errs"] == [None, "RuntimeError: rank 1 fails"]
        # device identity: two ranks on one card = one GPU, a rehearsal (no scaling claim)
        assert r["dev_same"] == {"distinct_devices": 1, "shared_devices": True, "ranks_per_device": [2]}
        assert r["dev_two"] == {"distinct_devices": 2, "shared_devices": False, "ranks_per_device": [1, 1]}


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


def test_aggregate_devices_fallbacks():
    import bench
    # no bus id: the device number per host stands in for it
    rows = [{"rank": 0, "device": 0, "pci_bus_id": None, "host": "a"},
            {"rank": 1, "device": 0, "pci_bus_id": None, "host": "a"},
            {"rank": 2, "device": 0, "pci_bus_id": None, "host": "b"}]
    agg = bench.aggregate_devices(rows)
    assert agg["distinct_devices"] == 2 and agg["shared_devices"] is True
    rows = [{"rank": i, "device": i, "pci_bus_id": f"0000:{i:02x}:00.0", "host": "a"} for i in range(8)]
    assert bench.aggregate_devices(rows) == {"distinct_devices": 8, "shared_devices": False,
                                             "ranks_per_device": [1] * 8}


def test_steps_and_phases():
    import bench
    S = bench.Steps()
    assert S.run(lambda x: x + 1, 1) == 2 and S.ok
    assert S.run(lambda: 1 / 0) is None and not S.ok and S.err.startswith("ZeroDivisionError")
    assert S.run(lambda: 5) is None                    # later steps skipped
    ph = bench.Phases()
    ph.mark("a")
    ph.mark("b")
    ph.mark("a")                                       # accumulates
    assert set(ph.rows) == {"a", "b"} and all(v >= 0 for v in ph.rows.values())
    assert bench.Phases.peak_rss_gb() > 0
