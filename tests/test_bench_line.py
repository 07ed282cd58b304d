"""bench.py's JSON line: the driver keeps an 8 KB
tail of stdout, so the line is the last thing printed and at most
bench.LINE_MAX (6000) bytes at any N; the full record goes to a side file
whose path the line carries; ranks other than 0 write nothing to the shared
streams.  CPU only: the records are the committed round-4 bench lines (N = 1
and an N = 8 rehearsal) with their per-rank arrays filled out to 8 ranks."""
import copy
import json
import os
import subprocess
import sys
import textwrap

import pytest

import bench
from util import REPO

R4 = REPO / "profiles" / "r04"
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _record(name):
    return json.loads((R4 / name).read_text().strip().splitlines()[-1])


def _fill_ranks(d, n=8):
    """Every per-rank array of the record at n ranks, each row a copy of rank
    0's (the shape an N = 8 run on eight GPUs produces)."""
    d = copy.deepcopy(d)
    rows = d["ranks"]["ranks"]
    d["ranks"]["ranks"] = [dict(rows[0], rank=r, device=r, pci_bus_id=f"0000:{r:02x}:00.0") for r in range(n)]
    d["ranks"]["n_ranks"] = n
    d["devices"]["per_rank"] = [dict(d["devices"]["per_rank"][0], rank=r, local_rank=r, device=r) for r in range(n)]
    d["devices"].update(distinct_devices=n, shared_devices=False, ranks_per_device=[1] * n)
    ph = d["phases"]["per_rank"][0]
    d["phases"]["per_rank"] = [dict(ph, rank=r) for r in range(n)]
    c5 = d["variants"].get("config5")
    if c5:
        for k, v in list(c5.items()):
            if k.endswith("_per_rank") and isinstance(v, list):
                c5[k] = [v[0]] * n
        h = c5.get("host_to_host") or {}
        for sub in (h, h.get("streamed") or {}):
            for k, v in list(sub.items()):
                if k.endswith("_per_rank") and isinstance(v, list):
                    sub[k] = [v[0]] * n
    d["n_gpus"], d["ranks_launched"], d["launcher"] = n, n, "external"
    return d


@pytest.mark.parametrize("name,n", [("bench_r4z3.json", 1), ("bench_r4z3.json", 8), ("bench_r4v_n8full.json", 8)])
def test_line_fits_the_driver_tail(tmp_path, name, n):
    d = _record(name)
    if n > 1:
        d = _fill_ranks(d, n)
    assert len(json.dumps(d)) > 9000                  # the full record would not fit
    d["configs"] = bench.config_rows(d)
    path = bench.write_detail(d, str(tmp_path / "detail.json"), n)
    line = bench.compact_line(d, path)
    s = json.dumps(line, separators=(",", ":"))
    assert len(s) <= bench.LINE_MAX, len(s)
    assert all(k in line for k in REQUIRED)
    for k in ("bound", "achieved", "peak", "frac", "bytes_per_launch", "traffic", "traffic_over_algorithmic",
              "line_requests_per_query", "line_request_frac", "lf_ms"):
        assert k in line["roofline"], k
    for k in ("value", "cores", "threads", "kind", "cpu_model", "cgroup_cpu_quota", "parity_with_gpu"):
        assert k in line["cpu_baseline"], k
    assert line["parity"]["results_md5_pinned"] is True and line["ranks"]["n"] == n
    assert json.loads((tmp_path / "detail.json").read_text())["variants"] == d["variants"]
    assert line["detail"] == path
    # nothing above the achievable-HBM ratio under an HBM label
    def walk(x, key=""):
        if isinstance(x, dict):
            for k, v in x.items():
                yield from walk(v, k)
        elif isinstance(x, (int, float)) and not isinstance(x, bool):
            yield key, x
    for k, v in walk(line):
        if "hbm" in k.lower():
            assert v <= 6.29 / 8, (k, v)


def test_config_rows_cover_every_baseline_config():
    d = _record("bench_r4z3.json")
    rows = bench.config_rows(d)
    assert set(rows) >= {"1", "2", "3", "4", "5", "k4"}
    assert set(rows["2"]) >= {"task-mid", "task"} and set(rows["3"]) >= {"coop-mid", "coop"}
    assert set(rows["4"]) >= {"task-ac", "task-ac-mid"}
    for key, b in (("2", "task"), ("3", "coop"), ("4", "task-ac")):
        r = rows[key][b]
        assert r["frac"] > 0 and r["lrpq"] > 0 and r["eq"] is True
    assert rows["2"]["task-mid"]["md5"] is True and rows["1"]["gpu"]["md5"] is True
    assert rows["k4"]["md5"] is True and rows["5"]["oracle_ok"] is True


def test_line_guard_drops_rows_before_overflowing():
    d = _record("bench_r4z3.json")
    d["configs"] = {str(i): {"what": "x" * 200, "pad": "y" * 200} for i in range(40)}
    line = bench.compact_line(d, None)
    assert len(json.dumps(line, separators=(",", ":"))) <= bench.LINE_MAX
    assert line["configs"] == {"in_detail_file": True}


def test_kernel_prefix_names_the_timed_kernels():
    """The names rocprofv3 prints for the LF kernels (profiles/r04 kernel stats)."""
    assert bench.kernel_prefix("task-mid", 2, 64, 100) == "kfmi::task_kernel<kfmi::Geo<2, 2, 3>, 1, 8,"
    assert bench.kernel_prefix("task-mid", 2, 64, 150) == "kfmi::task_kernel<kfmi::Geo<2, 2, 3>, 1, 16,"
    assert bench.kernel_prefix("coop", 2, 64, 100) == "kfmi::coop_kernel<kfmi::Geo<2, 2, 0>, 8>"
    assert bench.kernel_prefix("coop-grp", 4, 64, 150) == "kfmi::coop_kernel<kfmi::Geo<4, 2, 6>, 16>"
    stats = (R4 / "bench_r4z4_kernel_stats.csv").read_text()
    for b, k in (("task-mid", 2), ("task", 2), ("coop-mid", 2), ("task-ac-mid", 2), ("coop-grp", 4)):
        assert bench.kernel_prefix(b, k, 64, 100) in stats, b


STUB = textwrap.dedent(r"""
    import json, os, sys
    sys.path.insert(0, %(repo)r); sys.path.insert(0, %(pkg)r)
    import bench
    rank = int(os.environ["RANK"])
    bench.setup_logging(rank)
    D = bench.Dist(int(os.environ["WORLD_SIZE"]))
    for i in range(200):                               # a chatty run: only rank 0's brief lines may show
        bench.log(f"rank {rank} detail line {i} " + "z" * 100)
        print(f"rank {rank} raw stdout {i}", flush=True) if rank else None
        print(f"rank {rank} raw stderr {i}", file=sys.stderr, flush=True) if rank else None
    bench.log(f"rank {rank}: progress", brief=True)
    D.barrier()
    if rank == 0:
        d = json.loads(open(%(rec)r).read().strip().splitlines()[-1])
        d["configs"] = bench.config_rows(d)
        line = bench.compact_line(d, bench.write_detail(d, os.path.join(os.environ["TMPDIR"], "det.json"), D.world))
        sys.stderr.flush()
        print(json.dumps(line, separators=(",", ":")), flush=True)
    D.barrier()
    D.close()
""")


def test_eight_stub_ranks_keep_stderr_small_and_stdout_one_line(tmp_path):
    """at N = 8 ranks > 0 log only to their own files; the
    parent's stderr stays under 2 KB and stdout is rank 0's one line."""
    s = tmp_path / "stub.py"
    s.write_text(STUB % {"repo": str(REPO), "pkg": str(REPO / "k-step_fm-index_amd"),
                         "rec": str(R4 / "bench_r4z3.json")})
    drv = (f"import sys; sys.path.insert(0, {str(REPO)!r}); sys.path.insert(0, {str(REPO / 'k-step_fm-index_amd')!r});"
           f"import bench; sys.exit(bench.spawn_ranks(8, [], script={str(s)!r}, grace_s=5))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT",
                                                            "KFMI_BENCH_VERBOSE", "KFMI_BENCH_LOGDIR")}
    env.update(OMP_NUM_THREADS="1", TMPDIR=str(tmp_path))
    p = subprocess.run([sys.executable, "-c", drv], capture_output=True, text=True, env=env, timeout=240,
                       cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(p.stderr.encode()) < 2048, p.stderr
    assert "raw stderr" not in p.stderr and "detail line" not in p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and len(lines[0]) <= bench.LINE_MAX
    assert json.loads(lines[0])["metric"].startswith("Mqueries/s")
    logs = sorted(tmp_path.glob("kfmi_bench_rank*_*.log"))
    assert len(logs) == 8
    r3 = next(x for x in logs if x.name.startswith("kfmi_bench_rank3_")).read_text()
    assert "raw stderr 199" in r3 and "raw stdout 199" in r3 and "detail line 199" in r3
