"""bench.py --gpus N without a launcher: the parent starts N
fresh rank processes itself (bench.spawn_ranks, before any HIP call, no exec),
relays rank 0's line, fails when a rank fails, and refuses a --gpus /
WORLD_SIZE mismatch.  CPU only: the ranks here are stub scripts over gloo, and
the real bench.py path is run up to its device check."""
import json
import os
import subprocess
import sys
import textwrap

from util import REPO

STUB = textwrap.dedent(r"""
    import json, os, sys, time
    sys.path.insert(0, %(repo)r); sys.path.insert(0, %(pkg)r)
    import bench
    mode = sys.argv[1]
    D = bench.Dist(int(os.environ["WORLD_SIZE"]))
    if mode == "fail" and D.rank == 1:
        sys.exit(3)                                  # rank 0 then waits at the barrier below
    D.barrier()
    # node-shared text (bench_text): local rank 0 writes, every rank maps it
    txt = bench.bench_text(D, 50_000)
    env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                                      "MASTER_PORT", "KFMI_BENCH_LAUNCHER")}
    rows = D.gather(dict(env, pid=os.getpid(), text_head=bytes(txt[:32]).decode(), text_len=len(txt),
                         shared=type(txt).__name__ == "mmap"))
    if D.rank == 0:
        print(json.dumps({"rows": rows}), flush=True)
    else:
        print("rank %%d stdout line" %% D.rank, flush=True)    # must not reach the parent's stdout
    D.close()
""")


def _stub(tmp_path):
    s = tmp_path / "stub.py"
    s.write_text(STUB % {"repo": str(REPO), "pkg": str(REPO / "k-step_fm-index_amd")})
    return s


def _spawn(tmp_path, n, mode, timeout=180, extra_env=None):
    drv = (f"import sys; sys.path.insert(0, {str(REPO)!r}); sys.path.insert(0, {str(REPO / 'k-step_fm-index_amd')!r});"
           f"import bench; sys.exit(bench.spawn_ranks({n}, [{mode!r}], script={str(_stub(tmp_path))!r}, grace_s=5))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", TMPDIR=str(tmp_path), **(extra_env or {}))
    return subprocess.run([sys.executable, "-c", drv], capture_output=True, text=True, env=env, timeout=timeout,
                          cwd=str(tmp_path))


def test_spawn_ranks_starts_n_ranks_and_relays_rank0(tmp_path):
    p = _spawn(tmp_path, 3, "ok")
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout                 # only rank 0's line on stdout
    rows = json.loads(lines[0])["rows"]
    assert [r["RANK"] for r in rows] == ["0", "1", "2"]
    assert [r["LOCAL_RANK"] for r in rows] == ["0", "1", "2"]
    assert {r["WORLD_SIZE"] for r in rows} == {"3"} and {r["LOCAL_WORLD_SIZE"] for r in rows} == {"3"}
    assert {r["MASTER_ADDR"] for r in rows} == {"127.0.0.1"} and len({r["MASTER_PORT"] for r in rows}) == 1
    assert {r["KFMI_BENCH_LAUNCHER"] for r in rows} == {"self-spawned"}
    assert len({r["pid"] for r in rows}) == 3        # fresh processes, not threads or an exec
    # one text for the node, the same bytes on every rank, file gone afterwards
    assert len({r["text_head"] for r in rows}) == 1 and {r["text_len"] for r in rows} == {50_000}
    assert not list(tmp_path.glob("kfmi_bench_*"))
    assert all(r["shared"] for r in rows)
    assert "rank 1 stdout line" in p.stderr and "rank 2 stdout line" in p.stderr


def test_node_shared_text_falls_back_to_private_copies(tmp_path):
    """No room for the node-shared file (forced here): every rank keeps its own
    copy of the same text, and the run goes on."""
    p = _spawn(tmp_path, 2, "ok", extra_env={"KFMI_BENCH_NODE_SHARED": "0"})
    assert p.returncode == 0, p.stderr[-2000:]
    rows = json.loads([ln for ln in p.stdout.splitlines() if ln.strip()][0])["rows"]
    assert not any(r["shared"] for r in rows) and len({r["text_head"] for r in rows}) == 1
    assert "KFMI_BENCH_NODE_SHARED=0" in p.stderr


def test_spawn_ranks_fails_when_a_rank_fails(tmp_path):
    p = _spawn(tmp_path, 2, "fail", timeout=120)
    assert p.returncode == 3, p.stderr[-2000:]
    assert "rank 1 exited with 3" in p.stderr
    assert not p.stdout.strip()                      # no line for a failed run


def test_bench_text_matches_recipe():
    """N = 1 keeps the text in-process; its bytes are the seeded recipe."""
    import random
    import bench
    from kstep_fmi import synth

    class One:
        world, local = 1, 0
    t = bench.bench_text(One(), 300_000)
    rng = random.Random(300_000)
    assert bytes(t) == rng.randbytes(300_000).translate(synth.TBL)


def _bench(args, env_extra, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True, text=True, env=env,
                          timeout=timeout, cwd=str(REPO))


def test_bench_refuses_gpus_world_size_mismatch():
    for gpus, ws in (("2", "3"), ("1", "2"), ("8", "1")):
        p = _bench(["--gpus", gpus], {"WORLD_SIZE": ws, "RANK": "0"}, timeout=60)
        assert p.returncode != 0
        assert f"--gpus {gpus} but the launcher started WORLD_SIZE={ws}" in p.stderr, p.stderr[-1000:]
        assert not p.stdout.strip()


def test_bench_gpus2_spawns_two_ranks_to_the_device_check(tmp_path):
    """The real bench.py path: `--gpus 2` with no launcher starts two ranks,
    which form their gloo group and stop at the device check on this GPU-less
    host; the parent fails with them and prints no line."""
    p = _bench(["--gpus", "2", "--steps", "1"], {"TMPDIR": str(tmp_path), "OMP_NUM_THREADS": "1"})
    assert p.returncode != 0
    assert "launcher: 2 ranks started" in p.stderr, p.stderr[-2000:]
    assert "no HIP device visible" in p.stderr
    assert not p.stdout.strip()
