#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: Mqueries/s of batched k-step FM-index
backward search (3 Gbase synthetic reference, 10M x 100 bp reads, K=2, d=64)
on N MI355X, one process per GPU, plus the achieved HBM fraction of the LF
kernel and the CPU oracle timed on the host cores.

  python bench.py --gpus 1 --steps 10 --warmup 20
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N

A step = one searchIndexGPU() over the rank's whole batch (query packing +
LF kernel, inputs resident in HBM).  Each rank builds its own replica of the
index on its GPU (no collective on the data path) and searches its own 10M
reads (weak scaling).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "k-step_fm-index_amd"))

import kstep_fmi as K  # noqa: E402
from kstep_fmi import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PROBE_CEILING_GLINES = 56.0   # gather_probe, 200 MB table (Infinity-Cache resident), profiles/r03/gather_probe_r3g.jsonl


_LOG = {"file": None, "echo": True}


def setup_logging(rank: int) -> Path | None:
    """Every rank logs to its own file (KFMI_BENCH_LOGDIR, else TMPDIR): rank
    0 also echoes the brief progress lines to stderr; ranks > 0 send their fds
    1 and 2 to the file, so nothing of theirs (gloo's connect lines, library
    messages) reaches the stream rank 0's JSON line is printed on."""
    d = Path(os.environ.get("KFMI_BENCH_LOGDIR") or os.environ.get("TMPDIR") or "/tmp")
    fn = d / f"kfmi_bench_rank{rank}_{os.environ.get('MASTER_PORT', '0')}_{os.getpid()}.log"
    try:
        d.mkdir(parents=True, exist_ok=True)
        f = open(fn, "a", buffering=1)
    except OSError:
        f, fn = None, None
    _LOG["file"] = f
    if rank != 0:
        _LOG["echo"] = False
        if f is not None:
            sys.stdout.flush()
            sys.stderr.flush()
            os.dup2(f.fileno(), 1)
            os.dup2(f.fileno(), 2)
    return fn


def log(*a, brief: bool = False):
    """A line in this rank's log file; on rank 0 the `brief` ones (a dozen
    progress lines per run) also go to stderr, cut to 160 characters
    (KFMI_BENCH_VERBOSE=1: every line, whole)."""
    msg = " ".join(str(x) for x in a)
    line = f"[bench {time.strftime('%H:%M:%S')}] {msg}"
    f = _LOG["file"]
    if f is not None:
        try:
            f.write(line + "\n")
        except (OSError, ValueError):
            pass
    verbose = os.environ.get("KFMI_BENCH_VERBOSE") == "1"
    if _LOG["echo"] and (brief or verbose or f is None):
        print(line if verbose else line[:160], file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    # right after the upload the LF kernel needs ~10 steps to reach its steady
    # rate (9.9 -> 9.55 ms, profiles/r01/idle_probe.jsonl); 20 warmup steps = 0.2 s
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--backend", default="task-mid")
    p.add_argument("--ref-size", type=int, default=3_000_000_000)
    p.add_argument("--queries", type=int, default=10_000_000)
    p.add_argument("--qlen", type=int, default=100)
    p.add_argument("--e2e-steps", type=int, default=3, help="streamed host-to-host passes (0: skip)")
    p.add_argument("--k", type=int, default=2)
    p.add_argument("--d", type=int, default=64)
    p.add_argument("--cpu-sample", type=int, default=2_000_000,
                   help="queries of the CPU-oracle baseline sample (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the CPU baseline (0: every core in this process's affinity mask)")
    p.add_argument("--parity-sample", type=int, default=100_000,
                   help="reads per rank checked against the CPU oracle after the timed region (0 = skip)")
    p.add_argument("--cpu-port-only", action="store_true",
                   help="time only our restatement, not the reference's CPU binary (oracle/_ref)")
    p.add_argument("--variants", default="task,coop,task-ac,coop-ac,task-ac-mid,coop-ac-mid,"
                                         "task-mid,coop-mid,task-mid+ftab14,task-mid+ftab16",
                   help="other backends timed on rank 0 at N=1 (empty = none)")
    p.add_argument("--variant-steps", type=int, default=5)
    p.add_argument("--config5-queries", type=int, default=10_000_000,
                   help="reads per GPU of the config #5 leg (0 = skip)")
    p.add_argument("--config5-qlen", type=int, default=150)
    p.add_argument("--no-kstep4", dest="kstep4", action="store_false",
                   help="skip the K=4 (coop-grp) leg at N=1")
    p.add_argument("--ingest", choices=("auto", "on", "off"), default="auto",
                   help="FASTA file -> loadQueries -> search -> results legs (f2); auto: on at N <= 2 (each rank "
                        "writes 2.6 GB of FASTA to TMPDIR and parses it on 16 host threads)")
    p.add_argument("--no-ingest", dest="ingest", action="store_const", const="off", help="= --ingest off")
    p.add_argument("--no-md5", action="store_true")
    p.add_argument("--traffic-json", default=str(ROOT / "profiles" / "traffic.json"))
    p.add_argument("--sa-rate", type=int, default=32,
                   help="SA sampling rate of the index for the locate leg (0 = no locate)")
    p.add_argument("--locate-steps", type=int, default=3)
    p.add_argument("--no-config1", dest="config1", action="store_false",
                   help="skip the 64 Mbase / 2^20-read leg (BASELINE config #1)")
    p.add_argument("--detail", default=None,
                   help="where the full record goes (default gpurun_out/bench_detail_n<N>.json, else TMPDIR); "
                        "the JSON line carries its path")
    return p.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list, script: str | None = None, grace_s: float = 20.0) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh child processes of
    `script` (default this file) with argv, one per rank, with the environment
    torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, GROUP_RANK, MASTER_ADDR=127.0.0.1, MASTER_PORT), and
    wait.  Called before this process touches HIP; the children are started,
    never exec'd into.  Rank 0 shares this process's stdout (its JSON line is
    the run's line), the others print to stderr.  The first child that exits
    non-zero ends the run: the rest are terminated (they would wait for it at
    their next barrier) and its code is returned; 0 when every rank exits 0."""
    import signal
    import subprocess
    port = _free_port()
    procs = []

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.monotonic() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def on_signal(signum, frame):
        stop_all()
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    failed = None
    try:
        sys.stdout.flush()
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", ROLE_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       KFMI_BENCH_LAUNCHER="self-spawned")
            procs.append(subprocess.Popen([sys.executable, script or str(Path(__file__).resolve()), *argv], env=env,
                                          stdout=None if r == 0 else sys.stderr))
        log(f"launcher: {n} ranks started (pids {[p.pid for p in procs]}, master port {port})")
        while failed is None and any(p.poll() is None for p in procs):
            for r, p in enumerate(procs):
                rc = p.poll()
                if rc is not None and rc != 0:
                    failed = (r, rc)
                    break
            time.sleep(0.2)
        if failed is None:
            failed = next(((r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0), None)
    finally:
        stop_all()
        for s, h in old.items():
            signal.signal(s, h)
    if failed is not None:
        log(f"launcher: rank {failed[0]} exited with {failed[1]}; the other ranks were stopped")
        return failed[1] if failed[1] > 0 else 1
    return 0


class Dist:
    def __init__(self, gpus: int):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo's C++ layer prints "[Gloo] Rank r is connected to ..." on
            # fd 1 while the group forms; keep stdout for rank 0's JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo")    # control plane only: barrier + timing max
                dist.barrier()
            finally:
                os.dup2(saved, 1)
                os.close(saved)
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def max(self, x: float) -> float:
        if not self.pg:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if not self.pg:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.SUM)
        return float(t.item())

    def gather(self, obj) -> list:
        """Every rank's `obj` (JSON-able), in rank order, on every rank."""
        if not self.pg:
            return [obj]
        out = [None] * self.world
        self.pg.all_gather_object(out, obj)
        return out

    def all_ok(self, ok: bool) -> bool:
        """True on every rank iff `ok` on every rank (one collective, every rank calls it)."""
        if not self.pg:
            return bool(ok)
        import torch
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MIN)
        return bool(t.item())

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


class Steps:
    """A leg's local work on this rank, one step at a time: the first step that
    raises ends the rank's local work for the leg (its error is kept), while the
    leg itself keeps making every collective call (barrier, max, gather) in the
    same order on every rank -- a rank that fails part-way never leaves the
    others waiting at a barrier it skips.  Timed sections ask D.all_ok first and
    are skipped by every rank together."""

    def __init__(self):
        self.err = None

    @property
    def ok(self) -> bool:
        return self.err is None

    def run(self, fn, *a, **kw):
        if self.err is not None:
            return None
        try:
            return fn(*a, **kw)
        except Exception as e:          # reported in the leg's output, never fatal
            self.err = f"{type(e).__name__}: {e}"
            return None


class Phases:
    """Wall time of each bench phase on this rank, and the process's peak RSS."""

    def __init__(self):
        self.t = time.perf_counter()
        self.rows = {}
        self.anon_peak = 0.0

    def mark(self, name: str) -> None:
        now = time.perf_counter()
        self.rows[name] = round(self.rows.get(name, 0.0) + now - self.t, 2)
        self.t = now
        self.anon_peak = max(self.anon_peak, self.rss_anon_gb())

    @staticmethod
    def rss_anon_gb() -> float:
        """This process's private resident memory now (RssAnon: excludes the
        page-cache pages of the node-shared text and image mappings)."""
        try:
            for ln in open("/proc/self/status"):
                if ln.startswith("RssAnon:"):
                    return round(int(ln.split()[1]) / 1e6, 2)
        except OSError:
            pass
        return 0.0

    @staticmethod
    def peak_rss_gb() -> float:
        import resource
        return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2)   # ru_maxrss is KiB


def device_rows(D, dev: int) -> list:
    """Every rank's (rank, local rank, device number, PCI bus id of that device),
    in rank order on every rank: the bus id names the physical GPU, which device
    numbers do not across processes (HIP_VISIBLE_DEVICES)."""
    try:
        bus = K.device_pci_bus_id(dev)
    except K.KfmiError:
        bus = None
    return D.gather({"rank": D.rank, "local_rank": D.local, "device": dev, "pci_bus_id": bus,
                     "host": os.uname().nodename})


def aggregate_devices(rows: list) -> dict:
    """Distinct physical GPUs behind the ranks (host + PCI bus id; a rank whose
    bus id is unknown counts as its own GPU only if no other rank on its host
    has the same device number).  shared_devices: two ranks on one GPU -- then
    the run is a rehearsal, not a multi-GPU measurement."""
    keys = []
    for r in rows:
        keys.append((r.get("host"), r["pci_bus_id"]) if r.get("pci_bus_id") else (r.get("host"), f"dev{r['device']}"))
    per = {}
    for k in keys:
        per[k] = per.get(k, 0) + 1
    distinct = len(per)
    return {"distinct_devices": distinct, "shared_devices": distinct < len(rows),
            "ranks_per_device": sorted(per.values(), reverse=True)}


def cuda_sync(dev: int):
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize(dev)
    except Exception:
        pass


def bench_text(D, n: int):
    """The reference text, generated once per node (synth.text_chunks: the
    md5-pinned 3 Gbase recipe, or random.Random(n) for other sizes).  N = 1:
    filled into one bytearray chunk by chunk (peak = the text, not text + the
    joined chunks).  N > 1: local rank 0 streams it to a file in TMPDIR, every
    rank maps that file read-only -- one copy in the node's page cache instead
    of one 3 GB object per rank -- and the file is unlinked once every rank
    holds its mapping."""
    if D.world > 1:
        mm = _node_shared(D, f"text_{n}", n, lambda f: [f.write(ch) for ch in synth.text_chunks(n)])
        if mm is not None:
            return mm
        log(f"rank {D.rank}: no room for the node-shared text: generating it in this process", brief=True)
    buf = bytearray(n)
    off = 0
    for ch in synth.text_chunks(n):
        buf[off:off + len(ch)] = ch
        off += len(ch)
    return buf


def _node_shared(D, name: str, nbytes: int, write):
    """A file of `nbytes` written once per node by local rank 0 (`write(f)`) in
    TMPDIR, then mapped read-only by every rank of the node; returns the mmap,
    or None on every rank when local rank 0 could not write it (no room: the
    caller then keeps a private copy per rank).  Collective: every rank calls
    it."""
    import mmap
    import shutil
    d = Path(os.environ.get("TMPDIR") or "/tmp")
    fn = d / f"kfmi_bench_{name}_{os.environ.get('MASTER_PORT', '0')}.bin"
    err = None
    if D.local == 0:
        tmp = fn.with_suffix(".part")
        try:
            if os.environ.get("KFMI_BENCH_NODE_SHARED", "1") == "0":
                raise OSError("KFMI_BENCH_NODE_SHARED=0")
            if shutil.disk_usage(d).free < nbytes + (1 << 30):
                raise OSError(f"{d}: {shutil.disk_usage(d).free} bytes free, {nbytes} needed")
            with open(tmp, "wb") as f:
                write(f)
            os.replace(tmp, fn)
        except OSError as e:
            err = f"{type(e).__name__}: {e}"
            tmp.unlink(missing_ok=True)
    if not D.all_ok(err is None):
        if err:
            log(f"node-shared {name}: {err}", brief=True)
        return None
    with open(fn, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    D.barrier()                      # every rank holds its mapping: the name can go
    if D.local == 0:
        fn.unlink(missing_ok=True)
    return mm


def shared_image(D, idx) -> np.ndarray:
    """The index's tag-100 image for the CPU oracle.  N = 1: the handle's own
    host image.  N > 1: every rank built the same index from the same text (on
    its own GPU, without a host image); local rank 0 fetches its image from
    the device and the others map rank 0's copy (the parity samples then check
    each rank's GPU results against that image)."""
    if D.world == 1:
        return idx.image()
    h = idx.header()
    nbytes = 24 + 8 * h["steps"] + 4 * h["nentries"] * ((2 * h["chunk"] // 32 * h["steps"]) + h["ncounters"])
    mm = _node_shared(D, "image", nbytes, lambda f: idx.image().tofile(f))
    if mm is None:
        return idx.image()           # no room on the node: each rank fetches its own
    return np.frombuffer(mm, dtype=np.uint8)


def cpu_threads() -> int:
    """Every core this process may run on (its affinity mask), SURVEY 8(d)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_quota() -> float | None:
    """CPUs granted by the cgroup (cpu.max quota / period), None when unlimited."""
    for fn in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(fn).read().split()[:2]
            if q != "max":
                return round(int(q) / int(per), 2)
        except (OSError, ValueError):
            pass
    return None


def cpu_effective() -> int:
    """CPUs this process can actually use: the affinity mask capped by the cgroup quota."""
    q = cpu_quota()
    return max(1, min(cpu_threads(), int(round(q)) if q else 1 << 30))


def ingest_leg(idx, reads: np.ndarray, res: np.ndarray, world: int) -> dict:
    """this rank's reads as a multi-FASTA file (">r" headers,
    in TMPDIR, so in the page cache), then loadQueries (parallel mapped parse;
    the line-by-line loop beside it) + queries H2D + search + results D2H,
    timed as one host-file-to-host-results pass on the resident index."""
    import tempfile
    n, m = reads.shape
    out = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        fn = Path(td) / "reads.fa"
        rec = np.empty((n, m + 4), dtype=np.uint8)
        rec[:, :3] = np.frombuffer(b">r\n", dtype=np.uint8)
        rec[:, 3:3 + m] = reads
        rec[:, -1] = 10
        rec.tofile(fn)
        del rec
        out["file_bytes"] = fn.stat().st_size
        modes = (("parallel", "1"), ("line_loop", "0")) if world == 1 else (("parallel", "1"),)
        for mode, mm in modes:
            os.environ["KFMI_LOAD_MMAP"] = mm
            t = time.perf_counter()
            q2 = K.Queries.load(fn, m, n)
            out[f"load_s_{mode}"] = round(time.perf_counter() - t, 3)
            if mode != "parallel":
                q2.close()
            else:
                qp = q2
        os.environ.pop("KFMI_LOAD_MMAP", None)
        # the same file parsed on the device (kfmi_load_queries_gpu): file -> device reads
        try:
            rd = K.Results.alloc(n)
            t = time.perf_counter()
            qd = K.Queries.load_gpu(fn, m, n)
            out["device_parse_load_s"] = round(time.perf_counter() - t, 3)
            t = time.perf_counter()
            K.transfer_to_gpu(idx, qd, rd)
            K.search(idx, qd, rd)
            K.transfer_to_cpu(rd)
            tot_d = out["device_parse_load_s"] + time.perf_counter() - t
            out["device_parse_total_s"] = round(tot_d, 3)
            out["device_parse_mqps_file_to_results"] = round(n / tot_d / 1e6, 2)
            out["device_parse_results_equal"] = bool(np.array_equal(rd.array(), res))
            qd.close()
            rd.close()
        except K.KfmiError as e:
            out["device_parse_error"] = str(e)
    r2 = K.Results.alloc(n)
    t = time.perf_counter()
    K.transfer_to_gpu(idx, qp, r2)
    out["h2d_s"] = round(time.perf_counter() - t, 3)
    t = time.perf_counter()
    K.search(idx, qp, r2)
    out["search_s"] = round(time.perf_counter() - t, 4)
    t = time.perf_counter()
    K.transfer_to_cpu(r2)
    out["d2h_s"] = round(time.perf_counter() - t, 4)
    tot = out["load_s_parallel"] + out["h2d_s"] + out["search_s"] + out["d2h_s"]
    out["total_s"] = round(tot, 3)
    out["mqps_file_to_results"] = round(n / tot / 1e6, 2)
    out["load_GB_per_s"] = round(out["file_bytes"] / out["load_s_parallel"] / 1e9, 2)
    out["results_equal"] = bool(np.array_equal(r2.array(), res))
    out["host_threads"] = K.host_threads()
    qp.close()
    r2.close()
    return out


def aggregate_ranks(rows: list) -> dict:
    """Whole-job view of the per-rank rows (rank, device, lf_ms, step_ms,
    queries, parity_ok, ...): min/max LF time over ranks and the AND of every
    rank's oracle-sample parity."""
    lf = [r["lf_ms"] for r in rows]
    st = [r["step_ms"] for r in rows]
    oks = [r.get("parity_ok") for r in rows]
    return {"n_ranks": len(rows),
            "lf_ms_min": round(min(lf), 4), "lf_ms_max": round(max(lf), 4),
            "step_ms_min": round(min(st), 4), "step_ms_max": round(max(st), 4),
            "queries": int(sum(r["queries"] for r in rows)),
            "parity_ok_all": None if any(o is None for o in oks) else bool(all(oks)),
            "ranks": rows}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cores_used(threads: int) -> int:
    """CPUs a run of `threads` OS threads actually had: the thread count capped
    by what this process can use (affinity mask and cgroup quota).  256 threads
    on a 16-CPU quota ran on 16 cores; `threads` is reported beside it."""
    return max(1, min(int(threads), cpu_effective()))


def baseline_thread_counts() -> list:
    """Thread counts the CPU baseline is timed at: every core of the affinity
    mask and, when the cgroup grants fewer CPUs than that (the GPU boxes show
    256 cores but a 16-CPU quota), the quota as well."""
    aff = cpu_threads()
    q = cpu_quota()
    out = [aff]
    if q and int(round(q)) < aff:
        out.append(max(1, int(round(q))))
    return out


def cpu_reference_baseline(idx, reads, ns, k, d, thr, res_gpu):
    """The reference's own CPU searcher (common/searchQueries.c +
    src/fmIndexCPUBaseline.c, compiled from /root/reference sources into
    oracle/_ref by oracle/Makefile) on the first `ns` reads: its file interface
    (tag-100 index file, multi-FASTA queries, 5 timed iterations, "TIME:" = mean
    seconds per iteration, results in <index>.res.cpu).  `thr` is a thread
    count or a list of them (one run each, same files); the fastest run is
    returned, the others under "other_runs".  None when the binary for (k, d)
    is not there."""
    thrs = thr if isinstance(thr, (list, tuple)) else [thr]
    import subprocess
    import tempfile
    binp = ROOT / "oracle" / "_ref" / f"cpu_{k}_{d}"
    if not binp.exists():
        return None
    m = reads.shape[1]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        ip, qp = Path(td) / "index.fmi", Path(td) / "q.qry"
        idx.image().tofile(ip)
        rec = np.empty((ns, m + 4), dtype=np.uint8)
        rec[:, :3] = np.frombuffer(b">r\n", dtype=np.uint8)
        rec[:, 3:3 + m] = reads[:ns]
        rec[:, -1] = 10
        rec.tofile(qp)
        runs = []
        for thr in thrs:
            env = dict(os.environ, OMP_NUM_THREADS=str(thr))
            p = subprocess.run([str(binp), str(ip), str(qp), str(m), str(ns)], env=env, capture_output=True,
                               text=True, timeout=900)
            if p.returncode != 0 or "TIME:" not in p.stdout:
                log(f"reference cpu baseline failed: rc={p.returncode} {p.stdout[-300:]} {p.stderr[-300:]}", brief=True)
                return None
            t_iter = float(p.stdout.split("TIME:")[1].split()[0])
            vals = np.array((Path(str(ip) + ".res.cpu")).read_bytes().split(), dtype=np.uint64)
            ok = int(vals[0]) == ns and bool(np.array_equal(vals[1:].astype(np.uint32), res_gpu[:2 * ns]))
            runs.append({"value": round(ns / t_iter / 1e6, 4), "unit": "Mqueries/s", "cores": cores_used(thr),
                         "threads": thr, "kind": "reference",
                         "sample": f"first {ns} of the same 10M reads; oracle/_ref/cpu_{k}_{d} = the reference's "
                                   f"searchQueries.c + fmIndexCPUBaseline.c built from its sources, OMP "
                                   f"threads={thr}, 5 iterations, TIME {t_iter:.3f} s/iteration",
                         "parity_with_gpu": ok})
    best = max(runs, key=lambda x: x["value"])
    if len(runs) > 1:
        best = dict(best, other_runs=[{"cores": x["cores"], "threads": x["threads"], "value": x["value"]}
                                      for x in runs if x is not best])
    return best


def probe_rows(stdout: str, gb: str) -> tuple[int | None, list]:
    """gather_probe's JSON rows for its main table of `gb` GB (the tool also
    probes 4 MB / 200 MB tables after the main one; those rows are dropped)."""
    rows, table, want = [], None, int(float(gb) * 1e9) & ~127
    for ln in stdout.splitlines():
        try:
            d = json.loads(ln)
        except ValueError:
            continue
        if "table_bytes" in d:
            table = d["table_bytes"]
        elif "kind" in d and table == want:
            rows.append(d)
    return (want if rows else None), rows


def best_of_runs(runs: list) -> list:
    """Per (kind, line size), the fastest of several runs' rows (a ceiling is
    the rate the path can reach: the max over repeats, not their mean)."""
    best = {}
    for rows in runs:
        for r in rows:
            k = (r["kind"], r["line_B"])
            if k not in best or r["Glines_s"] > best[k]["Glines_s"]:
                best[k] = dict(r)
    return list(best.values())


def probe_leg(ic_runs: int = 2) -> dict | None:
    """The random-line request ceiling on this box, measured beside the kernel:
    bin/gather_probe (csrc/tools/gather_probe.hip) reads uniformly random lines
    -- independent per lane, cooperative, and dependent chains (the LF shape) --
    of a 3 GB table (every request an L2 and Infinity-Cache miss: HBM) and of
    a 200 MB one (past the L2s, inside the 256 MB Infinity Cache: the request
    path's own limit, with no DRAM behind it).  The LF kernel's requests are a
    mix of both (its early steps' lines stay in the caches), so the ceiling it
    is held against is the larger rate, the Infinity-Cache-resident one
    (DESIGN.md 5); that table is probed `ic_runs` times and each kind keeps
    its best run, so one slow run does not put the ceiling under the kernel.
    Run as a child process while this one idles.  None when the tool is
    missing or fails."""
    import subprocess
    exe = ROOT / "k-step_fm-index_amd" / "bin" / "gather_probe"
    if not exe.exists():
        return None
    out = {}
    for gb, key, n in (("3", "hbm_3GB", 1), ("0.2", "infinity_cache_200MB", max(1, ic_runs))):
        runs, table = [], None
        for _ in range(n):
            try:
                p = subprocess.run([str(exe), gb, "512"], capture_output=True, text=True, timeout=300)
            except (OSError, subprocess.SubprocessError):
                return None
            if p.returncode != 0:
                return None
            table, rows = probe_rows(p.stdout, gb)
            if not rows:
                return None
            runs.append(rows)
        rows = best_of_runs(runs)
        best = max(rows, key=lambda x: x["Glines_s"])
        chain = [x for x in rows if x["kind"].startswith("chain")]
        out[key] = {"best_G_lines_per_s": best["Glines_s"], "best_kind": f"{best['kind']} {best['line_B']} B",
                    "chain_G_lines_per_s": max(x["Glines_s"] for x in chain) if chain else None,
                    "table_bytes": table, "runs": n, "rows": rows}
    ceil_key = max(out, key=lambda k: out[k]["best_G_lines_per_s"])
    return dict(out, ceiling_G_lines_per_s=out[ceil_key]["best_G_lines_per_s"], ceiling_from=ceil_key)


def replay_requests(replay: list | None, pmc: dict | None) -> dict | None:
    """The replay probe's fabric request rate per mode: requests per launch
    from the committed PMC pass of kfmi_probe_replay on the bench batch
    (scripts/pmc_replay.py; the line stream is the same in every mode, so a
    mode the pass did not cover takes the median of the measured ones) over
    this run's replay time.  None without the probe or the counts."""
    if not replay or not pmc or not pmc.get("rdreq_per_launch"):
        return None
    counts = pmc["rdreq_per_launch"]
    med = float(np.median(list(counts.values())))
    req, rate = {}, {}
    for x in replay:
        m = f"u{x['unroll']}g{x['groups']}"
        req[m] = int(counts.get(m, med))
        rate[m] = round(req[m] / (x["ms"] / 1e3) / 1e9, 2)
    best = max(rate, key=rate.get)
    return {"requests": req, "G_requests_per_s": rate, "best_G_requests_per_s": rate[best], "best_mode": best}


# the newest committed pass (this round's, else round 4's)
VARIANTS_PMC = next((p for p in (ROOT / "profiles" / r / "traffic_variants.json" for r in ("r05", "r04"))
                     if p.exists()), ROOT / "profiles" / "r05" / "traffic_variants.json")
VARIANTS_PMC_Q150 = ROOT / "profiles" / "r05" / "traffic_variants_q150.json"

# backend -> layout id of its kernels' Geo<K, NB, LAY> (kfmi_device.h Layout)
LAYOUT = {"task": 0, "coop": 0, "task-ac": 1, "coop-ac": 1, "task-mid": 3, "coop-mid": 3, "task-ac-mid": 5,
          "coop-ac-mid": 5, "task-grp": 6, "coop-grp": 6}   # 2 and 4: the retired packed / ac128 layouts


def kernel_prefix(backend: str, k: int, d: int, qlen: int) -> str:
    """The demangled-name prefix of `backend`'s LF kernel for reads of qlen
    bases (fused packing: 8 code words up to 128 bases of K-steps, else 16;
    kfmi_search.hip fused_maxw), as rocprofv3 prints it."""
    name = backend.partition("+")[0]
    maxw = 8 if k * (qlen // k) <= 128 else 16
    geo = f"kfmi::Geo<{k}, {d // 32}, {LAYOUT[name]}>"
    return f"kfmi::coop_kernel<{geo}, {maxw}>" if name.startswith("coop") else f"kfmi::task_kernel<{geo}, 1, {maxw},"


def launch_spec(backend: str, k: int, d: int, qlen: int, num: int, first: int, count: int) -> dict:
    """Where a row's timed LF launches sit in a rocprofv3 kernel trace of this
    run: the launches of kernel `kernel` whose grid covers `num` reads, in
    dispatch order, [first, first + count) (scripts/rows_from_trace.py)."""
    return {"kernel": kernel_prefix(backend, k, d, qlen), "num": int(num), "first": int(first), "count": int(count)}


def load_variants_pmc(queries: int, ref_size: int, qlen: int, d: int, path: Path | None = None) -> dict | None:
    """Per-backend fabric read requests per launch (TCC_EA0_RDREQ) of the 3 Gbase
    LF kernels, from a committed PMC pass (scripts/traffic_variants.py over
    scripts/pmc_variants.py under rocprofv3): the 10M x 100 bp batch, or with
    `path` = VARIANTS_PMC_Q150 config #5's 10M x 150 bp shard; None unless it
    was taken on that config."""
    try:
        tv = json.loads((path or VARIANTS_PMC).read_text())
    except (OSError, ValueError):
        return None
    cfg = tv.get("config", {})
    if (cfg.get("queries") != queries or cfg.get("ref_size") != ref_size or cfg.get("qlen") != qlen
            or cfg.get("d") != d):
        return None
    return tv


def variant_roofline(blocks: int, b_lf: int, lf_ms: float, a, backend: str, pmc: dict | None,
                     ceiling: float, k: int | None = None, queries: int | None = None) -> dict:
    """Roofline of one backend's LF launch on the bench batch: SURVEY 8(d)
    algorithmic bytes (K*d/4 + 4 B per distinct block) over its HIP-event time,
    against the HBM peak; and, when the committed PMC pass holds this backend,
    its fabric read requests per launch and per query, their rate, and that
    rate against the random-line request ceiling."""
    bytes_alg = blocks * b_lf
    out = {"distinct_blocks": int(blocks), "bytes_per_block": b_lf, "bytes_per_launch": int(bytes_alg),
           "achieved_GBs": round(bytes_alg / (lf_ms / 1e3) / 1e9, 1),
           "frac": round(bytes_alg / (lf_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    row = (pmc or {}).get("backends", {}).get(f"{backend}@k{k or a.k}")
    if row:
        req = row["rdreq_per_launch"]
        # no ceiling fraction here: the probe's ceiling is measured on uniformly
        # random 64/128-B lines, and other layouts' request mixes (64-B lines,
        # an L2-resident superblock table, 96 GB tables) sit on either side of
        # it -- the retired coop-packed issued 58.6 G/s, coop-grp 49.9
        out.update({"fabric_read_requests_per_launch": req,
                    "line_requests_per_query": round(req / (queries or a.queries), 2),
                    "line_requests_G_per_s": round(req / (lf_ms / 1e3) / 1e9, 2),
                    "l2_requests_per_launch": row.get("tcc_req_per_launch"),
                    "pmc_kernel_ms": row.get("kernel_ms_under_pmc"), "pmc_source": pmc.get("source"),
                    # every random L2 miss on gfx950 is one 128-B request, whatever the line
                    # width the layout reads (TCC_EA0_RDREQ_128B, profiles/r04/pmc_r4k_*_sizes):
                    # the guide's FETCH_SIZE x 2, Infinity-Cache hits included
                    "traffic": req * 128, "traffic_GB_per_s": round(req * 128 / (lf_ms / 1e3) / 1e9, 1),
                    # whole-line bytes at the L2/fabric boundary (Infinity-Cache hits included)
                    # against 8 TB/s: NOT an HBM fraction -- that is `frac` above
                    "l2_fabric_line_bytes_vs_8TBs_incl_ic_hits": round(req * 128 / (lf_ms / 1e3) / 1e9
                                                                       / HBM_PEAK_GBS, 4),
                    "traffic_over_algorithmic": round(req * 128 / bytes_alg, 3) if bytes_alg else None})
    return out


def cpu_product_rows(idx, reads: np.ndarray, want: np.ndarray, thrs: list) -> list:
    """searchIndexCPU of the library (kfmi_search_cpu) on `reads` at each
    thread count: rate and equality with the GPU results."""
    rows = []
    for thr in thrs:
        t = time.perf_counter()
        got = K.search_cpu_array(idx, reads, nthreads=thr)
        s_ = time.perf_counter() - t
        rows.append({"value": round(reads.shape[0] / s_ / 1e6, 4), "unit": "Mqueries/s", "cores": cores_used(thr),
                     "threads": thr, "kind": "product (searchIndexCPU)", "equal_gpu": bool(np.array_equal(got, want))})
    return rows


def config1_leg(backend: str, thr, steps: int = 5) -> dict:
    """BASELINE config #1 (64 Mbase recipe text, 2^20 x 100 bp reads): GPU
    search rate on the md5-pinned inputs and the reference's CPU searcher on
    the same reads (its 'plumbing' config)."""
    text, rng = synth.text_64m()
    idx = K.Index.build(text, k=2, d=64, gpu=True)
    reads = synth.reads_64m(text, rng)
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    wall, lf, tot = time_backend(idx, q, r, backend, steps, 20)
    res = r.array().copy()
    blocks = K.count_blocks(idx, q)
    b_lf = 2 * 64 // 4 + 4
    out = {"backend": backend, "mqps": round(reads.shape[0] / float(np.median(wall)) / 1e6, 2), "lf_ms": round(lf, 3),
           "results_md5_pinned": synth.results_md5(res) == synth.MD5["res64"],
           # 36 B x distinct blocks over the HIP-event LF time against 8 TB/s; the
           # 64 MB MID128 table sits in the 256 MB Infinity Cache, so this row is
           # not HBM-bound and may exceed the 3 Gbase rows' fraction
           "bytes_per_launch": int(blocks * b_lf), "frac": round(blocks * b_lf / (lf / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
           "launches": launch_spec(backend, 2, 64, reads.shape[1], reads.shape[0], 20, steps)}
    thrs = thr if isinstance(thr, (list, tuple)) else [thr]
    ref = cpu_reference_baseline(idx, reads, reads.shape[0], 2, 64, thrs, res)
    if ref:
        out["cpu_reference"] = {k: ref[k] for k in ("value", "unit", "cores", "threads", "parity_with_gpu")}
    # config #1 is the reference's CPU searcher: the product's searchIndexCPU
    # beside it, at the same thread counts (the faster run reported)
    rows = cpu_product_rows(idx, reads, res, thrs)
    out["cpu_product"] = max(rows, key=lambda x: x["value"])
    q.close()
    r.close()
    idx.close()
    return out


def config5_leg(D, idx, text: bytes, backend: str, qlen: int, nq: int, steps: int, warmup: int, ac: bool,
                oracle_img=None, ingest: bool = False, k: int = 2, d: int = 64, pmc: dict | None = None) -> dict:
    """BASELINE config #5's read shape on every rank: this rank's shard of nq
    reads of qlen bases (seed 20 + rank; 10M x 150 bp = one eighth of the
    80M x 150 bp batch at N = 8), searched on the resident index; timed like
    the main leg (barrier + synchronize, max over ranks), then an evenly spread
    100 K-read sample of every rank checked against the CPU oracle (on
    `oracle_img` when given: the image of another index of the same text, or
    the node-shared image at N > 1; AltCounters semantics from `idx`).  Every
    rank makes the same collective calls whatever fails locally (Steps)."""
    from oracle import oracle
    S = Steps()
    h = {}

    def setup():
        h["reads"] = synth.gather_reads(text, synth.read_starts(len(text), nq, qlen, seed=20 + D.rank), qlen)
        h["q"] = K.Queries.from_array(h["reads"])
        h["r"] = K.Results.alloc(nq)
        K.set_backend(backend)
        K.transfer_to_gpu(idx, h["q"], h["r"])
        for _ in range(warmup):
            K.search(idx, h["q"], h["r"])

    def timed(lf):
        for _ in range(steps):
            K.search(idx, h["q"], h["r"])
            lf.append(K.last_timing()["lf_ms"])

    def fetch():
        K.transfer_to_cpu(h["r"])
        h["res"] = h["r"].array().copy()

    def host_to_host():
        K.transfer_to_gpu(idx, h["q"], h["r"])
        K.search(idx, h["q"], h["r"])
        K.transfer_to_cpu(h["r"])

    S.run(setup)
    out = {"what": f"config #5 shape: {nq // 1_000_000}M x {qlen} bp reads per GPU (seed 20 + rank), "
                   f"{D.world} GPU(s), index replicated"}
    lf = []
    if D.all_ok(S.ok):
        D.barrier()
        t0 = time.perf_counter()
        S.run(timed, lf)
        D.barrier()
        el = D.max(time.perf_counter() - t0)
        S.run(fetch)
        total = D.sum(float(nq))
        out.update({"mqps": round(total * steps / el / 1e6, 2), "ms_per_step": round(el / steps * 1e3, 4),
                    "lf_ms_per_rank": D.gather(round(float(np.mean(lf)), 4) if lf else None)})
        # this rank's roofline: SURVEY 8(d) bytes (K*d/4 + 4 per distinct block,
        # counted on the device over the same shard) over its HIP-event LF time
        blocks = S.run(K.count_blocks, idx, h["q"]) if lf else None
        if blocks is not None:
            b_lf = k * d // 4 + 4
            lfm = float(np.mean(lf))
            out["roofline"] = variant_roofline(blocks, b_lf, lfm, argparse.Namespace(queries=nq, k=k), backend, pmc,
                                               PROBE_CEILING_GLINES, k=k, queries=nq)
            out["roofline"]["lf_ms"] = round(lfm, 4)
            out["launches"] = launch_spec(backend, k, d, qlen, nq, warmup, steps)
    # host memory to host memory on every rank (config #5's wall
    # time across the GPUs): this rank's reads H2D, search, results D2H on the
    # resident index, bracketed by barriers, max over ranks
    if D.all_ok(S.ok):
        D.barrier()
        t0 = time.perf_counter()
        S.run(host_to_host)
        D.barrier()
        e2e = D.max(time.perf_counter() - t0)
        e2e_eq = D.gather(S.ok and bool(np.array_equal(h["r"].array(), h["res"])))
        out["host_to_host"] = {"wall_s": round(e2e, 4), "mqps": round(D.sum(float(nq)) / e2e / 1e6, 2),
                               "results_equal_per_rank": e2e_eq,
                               "what": "every rank: its reads (pageable host memory) H2D + search + results D2H "
                                       "on the resident index through the reference's trio (ASCII upload), "
                                       "barriers around, max over ranks"}
        # the same through kfmi_search_stream (chunks packed to 2-bit words on the
        # host, H2D / LF / D2H overlapped): one warm-up call, then one timed call
        outb = np.empty(2 * nq, dtype=np.uint32)
        err = None
        try:
            K.search_stream(idx, h["reads"], out=outb)
        except K.KfmiError as e:
            err = str(e)
        D.barrier()
        t0 = time.perf_counter()
        if err is None:
            try:
                K.search_stream(idx, h["reads"], out=outb)
            except K.KfmiError as e:
                err = str(e)
        D.barrier()
        sw = D.max(time.perf_counter() - t0)
        errs = D.gather(err)
        st_eq = D.gather(err is None and bool(np.array_equal(outb, h["res"])))
        if any(errs):
            out["host_to_host"]["streamed"] = {"error_per_rank": errs}
        else:
            out["host_to_host"]["streamed"] = {"wall_s": round(sw, 4), "mqps": round(D.sum(float(nq)) / sw / 1e6, 2),
                                               "results_equal_per_rank": st_eq,
                                               "host_threads": K.host_threads()}
        del outb

    def parity():
        sel = np.linspace(0, nq - 1, min(100_000, nq)).astype(np.int64)
        if ac:
            img_idx = idx.alt_counters()[0]
            want, _ = oracle.search(img_idx.image(), h["reads"][sel], nthreads=max(1, cpu_effective() // D.world))
            img_idx.close()
        else:
            img = oracle_img if oracle_img is not None else idx.image()
            want, _ = oracle.search(img, h["reads"][sel], nthreads=max(1, cpu_effective() // D.world))
        h["n_sample"] = int(sel.size)
        return bool(np.array_equal(want.reshape(-1, 2), h["res"].reshape(-1, 2)[sel]))

    ok = S.run(parity)
    out["oracle_sample_ok_per_rank"] = D.gather(ok if S.ok else None)
    out["oracle_sample_per_rank"] = h.get("n_sample", 0)
    for k in ("q", "r"):
        if k in h:
            h[k].close()
    if ingest:
        # this rank's shard as a FASTA file -> results (host parser and device parser)
        ing = S.run(ingest_leg, idx, h["reads"], h["res"], D.world) if S.ok else None
        os.environ.pop("KFMI_LOAD_MMAP", None)
        out["ingest_file_per_rank"] = D.gather(ing if ing is not None else {"error": S.err})
    errs = D.gather(S.err)
    if any(errs):
        out["error_per_rank"] = errs
    return out


def kstep4_leg(D, text: bytes, reads: np.ndarray, res: np.ndarray, img2, steps: int, pinned_md5: str | None,
               c5_qlen: int, c5_queries: int, a=None, pmc: dict | None = None, ceiling: float | None = None,
               pmc150: dict | None = None) -> dict:
    """Every rank's reads on a K = 4 index (the reference's K_STEPS parameter;
    its GPU files stop at K = 2): built on the device with no host image (the
    51 GB of tag-100 entries stay in HBM), laid out as LAY_GRP -- one 128-B line
    per (block, 16-code group) -- and searched by the wave64 cooperative kernel
    in 25 K-steps per 100-bp read.  Timed like the main leg (barrier, max over
    ranks).  The intervals do not depend on K, so every rank's results must
    equal its K = 2 results (rank 0: and the pinned md5).  Config #5's read
    shape runs on it too (150 % 4 = 2: the last two bases of each read from the
    remainder table, then 37 K-steps), oracle-sampled against the K = 2 image.
    Every rank makes the same collective calls whatever fails locally (Steps)."""
    out = {"what": "coop-grp: K=4, d=64 index (LAY_GRP lines, device_index_bytes), wave64 cooperative LF, "
                   "the main leg's reads on every rank"}
    S = Steps()
    h = {}

    def setup():
        t = time.perf_counter()
        h["i4"] = K.Index.build(text, k=4, d=64, gpu=True, host_image=False)
        h["build_s"] = time.perf_counter() - t
        h["q"] = K.Queries.from_array(reads)
        h["r"] = K.Results.alloc(reads.shape[0])
        t = time.perf_counter()
        K.set_backend("coop-grp")
        K.transfer_to_gpu(h["i4"], h["q"], h["r"])
        h["upload_s"] = time.perf_counter() - t
        # 60 untimed searches: the first 30-40 after the 96 GB table's upload
        # run ~2 % slow (the fresh allocation warming up,
        # profiles/r03/sweep_k4_r3y.jsonl), a one-time cost of the upload
        for _ in range(60):
            K.search(h["i4"], h["q"], h["r"])

    def timed(lf):
        for _ in range(steps):
            K.search(h["i4"], h["q"], h["r"])
            lf.append(K.last_timing()["lf_ms"])

    def fetch():
        K.transfer_to_cpu(h["r"])
        return h["r"].array().copy()

    S.run(setup)
    got = None
    if D.all_ok(S.ok):
        lf = []
        D.barrier()
        t0 = time.perf_counter()
        S.run(timed, lf)
        D.barrier()
        el = D.max(time.perf_counter() - t0)
        got = S.run(fetch)
        total = D.sum(float(reads.shape[0]))
        lfm = float(np.mean(lf)) if lf else float("nan")
        out.update({"mqps": round(total * steps / el / 1e6, 2), "ms_per_step": round(el / steps * 1e3, 4),
                    "lf_ms": round(lfm, 3), "lf_ms_per_rank": D.gather(round(lfm, 4) if lf else None),
                    "device_index_bytes": h["i4"].device_bytes(),
                    "build_s_max": round(D.max(h["build_s"]), 2), "upload_s_max": round(D.max(h["upload_s"]), 2),
                    "results_equal_k2_per_rank": D.gather(got is not None and bool(np.array_equal(got, res)))})
        if pinned_md5 and D.rank == 0 and got is not None:
            out["results_md5_pinned"] = synth.results_md5(got) == pinned_md5
        blocks = S.run(K.count_blocks, h["i4"], h["q"])
        if blocks is not None and lf:
            # K*d/4 + 4 = 68 B per distinct block at K = 4
            out["roofline"] = dict(variant_roofline(blocks, 4 * 64 // 4 + 4, lfm, a, "coop-grp", pmc,
                                                    ceiling or PROBE_CEILING_GLINES, k=4), note="rank 0's launch")
            out["launches"] = launch_spec("coop-grp", 4, 64, reads.shape[1], reads.shape[0], 60, steps)
        if D.world == 1 and S.ok:
            i4, q, r = h["i4"], h["q"], h["r"]
            # opt-in jump start on the K = 4 index: the first 16 bases
            # (4 K-steps, most with L and R in different blocks) from a 34 GB table
            wall, lf1, tot1 = time_backend(i4, q, r, "coop-grp+ftab16", steps, 5)
            out["coop-grp+ftab16"] = {"mqps": round(reads.shape[0] / float(np.median(wall)) / 1e6, 2), "lf_ms": round(lf1, 3),
                                      "results_equal_k2": bool(np.array_equal(r.array(), res)),
                                      "device_bytes_incl_ftab": i4.device_bytes() + 8 * 4 ** 16}
            # the per-lane kernel on the same 96 GB lines, with its default
            # split-issue gathers (4 exec-masked groups of 16 lanes)
            wall, lf1, tot1 = time_backend(i4, q, r, "task-grp", steps, 5)
            out["task-grp"] = {"mqps": round(reads.shape[0] / float(np.median(wall)) / 1e6, 2), "lf_ms": round(lf1, 3),
                               "results_equal_k2": bool(np.array_equal(r.array(), res))}
    for k in ("q", "r"):
        if k in h:
            h[k].close()
    if c5_queries > 0:
        if D.all_ok(S.ok):
            out["config5"] = config5_leg(D, h["i4"], text, "coop-grp", c5_qlen, c5_queries, steps, 5, False,
                                         oracle_img=img2, k=4, pmc=pmc150)
    if "i4" in h:
        try:
            h["i4"].free_gpu()
            h["i4"].close()
        except K.KfmiError as e:
            S.err = S.err or str(e)
    errs = D.gather(S.err)
    if any(errs):
        out["error_per_rank"] = errs
    return out


def kstep3_leg(text: bytes, reads: np.ndarray, res: np.ndarray, steps: int) -> dict:
    """The main leg's reads on a K = 3 index (LAY_GRP, 4 lines per block; 100 %
    3 = 1 base from the remainder table, then 33 K-steps), one GPU."""
    t = time.perf_counter()
    i3 = K.Index.build(text, k=3, d=64, gpu=True, host_image=False)
    out = {"what": "coop-grp: K=3, d=64 index (LAY_GRP lines), wave64 cooperative LF, the main leg's reads",
           "build_s": round(time.perf_counter() - t, 2)}
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    try:
        wall, lf, tot = time_backend(i3, q, r, "coop-grp", steps, 5)
        out.update({"mqps": round(reads.shape[0] / float(np.median(wall)) / 1e6, 2), "lf_ms": round(lf, 3),
                    "device_index_bytes": i3.device_bytes(),
                    "results_equal_k2": bool(np.array_equal(r.array(), res))})
    finally:
        q.close()
        r.close()
        i3.free_gpu()
        i3.close()
    return out


def derived_leg(idx, reads: np.ndarray, res: np.ndarray, steps: int) -> dict:
    """The bench's K = 2 index, without its text, derived on the device into
    the K = 4 index (kfmi_derive_index_gpu, DESIGN.md 5d') and searched on the
    K = 4 grouped-counter layout: the reference's K = 2 file at K = 4 speed.
    The results must equal the K = 2 (md5-pinned) ones."""
    t = time.perf_counter()
    i4 = idx.derive(4)
    out = {"what": "K=4 index derived on the device from the K=2 index (no text), coop-grp",
           "derive_s": round(time.perf_counter() - t, 2)}
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    try:
        wall, lf, tot = time_backend(i4, q, r, "coop-grp", steps, 60)
        out.update({"mqps": round(q.num() / float(np.median(wall)) / 1e6, 2), "lf_ms": round(lf, 3),
                    "results_equal": bool(np.array_equal(r.array(), res)), "device_index_bytes": i4.device_bytes()})
        wall, lf, tot = time_backend(i4, q, r, "coop-grp+ftab16", steps, 5)
        out["ftab16"] = {"mqps": round(q.num() / float(np.median(wall)) / 1e6, 2), "lf_ms": round(lf, 3),
                         "results_equal": bool(np.array_equal(r.array(), res))}
    finally:
        q.close()
        r.close()
        i4.free_gpu()
        i4.close()
    return out


def time_backend(idx, q, r, backend, steps, warmup):
    """`backend` may carry "+ftabN": the Bowtie-style jump-start table of N bases."""
    name, _, opt = backend.partition("+")
    K.set_backend(name)
    K.set_ftab(int(opt[4:]) if opt.startswith("ftab") else 0)
    K.transfer_to_gpu(idx, q, r)
    for _ in range(warmup):
        K.search(idx, q, r)
    lf, tot, walls = [], [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        K.search(idx, q, r)
        walls.append(time.perf_counter() - t0)
        t = K.last_timing()
        lf.append(t["lf_ms"])
        tot.append(t["total_ms"])
    K.transfer_to_cpu(r)
    K.set_ftab(0)
    return walls, float(np.mean(lf)), float(np.mean(tot))


def _compact_row(v: dict | None, extra: tuple = ()) -> dict | None:
    """One backend's row for the line: Mq/s, HIP-event LF ms, algorithmic HBM
    fraction, fabric line requests per read (committed PMC pass), equality
    with the headline's md5-pinned results."""
    if not v:
        return None
    if "error" in v:
        return {"error": str(v["error"])[:120]}
    rf = v.get("roofline") or {}
    out = {"mqps": v.get("mqps"), "lf_ms": v.get("lf_ms", rf.get("lf_ms")), "frac": rf.get("frac", v.get("frac")),
           "lrpq": rf.get("line_requests_per_query")}
    if "results_equal" in v:
        out["eq"] = v["results_equal"]
    for k in extra:
        if k in v:
            out[k] = v[k]
    return {k: x for k, x in out.items() if x is not None}


def _all_true(xs) -> bool | None:
    xs = list(xs or [])
    return None if not xs or any(x is None for x in xs) else bool(all(xs))


def _max(xs):
    xs = [x for x in (xs or []) if x is not None]
    return max(xs) if xs else None


def config_rows(detail: dict, a=None) -> dict:
    """One short row per BASELINE.json config, from the full
    record: #1 the 64 Mbase plumbing case (GPU and the reference's CPU
    searcher), #2-#4 the reference's Task/Coop/AltCounters kernels -- each
    with its layout-matched MID form beside the reference layout -- #5 the
    per-GPU 150 bp shard, and K = 4 (coop-grp) on the same reads."""
    V = detail.get("variants") or {}
    rf = detail.get("roofline") or {}
    backend = (detail.get("config") or {}).get("backend")
    head = {"mqps": detail.get("value"), "lf_ms": rf.get("lf_ms"), "frac": rf.get("frac"),
            "lrpq": rf.get("line_requests_per_query"), "md5": (detail.get("parity") or {}).get("results_md5_pinned")}
    head = {k: x for k, x in head.items() if x is not None}

    def pick(b):
        if b == backend:
            return head
        r = _compact_row(V.get(b), extra=("derive_s",))
        if r and b == "derived_k4" and (V.get(b) or {}).get("ftab16"):
            r["ftab16"] = (V[b]["ftab16"] or {}).get("mqps")
        return r

    rows = {}
    c1 = V.get("config1_64mbase")
    if c1:
        if "error" in c1:
            rows["1"] = {"error": str(c1["error"])[:120]}
        else:
            ref = c1.get("cpu_reference") or {}
            prod = c1.get("cpu_product") or {}
            rows["1"] = {"what": "64 Mbase, 1M x 100 bp",
                         "gpu": {k: x for k, x in (("mqps", c1.get("mqps")), ("lf_ms", c1.get("lf_ms")),
                                                   ("frac", c1.get("frac")), ("md5", c1.get("results_md5_pinned")))
                                 if x is not None},
                         "cpu_ref": {k: x for k, x in (("mqps", ref.get("value")), ("cores", ref.get("cores")),
                                                       ("threads", ref.get("threads")),
                                                       ("eq", ref.get("parity_with_gpu"))) if x is not None},
                         "cpu_product": {k: x for k, x in (("mqps", prod.get("value")), ("cores", prod.get("cores")),
                                                           ("threads", prod.get("threads")),
                                                           ("eq", prod.get("equal_gpu"))) if x is not None}}
    for key, what, pair in (("2", "Task-2Step, 3 Gbase, 10M x 100 bp",
                             ("task-mid", "task", "task-mid+ftab16", "derived_k4")),
                            ("3", "Coop-2Step, same index and reads", ("coop-mid", "coop")),
                            ("4", "Task-2Step-AltCounters, same", ("task-ac", "task-ac-mid"))):
        r = {b: pick(b) for b in pair}
        if any(r.values()):
            rows[key] = dict(what=what, **{b: x for b, x in r.items() if x})

    def c5_row(c5):
        if not c5:
            return None
        if "mqps" not in c5:
            return {"error": str(c5.get("error_per_rank") or "no timing")[:120]}
        crf = c5.get("roofline") or {}
        h2h = c5.get("host_to_host") or {}
        out = {"mqps": c5.get("mqps"), "ms_per_step": c5.get("ms_per_step"),
               "lf_ms_max": _max(c5.get("lf_ms_per_rank")), "frac": crf.get("frac"),
               "lrpq": crf.get("line_requests_per_query"), "oracle_ok": _all_true(c5.get("oracle_sample_ok_per_rank")),
               "h2h_mqps": h2h.get("mqps"), "stream_mqps": (h2h.get("streamed") or {}).get("mqps")}
        return {k: x for k, x in out.items() if x is not None}

    c5 = c5_row(V.get("config5"))
    if c5:
        qlen = getattr(a, "config5_qlen", 150)
        nq = getattr(a, "config5_queries", 10_000_000)
        rows["5"] = dict(what=f"{nq // 1_000_000}M x {qlen} bp per GPU, index replicated", **c5)
    k4 = V.get("kstep4")
    if k4:
        r = _compact_row(k4) or {}
        if "results_md5_pinned" in k4:
            r["md5"] = k4["results_md5_pinned"]
        if k4.get("results_equal_k2_per_rank") is not None:
            r["eq_k2"] = _all_true(k4.get("results_equal_k2_per_rank"))
        k4c5 = c5_row(k4.get("config5"))
        ft = _compact_row(k4.get("coop-grp+ftab16"))
        if ft:
            ft.pop("eq", None)
            ft["eq_k2"] = (k4.get("coop-grp+ftab16") or {}).get("results_equal_k2")
        rows["k4"] = dict(what="K=4 index, coop-grp, same reads", **r, **({"c5": k4c5} if k4c5 else {}),
                          **({"ftab16": ft} if ft else {}))
    return rows


LINE_MAX = 6000   # bytes of the JSON line: the driver keeps an 8 KB stdout tail


def compact_line(detail: dict, detail_path: str | None) -> dict:
    """The one JSON line rank 0 prints: the contract's keys, a compact
    roofline and cpu_baseline, parity, launcher, whole-job rank summary and
    the per-config rows; everything else stays in the detail file whose path
    the line carries.  Held to LINE_MAX bytes: past it the rows' labels go,
    then the rows themselves (still in the detail file)."""
    line = {k: detail.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                       "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    cfg = detail.get("config") or {}
    line["config"] = {k: cfg[k] for k in ("workload", "backend", "k", "d", "ref_size", "queries_per_gpu", "qlen",
                                          "query_upload", "parallelism") if k in cfg}
    rf = detail.get("roofline") or {}
    line["roofline"] = {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                "bytes_per_launch", "traffic_over_algorithmic",
                                                "line_requests_per_query", "line_request_frac",
                                                "line_request_ceiling_G_per_s", "lf_ms", "kernel")}
    line["roofline"]["frac_is"] = "achieved HBM fraction: SURVEY 8(d) algorithmic bytes / LF time / 8 TB/s"
    cpu = detail.get("cpu_baseline")
    if cpu:
        line["cpu_baseline"] = {k: cpu.get(k) for k in ("value", "unit", "cores", "threads", "kind", "cpu_model",
                                                        "cgroup_cpu_quota", "parity_with_gpu")}
        line["cpu_baseline"]["sample"] = str(cpu.get("sample", ""))[:200]
    else:
        line["cpu_baseline"] = None
    line["parity"] = detail.get("parity")
    line["ranks_launched"] = detail.get("ranks_launched")
    line["launcher"] = detail.get("launcher")
    rk = detail.get("ranks") or {}
    dv = detail.get("devices") or {}
    line["ranks"] = {k: x for k, x in (("n", rk.get("n_ranks")), ("lf_ms_min", rk.get("lf_ms_min")),
                                       ("lf_ms_max", rk.get("lf_ms_max")), ("step_ms_max", rk.get("step_ms_max")),
                                       ("parity_ok_all", rk.get("parity_ok_all")),
                                       ("distinct_gpus", dv.get("distinct_devices")),
                                       ("shared_gpus", dv.get("shared_devices"))) if x is not None}
    line["configs"] = detail.get("configs") or {}
    line["detail"] = detail_path
    if len(json.dumps(line, separators=(",", ":"))) > LINE_MAX:
        line["configs"] = {k: {kk: vv for kk, vv in v.items() if kk != "what"} for k, v in line["configs"].items()}
    if len(json.dumps(line, separators=(",", ":"))) > LINE_MAX:
        line["configs"] = {"in_detail_file": True}
    if len(json.dumps(line, separators=(",", ":"))) > LINE_MAX:
        line["roofline"].pop("frac_is", None)
        line["cpu_baseline"] and line["cpu_baseline"].pop("sample", None)
    return line


def write_detail(detail: dict, path: str | None, world: int) -> str | None:
    """The full record (every leg, per-rank rows, probes, variants) as JSON:
    `path`, else gpurun_out/bench_detail_n<N>.json, else TMPDIR; its path, or
    None when nothing could be written."""
    tmp = Path(os.environ.get("TMPDIR") or "/tmp")
    cands = [Path(path)] if path else [ROOT / "gpurun_out" / f"bench_detail_n{world}.json",
                                       tmp / f"kfmi_bench_detail_n{world}_{os.getpid()}.json"]
    for p in cands:
        try:
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_text(json.dumps(detail, indent=1, default=str))
            return str(p)
        except OSError:
            continue
    return None


def main():
    a = parse()
    ws = os.environ.get("WORLD_SIZE")
    if a.gpus < 1:
        raise SystemExit(f"bench.py: --gpus {a.gpus}: need at least one rank")
    if ws is None and a.gpus > 1:
        # no launcher around us: start the N ranks here, before anything in
        # this process touches HIP (bench.spawn_ranks; no exec)
        raise SystemExit(spawn_ranks(a.gpus, sys.argv[1:]))
    if ws is not None and int(ws) != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={ws} ranks; "
                         "refusing to report a run of a different size")
    setup_logging(int(os.environ.get("RANK", "0")))
    D = Dist(a.gpus)
    ph = Phases()
    K.load()
    ndev = K.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no HIP device visible")
    # one rank per GPU: local rank r on device r.  With fewer devices than local
    # ranks (a rehearsal on one card) ranks wrap onto shared devices -- detected
    # below from the PCI bus ids and reported, never claimed as N GPUs
    dev = D.local % ndev
    K.set_device(dev)
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_device(dev)
    except Exception:
        pass
    dev_rows = device_rows(D, dev)
    dev_agg = aggregate_devices(dev_rows)
    if dev_agg["shared_devices"] and D.rank == 0:
        log(f"WARNING: {D.world} ranks on {dev_agg['distinct_devices']} distinct GPU(s) -- a rehearsal, "
            "not a multi-GPU measurement (n_gpus reports distinct devices, no scaling claim)", brief=True)
    if dev_agg["shared_devices"]:
        # ranks rehearsing on one card share its PCIe link: the streamed
        # search's transfer-mode model charges its link by that many
        # (kfmi_search_stream, KFMI_LINK_SHARERS)
        os.environ.setdefault("KFMI_LINK_SHARERS", str(max(dev_agg["ranks_per_device"])))
    ingest_on = a.ingest == "on" or (a.ingest == "auto" and D.world <= 2)
    # the reads sit in HBM as ASCII (the library's default upload, as the
    # reference's transferCPUtoGPU leaves them), so the timed search packs them
    # (fused into the LF kernel); the opt-in host-packed upload
    # (KFMI_UPLOAD=packed, DESIGN.md 6a') is timed in the end-to-end trio
    upload_form = os.environ.get("KFMI_UPLOAD", "ascii")
    ph.mark("init")

    # ---- inputs: reference text, index replica, this rank's reads ----------
    t = time.perf_counter()
    text = bench_text(D, a.ref_size)
    log(f"rank {D.rank}: text {len(text)} bases in {time.perf_counter() - t:.1f}s", brief=True)
    ph.mark("text")
    t = time.perf_counter()
    # N = 1: host image + SA samples (locate runs at N = 1 only).  N > 1: no
    # host image per rank; the oracle's image is shared on the node (shared_image)
    if D.world == 1:
        idx = K.Index.build(text, k=a.k, d=a.d, gpu=True, sa_rate=a.sa_rate)
    elif not dev_agg["shared_devices"]:
        idx = K.Index.build(text, k=a.k, d=a.d, gpu=True, host_image=False)
    else:
        # a rehearsal with ranks sharing a card: the builders' transient device
        # memory (the suffix sort) would peak on one card at once, so the ranks
        # take turns; on a node with a GPU per rank they build concurrently
        idx, err = None, None
        for r in range(D.world):
            if r == D.rank:
                try:
                    idx = K.Index.build(text, k=a.k, d=a.d, gpu=True, host_image=False)
                except K.KfmiError as e:
                    err = str(e)
            D.barrier()
        if not D.all_ok(err is None):
            raise SystemExit(f"bench.py: rank {D.rank}: index build failed: {err}")
    build_s = time.perf_counter() - t
    log(f"rank {D.rank}: GPU index build {build_s:.1f}s", brief=True)
    img = shared_image(D, idx)
    ph.mark("index_build")
    pinned = (a.ref_size == 3_000_000_000 and a.k == 2 and a.d == 64)
    index_md5_ok = None
    if pinned and D.rank == 0 and not a.no_md5:
        h = hashlib.md5(idx.image()).hexdigest()
        index_md5_ok = h == synth.MD5["ref3g.k2d64.fmi"]
        log(f"index md5 {h} pinned-ok={index_md5_ok}", brief=True)
    t = time.perf_counter()
    starts = synth.read_starts(len(text), a.queries, a.qlen, seed=10 + D.rank)
    reads = synth.gather_reads(text, starts, a.qlen)
    del starts
    log(f"rank {D.rank}: {reads.shape[0]} reads in {time.perf_counter() - t:.1f}s")
    ph.mark("reads")

    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    K.set_backend(a.backend)
    t = time.perf_counter()
    K.transfer_to_gpu(idx, q, r)
    upload_s = time.perf_counter() - t
    dev_index_bytes = idx.device_bytes()

    # ---- timed region --------------------------------------------------------
    for _ in range(a.warmup):
        K.search(idx, q, r)
    cuda_sync(dev)
    D.barrier()
    lf_ms, tot_ms, pack_ms = [], [], []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        K.search(idx, q, r)
        tm = K.last_timing()
        lf_ms.append(tm["lf_ms"])
        tot_ms.append(tm["total_ms"])
        pack_ms.append(tm["pack_ms"])
    cuda_sync(dev)
    D.barrier()
    elapsed = time.perf_counter() - t0
    ph.mark("upload_warmup_timed")
    elapsed_max = D.max(elapsed)
    total_queries = D.sum(float(reads.shape[0]))
    ms_per_step = elapsed_max / a.steps * 1e3
    value = total_queries * a.steps / elapsed_max / 1e6      # Mqueries/s, whole job

    # ---- correctness of the timed results -----------------------------------
    t = time.perf_counter()
    K.transfer_to_cpu(r)
    d2h_s = time.perf_counter() - t
    res = r.array().copy()
    results_md5_ok = None
    if pinned and a.qlen == 100 and a.queries == 10_000_000 and D.rank == 0 and not a.no_md5:
        results_md5_ok = synth.results_md5(res) == synth.MD5["res3g.q10M"]
        log(f"timed: {value:.1f} Mq/s, LF {np.mean(lf_ms):.3f} ms; results md5 pinned-ok={results_md5_ok}", brief=True)
    # every rank: an evenly spread sample of its own results against the CPU
    # oracle (oracle/fmi_oracle.c, test infrastructure; never on the timed path),
    # with the semantics of the backend (AltCounters for the *-ac backends)
    parity_ok, ns_par = None, min(a.parity_sample, reads.shape[0])
    if ns_par > 0:
        from oracle import oracle
        t = time.perf_counter()
        sel = np.linspace(0, reads.shape[0] - 1, ns_par).astype(np.int64)
        ac = a.backend in ("task-ac", "coop-ac")
        img_idx = idx.alt_counters()[0] if ac else None
        want, _ = oracle.search(img_idx.image() if ac else img, reads[sel],
                                nthreads=max(1, cpu_effective() // D.world))
        parity_ok = bool(np.array_equal(want.reshape(-1, 2), res.reshape(-1, 2)[sel]))
        if ac:
            img_idx.close()
        log(f"rank {D.rank}: oracle sample {ns_par} reads parity_ok={parity_ok} ({time.perf_counter() - t:.1f}s)", brief=True)
    ph.mark("parity")

    # ---- roofline: algorithmic bytes of the LF kernel ------------------------
    blocks = K.count_blocks(idx, q)
    b_lf = a.k * a.d // 4 + 4                               # bit planes of one block + one counter
    bytes_alg = blocks * b_lf                               # 36 B x distinct blocks
    # reported beside it: what the LF kernel also reads per query (the ASCII row
    # when packing is fused into the task kernel, else the packed code words)
    # and the (L, R) it writes
    spw = 16 // a.k
    nwords = (a.qlen // a.k + spw - 1) // spw
    fused = os.environ.get("KFMI_FUSED", "1") != "0" and nwords <= 16
    q_in = a.qlen if fused else 4 * nwords
    bytes_io = reads.shape[0] * (q_in + 8)
    lf_avg_ms = float(np.mean(lf_ms))
    achieved = bytes_alg / (lf_avg_ms / 1e3) / 1e9
    # traffic per launch from the committed PMC profile of the same config, by
    # the guide's recipe (MI355X_MICROARCH.md HBM section): FETCH_SIZE in its own
    # pass, doubled (gfx950 tallies a 128-B request at 64 B; every request here
    # is 128 B, TCC_EA0_RDREQ_128B).  It counts every L2 miss, Infinity-Cache
    # hits included, so it is the L2/fabric traffic and bounds the HBM bytes
    # from above; no gfx950 counter separates the Infinity-Cache hits.
    traffic, traffic_src, traffic_note, rdreq, replay_pmc = None, None, None, None, None
    tj = Path(a.traffic_json)
    if tj.exists() and D.world == 1:   # a one-GPU PMC profile says nothing about N > 1 runs
        try:
            tr = json.loads(tj.read_text())
            if (tr.get("backend") == a.backend and tr.get("queries") == a.queries and tr.get("ref_size") == a.ref_size
                    and tr.get("qlen", 100) == a.qlen and tr.get("k", 2) == a.k and tr.get("d", 64) == a.d):
                traffic = tr.get("fetch_size_corrected_bytes_per_launch")
                traffic_src, traffic_note = tr.get("fetch_size_source"), tr.get("fetch_size_correction")
                rdreq = tr.get("rdreq_per_launch")
                replay_pmc = tr.get("replay")
        except Exception:
            traffic = None
    # the kernel's own request stream replayed without its LF dependence
    # (kfmi_probe_replay: MID layouts): a measured ceiling for that exact mix
    replay = None
    if D.world == 1 and D.rank == 0 and a.backend in ("task-mid", "coop-mid") and a.k == 2 and a.d == 64:
        try:
            replay = [K.probe_replay(idx, q, unroll=u, groups=g, reps=5)
                      for u, g in ((0, 1), (0, 2), (1, 1), (1, 2), (2, 2), (4, 2), (8, 2))]
        except K.KfmiError as e:
            log(f"replay probe unavailable: {e}")
    ph.mark("count_blocks")
    # ---- auxiliary legs: each makes the same collective calls on every rank
    # whatever fails locally (Steps), so one failing rank never hangs the rest
    # the committed PMC passes (one GPU; not applied to N > 1 runs)
    pmc100 = load_variants_pmc(a.queries, a.ref_size, a.qlen, a.d) if D.world == 1 else None
    pmc150 = (load_variants_pmc(a.config5_queries, a.ref_size, a.config5_qlen, a.d, VARIANTS_PMC_Q150)
              if D.world == 1 else None)
    c5 = None
    if a.config5_queries > 0:
        c5 = config5_leg(D, idx, text, a.backend, a.config5_qlen, a.config5_queries, a.steps, 5,
                         a.backend in ("task-ac", "coop-ac", "task-ac-mid",
                                       "coop-ac-mid"), oracle_img=img, ingest=ingest_on, k=a.k, d=a.d, pmc=pmc150)
        log(f"rank {D.rank}: config #5 leg {c5}")
        log(f"config #5 leg: {c5.get('mqps')} Mq/s", brief=True)
        ph.mark("config5")
    ingest = None
    if ingest_on:
        S = Steps()
        ingest = S.run(ingest_leg, idx, reads, res, D.world) or {"error": S.err}
        os.environ.pop("KFMI_LOAD_MMAP", None)
        log(f"rank {D.rank}: ingest {ingest}")
        ph.mark("ingest")
    k4 = None
    if a.kstep4 and a.k == 2 and a.d == 64:
        # ---- K = 4 on every rank's reads (LAY_GRP, coop kernel) --------------
        k4 = kstep4_leg(D, text, reads, res, img, a.steps,
                        synth.MD5["res3g.q10M"] if (pinned and a.qlen == 100 and a.queries == 10_000_000)
                        else None, a.config5_qlen, a.config5_queries, a=a,
                        pmc=pmc100, pmc150=pmc150)
        log(f"rank {D.rank}: K=4 leg {k4}")
        log(f"K=4 leg: {k4.get('mqps')} Mq/s", brief=True)
        ph.mark("kstep4")
    rank_rows = D.gather({"ingest": ingest, "rank": D.rank, "device": dev,
                          "pci_bus_id": dev_rows[D.rank]["pci_bus_id"], "queries": int(reads.shape[0]),
                          "lf_ms": round(float(np.mean(lf_ms)), 4), "step_ms": round(float(np.mean(tot_ms)), 4),
                          "elapsed_s": round(elapsed, 4), "distinct_blocks": int(blocks),
                          "parity_ok": parity_ok, "parity_sample": int(ns_par),
                          "results_md5_pinned": results_md5_ok})
    ranks = aggregate_ranks(rank_rows)

    extra = {}
    ph.mark("gather")
    probe = probe_leg() if D.world == 1 and D.rank == 0 else None
    ceiling = probe["ceiling_G_lines_per_s"] if probe else PROBE_CEILING_GLINES
    ceiling_src = ((f"gather_probe on this box, this run: the larger of the 3 GB (HBM) and 200 MB "
                    f"(Infinity-Cache-resident, best of {probe['infinity_cache_200MB']['runs']} runs per kind) "
                    f"random-line rates ({probe['ceiling_from']})") if probe else
                   "profiles/r03/gather_probe_r3g.jsonl: 200 MB table, Infinity-Cache resident (another box)")
    if probe:
        extra["line_request_probe"] = probe
        log(f"gather probe: ceiling {ceiling} G lines/s ({probe['ceiling_from']})")
    rp = replay_requests(replay, replay_pmc)
    if rp and rp["best_G_requests_per_s"] > ceiling:
        # the kernel's own line stream without its dependence issued faster than
        # the probe's uniform lines: that rate is the ceiling for this mix
        ceiling = rp["best_G_requests_per_s"]
        ceiling_src = (f"kfmi_probe_replay on this box, this run: the kernel's own line stream re-issued without "
                       f"its LF dependence ({rp['best_mode']}), fabric requests per launch from "
                       f"{replay_pmc.get('source', 'the committed PMC pass')}; above the gather_probe rate")
    if c5 is not None:
        extra["config5"] = c5
    if k4 is not None:
        extra["kstep4"] = k4
    if a.kstep4 and a.k == 2 and a.d == 64 and D.world == 1:
        try:
            extra["kstep3"] = kstep3_leg(text, reads, res, a.steps)
            log(f"K=3 leg {extra['kstep3']}")
        except K.KfmiError as e:
            extra["kstep3"] = {"error": str(e)}
    if a.kstep4 and a.k == 2 and a.d == 64 and D.world == 1:
        try:
            extra["derived_k4"] = derived_leg(idx, reads, res, a.steps)
            log(f"derived K=4 leg {extra['derived_k4']}")
            log(f"derived K=4 leg: {extra['derived_k4'].get('mqps')} Mq/s", brief=True)
        except K.KfmiError as e:
            extra["derived_k4"] = {"error": str(e)}
        K.set_backend(a.backend)
    if ingest is not None:
        extra["ingest_file"] = ingest          # rank 0's; every rank's is under "ranks"
    cpu = None
    if D.rank == 0 and D.world == 1 and a.sa_rate:
        # ---- locate: text positions of every [L, R) ---------
        loc = K.locate(idx, r)                                  # warm-up (SA upload)
        loc.close()
        lms, kms = [], []
        for _ in range(a.locate_steps):
            t = time.perf_counter()
            loc = K.locate(idx, r)
            lms.append((time.perf_counter() - t) * 1e3)
            kms.append(K.last_timing()["lf_ms"])
            if _ < a.locate_steps - 1:
                loc.close()
        off, pos = loc.offsets(), loc.positions()
        # property check on a sample: every first position starts its read
        t8 = np.frombuffer(text, dtype=np.uint8)
        smp = np.arange(0, reads.shape[0], max(1, reads.shape[0] // 100_000))
        has = off[smp + 1] > off[smp]
        p0 = pos[off[smp[has]].astype(np.int64)].astype(np.int64)
        ok = bool(has.all()) and bool(np.array_equal(t8[p0[:, None] + np.arange(a.qlen)[None, :]], reads[smp[has]]))
        extra["locate"] = {"sa_rate": a.sa_rate, "positions": int(loc.total()),
                           "kernel_ms": round(float(np.median(kms)), 3),
                           "call_ms": round(float(np.median(lms)), 3),
                           "Mpositions_per_s": round(loc.total() / (float(np.median(kms)) / 1e3) / 1e6, 1),
                           "sample_checked": int(has.sum()), "positions_start_reads": ok,
                           "what": "kfmi_locate on the timed batch's device results: count + scan + LF_K walk "
                                   "to a sampled row (kernel_ms = walk kernel, call_ms = incl. D2H of positions)"}
        log(f"locate {extra['locate']}")
        loc.close()
    variants_pmc = pmc100
    if D.rank == 0 and D.world == 1:
        # ---- other backends (same index, same reads) ------------------------
        for b in [x for x in a.variants.split(",") if x and x != a.backend]:
            try:
                walls, lf, tot = time_backend(idx, q, r, b, a.variant_steps, 10)
                ok = bool(np.array_equal(r.array(), res))
                # per-call wall clock (search + sync through the C ABI), median
                # over the steps so one host hiccup on a shared box does not
                # stand in for the backend; the mean is kept beside it
                extra[b] = {"mqps": round(reads.shape[0] / float(np.median(walls)) / 1e6, 2),
                            "mqps_mean_wall": round(reads.shape[0] * len(walls) / float(np.sum(walls)) / 1e6, 2),
                            "lf_ms": round(lf, 3), "step_ms": round(tot, 3), "results_equal": ok,
                            "device_index_bytes": idx.device_bytes()}
                if "+" not in b:
                    # the row's own roofline: algorithmic bytes of this backend's
                    # launch (36 B x distinct blocks, counted on the device with
                    # the backend's own LF semantics), its HIP-event LF time, and
                    # its fabric read requests from the committed PMC pass
                    extra[b]["roofline"] = variant_roofline(K.count_blocks(idx, q), b_lf, lf, a, b, variants_pmc,
                                                            ceiling)
                    extra[b]["launches"] = launch_spec(b, a.k, a.d, a.qlen, reads.shape[0], 10, a.variant_steps)
                log(f"variant {b}: {extra[b]}")
            except K.KfmiError as e:
                extra[b] = {"error": str(e)}
            idx.free_gpu()
        log("variants: " + ", ".join(f"{b} {extra[b].get('mqps')}" for b in a.variants.split(",")
                                     if b in extra and b != a.backend), brief=True)
        # ---- device-group replication (kfmi_set_devices): the layout is built
        # once and fanned out device-to-device; here one card listed n times ----
        try:
            K.set_backend(a.backend)
            reps, parts = {}, {}
            for nrep in (1, 2, 4):
                K.set_devices([dev] * nrep if nrep > 1 else [])
                idx.free_gpu()
                t = time.perf_counter()
                K.transfer_to_gpu(idx, None, None)
                reps[str(nrep)] = round(time.perf_counter() - t, 3)
                if nrep > 1:
                    lt = K.last_timing()
                    parts[str(nrep)] = {"members_streams_events_ms": round(lt["pack_ms"], 2),
                                        "fan_out_ms": round(lt["lf_ms"], 2),
                                        "first_member_upload_ms": round(lt["total_ms"] - lt["pack_ms"] - lt["lf_ms"], 2)}
            K.set_devices([])
            idx.free_gpu()
            extra["group_replication"] = {"setup_s_by_replicas": reps, "breakdown_by_replicas": parts,
                                          "what": "transferCPUtoGPU(index) for a device group of n replicas "
                                                  "on this card: host upload + relayout on the first, "
                                                  "hipMemcpyPeerAsync to the others (kfmi_last_timing split)"}
            log(f"group replication {extra['group_replication']}")
        except Exception as e:
            K.set_devices([])
            extra["group_replication"] = {"error": repr(e)}
        # ---- end to end from host memory: streamed H2D + search + D2H ------
        if a.e2e_steps > 0:
            try:
                K.set_backend(a.backend)
                K.transfer_to_gpu(idx, None, None)
                e2e = {}
                pin = K.pinned_empty(reads.shape, np.uint8)
                pin[:] = reads
                pout = K.pinned_empty((2 * reads.shape[0],), np.uint32)
                for kind, src, dst in (("pinned", pin, pout), ("pageable", reads, None)):
                    out = K.search_stream(idx, src, out=dst)          # warm-up (buffer allocation)
                    t = time.perf_counter()
                    for _ in range(a.e2e_steps):
                        out = K.search_stream(idx, src, out=dst)
                    w = (time.perf_counter() - t) / a.e2e_steps
                    lt = K.last_timing()
                    e2e[kind] = {"mqps": round(reads.shape[0] / w / 1e6, 2), "ms": round(w * 1e3, 3),
                                 "host_ms": round(lt["pack_ms"], 3), "wait_ms": round(lt["lf_ms"], 3),
                                 "hostpacked_fraction": round(K.load().kfmi_stream_hostpacked_fraction(), 3),
                                 "results_equal": bool(np.array_equal(out, res))}
                hp_mode = os.environ.get("KFMI_STREAM_HOSTPACK", "2")
                e2e["chunk_queries"] = int(os.environ.get("KFMI_STREAM_CHUNK", (1 << 16) if hp_mode == "0" else (1 << 19)))
                e2e["host_pack"] = {"0": "never", "1": "always", "3": "alternate"}.get(hp_mode, "adaptive")
                e2e["what"] = "kfmi_search_stream: ASCII reads in host memory -> results in host memory; " \
                              "per chunk host 2-bit packing (qpack.c, KFMI_HOST_THREADS) + code-word H2D, or " \
                              "ASCII H2D + device packing, chosen from measured rates; LF / D2H of successive " \
                              "chunks overlapped on KFMI_STREAM_SLOTS (default 6) HIP streams"
                # the reference's own trio from pageable memory (transferCPUtoGPU,
                # searchIndexGPU, transferGPUtoCPU on the resident index): the
                # ASCII upload (default) and the opt-in host-packed one
                trio, prev_upload = {}, os.environ.get("KFMI_UPLOAD")
                for form in ("ascii", "packed"):
                    os.environ["KFMI_UPLOAD"] = form
                    tq = K.Queries.from_array(reads)
                    tr = K.Results.alloc(reads.shape[0])
                    walls, parts = [], []
                    for i in range(a.e2e_steps + 1):
                        t0 = time.perf_counter()
                        K.transfer_to_gpu(idx, tq, tr)
                        t1 = time.perf_counter()
                        K.search(idx, tq, tr)
                        t2 = time.perf_counter()
                        K.transfer_to_cpu(tr)
                        t3 = time.perf_counter()
                        if i:                               # the first round allocates
                            walls.append(t3 - t0)
                            parts.append((t1 - t0, t2 - t1, t3 - t2))
                    w = float(np.median(walls))
                    med = np.median(np.array(parts), axis=0) * 1e3
                    trio[form] = {"mqps": round(reads.shape[0] / w / 1e6, 2), "ms": round(w * 1e3, 3),
                                  "transfer_to_gpu_ms": round(float(med[0]), 3), "search_ms": round(float(med[1]), 3),
                                  "lf_ms": round(K.last_timing()["lf_ms"], 4),
                                  "transfer_to_cpu_ms": round(float(med[2]), 3),
                                  "results_equal": bool(np.array_equal(tr.array(), res))}
                    tq.close()
                    tr.close()
                if prev_upload is None:
                    os.environ.pop("KFMI_UPLOAD", None)
                else:
                    os.environ["KFMI_UPLOAD"] = prev_upload
                trio["what"] = ("the reference's transfer/search/transfer trio from pageable host memory, "
                                "median of e2e_steps rounds: `ascii` (the default) uploads the reads as they "
                                "are (packed inside the search), `packed` (KFMI_UPLOAD=packed) packs them to "
                                "2-bit words on the host during the upload (DESIGN.md 6a')")
                e2e["trio"] = trio
                extra["end_to_end"] = e2e
                log(f"end to end {e2e}")
                del pin, pout
                K.load().kfmi_stream_release()
            except K.KfmiError as e:
                extra["end_to_end"] = {"error": str(e)}
    # ---- CPU baseline on rank 0 at any N: the reference's CPU searcher and the
    # restatement on every core of the affinity mask (other ranks wait) --------
    if D.rank == 0 and a.cpu_sample > 0:
        from oracle import oracle
        thrs = [a.cpu_threads] if a.cpu_threads else baseline_thread_counts()
        ns = min(a.cpu_sample, reads.shape[0])
        ports = []
        for thr in thrs:
            t = time.perf_counter()
            cres, _ = oracle.search(img, reads[:ns], nthreads=thr)
            cpu_s = time.perf_counter() - t
            ports.append({"value": round(ns / cpu_s / 1e6, 4), "unit": "Mqueries/s", "cores": cores_used(thr),
                          "threads": thr, "kind": "port",
                          "sample": f"first {ns} of the same 10M reads, 1 pass, oracle/fmi_oracle.c "
                                    f"(restatement of fmIndexCPUBaseline.c), OMP threads={thr}, {cpu_s:.2f}s",
                          "parity_with_gpu": bool(np.array_equal(cres, res[:2 * ns]))})
        port = max(ports, key=lambda x: x["value"])
        if len(ports) > 1:
            port = dict(port, other_runs=[{"cores": x["cores"], "threads": x["threads"], "value": x["value"]}
                                          for x in ports if x is not port])
        log(f"cpu baseline (port) {port}")
        cpu = None
        if not a.cpu_port_only:
            try:
                cpu = cpu_reference_baseline(idx, reads, ns, a.k, a.d, thrs, res)
            except Exception as e:          # the reference binary is a baseline, never the product
                log(f"reference cpu baseline unavailable: {e}")
        if cpu is None:
            cpu = port
        else:
            extra["cpu_port"] = port
        cpu["cpu_model"] = cpu_model()
        cpu["affinity_cores"] = cpu_threads()
        cpu["os_cpu_count"] = os.cpu_count()
        cpu["cgroup_cpu_quota"] = cpu_quota()
        if a.config1 and D.world == 1:
            try:
                extra["config1_64mbase"] = config1_leg(a.backend, thrs)
                log(f"config #1 {extra['config1_64mbase']}")
            except K.KfmiError as e:
                extra["config1_64mbase"] = {"error": str(e)}
        # single-thread rate of the restatement on a small slice
        n1 = min(100_000, ns)
        t = time.perf_counter()
        oracle.search(img, reads[:n1], nthreads=1)
        extra["cpu_port_1thread"] = {"value": round(n1 / (time.perf_counter() - t) / 1e6, 4),
                                     "unit": "Mqueries/s", "cores": 1, "threads": 1, "sample": f"first {n1} reads"}
        # the product's own host search (searchIndexCPU, csrc/host/cpu_search.c: batched
        # prefetch, the reference CPU driver's drop-in) on the same sample and cores
        extra["cpu_product"] = cpu_product_rows(idx, reads[:ns], res[:2 * ns], thrs)
        log(f"cpu product {extra['cpu_product']}")
        log(f"cpu baseline {cpu}")
        log(f"cpu baseline: {cpu.get('value')} Mq/s, {cpu.get('threads')} threads on {cpu.get('cores')} cores "
            f"({cpu.get('kind')})", brief=True)
    ph.mark("rank0_n1_legs_and_cpu_baseline")
    # per-rank phase wall times and peak host RSS (the N = 8 budget: DESIGN.md 7)
    ph_rows = D.gather({"rank": D.rank, "phases_s": ph.rows, "peak_rss_gb": Phases.peak_rss_gb(),
                        "rss_anon_peak_gb": ph.anon_peak})
    phases = {"per_rank": ph_rows,
              "max_over_ranks_s": {k: max(r["phases_s"].get(k, 0.0) for r in ph_rows) for k in ph.rows},
              "wall_s_max": round(max(sum(r["phases_s"].values()) for r in ph_rows), 1),
              "peak_rss_gb_max": max(r["peak_rss_gb"] for r in ph_rows),
              # private memory (sampled at every phase end): the node-shared text
              # and image mappings (N > 1) are page cache, counted once per node
              "rss_anon_peak_gb_max": max(r["rss_anon_peak_gb"] for r in ph_rows),
              "shared_text_and_image": D.world > 1,
              "host_threads_per_rank": K.host_threads(),
              "ingest_legs": ingest_on}

    if D.rank == 0:
        detail = {
            "metric": f"Mqueries/s ({a.qlen} bp reads, {a.ref_size / 1e9:g} Gbase index)",
            "value": round(value, 3),
            "unit": "Mqueries/s",
            # distinct physical GPUs (PCI bus ids), not ranks: a one-card rehearsal
            # with two ranks reports 1 and makes no scaling claim
            "n_gpus": dev_agg["distinct_devices"],
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": None if dev_agg["shared_devices"] else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: seeded uniform-ACGT reference + exact-substring reads (SURVEY App. C recipe, md5-pinned)",
            "config": {"workload": f"{'Task' if a.backend.startswith('task') else 'Coop'}-{a.k}Step backward search, "
                                   f"{a.ref_size / 1e9:g} Gbase index, {a.queries // 1_000_000}M x {a.qlen} bp reads per GPU",
                       "backend": a.backend, "k": a.k, "d": a.d, "ref_size": a.ref_size,
                       "queries_per_gpu": a.queries, "qlen": a.qlen, "query_upload": upload_form,
                       "parallelism": f"query-sharded dp{D.world}, index replicated per GPU, no collective"
                                      + (f" (REHEARSAL: {D.world} ranks on {dev_agg['distinct_devices']} GPU(s))"
                                         if dev_agg["shared_devices"] else "")},
            "ranks_launched": D.world,
            "launcher": os.environ.get("KFMI_BENCH_LAUNCHER", "external" if D.world > 1 else "none"),
            "devices": dict(dev_agg, per_rank=dev_rows),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": kernel_prefix(a.backend, a.k, a.d, a.qlen).split("<", 1)[0].replace("kfmi::", "")
                                   + f" {a.backend}, HIP-event average over the timed steps",
                         "launches": launch_spec(a.backend, a.k, a.d, a.qlen, reads.shape[0], a.warmup, a.steps),
                         "bytes_per_launch": bytes_alg, "distinct_blocks": blocks, "bytes_per_block": b_lf,
                         "bytes_per_query_io": q_in + 8,
                         "achieved_incl_query_io": round((bytes_alg + bytes_io) / (lf_avg_ms / 1e3) / 1e9, 1),
                         "lf_ms": round(lf_avg_ms, 4), "pack_ms": round(float(np.mean(pack_ms)), 4),
                         "naive_bytes_per_launch": 2 * (a.qlen // a.k) * b_lf * a.queries,
                         "traffic_source": traffic_src,
                         "traffic_method": traffic_note,
                         # the L2/fabric bytes per second the kernel moves (whole 128-B lines), and
                         # how many of them per algorithmic byte: a random LF reads 36 B of a line
                         # that can only be fetched whole, not a re-read
                         "traffic_GB_per_s": round(traffic / (lf_avg_ms / 1e3) / 1e9, 1) if traffic else None,
                         "traffic_over_algorithmic": round(traffic / bytes_alg, 3) if traffic else None,
                         # those bytes against 8 TB/s: NOT the HBM fraction (Infinity-Cache hits
                         # are in the count; it can exceed the 6.29 TB/s achievable HBM rate).
                         # BASELINE's "achieved HBM GB/s %" is `frac`
                         "l2_fabric_line_bytes_vs_8TBs_incl_ic_hits":
                             round(traffic / (lf_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                         # every LF is a random 128-B line: the binding limit is the rate of random line
                         # requests at the L2/fabric boundary, calibrated by gather_probe on the same 3 GB
                         # table size.  Requests x 128 B includes Infinity-Cache hits: an upper bound on HBM
                         # bytes, compared with the probe's request ceiling, never with the HBM peak
                         "fabric_read_requests_per_launch": rdreq,
                         "fabric_request_bytes_upper_bound": rdreq * 128 if rdreq else None,
                         "line_requests_per_query": round(rdreq / a.queries, 2) if rdreq else None,
                         "line_requests_G_per_s": round(rdreq / (lf_avg_ms / 1e3) / 1e9, 2) if rdreq else None,
                         "line_request_ceiling_G_per_s": ceiling,
                         "line_request_ceiling_source": ceiling_src,
                         "line_request_frac": round(rdreq / (lf_avg_ms / 1e3) / 1e9 / ceiling, 3) if rdreq else None,
                         # the same question on the kernel's own fetches (distinct blocks = lines it loads):
                         # its rate against the fastest replay of the identical request stream
                         "replay": None if not replay else {
                             "kernel_G_lines_per_s": round(blocks / (lf_avg_ms / 1e3) / 1e9, 2),
                             "replay_G_lines_per_s": {f"u{x['unroll']}g{x['groups']}": round(x["G_lines_per_s"], 2)
                                                      for x in replay},
                             "replay_ms": {f"u{x['unroll']}g{x['groups']}": round(x["ms"], 4) for x in replay},
                             "lines_per_launch": replay[0]["lines"], "trace_bytes_per_launch": replay[0]["trace_bytes"],
                             # requests: the replay's lines plus its trace stream, counted by the
                             # committed PMC pass of the same kernels on the same batch (rocprofv3
                             # TCC_EA0_RDREQ; modes that pass did not cover take the median count)
                             "kernel_G_requests_per_s": round(rdreq / (lf_avg_ms / 1e3) / 1e9, 2) if rdreq else None,
                             **({"replay_requests_per_launch": rp["requests"],
                                 "replay_G_requests_per_s": rp["G_requests_per_s"],
                                 "replay_best_G_requests_per_s": rp["best_G_requests_per_s"],
                                 "replay_best_mode": rp["best_mode"],
                                 "replay_requests_source": replay_pmc.get("source")} if rp else {}),
                             "note": "the replay streams its trace beside the lines (its requests include "
                                     "it); it shows whether lifting the LF dependence (1-8 K-steps of loads in "
                                     "flight per lane) raises the request rate, and when its rate is above the "
                                     "gather_probe's it is the stated ceiling (DESIGN.md 5)",
                             "what": "kfmi_probe_replay: every (K-step, read) end's MID128 line recorded by a trace "
                                     "launch, then the task kernel's loads for them issued from the trace (no LF "
                                     "dependence): uU = U K-steps of C++ loads in flight per lane, u0 = the kernel's "
                                     "own asm fetch (one K-step in flight); gG = G exec-masked lane groups; rate = "
                                     "lines / replay time (the trace, 8 B per read per K-step, streams beside them)"}},
            "cpu_baseline": cpu,
            "parity": {"index_md5_pinned": index_md5_ok, "results_md5_pinned": results_md5_ok,
                       "oracle_sample_ok": ranks["parity_ok_all"], "oracle_sample_per_rank": int(ns_par)},
            "ranks": ranks,
            "setup_s": {"gpu_index_build": round(build_s, 2), "h2d": round(upload_s, 2), "d2h": round(d2h_s, 3)},
            "device_index_bytes": dev_index_bytes,
            "phases": phases,
            "variants": extra,
        }
        detail["configs"] = config_rows(detail, a)
        dpath = write_detail(detail, a.detail, D.world)
        line = compact_line(detail, dpath)
        log(f"detail: {dpath}; line {len(json.dumps(line))} B", brief=True)
        # the line is the last thing on stdout, after everything on stderr
        sys.stderr.flush()
        print(json.dumps(line, separators=(",", ":")), flush=True)
    D.barrier()          # every rank leaves together (rank 0 ran the CPU baseline)
    D.close()


if __name__ == "__main__":
    main()
