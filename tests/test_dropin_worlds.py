"""Seeded random worlds through the reference's own driver.

common/searchQueries.c, compiled unmodified against libkstepfmi.so
(oracle/Makefile: searchQueries_cpu_dropin without -DCUDA, searchQueries_dropin
with it), reads an index file written by the reference's builder and
transforms (oracle/_ref/gfmi_K_d, tfmiBMP_K_d, tfmiAC_K_d) and a query FASTA,
and writes its results file; the reference's own CPU searchers
(oracle/_ref/cpu_K_d, cpuac_K_d: searchQueries.c + fmIndexCPUBaseline*.c) write
theirs from the same files.  The two must be byte-identical: through the
library's searchIndexCPU in the CPU suite, through every GPU backend that takes
the file's tag in the GPU suite.  Worlds avoid the geometries where the
reference's own result is undefined: (n+1) % d == 0 (B5; and, for the
AltCounters files, (n+1) % d >= d - K, tests/test_gpu_parity.py
test_ac_tail_blocks) and m % K != 0 (B6)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from util import REPO

REF = REPO / "oracle" / "_ref"
ACGT = np.frombuffer(b"ACGT", np.uint8)
WORLDS = 40
GEOMS = [(1, 64), (2, 64), (1, 192), (2, 192), (3, 64), (4, 64)]
TAGS = {100: "", 101: ".interleaving", 200: ".ac", 201: ".interleaving.ac"}
PLAIN = ("task", "coop", "task-mid", "coop-mid")
ALT = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")


def world(i):
    rng = np.random.default_rng(60_000 + i)
    k, d = GEOMS[int(rng.integers(0, len(GEOMS)))]
    while True:
        n = int(rng.integers(300, 20_000))
        r = (n + 1) % d
        if r != 0 and r < d - k:
            break
    kind = int(rng.integers(0, 3))
    if kind == 0:
        t = ACGT[rng.integers(0, 4, size=n)]
    elif kind == 1:
        t = np.repeat(ACGT[rng.integers(0, 4, size=n)], rng.integers(1, 25, size=n))[:n]
    else:
        t = ACGT[rng.integers(0, 4, size=n)]
        for _ in range(8):   # copies: wide intervals
            a, b = rng.integers(0, n - 200, size=2)
            t[b:b + 150] = t[a:a + 150]
    t = np.ascontiguousarray(t, np.uint8)
    m = k * int(rng.integers(1, 160 // k + 1))
    nq = int(rng.integers(1, 3000))
    st = rng.integers(0, n - m + 1, size=nq)
    q = np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                        rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(nq // 5 + 1, m))])
    return k, d, t.tobytes(), q, rng


def _prepare(tmp_path, k, d, text, q):
    for tool in ("gfmi", "tfmiBMP", "tfmiAC", "cpu", "cpuac"):
        if k > 2 and tool != "gfmi" and tool != "cpu":
            continue
        if not (REF / f"{tool}_{k}_{d}").exists():
            pytest.skip("oracle/_ref not built (needs /root/reference)")
    n = len(text)
    (tmp_path / "ref.fa").write_bytes(b">w\n" + b"\n".join(text[j:j + 70] for j in range(0, n, 70)) + b"\n")
    run = lambda *a: subprocess.run([str(x) for x in a], cwd=tmp_path, check=True, capture_output=True,  # noqa: E731
                                    timeout=300)
    run(REF / f"gfmi_{k}_{d}", "ref.fa", n)
    fn = f"ref.fa.{n}.{d}fmi{k}steps.fmi"
    if k <= 2:
        run(REF / f"tfmiBMP_{k}_{d}", fn)
        run(REF / f"tfmiAC_{k}_{d}", fn)
    (tmp_path / "q.qry").write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in q))
    return fn, run


def _reference_results(tmp_path, run, fn, k, d, tag, q):
    """The reference CPU searcher's results file for the tag's semantics (its
    loaders take tag 100 / 200 only; 101 / 201 are the same indexes laid out
    for the GPU kernels, transformIndexBitmaps.c:269-295)."""
    tag = 200 if tag >= 200 else 100
    src = tmp_path / (fn + TAGS[tag])
    ref_dir = tmp_path / f"ref{tag}"
    ref_dir.mkdir(exist_ok=True)
    shutil.copy(src, ref_dir / src.name)
    tool = "cpuac" if tag >= 200 else "cpu"
    subprocess.run([str(REF / f"{tool}_{k}_{d}"), src.name, str(tmp_path / "q.qry"), str(q.shape[1]),
                    str(q.shape[0])], cwd=ref_dir, check=True, capture_output=True, timeout=300,
                   env=dict(os.environ, OMP_NUM_THREADS="2"))
    return (ref_dir / (src.name + ".res.cpu")).read_bytes()


def _driver(tmp_path, binary, fn, tag, q, env, suffix):
    src = tmp_path / (fn + TAGS[tag])
    out_dir = tmp_path / f"{binary.name}{tag}{env.get('KFMI_BACKEND', '')}"
    out_dir.mkdir(exist_ok=True)
    shutil.copy(src, out_dir / src.name)
    p = subprocess.run([str(binary), src.name, str(tmp_path / "q.qry"), str(q.shape[1]), str(q.shape[0])],
                       cwd=out_dir, capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
    assert p.returncode == 0, p.stdout + p.stderr
    return (out_dir / (src.name + suffix)).read_bytes()


@pytest.mark.parametrize("i", range(WORLDS))
def test_dropin_world_cpu(tmp_path, i):
    k, d, text, q, rng = world(i)
    fn, run = _prepare(tmp_path, k, d, text, q)
    binary = REF / "searchQueries_cpu_dropin"
    if not binary.exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    for tag in ((100, 101, 200, 201) if k <= 2 else (100,)):
        want = _reference_results(tmp_path, run, fn, k, d, tag, q)
        got = _driver(tmp_path, binary, fn, tag, q, {"OMP_NUM_THREADS": "3"}, ".res.cpu")
        assert got == want, dict(world=i, k=k, d=d, tag=tag, m=q.shape[1], n=len(text))


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(WORLDS))
def test_dropin_world_gpu(tmp_path, i):
    k, d, text, q, rng = world(i)
    binary = REF / "searchQueries_dropin"
    if not binary.exists():
        pytest.fail("oracle/_ref/searchQueries_dropin missing on the GPU box")
    fn, run = _prepare(tmp_path, k, d, text, q)
    for tag in ((100, 101, 200, 201) if k <= 2 else (100,)):
        want = _reference_results(tmp_path, run, fn, k, d, tag, q)
        if k > 2:
            pool = ("coop-grp", "task-grp")
        elif tag >= 200:
            pool = ("task-ac", "task-ac-mid", "coop-ac-mid") + (("coop-ac",) if k == 2 else ())
        else:
            pool = PLAIN + (("coop-grp",) if (k, d) == (2, 64) else ())
        for b in rng.choice(pool, size=2, replace=False):
            got = _driver(tmp_path, binary, fn, tag, q, {"KFMI_BACKEND": str(b)}, ".res.gpu")
            assert got == want, dict(world=i, k=k, d=d, tag=tag, backend=str(b), m=q.shape[1], n=len(text))
