"""Seeded random builder worlds against the reference's own tools.

Each world draws a text (length 2 .. 5,000: uniform, homopolymer runs, a
tandem repeat, two letters; lengths on and off the (n+1) % d == 0 boundary)
and a geometry the reference binaries were compiled for (oracle/Makefile:
K, d in {1, 2} x {64, 192} and K in {3, 4} at d = 64), runs the reference's
builder (genFMindex.c:457-543, oracle/_ref/gfmi_K_d) and, at K <= 2, its
transforms (transformIndexBitmaps.c:269-295, oracle/_ref/tfmiBMP_K_d;
transformIndexAlternateCounters.c:387-479, oracle/_ref/tfmiAC_K_d) on the
text, and compares their files byte for byte with this build's host builder,
GPU builder (GPU suite) and transforms.  Skipped where oracle/_ref was not
built (it needs /root/reference)."""
import hashlib
import subprocess

import numpy as np
import pytest

ACGT = np.frombuffer(b"ACGT", np.uint8)
WORLDS = 120
GEOMS = [(1, 64), (2, 64), (1, 192), (2, 192), (3, 64), (4, 64)]


def _text(rng, n):
    kind = rng.integers(0, 4)
    if kind == 0:
        t = ACGT[rng.integers(0, 4, size=n)]
    elif kind == 1:
        t = np.repeat(ACGT[rng.integers(0, 4, size=n)], rng.integers(1, 30, size=n))[:n]
    elif kind == 2:
        unit = ACGT[rng.integers(0, 4, size=int(rng.integers(1, 9)))]
        t = np.resize(unit, n).copy()
        t[rng.integers(0, n, size=max(1, n // 300))] = ACGT[rng.integers(0, 4)]
    else:
        t = ACGT[rng.integers(0, 4, size=2)][rng.integers(0, 2, size=n)]
    return np.ascontiguousarray(t, dtype=np.uint8).tobytes()


def world(i):
    rng = np.random.default_rng(70_000 + i)
    k, d = GEOMS[int(rng.integers(0, len(GEOMS)))]
    n = int(rng.choice([d - 1, 2 * d - 1, 3 * d - 1, d, d + 1, int(rng.integers(2 * k + 1, 5001)),
                        int(rng.integers(2 * k + 1, 400))]))
    return k, d, max(n, 2 * k + 1), rng


def _ref_files(oracle_mod, tmp_path, k, d, text):
    gfmi = oracle_mod.ref_binary("gfmi", k, d)
    if not gfmi.exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    n = len(text)
    (tmp_path / "ref.fa").write_bytes(b">w\n" + b"\n".join(text[j:j + 70] for j in range(0, n, 70)) + b"\n")
    subprocess.run([str(gfmi), "ref.fa", str(n)], cwd=tmp_path, check=True, capture_output=True, timeout=120)
    fn = tmp_path / f"ref.fa.{n}.{d}fmi{k}steps.fmi"
    out = {100: fn.read_bytes()}
    if k <= 2:
        for tool, tags in (("tfmiBMP", ((101, ".interleaving"),)), ("tfmiAC", ((200, ".ac"), (201, ".interleaving.ac")))):
            subprocess.run([str(oracle_mod.ref_binary(tool, k, d)), fn.name], cwd=tmp_path, check=True,
                           capture_output=True, timeout=120)
            for tag, suffix in tags:
                out[tag] = (tmp_path / (fn.name + suffix)).read_bytes()
    return out


def _md5(b):
    return hashlib.md5(bytes(b)).hexdigest()


@pytest.mark.parametrize("i", range(WORLDS))
def test_builder_world_host(kfmi_mod, oracle_mod, tmp_path, i):
    k, d, n, rng = world(i)
    text = _text(rng, n)
    ref = _ref_files(oracle_mod, tmp_path, k, d, text)
    idx = kfmi_mod.Index.build(text, k=k, d=d, gpu=False)
    try:
        assert _md5(idx.image()) == _md5(ref[100]), dict(world=i, k=k, d=d, n=n)
        if k <= 2:
            i101 = idx.interleave()
            a200, a201 = idx.alt_counters()
            for tag, x in ((101, i101), (200, a200), (201, a201)):
                assert _md5(x.image()) == _md5(ref[tag]), dict(world=i, k=k, d=d, n=n, tag=tag)
                x.close()
    finally:
        idx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(WORLDS))
def test_builder_world_gpu(kfmi_mod, oracle_mod, tmp_path, i):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    k, d, n, rng = world(i)
    text = _text(rng, n)
    ref = _ref_files(oracle_mod, tmp_path, k, d, text)
    idx = K.Index.build(text, k=k, d=d, gpu=True)
    try:
        assert _md5(idx.image()) == _md5(ref[100]), dict(world=i, k=k, d=d, n=n)
    finally:
        idx.close()
