"""GPU index builder (kfmi_build_index_gpu) pinned bit-exactly against the
reference builder's .fmi files (tests/golden)."""
import hashlib

import numpy as np
import pytest

import util
from util import GOLDEN, manifest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible")
    kfmi_mod.set_device(0)
    return kfmi_mod


@pytest.mark.parametrize("case", sorted(manifest()))
def test_gpu_builder_matches_reference_builder(gpu, case):
    c = manifest()[case]
    text = util.read_fasta_text(GOLDEN / case / "ref.fa").encode()
    for key, ent in sorted(c["indexes"].items()):
        idx = gpu.Index.build(text, k=ent["k"], d=ent["d"], gpu=True)
        assert hashlib.md5(idx.image().tobytes()).hexdigest() == ent["files"]["100"]["md5"], (case, key)


@pytest.mark.parametrize("k,d", [(1, 32), (2, 64), (3, 64), (4, 128), (2, 960)])
def test_gpu_builder_equals_host_builder(gpu, k, d):
    rng = np.random.default_rng(k * 1000 + d)
    for n in (1, 5, 63, 64, 65, 1000, 250_000):
        text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n).tobytes()
        if n + 1 < k:      # a D_s would not exist: both builders refuse
            for g in (True, False):
                with pytest.raises(gpu.KfmiError):
                    gpu.Index.build(text, k=k, d=d, gpu=g)
            continue
        a = gpu.Index.build(text, k=k, d=d, gpu=True).image().tobytes()
        b = gpu.Index.build(text, k=k, d=d, gpu=False).image().tobytes()
        assert a == b, (k, d, n)


def test_gpu_builder_repetitive_text(gpu):
    """Many equal 32-base keys: the device prefix doubling must order them
    (and the suffixes whose '$' falls inside their first 32 bases)."""
    for text in (b"A" * 5000, b"ACGT" * 3000 + b"A", b"AC" * 2000 + b"G" + b"AC" * 2000,
                 (b"ACGTTGCA" * 100 + b"T") * 20, b"A" * 40, b"C" + b"A" * 70, b"AAAAT" * 9):
        a = gpu.Index.build(text, k=2, d=64, gpu=True).image().tobytes()
        st = gpu.build_stats()
        b = gpu.Index.build(text, k=2, d=64, gpu=False).image().tobytes()
        assert a == b, text[:20]
        assert st["ties"] > 0 and st["rounds"] > 0, st


@pytest.mark.parametrize("seed", range(6))
def test_gpu_builder_random_repeats(gpu, seed):
    """Random texts with copied segments (exact and with one mismatch), runs and
    near-end repeats: every tie pattern the doubling rounds must untangle."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    for n in (200, 5_000, 60_000):
        t = acgt[rng.integers(0, 4, size=n)].copy()
        for _ in range(rng.integers(1, 30)):
            ln = int(rng.integers(20, max(21, n // 4)))
            a, b = rng.integers(0, n - ln, size=2)
            t[b:b + ln] = t[a:a + ln]
            if rng.random() < 0.5:
                t[b + ln // 2] = acgt[rng.integers(0, 4)]
        if rng.random() < 0.5:
            ln = int(rng.integers(1, 100))
            t[n - ln:] = t[:ln] if rng.random() < 0.5 else ord("A")
        text = t.tobytes()
        for k, d in ((2, 64), (1, 32)):
            a = gpu.Index.build(text, k=k, d=d, gpu=True).image().tobytes()
            b = gpu.Index.build(text, k=k, d=d, gpu=False).image().tobytes()
            assert a == b, (seed, n, k, d)


def test_gpu_builder_repeat_rich_50mbase(gpu):
    """50 Mbase with 10^4 inserted 1-kb repeats of 20 families, a 1 Mbase
    homopolymer and a 400 kbase tandem repeat: the GPU image equals the host
    (SA-IS) image bit for bit, with no host fallback."""
    import time
    rng = np.random.default_rng(3)
    n = 50_000_000
    acgt = np.frombuffer(b"ACGT", np.uint8)
    t = acgt[rng.integers(0, 4, size=n, dtype=np.uint8)].copy()
    fam = [acgt[rng.integers(0, 4, size=1000, dtype=np.uint8)] for _ in range(20)]
    for i, p in enumerate(rng.choice(n // 1000, size=10_000, replace=False) * 1000):
        t[p:p + 1000] = fam[i % 20]
    t[1_000_000:2_000_000] = ord("A")
    t[3_000_000:3_400_000] = np.tile(np.frombuffer(b"ACGTTG", np.uint8), 400_000 // 6 + 1)[:400_000]
    text = t.tobytes()
    t0 = time.perf_counter()
    a = gpu.Index.build(text, k=2, d=64, gpu=True)
    gpu_s = time.perf_counter() - t0
    st = gpu.build_stats()
    t0 = time.perf_counter()
    b = gpu.Index.build(text, k=2, d=64, gpu=False)
    host_s = time.perf_counter() - t0
    print(f"repeat-rich 50 Mbase: GPU build {gpu_s:.2f} s ({st['ties']} tied positions, {st['rounds']} doubling "
          f"rounds), host SA-IS build {host_s:.2f} s")
    assert st["ties"] > 10_000_000 and st["rounds"] >= 5, st
    assert hashlib.md5(a.image().tobytes()).hexdigest() == hashlib.md5(b.image().tobytes()).hexdigest()


def test_gpu_builder_rejects_non_acgt(gpu):
    with pytest.raises(gpu.KfmiError):
        gpu.Index.build(b"ACGTNACGT" * 10, k=2, d=64, gpu=True)


def test_gpu_builder_64mbase_md5(gpu):
    from kstep_fmi import synth
    text, _ = synth.text_64m()
    for k, key in ((2, "ref64.k2d64.fmi"), (1, "ref64.k1d64.fmi")):
        idx = gpu.Index.build(text, k=k, d=64, gpu=True)
        assert hashlib.md5(idx.image().tobytes()).hexdigest() == synth.MD5[key]
