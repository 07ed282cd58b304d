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
    """Many equal 32-base keys: the host tie breaker must order them."""
    for text in (b"A" * 5000, b"ACGT" * 3000 + b"A", b"AC" * 2000 + b"G" + b"AC" * 2000,
                 (b"ACGTTGCA" * 100 + b"T") * 20):
        a = gpu.Index.build(text, k=2, d=64, gpu=True).image().tobytes()
        b = gpu.Index.build(text, k=2, d=64, gpu=False).image().tobytes()
        assert a == b


def test_gpu_builder_rejects_non_acgt(gpu):
    with pytest.raises(gpu.KfmiError):
        gpu.Index.build(b"ACGTNACGT" * 10, k=2, d=64, gpu=True)


def test_gpu_builder_64mbase_md5(gpu):
    from kstep_fmi import synth
    text, _ = synth.text_64m()
    for k, key in ((2, "ref64.k2d64.fmi"), (1, "ref64.k1d64.fmi")):
        idx = gpu.Index.build(text, k=k, d=64, gpu=True)
        assert hashlib.md5(idx.image().tobytes()).hexdigest() == synth.MD5[key]
