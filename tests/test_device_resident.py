"""An index built on the device without a host image (kfmi_build_index_gpu with
want_host_image = 0): its tag-100 entries stay in HBM, uploads relayout them
device to device, and the host image is fetched only when something asks for
it (image, saveIndex, the host transforms).  At 3 Gbase / K = 4 that keeps a
51 GB image out of host memory (builder).

Pins: every search equals the one on the host-image build of the same text;
the lazily fetched image is byte-identical to the host-image build's (whose
md5 the builder tests pin against the reference builder)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    return kfmi_mod


def _text(n, seed):
    rng = np.random.default_rng(seed)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n)].copy()
    for _ in range(30):                      # some repeats, so the builder resolves ties
        a, b = rng.integers(0, n - 2000, size=2)
        t[b:b + 1500] = t[a:a + 1500]
    return t


def _reads(t, n, m, seed):
    rng = np.random.default_rng(seed)
    st = rng.integers(0, t.size - m, size=n)
    return np.ascontiguousarray(np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                                                rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(n // 4, m))]))


@pytest.mark.parametrize("k,backends", [(2, ("task-mid", "coop-mid", "task")),
                                        (4, ("coop-grp", "task-grp"))])
def test_device_only_build_equals_host_image_build(gpu, tmp_path, k, backends):
    t = _text(2_000_003, k)
    text = t.tobytes()
    ref = gpu.Index.build(text, k=k, d=64, gpu=True)
    dev = gpu.Index.build(text, k=k, d=64, gpu=True, host_image=False)
    q = _reads(t, 20_000, 100, 3)
    for b in backends:
        assert np.array_equal(gpu.search_array(dev, q, b), gpu.search_array(ref, q, b)), b
        dev.free_gpu()
        ref.free_gpu()
    # odd length through the remainder table, and a device group of one card twice
    q7 = _reads(t, 3000, 99 if k == 2 else 102, 4)
    want = gpu.search_array(ref, q7, backends[0])
    gpu.set_devices([0, 0])
    try:
        assert np.array_equal(gpu.search_array(dev, q7, backends[0]), want)
    finally:
        gpu.set_devices([])
    # the host image appears on demand, identical to the host-image build
    assert hashlib.md5(dev.image().tobytes()).hexdigest() == hashlib.md5(ref.image().tobytes()).hexdigest()
    dev.save(tmp_path / "dev")
    ref.save(tmp_path / "ref")
    fd = sorted(tmp_path.glob("dev*"))
    fr = sorted(tmp_path.glob("ref*"))
    assert len(fd) == len(fr) == 1 and fd[0].read_bytes() == fr[0].read_bytes()
    # and searching after the fetch still works (both copies kept)
    assert np.array_equal(gpu.search_array(dev, q, backends[0]), gpu.search_array(ref, q, backends[0]))
    dev.close()
    ref.close()


def test_device_only_index_host_transforms(gpu):
    """AltCounters layouts need the host tfmiAC transform: it fetches the image."""
    t = _text(300_001, 9)
    text = t.tobytes()
    ref = gpu.Index.build(text, k=2, d=64, gpu=True)
    dev = gpu.Index.build(text, k=2, d=64, gpu=True, host_image=False)
    q = _reads(t, 5000, 100, 5)
    for b in ("task-ac", "coop-ac", "task-ac-mid"):
        assert np.array_equal(gpu.search_array(dev, q, b), gpu.search_array(ref, q, b)), b
    a200, a201 = dev.alt_counters()
    r200, r201 = ref.alt_counters()
    assert bytes(a201.image()) == bytes(r201.image())
    for x in (a200, a201, r200, r201, dev, ref):
        x.close()
