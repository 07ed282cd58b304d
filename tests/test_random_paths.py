"""The random worlds of tests/test_random_worlds.py through the paths around
the search: the device derivation of a 2K-step index (kfmi_derive_index_gpu,
byte-equal to the index built from the text), the GPU builder's
device-resident index (no host image), the streamed search at a random
chunk size and slot count, from pinned or pageable memory, host-packed or
not, and a device group (device 0 listed 2-3 times: independent replicas,
streams and slices on the one card of the box).  Oracle: brute-force suffix
ranks, as there."""
import numpy as np
import pytest

from test_random_worlds import WORLDS, _takes, world

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    yield kfmi_mod
    kfmi_mod.set_devices([0])


@pytest.mark.parametrize("i", range(0, WORLDS, 3))
def test_world_derived_index(K, i):
    n, k, d, m, text, q, want = world(i)
    if k > 2 or n < 4 * k:
        pytest.skip("derivation: K = 1 -> 2 or 2 -> 4 on texts of at least 2 * 2K bases")
    src = K.Index.build(text, k=k, d=d)
    built = K.Index.build(text, k=2 * k, d=d)
    got = src.derive(2 * k, host_image=True)
    try:
        assert got.header() == built.header(), (i, n, k, d)
        assert np.array_equal(np.asarray(got.image()), np.asarray(built.image())), (i, n, k, d)
        if 2 * k == 4 and d == 64:
            res = K.search_array(got, q, "coop-grp")
            assert np.array_equal(res, want), (i, n, k, d, m)
    finally:
        for x in (src, built, got):
            x.close()


@pytest.mark.parametrize("i", range(1, WORLDS, 3))
def test_world_device_resident_and_stream(K, i, monkeypatch):
    n, k, d, m, text, q, want = world(i)
    rng = np.random.default_rng(500 + i)
    idx = K.Index.build(text, k=k, d=d, gpu=True, host_image=False)
    try:
        pool = [b for b in ("task-mid", "coop-mid", "task", "task-grp", "coop-grp") if _takes(b, k, d, n)]
        b = str(rng.choice(pool))
        assert np.array_equal(K.search_array(idx, q, b), want), (i, b)
        monkeypatch.setenv("KFMI_STREAM_HOSTPACK", str(int(rng.integers(0, 3))))
        monkeypatch.setenv("KFMI_STREAM_SLOTS", str(int(rng.integers(2, 9))))
        K.set_backend(b)
        K.transfer_to_gpu(idx, None, None)
        chunk = int(rng.choice([1, 7, 64, 100, 1000]))
        src = K.pinned_empty(q.shape) if rng.random() < 0.5 else np.empty_like(q)
        src[...] = q
        got = K.search_stream(idx, src, chunk=chunk)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, dict(world=i, backend=b, chunk=chunk, first=int(bad[0]) if bad.size else None)
    finally:
        idx.close()


@pytest.mark.parametrize("i", range(2, WORLDS, 3))
def test_world_device_group(K, i):
    n, k, d, m, text, q, want = world(i)
    rng = np.random.default_rng(900 + i)
    idx = K.Index.build(text, k=k, d=d)
    pool = [b for b in ("task-mid", "coop-mid", "task", "coop", "task-grp", "coop-grp") if _takes(b, k, d, n)]
    b = str(rng.choice(pool))
    try:
        K.set_devices([0] * int(rng.integers(2, 4)))
        got = K.search_array(idx, q, b)
        assert np.array_equal(got, want), (i, b)
        K.transfer_to_gpu(idx, None, None)
        got = K.search_stream(idx, q, chunk=int(rng.choice([5, 64, 300])))
        assert np.array_equal(got, want), (i, b, "stream")
    finally:
        K.set_devices([0])
        idx.close()
