"""kfmi_derive_index_gpu (DESIGN.md 5d'): a 2K-step index derived on the
device from a K-step one, without the text, equals the index the builders
write from the text at 2K -- the whole tag-100 image, byte for byte (header,
'$' rows and their codes, planes, counters) -- for K = 1 -> 2 and 2 -> 4,
several d, texts whose tails put '$' rows in the last block and (n+1) % d == 0;
the reference's own tag-101 file derives the same; searches on the derived
K = 4 index equal the K = 2 ones."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    return kfmi_mod


def _text(n, tail, seed):
    rng = np.random.default_rng(seed)
    t = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n)
    if tail == "T-run":
        t[-min(n, 70):] = ord("T")
    elif tail == "A-run":
        t[-min(n, 70):] = ord("A")
    elif tail == "periodic":
        t[:] = np.resize(np.frombuffer(b"ACGTTGCA", np.uint8), n)
    return t.tobytes()


@pytest.mark.parametrize("kin", [1, 2])
@pytest.mark.parametrize("d", [32, 64, 128])
@pytest.mark.parametrize("n,tail", [(9, "random"), (100, "random"), (127, "T-run"), (191, "A-run"), (255, "random"),
                                    (1000, "periodic"), (5_000, "T-run"), (200_001, "random")])
def test_derived_image_equals_built(K, kin, d, n, tail):
    text = _text(n, tail, n + d + kin)
    src = K.Index.build(text, k=kin, d=d)
    want = K.Index.build(text, k=2 * kin, d=d)
    got = src.derive(2 * kin, host_image=True)
    assert got.header() == want.header()
    assert np.array_equal(np.asarray(got.image()), np.asarray(want.image())), (kin, d, n, tail)
    for x in (src, want, got):
        x.close()


def test_derived_from_tag101_and_device_resident(K):
    """The reference's interleaved file derives the same index, and a
    device-resident result (no host image) fetches the same bytes."""
    text = _text(50_001, "random", 3)
    src = K.Index.build(text, k=2, d=64)
    want = K.Index.build(text, k=4, d=64)
    for s in (src.interleave(), K.Index.build(text, k=2, d=64, gpu=True, host_image=False)):
        got = s.derive(4)
        assert np.array_equal(np.asarray(got.image()), np.asarray(want.image()))
        got.close()
        s.close()


def test_derived_k4_searches_equal_k2(K):
    rng = np.random.default_rng(5)
    text = _text(300_001, "random", 11)
    t = np.frombuffer(text, np.uint8)
    i2 = K.Index.build(text, k=2, d=64, gpu=True)
    i4 = i2.derive(4)
    for m in (100, 150, 102, 8):
        reads = np.ascontiguousarray(np.concatenate([
            t[rng.integers(0, len(t) - m, size=4000)[:, None] + np.arange(m)],
            rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(500, m))]))
        want = K.search_array(i2, reads, "task-mid")
        for be in ("coop-grp", "task-grp"):
            assert np.array_equal(K.search_array(i4, reads, be), want), (m, be)
    i4.close()
    i2.close()


def test_derive_rejects(K):
    text = _text(1000, "random", 1)
    i2 = K.Index.build(text, k=2, d=64)
    for kout in (2, 3, 8):
        with pytest.raises(K.KfmiError):
            i2.derive(kout)
    i4 = K.Index.build(text, k=4, d=64)
    with pytest.raises(K.KfmiError):
        i4.derive(8)
    ac = i2.alt_counters()[0]
    with pytest.raises(K.KfmiError):
        ac.derive(4)
    tiny = K.Index.build(b"ACGTACG", k=2, d=64)   # n = 7 < 2 * 4: row 0's LF would be a '$' row
    with pytest.raises(K.KfmiError):
        tiny.derive(4)
    for x in (i2, i4, ac, tiny):
        x.close()


def test_grouped_backends_derive_on_upload(K):
    """transferCPUtoGPU of a K = 2 index for coop-grp / task-grp derives its
    K = 4 index on the device and searches it (the queries are packed for
    K = 4); streamed search, block counts and locate through the row-sampled
    SA of the K = 2 handle (the suffix array is the same) follow."""
    rng = np.random.default_rng(9)
    text = _text(100_001, "random", 21)
    t = np.frombuffer(text, np.uint8)
    i2 = K.Index.build(text, k=2, d=64, gpu=True, sa_rate=8)
    reads = np.ascontiguousarray(t[rng.integers(0, len(t) - 100, size=3000)[:, None] + np.arange(100)])
    want = K.search_array(i2, reads, "task-mid")
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    K.set_backend("task-mid")
    K.transfer_to_gpu(i2, q, r)
    K.search(i2, q, r)
    loc_want = K.locate(i2, r)
    off_w, pos_w = loc_want.offsets().copy(), loc_want.positions().copy()
    loc_want.close()
    for be in ("coop-grp", "task-grp"):
        K.set_backend(be)
        K.transfer_to_gpu(i2, q, r)
        K.search(i2, q, r)
        K.transfer_to_cpu(r)
        assert np.array_equal(r.array(), want), be
        assert np.array_equal(K.search_stream(i2, reads), want), be
        assert K.count_blocks(i2, q) > 0
        loc = K.locate(i2, r)
        assert np.array_equal(loc.offsets(), off_w) and np.array_equal(loc.positions(), pos_w), be
        loc.close()
    K.set_backend("task-mid")
    q.close()
    r.close()
    i2.close()


def test_ref_alphabet_derivation_and_locate(K):
    """'ref'-mode indexes (the reference builder's byte semantics, DESIGN.md
    4a).  A text of A/C/G/T only is an ordinary index: it derives to the K = 4
    index built from the text and its searches on coop-grp equal the K = 2
    ones, and locate works.  A text with N runs and lowercase letters makes
    the reference walk's LF_K not a permutation (genFMindex.c:347-391): the
    derivation and locate refuse it (KFMI_E_BUILDING_FMI = 9, the
    check_lf_walks cycle check) instead of returning a wrong index or walking n/K
    steps per slot."""
    rng = np.random.default_rng(11)
    pure = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=40_001)
    mixed = pure.copy()
    mixed[1000:1300] = ord("N")
    mixed[5000:5050] = np.frombuffer(b"acgt", np.uint8)[rng.integers(0, 4, 50)]
    reads = pure[rng.integers(0, pure.size - 100, size=2000)[:, None] + np.arange(100)]
    try:
        K.set_alphabet("ref")
        src = K.Index.build(pure.tobytes(), k=2, d=64, sa_rate=8)
        want4 = K.Index.build(pure.tobytes(), k=4, d=64)
        got4 = src.derive(4, host_image=True)
        assert np.array_equal(np.asarray(got4.image()), np.asarray(want4.image()))
        k2 = K.search_array(src, reads, "task-mid")
        assert np.array_equal(K.search_array(src, reads, "coop-grp"), k2)
        res, off, pos = K.locate_array(src, reads[:200], "task-mid")
        assert off[-1] == int(np.sum(res[1::2].astype(np.int64) - res[0::2]))
        for x in (src, want4, got4):
            x.close()
        bad = K.Index.build(mixed.tobytes(), k=2, d=64, sa_rate=8)
        with pytest.raises(K.KfmiError) as e:
            bad.derive(4)
        assert e.value.code == 9
        with pytest.raises(K.KfmiError) as e:
            K.locate_array(bad, reads[:50], "task-mid")
        assert e.value.code == 9
        assert K.search_array(bad, reads, "task-mid").shape == (4000,)   # the K = 2 search itself runs
        bad.close()
    finally:
        K.set_alphabet(None)
