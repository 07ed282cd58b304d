"""Locate: SA interval -> text positions.

The reference has no locate (it stops at [L, R), fmIndexCPUBaseline.c:288-290),
so there is no reference vector for this row: it is pinned against the
brute-force suffix array of T$ (tests/util.suffix_array, '$' lowest), and at
any size by the property text[p : p+m] == read for every reported p.

CPU tests: the builders' SA samples, the sample file, argument checks.
GPU tests (-m gpu): the device walk on every backend / (K, d) / sampling rate.
"""
import numpy as np
import pytest

import util

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
PLAIN = ("task", "coop", "task-mid", "coop-mid")
ALT = ("task-ac", "coop-ac")


def _text(n, seed):
    return np.random.default_rng(seed).choice(ACGT, size=n).tobytes()


# ----------------------------------------------------------------- CPU ------

@pytest.mark.parametrize("k", [1, 2])
def test_cpu_builder_sa_samples_equal_bruteforce(kfmi_mod, k):
    for n in (1, 2, 5, 63, 64, 65, 1000, 20_000):
        if n + 1 < k:
            continue
        text = _text(n, n + k)
        sa = util.suffix_array(text + b"$")
        for rate in (1, 2, 8, 32):
            idx = kfmi_mod.Index.build(text, k=k, d=64, sa_rate=rate)
            got_rate, got = idx.sa()
            assert got_rate == rate
            assert np.array_equal(got, sa[::rate].astype(np.uint32)), (n, k, rate)
            idx.close()


def test_sa_samples_leave_the_index_unchanged(kfmi_mod):
    text = _text(5000, 3)
    a = kfmi_mod.Index.build(text, k=2, d=64).image().tobytes()
    b = kfmi_mod.Index.build(text, k=2, d=64, sa_rate=4).image().tobytes()
    assert a == b


def test_sa_file_roundtrip(kfmi_mod, tmp_path):
    text = _text(3000, 4)
    idx = kfmi_mod.Index.build(text, k=2, d=64, sa_rate=4)
    idx.save_sa(tmp_path / "x.sa")
    other = kfmi_mod.Index.from_image(idx.image())
    assert other.sa()[0] == 0
    other.load_sa(tmp_path / "x.sa")
    rate, s = other.sa()
    assert rate == 4 and np.array_equal(s, idx.sa()[1])
    # a different text length is refused, a missing file reported
    small = kfmi_mod.Index.build(_text(2999, 4), k=2, d=64)
    with pytest.raises(kfmi_mod.KfmiError) as e:
        small.load_sa(tmp_path / "x.sa")
    assert e.value.code == 5
    with pytest.raises(kfmi_mod.KfmiError) as e:
        small.load_sa(tmp_path / "missing.sa")
    assert e.value.code == 1
    with pytest.raises(kfmi_mod.KfmiError):
        small.save_sa(tmp_path / "y.sa")          # no samples to save


def test_sa_rate_must_be_power_of_two(kfmi_mod):
    for rate in (3, 6, 1 << 17):
        with pytest.raises(kfmi_mod.KfmiError) as e:
            kfmi_mod.Index.build(b"ACGTACGTAC", k=2, d=64, sa_rate=rate)
        assert e.value.code == 33


def test_locate_argument_errors_without_device(kfmi_mod):
    idx = kfmi_mod.Index.build(_text(500, 5), k=2, d=64, sa_rate=4)
    r = kfmi_mod.Results.alloc(4)
    with pytest.raises(kfmi_mod.KfmiError) as e:
        kfmi_mod.locate(idx, r)
    assert e.value.code == 34                    # nothing on the device yet


# ----------------------------------------------------------------- GPU ------

def _expected(sa, res, max_occ=0):
    offs, pos = [0], []
    for q in range(res.size // 2):
        L, R = int(res[2 * q]), int(res[2 * q + 1])
        hi = R if not max_occ else min(R, L + max_occ)
        rows = sa[L:hi] if hi > L else sa[:0]
        pos.append(rows)
        offs.append(offs[-1] + rows.size)
    return np.array(offs, dtype=np.uint64), np.concatenate(pos).astype(np.uint32)


def _reads(text, rng):
    t = np.frombuffer(text, dtype=np.uint8)
    n = len(t)
    out = []
    for m, cnt in ((2, 64), (4, 256), (6, 512), (12, 512), (100, 256)):
        if m > n:
            continue
        st = rng.integers(0, n - m + 1, size=cnt)
        reads = t[st[:, None] + np.arange(m)[None, :]]
        # '$' edges: the text's own prefix and suffix of length m
        edge = np.stack([t[:m], t[n - m:]])
        rnd = rng.choice(ACGT, size=(cnt // 4, m))
        out.append(np.concatenate([reads, edge, rnd]))
    return out


@pytest.fixture(scope="module")
def gpu(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    return kfmi_mod


def _coop_ok(backend, k, d):
    if not backend.startswith("coop"):
        return True
    bmw = 2 * (d // 32) * k
    if backend == "coop-ac":
        return k == 2 and bmw % 4 == 0
    if backend == "coop":
        return bmw % 4 == 0 and (bmw + 4 ** k) % 4 == 0
    return bmw % 4 == 0


@pytest.mark.gpu
@pytest.mark.parametrize("backend", PLAIN + ALT)
@pytest.mark.parametrize("k,d", [(2, 64), (1, 64), (2, 192), (1, 32)], ids=lambda x: str(x))
def test_locate_equals_bruteforce_sa(gpu, backend, k, d):
    if not _coop_ok(backend, k, d):
        pytest.skip("geometry not offered by this cooperative backend")
    text = _text(30_001, 100 * k + d)
    sa = util.suffix_array(text + b"$")
    rng = np.random.default_rng(k * d)
    for rate in (1, 8, 64):
        idx = gpu.Index.build(text, k=k, d=d, gpu=True, sa_rate=rate)
        for q in _reads(text, rng):
            if q.shape[1] % k:
                continue
            res, off, pos = gpu.locate_array(idx, q, backend)
            w_off, w_pos = _expected(sa, res)
            assert np.array_equal(off, w_off), (backend, k, d, rate, q.shape)
            assert np.array_equal(pos, w_pos), (backend, k, d, rate, q.shape)
        idx.close()


@pytest.mark.gpu
def test_locate_gpu_builder_samples_equal_host_builder(gpu):
    for n in (1, 64, 65, 4097, 100_000):
        text = _text(n, n)
        for k, rate in ((2, 1), (2, 16), (1, 4)):
            if n + 1 < k:
                continue
            a = gpu.Index.build(text, k=k, d=64, gpu=True, sa_rate=rate)
            b = gpu.Index.build(text, k=k, d=64, gpu=False, sa_rate=rate)
            assert a.image().tobytes() == b.image().tobytes()
            assert np.array_equal(a.sa()[1], b.sa()[1]), (n, k, rate)


@pytest.mark.gpu
def test_locate_max_occ_repeats_and_empty(gpu):
    # long runs: intervals of thousands of rows and long LF walks
    text = b"A" * 3000 + b"C" + b"ACGT" * 700 + b"G"
    sa = util.suffix_array(text + b"$")
    idx = gpu.Index.build(text, k=2, d=64, gpu=True, sa_rate=32)
    q = np.frombuffer(b"AAAA" + b"ACGT" + b"GGGG" + b"TACG", dtype=np.uint8).reshape(4, 4)
    for max_occ in (0, 1, 7, 5000):
        res, off, pos = gpu.locate_array(idx, q, "task-mid", max_occ=max_occ)
        w_off, w_pos = _expected(sa, res, max_occ)
        assert np.array_equal(off, w_off) and np.array_equal(pos, w_pos), max_occ
    # every reported position really starts an occurrence
    t = np.frombuffer(text, dtype=np.uint8)
    res, off, pos = gpu.locate_array(idx, q, "task-mid")
    for i in range(4):
        for p in pos[off[i]:off[i + 1]]:
            assert t[p:p + 4].tobytes() == q[i].tobytes()
    # empty batch
    res, off, pos = gpu.locate_array(idx, np.zeros((0, 4), dtype=np.uint8), "task-mid")
    assert res.size == 0 and off.tolist() == [0] and pos.size == 0


@pytest.mark.gpu
@pytest.mark.parametrize("queue,chunk", [("0", "256"), ("1", "256"), ("1", "64"), ("1", "4096"), ("1", "100")])
def test_locate_slot_queue_forced(gpu, monkeypatch, queue, chunk):
    # the cooperative walk's slot queue (default at SA rate >= 8) and the fixed
    # slot order, each forced at every rate: ~3 M positions, so every wave of
    # the grid takes several chunks of the queue and the last chunk is partial;
    # queue chunks of 64 (the floor: one take covers a wave), 100 (not a power
    # of two) and 4096 slots (KFMI_LOCATE_CHUNK) give the same positions
    monkeypatch.setenv("KFMI_LOCATE_QUEUE", queue)
    monkeypatch.setenv("KFMI_LOCATE_CHUNK", chunk)
    text = b"A" * 3000 + b"C" + b"ACGT" * 700 + b"G" + _text(5000, 77)
    sa = util.suffix_array(text + b"$")
    q = np.frombuffer(b"AAAA" * 999 + b"ACGT" + b"TTTT" + b"CGTA", dtype=np.uint8).reshape(-1, 4)
    for rate in (1, 8, 64):
        idx = gpu.Index.build(text, k=2, d=64, gpu=True, sa_rate=rate)
        for backend in ("task-mid", "coop-mid"):
            res, off, pos = gpu.locate_array(idx, q, backend)
            w_off, w_pos = _expected(sa, res)
            assert int(w_off[-1]) > 2_900_000
            assert np.array_equal(off, w_off), (queue, chunk, rate, backend)
            assert np.array_equal(pos, w_pos), (queue, chunk, rate, backend)
        idx.close()


@pytest.mark.gpu
def test_locate_errors(gpu):
    text = _text(2000, 9)
    idx = gpu.Index.build(text, k=2, d=64, gpu=True)          # no samples
    q = gpu.Queries.from_array(np.frombuffer(text[:16], dtype=np.uint8).reshape(1, 16))
    r = gpu.Results.alloc(1)
    gpu.set_backend("task-mid")
    gpu.transfer_to_gpu(idx, q, r)
    gpu.search(idx, q, r)
    with pytest.raises(gpu.KfmiError) as e:
        gpu.locate(idx, r)
    assert e.value.code == 33
    # samples attached after the upload are picked up by the next locate
    idx2 = gpu.Index.build(text, k=2, d=64, sa_rate=2)
    import tempfile, os
    with tempfile.TemporaryDirectory() as d:
        idx2.save_sa(os.path.join(d, "s.sa"))
        idx.load_sa(os.path.join(d, "s.sa"))
    loc = gpu.locate(idx, r)
    assert loc.total() == 1 and int(loc.positions()[0]) == 0


@pytest.mark.gpu
def test_locate_refuses_cyclic_walks_fast(gpu):
    """A 'ref'-mode index of a text with N runs and lowercase letters (the
    reference builder's byte semantics) has LF_K cycles that
    miss every '$' row: a walk there would take up to n/K dependent loads
    before walk_lost stops it.  Locate checks the walks once per
    device copy (check_lf_walks; at 4.5 Mbase, above 2^22 rows, the sampled
    check) and refuses with KFMI_E_BUILDING_FMI -- quickly -- while the same
    text's ACGT-only twin locates."""
    import time
    K = gpu
    rng = np.random.default_rng(21)
    pure = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=4_500_001)
    mixed = pure.copy()
    for s in rng.integers(0, pure.size - 500, size=40):
        mixed[s:s + int(rng.integers(1, 400))] = ord("N")
    mixed[100:160] = np.frombuffer(b"acgt", np.uint8)[rng.integers(0, 4, 60)]
    reads = pure[rng.integers(0, pure.size - 100, size=5000)[:, None] + np.arange(100)]
    try:
        K.set_alphabet("ref")
        for text, ok in ((pure, True), (mixed, False)):
            idx = K.Index.build(text.tobytes(), k=2, d=64, gpu=True, sa_rate=32)
            t0 = time.perf_counter()
            if ok:
                res, off, pos = K.locate_array(idx, reads, "task-mid")
                assert off[-1] == int(np.sum(res[1::2].astype(np.int64) - res[0::2]))
                assert K.walk_check_last() == 2          # decided by the sampled check alone
            else:
                with pytest.raises(K.KfmiError) as e:
                    K.locate_array(idx, reads, "task-mid")
                assert e.value.code == 9
                assert K.walk_check_last() in (2, 3)
            assert time.perf_counter() - t0 < 30
            idx.close()
    finally:
        K.set_alphabet(None)


def _walk_texts(rng):
    """Texts whose LF_K orders are far from random: runs, periods, repeats."""
    acgt = np.frombuffer(b"ACGT", np.uint8)
    rnd = rng.choice(acgt, size=300_001)
    rep = rnd.copy()
    rep[150_000:290_000] = np.tile(rnd[:14_000], 10)
    return {"random": rnd, "all-A": np.full(200_001, ord("A"), np.uint8),
            "ACGT-period": np.tile(acgt, 60_000), "AC-period": np.tile(acgt[:2], 90_001),
            "period-7": np.tile(rng.choice(acgt, 7), 40_000), "repeats": rep}


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2])
def test_walk_check_full_and_sampled_agree(gpu, k):
    """The sampled walk check (1-in-256 hashed sample rows, their paths marked,
    orphans walked, pointer jumping over the samples' skeleton) against full
    pointer jumping over every row, forced through kfmi_set_walk_check on
    indexes below the size switch: both accept every text of a valid index
    (random, a single letter, short periods, long repeats) and locate equals
    the brute-force suffix array; both refuse the 'ref'-mode N-rich text."""
    K = gpu
    rng = np.random.default_rng(5 + k)
    try:
        for name, t in _walk_texts(rng).items():
            text = t.tobytes()
            sa = np.array(util.suffix_array(text + b"$"), dtype=np.int64)
            q = t[rng.integers(0, t.size - 40, size=300)[:, None] + np.arange(40)]
            for mode in (1, 2):
                K.set_walk_check(mode)
                idx = K.Index.build(text, k=k, d=64, gpu=True, sa_rate=8)
                res, off, pos = K.locate_array(idx, q, "task-mid", max_occ=64)
                assert K.walk_check_last() == (1 if mode == 1 else 2), (name, mode)
                assert np.array_equal(pos, _expected(sa, res, 64)[1]), (name, mode)
                idx.close()
        mixed = _walk_texts(rng)["random"].copy()
        mixed[1000:1300] = ord("N")
        mixed[5000:5050] = np.frombuffer(b"acgt", np.uint8)[rng.integers(0, 4, 50)]
        K.set_alphabet("ref")
        for mode in (1, 2):
            K.set_walk_check(mode)
            bad = K.Index.build(mixed.tobytes(), k=2, d=64, gpu=True, sa_rate=8)
            with pytest.raises(K.KfmiError) as e:
                K.locate_array(bad, q, "task-mid")
            assert e.value.code == 9, mode
            bad.close()
    finally:
        K.set_alphabet(None)
        K.set_walk_check(0)


def test_walk_check_mode_argument(kfmi_mod):
    """kfmi_set_walk_check takes 0, 1 or 2 (no device needed)."""
    K = kfmi_mod
    with pytest.raises(K.KfmiError):
        K.set_walk_check(3)
    K.set_walk_check(1)
    K.set_walk_check(0)


@pytest.mark.gpu
def test_walk_check_modes_agree_on_corrupted_counters(gpu, tmp_path):
    """Indexes whose LF_K is not a text's: one counter of a valid image moved
    by a few rows, so that LF_K merges rows, skips rows, leaves the table or
    closes cycles.  Full pointer jumping and the sampled check (which falls
    back to full jumping when two walks meet) must give the same verdict on
    each: refuse with KFMI_E_BUILDING_FMI, or accept and locate."""
    from oracle import oracle
    K = gpu
    rng = np.random.default_rng(44)
    t = rng.choice(ACGT, size=60_001)
    src = K.Index.build(t.tobytes(), k=2, d=64, gpu=True, sa_rate=8)
    src.save_sa(str(tmp_path / "x.sa"))
    img = np.array(src.image(), dtype=np.uint8, copy=True)
    src.close()
    h = oracle.header(img)
    k, d, ne = h["steps"], h["chunk"], h["nentries"]
    nb = d // 32
    ew = 2 * nb * k + 4 ** k
    q = t[rng.integers(0, t.size - 40, size=200)[:, None] + np.arange(40)]
    verdicts = {}
    try:
        for trial in range(24):
            bad = img.copy()
            ent = bad[bad.size - 4 * ew * ne:].view(np.uint32).reshape(ne, ew)
            b, c = int(rng.integers(1, ne)), int(rng.integers(0, 4 ** k))
            delta = int(rng.choice([-3, -1, 1, 3, 64, -64]))
            if int(ent[b, 2 * nb * k + c]) + delta < 0:
                continue
            ent[b, 2 * nb * k + c] = np.uint32(int(ent[b, 2 * nb * k + c]) + delta)
            got = []
            for mode in (1, 2):
                K.set_walk_check(mode)
                idx = K.Index.from_image(bad)
                idx.load_sa(str(tmp_path / "x.sa"))
                try:
                    K.locate_array(idx, q, "task-mid", max_occ=16)
                    got.append("accepted")
                except K.KfmiError as e:
                    assert e.code == 9, (trial, mode, e.code)
                    got.append("refused")
                assert K.walk_check_last() in ((1,) if mode == 1 else (2, 3))
                idx.close()
            assert got[0] == got[1], (trial, b, c, delta, got)
            verdicts[got[0]] = verdicts.get(got[0], 0) + 1
    finally:
        K.set_walk_check(0)
    assert verdicts.get("refused", 0) > 0, verdicts


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["task", "coop", "task-mid", "coop-mid", "task-ac", "task-ac-mid"])
def test_corrupt_counters_stay_in_table(gpu, backend):
    """A loaded file with wrapped or oversized counters (every counter of some
    entries set to 0xFFFFFFFF, 2^31 or a random u32): the LF steps' results
    are capped at the last row of the last block the layout holds
    (IdxArgs::lf_cap; ac_clamp on the AltCounters layouts), so every search
    stays inside the table -- it returns, with some intervals, and the same
    batch on the intact file still equals the oracle."""
    from oracle import oracle
    K = gpu
    rng = np.random.default_rng(91)
    t = rng.choice(ACGT, size=40_001)
    src = K.Index.build(t.tobytes(), k=2, d=64, gpu=False)
    img = np.array(src.image(), dtype=np.uint8, copy=True)
    src.close()
    h = oracle.header(img)
    k, d, ne = h["steps"], h["chunk"], h["nentries"]
    nb = d // 32
    ew = 2 * nb * k + 4 ** k
    q = np.concatenate([t[rng.integers(0, t.size - 60, size=1500)[:, None] + np.arange(60)],
                        rng.choice(ACGT, size=(500, 60))])
    good = K.Index.from_image(img)
    want_img = good.alt_counters()[0].image() if "ac" in backend else img
    assert np.array_equal(K.search_array(good, q, backend), oracle.search(want_img, q)[0])
    good.close()
    for how in ("ones", "high", "random"):
        bad = img.copy()
        ent = bad[bad.size - 4 * ew * ne:].view(np.uint32).reshape(ne, ew)
        rows = rng.choice(ne, size=max(1, ne // 8), replace=False)
        if how == "ones":
            ent[rows, 2 * nb * k:] = 0xFFFFFFFF
        elif how == "high":
            ent[rows, 2 * nb * k:] = 0x80000000
        else:
            ent[rows, 2 * nb * k:] = rng.integers(0, 1 << 32, size=(rows.size, 4 ** k), dtype=np.uint64).astype(np.uint32)
        idx = K.Index.from_image(bad)
        got = K.search_array(idx, q, backend)
        assert got.shape == (2 * q.shape[0],)
        idx.close()
