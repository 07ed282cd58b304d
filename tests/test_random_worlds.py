"""Seeded random small worlds: every searcher against brute-force suffix ranks.

Each world draws a text (length 1 .. 6,000; uniform, homopolymer runs, a
tandem repeat, or two letters, so that intervals stay wide deep into a read),
a geometry (K in 1 .. 4, d in {32, 64, 128, 192, 448, 960}; the grouped
layout is d = 64 at K = 3, 4, or a K = 2 index derived to K = 4 on upload),
a read length (1 .. 400, so m % K != 0 occurs) and a batch size that is
rarely a multiple of the wave (1 .. 700), then searches sampled, random,
N-bearing and text-ending reads.

Oracle: [L, R) = the suffix-rank interval of the read over T$ (brute force,
tests/util.py), which is what fmIndexCPUBaseline.c:157-292 returns wherever
it is defined -- including (n+1) % d == 0, where the reference reads past its
index and this build reads the padding entry's end counters.
The AltCounters searchers (fmIndexCPUBaseline-AltCounters.c:145-310) differ
from the true rank past the last real block (their sentinel counts the '$'
rows as stored codes): they are checked against the AltCounters restatement
on the transformed index where the reference's result is defined (the
restatement refuses a search that reads past the file), else against the
host search and kept below the cap (tests/test_ac_drift.py).  A geometry a
backend does not take must be refused with code 33, never answered.
The host search (searchIndexCPU) runs in the CPU suite; the GPU
backends in the GPU suite."""
import numpy as np
import pytest

import util

PLAIN = ("task", "coop", "task-mid", "coop-mid")
ALT = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")
GRP = ("task-grp", "coop-grp")
ACGT = np.frombuffer(b"ACGT", np.uint8)
WORLDS = 160


def _takes(backend, k, d, n):
    """Geometries each backend is built for (kfmi_search.hip geometry_supported;
    a K = 2 index on the grouped layout is derived to K = 4 on upload, which
    needs n >= 8, kfmi_derive.hip)."""
    if backend in GRP:
        return d == 64 and (k in (3, 4) or (k == 2 and n >= 8))
    if k > 2:
        return False
    if not backend.startswith("coop"):
        return True
    bmw = 2 * (d // 32) * k
    if backend == "coop-ac":
        return k == 2 and bmw % 4 == 0
    return bmw % 4 == 0


def _text(rng, n):
    kind = rng.integers(0, 4)
    if kind == 0:
        t = ACGT[rng.integers(0, 4, size=n)]
    elif kind == 1:   # homopolymer runs
        t = np.repeat(ACGT[rng.integers(0, 4, size=n)], rng.integers(1, 40, size=n))[:n]
    elif kind == 2:   # a tandem repeat with a few point changes
        unit = ACGT[rng.integers(0, 4, size=int(rng.integers(1, 12)))]
        t = np.resize(unit, n).copy()
        t[rng.integers(0, n, size=max(1, n // 200))] = ACGT[rng.integers(0, 4)]
    else:             # two letters only
        t = ACGT[rng.integers(0, 4, size=2)][rng.integers(0, 2, size=n)]
    return np.ascontiguousarray(t, dtype=np.uint8)


def _reads(rng, t, m, nq):
    n = t.size
    parts = []
    if m <= n:
        st = rng.integers(0, n - m + 1, size=nq)
        parts.append(t[st[:, None] + np.arange(m)[None, :]])
        parts.append(t[n - m:][None, :])                                  # ends the text
    parts.append(rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(max(1, nq // 5), m)))
    parts.append(np.full((1, m), ord("A"), np.uint8))
    q = np.concatenate(parts)
    return np.ascontiguousarray(q[rng.permutation(q.shape[0])][:nq] if q.shape[0] > nq else q)


def world(i):
    """(n, k, d, m, text bytes, reads [N, m], brute-force [L0, R0, ...])."""
    rng = np.random.default_rng(90_000 + i)
    n = int(rng.choice([1, 2, 3, 5, 31, 63, 64, 127, 128, 191, 255, 447, 959, 1023, 2047, 6000,
                        int(rng.integers(4, 6000))]))
    k = int(rng.choice([1, 2, 2, 3, 4]))
    d = 64 if k > 2 else int(rng.choice([32, 64, 128, 192, 448, 960]))
    if n < 2 * k + 1:
        k = 1
    m = int(rng.integers(1, 401)) if rng.random() < 0.7 else int(rng.choice([k, 2 * k, 100, 150]))
    nq = int(rng.integers(1, 700))
    t = _text(rng, n)
    q = _reads(rng, t, m, nq)
    bf = util.BruteForce(t.tobytes().decode())
    want = np.array([x for r in q for x in bf.interval(r.tobytes())], dtype=np.uint32)
    return n, k, d, m, t.tobytes(), q, want


def _ac_cap(n, d):
    """The AltCounters step cap, (S+2)*d - 1 rows past the sentinel S
    (kfmi_device.h ac_clamp; tests/test_ac_drift.py)."""
    return ((n + 1 + d - 1) // d + 2) * d - 1


def _ac_want(K, oracle_mod, acs, q, n, d):
    """The AltCounters restatement on the tag-200 file where the reference is
    defined; where a step reads past its file, the host search (every GPU
    backend must agree with it there), kept below the cap."""
    try:
        return oracle_mod.search(acs[0].image(), q)[0]
    except ValueError:
        got = K.search_cpu_array(acs[0], q, 2)
        assert q.shape[0] == 0 or int(got.max()) <= _ac_cap(n, d)
        return got


@pytest.mark.parametrize("i", range(WORLDS))
def test_random_world_host_search(kfmi_mod, i):
    """searchIndexCPU (the library's host search, csrc/host/cpu_search.c) on
    the world's index and its tag-101 interleaving: any K, m % K != 0 through
    its remainder table."""
    K = kfmi_mod
    n, k, d, m, text, q, want = world(i)
    idx = K.Index.build(text, k=k, d=d)
    try:
        for tagged in (idx, idx.interleave()):
            got = K.search_cpu_array(tagged, q, 2)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, dict(world=i, n=n, k=k, d=d, m=m, tag=tagged.header()["tag"], first=int(bad[0]))
    finally:
        idx.close()


@pytest.mark.parametrize("i", range(WORLDS))
def test_random_world_host_search_ac(kfmi_mod, oracle_mod, i):
    """searchIndexCPU on the world's AltCounters files (tags 200, 201) against
    the AltCounters restatement wherever the reference is defined."""
    K = kfmi_mod
    n, k, d, m, text, q, want = world(i)
    if k > 2 or m % k:
        pytest.skip("AltCounters files exist for K = 1, 2 and take m % K == 0 only")
    idx = K.Index.build(text, k=k, d=d)
    acs = idx.alt_counters()
    try:
        w = _ac_want(K, oracle_mod, acs, q, n, d)
        for a in acs:
            got = K.search_cpu_array(a, q, 2)
            bad = np.flatnonzero(got != w)
            assert bad.size == 0, dict(world=i, n=n, k=k, d=d, m=m, tag=a.header()["tag"], first=int(bad[0]))
    finally:
        for x in (idx,) + tuple(acs):
            x.close()


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(WORLDS))
def test_random_world_gpu(kfmi_mod, oracle_mod, i):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    n, k, d, m, text, q, want = world(i)
    idx = K.Index.build(text, k=k, d=d)
    acs = ()
    want_ac = None
    if k <= 2 and m % k == 0:
        acs = idx.alt_counters()   # tags 200 and 201
        want_ac = _ac_want(K, oracle_mod, acs, q, n, d)
    try:
        order = ("task-ac",) + tuple(b for b in PLAIN + ALT + GRP if b != "task-ac")
        for b in order:
            if b in ALT and m % k:
                continue
            if not _takes(b, k, d, n):
                with pytest.raises(K.KfmiError) as e:
                    K.search_array(idx, q, b)
                assert e.value.code == 33, (b, k, d)
                continue
            got = K.search_array(idx, q, b)
            if b in ALT:
                w = want_ac
            else:
                w = want
            bad = np.flatnonzero(got != w)
            assert bad.size == 0, dict(world=i, backend=b, n=n, k=k, d=d, m=m, nq=q.shape[0], first=int(bad[0]))
    finally:
        for x in (idx,) + acs:
            x.close()


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(0, WORLDS, 2))
def test_random_world_locate_and_ftab(kfmi_mod, i):
    """The same worlds through locate ([L, R) -> SA[L .. R), the GPU builder's
    sampled suffix array at a random rate, max_occ truncation) and through the
    ftab jump start (kfmi_set_ftab: the first bases from a table)."""
    K = kfmi_mod
    K.set_device(0)
    n, k, d, m, text, q, want = world(i)
    rng = np.random.default_rng(i)
    rate = int(rng.choice([1, 2, 8, 32]))
    max_occ = int(rng.choice([0, 0, 1, 5]))
    sa = util.suffix_array(text + b"$")
    idx = K.Index.build(text, k=k, d=d, gpu=True, sa_rate=rate)
    try:
        for b in ("task-mid", "coop-mid", "task") if k <= 2 else GRP:
            if not _takes(b, k, d, n):
                continue
            res, off, pos = K.locate_array(idx, q, b, max_occ)
            assert np.array_equal(res, want), (i, b)
            w_off, w_pos = [0], []
            for j in range(q.shape[0]):
                L, R = int(want[2 * j]), int(want[2 * j + 1])
                hi = R if not max_occ else min(R, L + max_occ)
                w_pos.append(sa[L:hi] if hi > L else sa[:0])
                w_off.append(w_off[-1] + max(0, hi - L))
            assert np.array_equal(off, np.array(w_off, np.uint64)), (i, b, rate, max_occ)
            assert np.array_equal(pos, np.concatenate(w_pos).astype(np.uint32)), (i, b, rate, max_occ)
        bases = k * int(rng.integers(1, 12 // k + 1))   # a whole number of K-steps, <= 12 bases
        K.set_ftab(bases)
        try:
            for b in ("task-mid", "coop-mid") if k <= 2 else GRP:
                if _takes(b, k, d, n):
                    got = K.search_array(idx, q, b)
                    bad = np.flatnonzero(got != want)
                    assert bad.size == 0, dict(world=i, backend=b, ftab=bases, k=k, d=d, m=m, first=int(bad[0]))
        finally:
            K.set_ftab(0)
    finally:
        idx.close()
