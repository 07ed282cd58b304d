"""AltCounters results past n+1: texts that end in a run of A.

The tfmiAC file ends with a sentinel entry S = ceil((n+1)/d) whose rows read
as code 0 (transformIndexAC.c), so where the text ends in A's the
AltCounters searcher (fmIndexCPUBaseline-AltCounters.c:218-266) walks an
interval end past n+1 -- on a homopolymer of A, R = n+1, n+3, n+5, ... at
K = 2 -- and its result stays defined while every step reads inside the file:
up to (S+1)*d + K.  Round 5 capped every AltCounters step at n+d rows, which
cut those results short (the large random worlds, scripts/diag/worlds_large.py,
found one at n = 1,145,896; earlier rounds had the same cap); the cap is now (S+2)*d - 1 (kfmi_device.h
ac_clamp).  Oracle: the AltCounters restatement (oracle/fmi_oracle.c), which
refuses a search that reads past the file -- pinned here against the
reference's own searcher (oracle/_ref/cpuac_K_d) where it is built -- and,
where it refuses, the result is undefined: every searcher must stay below the
cap and the GPU backends must agree with the host search."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from util import REPO

REF = REPO / "oracle" / "_ref"
ALT = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")
ACGT = np.frombuffer(b"ACGT", np.uint8)


# cases whose all-A reads end past n+d where the reference is defined (a drift
# needs the padding's code 0 to be the text's largest code: a run of A only)
DRIFTS = {("A1001", 2, 64), ("A1001", 1, 64), ("A1000", 2, 64), ("A3001", 2, 32), ("A1145", 1, 32),
          ("A4000", 2, 128)}


def cases():
    """(name, text, k, d): homopolymers of A, (n+1) % d on both sides of d - K
    and at 0 (B5), and random texts ending in an A run (which stay below n+d:
    their R end leaves the sentinel block at the first step)."""
    out = []
    rng = np.random.default_rng(4242)
    for n, k, d in [(1001, 2, 64), (1001, 1, 64), (1000, 2, 64), (1023, 2, 64), (777, 1, 192),
                    (2000, 2, 192), (3001, 2, 32), (1145, 1, 32), (4000, 2, 128), (1150, 2, 32)]:
        out.append((f"A{n}", b"A" * n, k, d))
    for n, run, k, d in [(2940, 300, 2, 64), (2940, 150, 1, 64), (4990, 400, 2, 32), (2500, 700, 2, 192)]:
        t = ACGT[rng.integers(0, 4, size=n)].copy()
        t[-run:] = ord("A")
        out.append((f"rand{n}+A{run}", t.tobytes(), k, d))
    return out


def reads(text, k, d):
    """All-A reads of every length the cases need, with reads ending the text
    and a few random ones, as one batch per length."""
    t = np.frombuffer(text, np.uint8)
    rng = np.random.default_rng(len(text))
    for m in sorted({k, 2 * k, 10 * k, d, d + 2 * k, 2 * d, 2 * d + 6 * k, 3 * d}):
        if m % k or m > len(text):
            continue
        q = np.concatenate([np.full((3, m), ord("A"), np.uint8), t[len(t) - m:][None, :],
                            rng.choice(ACGT, size=(4, m)), np.full((1, m), ord("C"), np.uint8)])
        yield m, np.ascontiguousarray(q)


def cap(text, d):
    s = (len(text) + 1 + d - 1) // d
    return (s + 2) * d - 1


def oracle_or_none(oracle_mod, img, q):
    try:
        return oracle_mod.search(img, q)[0]
    except ValueError:   # a step reads past the file: the reference's result is undefined
        return None


@pytest.mark.parametrize("case", cases(), ids=lambda c: f"{c[0]}-K{c[2]}-d{c[3]}")
def test_ac_drift_host(kfmi_mod, oracle_mod, case):
    """searchIndexCPU on tags 200 and 201 equals the AltCounters oracle wherever
    it is defined, including results past n+d."""
    K = kfmi_mod
    name, text, k, d = case
    idx = K.Index.build(text, k=k, d=d)
    acs = idx.alt_counters()
    past = 0
    try:
        for m, q in reads(text, k, d):
            want = oracle_or_none(oracle_mod, acs[0].image(), q)
            for a in acs:
                got = K.search_cpu_array(a, q, 2)
                if want is None:
                    assert int(got.max()) <= cap(text, d), (name, m)
                else:
                    assert np.array_equal(got, want), (name, m, a.header()["tag"], got[:4], want[:4])
                    past += int((want > len(text) + d).any())
    finally:
        for x in (idx,) + tuple(acs):
            x.close()
    if (name, k, d) in DRIFTS:
        assert past, "the case no longer reaches past n+d"


def _ref_search(tmp_path, k, d, text, q):
    """The reference's own AltCounters searcher (searchQueries.c over
    fmIndexCPUBaseline-AltCounters.c) on the reference-built tag-200 file."""
    for tool in ("gfmi", "tfmiAC", "cpuac"):
        if not (REF / f"{tool}_{k}_{d}").exists():
            pytest.skip("oracle/_ref not built for this geometry (needs /root/reference)")
    n = len(text)
    (tmp_path / "ref.fa").write_bytes(b">w\n" + b"\n".join(text[j:j + 70] for j in range(0, n, 70)) + b"\n")
    run = lambda *a: subprocess.run([str(x) for x in a], cwd=tmp_path, check=True, capture_output=True,  # noqa: E731
                                    timeout=120)
    run(REF / f"gfmi_{k}_{d}", "ref.fa", n)
    fn = f"ref.fa.{n}.{d}fmi{k}steps.fmi"
    run(REF / f"tfmiAC_{k}_{d}", fn)
    (tmp_path / "q.qry").write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in q))
    ref_dir = tmp_path / "ref200"
    ref_dir.mkdir(exist_ok=True)
    shutil.copy(tmp_path / (fn + ".ac"), ref_dir)
    subprocess.run([str(REF / f"cpuac_{k}_{d}"), fn + ".ac", str(tmp_path / "q.qry"), str(q.shape[1]),
                    str(q.shape[0])], cwd=ref_dir, check=True, capture_output=True, timeout=120,
                   env=dict(os.environ, OMP_NUM_THREADS="1"))
    lines = (ref_dir / (fn + ".ac.res.cpu")).read_text().split("\n")
    assert int(lines[0]) == q.shape[0]
    return np.array([int(v) for ln in lines[1:1 + q.shape[0]] for v in ln.split()], dtype=np.uint32)


@pytest.mark.parametrize("case", [c for c in cases() if c[3] in (64, 192)], ids=lambda c: f"{c[0]}-K{c[2]}-d{c[3]}")
def test_ac_drift_oracle_is_the_reference(oracle_mod, tmp_path, case):
    """The oracle's AltCounters results past n+1 are the reference searcher's
    (its binary, oracle/_ref), on every read length where it is defined."""
    name, text, k, d = case
    import kstep_fmi as K
    idx = K.Index.build(text, k=k, d=d)
    ac = idx.alt_counters()[0]
    try:
        checked = 0
        for m, q in reads(text, k, d):
            want = oracle_or_none(oracle_mod, ac.image(), q)
            if want is None:
                continue
            sub = tmp_path / f"m{m}"
            sub.mkdir()
            assert np.array_equal(_ref_search(sub, k, d, text, q), want), (name, m)
            checked += 1
        assert checked or (len(text) + 1) % d == 0   # B5: every search reads past the file
    finally:
        idx.close()
        ac.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", cases(), ids=lambda c: f"{c[0]}-K{c[2]}-d{c[3]}")
def test_ac_drift_gpu(kfmi_mod, oracle_mod, case):
    """Every AltCounters GPU backend equals the oracle where it is defined and
    the host search everywhere (both stay below the cap where it is not)."""
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    name, text, k, d = case
    idx = K.Index.build(text, k=k, d=d)
    acs = idx.alt_counters()
    try:
        for m, q in reads(text, k, d):
            want = oracle_or_none(oracle_mod, acs[0].image(), q)
            host = K.search_cpu_array(acs[1], q, 2)
            if want is not None:
                assert np.array_equal(host, want), (name, m)
            for src in (idx,) + tuple(acs):
                for b in ALT:
                    try:
                        got = K.search_array(src, q, b)
                    except K.KfmiError as e:
                        assert e.code == 33, (name, b, e.code)   # a geometry the backend does not take
                        continue
                    assert np.array_equal(got, host), (name, m, b, src.header()["tag"], got[:4], host[:4])
    finally:
        for x in (idx,) + tuple(acs):
            x.close()


@pytest.mark.gpu
@pytest.mark.parametrize("k,rate", [(2, 1), (2, 8), (1, 32)])
def test_ac_drift_locate(kfmi_mod, k, rate):
    """Locate of AltCounters intervals that reach past n+1: rows from n+1 on
    hold no suffix, so each query reports the rows of [L, min(R, n+1)) -- no
    read of the sampled SA past its end, no walk from a row with no suffix
    (kfmi_locate.h walk_lost)."""
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    n, d = 1001, 64
    text = b"A" * n
    full = K.Index.build(text, k=k, d=d, sa_rate=1)
    sa = np.array(full.sa()[1], dtype=np.uint32)
    full.close()
    idx = K.Index.build(text, k=k, d=d, gpu=True, sa_rate=rate)
    try:
        for m in (2 * k, 64, 80):
            q = np.full((5, m), ord("A"), np.uint8)
            for b in ("task-ac", "task-ac-mid", "coop-ac-mid"):
                res, off, pos = K.locate_array(idx, q, b)
                assert int(res[1]) > n + 1 or m == 2 * k, (b, m, res[:2])   # the drift reaches past n+1
                w_pos, w_off = [], [0]
                for j in range(q.shape[0]):
                    lo, hi = int(res[2 * j]), min(int(res[2 * j + 1]), n + 1)
                    w_pos.append(sa[lo:hi] if hi > lo else sa[:0])
                    w_off.append(w_off[-1] + max(0, hi - lo))
                assert np.array_equal(off, np.array(w_off, np.uint64)), (b, m)
                assert np.array_equal(pos, np.concatenate(w_pos)), (b, m)
    finally:
        idx.close()


def _locate_case(name):
    rng = np.random.default_rng(99)
    if name == "A1023-B5":
        return b"A" * 1023
    if name == "T-head":   # the whole-text suffix sorts last: its '$' rows sit in the last block
        t = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=3000)
        t[:60] = ord("T")
        return t.tobytes()
    if name == "T-head-B5":
        t = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=4095)
        t[:60] = ord("T")
        return t.tobytes()
    return b"A" * 1001


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["A1023-B5", "T-head", "T-head-B5", "A1001"])
@pytest.mark.parametrize("k", [1, 2])
def test_locate_walks_on_altcounters_layouts(kfmi_mod, name, k):
    """A locate walk steps with the plain LF on every layout: on the
    AltCounters ones a step backward from the sentinel (the last real block)
    takes off what the sentinel adds there -- the block's '$' rows, and under
    B5 its padding (kfmi_search.hip ac_locate_fix).  Texts whose '$' rows sit in
    the last block (a homopolymer, a text that opens with a run of T), with and
    without (n+1) % d == 0; every row of every interval the walk can reach."""
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    text = _locate_case(name)
    n, d = len(text), 64
    t = np.frombuffer(text, np.uint8)
    full = K.Index.build(text, k=k, d=d, sa_rate=1)
    sa = np.array(full.sa()[1], dtype=np.uint32)
    full.close()
    idx = K.Index.build(text, k=k, d=d, gpu=True, sa_rate=16)
    try:
        st = np.arange(0, n - 4 * k + 1, 7)
        q = np.ascontiguousarray(np.concatenate([t[st[:, None] + np.arange(2 * k)[None, :]],
                                                 np.full((1, 2 * k), ord("T"), np.uint8)]))
        for b in ("task-ac", "task-ac-mid", "task-mid"):
            res, off, pos = K.locate_array(idx, q, b)
            w_pos = [sa[int(res[2 * j]):min(int(res[2 * j + 1]), n + 1)] for j in range(q.shape[0])]
            assert np.array_equal(pos, np.concatenate(w_pos)), (name, k, b)
    finally:
        idx.close()
