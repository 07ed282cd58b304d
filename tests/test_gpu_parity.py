"""GPU parity: every backend through the C ABI vs the reference's own result
files (tests/golden) and vs the CPU oracle (oracle/fmi_oracle.c) on seeded
inputs.  Bit-exact: the path is integer rank arithmetic.

Run on the GPU box:  python -m pytest tests -m gpu -x -q
"""
import hashlib

import numpy as np
import pytest

import util
from util import GOLDEN, manifest, read_qry

pytestmark = pytest.mark.gpu

PLAIN = ("task", "coop", "task-mid", "coop-mid")
ALT = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")
ACMID = ("task-ac-mid", "coop-ac-mid")     # AltCounters semantics on MID128 lines: from tag 100/101 (or 200/201, test_ac_inverse.py)


def coop_supported(backend, k, d):
    """Geometries the LDS-staged cooperative kernel accepts (16-byte chunks)."""
    if not backend.startswith("coop"):
        return True
    nb = d // 32
    bmw = 2 * nb * k
    if backend == "coop-ac":
        return k == 2 and bmw % 4 == 0
    if backend == "coop-ac-mid":
        return bmw % 4 == 0
    if backend == "coop":
        return bmw % 4 == 0 and (bmw + 4 ** k) % 4 == 0
    return bmw % 4 == 0


@pytest.fixture(scope="module")
def gpu(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    return kfmi_mod


def _cases():
    for case, c in sorted(manifest().items()):
        for key, ent in sorted(c["indexes"].items()):
            yield case, key


@pytest.mark.parametrize("backend", PLAIN + ALT)
@pytest.mark.parametrize("case,key", list(_cases()), ids=[f"{a}-{b}" for a, b in _cases()])
def test_backend_matches_reference_results(gpu, oracle_mod, backend, case, key):
    c = manifest()[case]
    ent = c["indexes"][key]
    k, d = ent["k"], ent["d"]
    ac = backend in ALT
    tags = (100, 101) if backend in ACMID else (200, 201, 100) if ac else (100, 101)
    checked = 0
    for tag in tags:
        idx = gpu.Index.load(GOLDEN / case / ent["files"][str(tag)]["file"])
        for m, qd in sorted(c["queries"].items()):
            m = int(m)
            if m % k:
                continue
            q = read_qry(GOLDEN / case / qd["file"], m)
            want = oracle_mod.read_results_file(
                GOLDEN / case / ent["results"][f"{m}.{200 if ac else 100}"]["file"])
            if not coop_supported(backend, k, d):
                with pytest.raises(gpu.KfmiError) as e:
                    gpu.search_array(idx, q, backend)
                assert e.value.code == 33          # KFMI_E_BAD_ARGUMENT at transferCPUtoGPU
                return
            got = gpu.search_array(idx, q, backend)
            assert np.array_equal(got, want), (backend, case, key, tag, m,
                                               int(np.flatnonzero(got != want)[0]))
            checked += 1
        idx.close()
    assert checked


@pytest.fixture(scope="module")
def random_index(kfmi_mod):
    rng = np.random.default_rng(2026)
    text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=3_000_001).tobytes()
    return text, {(k, d): kfmi_mod.Index.build(text, k=k, d=d) for k, d in
                  [(2, 64), (1, 64), (2, 192), (2, 448), (2, 960), (1, 32), (2, 128), (2, 256), (1, 128),
                   (2, 32)]}


def _reads(text, n, m, seed):
    rng = np.random.default_rng(seed)
    t = np.frombuffer(text, dtype=np.uint8)
    st = rng.integers(0, len(text) - m, size=n)
    samp = t[st[:, None] + np.arange(m)[None, :]]
    rnd = rng.choice(np.frombuffer(b"ACGTNacgt", dtype=np.uint8), size=(n // 4, m))
    return np.concatenate([samp, rnd])


@pytest.mark.parametrize("backend", PLAIN + ALT)
@pytest.mark.parametrize("kd", [(2, 64), (1, 64), (2, 192), (2, 448), (2, 960), (1, 32), (2, 128), (2, 256),
                                (1, 128), (2, 32)],
                         ids=lambda kd: f"k{kd[0]}d{kd[1]}")
def test_backend_matches_oracle_random(gpu, oracle_mod, random_index, backend, kd):
    text, idxs = random_index
    k, d = kd
    idx = idxs[kd]
    for m, n in ((100, 20000), (150, 4000), (2 * k, 4000)):
        q = _reads(text, n, m, seed=m * 7 + k)
        if backend in ALT:
            i200, _ = idx.alt_counters()
            want, _ = oracle_mod.search(i200.image(), q)
        else:
            want, _ = oracle_mod.search(idx.image(), q)
        if not coop_supported(backend, k, d):
            with pytest.raises(gpu.KfmiError) as e:
                gpu.search_array(idx, q, backend)
            assert e.value.code == 33
            return
        got = gpu.search_array(idx, q, backend)
        assert np.array_equal(got, want), (backend, kd, m)


def test_block_count_matches_oracle(gpu, oracle_mod, random_index):
    text, idxs = random_index
    idx = idxs[(2, 64)]
    q = _reads(text, 20000, 100, seed=3)
    _, want = oracle_mod.search(idx.image(), q)
    gpu.set_backend("task-mid")
    qq = gpu.Queries.from_array(q)
    r = gpu.Results.alloc(q.shape[0])
    gpu.transfer_to_gpu(idx, qq, r)
    assert gpu.count_blocks(idx, qq) == want


def test_edge_cases(gpu, oracle_mod, random_index):
    text, idxs = random_index
    idx = idxs[(2, 64)]
    # empty batch
    for b in PLAIN + ALT:
        out = gpu.search_array(idx, np.zeros((0, 100), dtype=np.uint8), b)
        assert out.size == 0
    # batches that are not multiples of the wave / block size
    for n in (1, 63, 65, 257, 1023):
        q = _reads(text, n, 100, seed=n)[:n]
        want, _ = oracle_mod.search(idx.image(), q)
        for b in PLAIN:
            assert np.array_equal(gpu.search_array(idx, q, b), want), (b, n)
    # m % K != 0 (reference reads query[-1]): the AltCounters
    # backends reject it, the plain ones take the remainder table
    # (tests/test_remainder.py): here 4 x "AAAAA" -> the interval of A^5
    with pytest.raises(gpu.KfmiError):
        gpu.search_array(idx, np.zeros((4, 5), dtype=np.uint8) + 65, "task-ac")
    a5 = gpu.search_array(idx, np.zeros((4, 5), dtype=np.uint8) + 65, "task")
    t8 = np.frombuffer(text, dtype=np.uint8)
    assert a5[1] - a5[0] == int(np.sum(np.all(np.lib.stride_tricks.sliding_window_view(t8, 5) == 65, axis=1)))
    # search before transfer
    q = gpu.Queries.from_array(np.zeros((4, 8), dtype=np.uint8) + 65)
    r = gpu.Results.alloc(4)
    fresh = gpu.Index.from_image(idx.image())
    with pytest.raises(gpu.KfmiError) as e:
        gpu.search(fresh, q, r)
    assert e.value.code == 34


def test_strict_tag_like_reference(gpu, monkeypatch):
    c = manifest()["textA"]["indexes"]["k2_d64"]["files"]
    monkeypatch.setenv("KFMI_STRICT_TAG", "1")
    gpu.set_backend("task")
    with pytest.raises(gpu.KfmiError) as e:
        gpu.Index.load(GOLDEN / "textA" / c["100"]["file"])
    assert e.value.code == 101
    gpu.Index.load(GOLDEN / "textA" / c["101"]["file"]).close()
    gpu.set_backend("task-ac")
    with pytest.raises(gpu.KfmiError) as e:
        gpu.Index.load(GOLDEN / "textA" / c["101"]["file"])
    assert e.value.code == 201


def test_config1_64mbase_md5_pinned(gpu):
    """BASELINE config #1 end to end: recipe text (md5), host builder (md5 of
    the reference-built .fmi), 2^20 reads (md5), GPU search on every backend
    -> md5 of the results file the reference CPU searcher wrote."""
    from kstep_fmi import synth
    text, rng = synth.text_64m()
    assert synth.fasta_md5(text, b">synthetic_64M\n") == synth.MD5["ref64.fa"]
    idx = gpu.Index.build(text, k=2, d=64)
    assert hashlib.md5(idx.image().tobytes()).hexdigest() == synth.MD5["ref64.k2d64.fmi"]
    q = synth.reads_64m(text, rng)
    for b in PLAIN + ALT:
        res = gpu.search_array(idx, q, b)
        assert synth.results_md5(res) == synth.MD5["res64"], b


@pytest.mark.parametrize("n", [63, 127, 191, 255, 1023, 4095, 100, 129])
def test_b5_boundary_against_bruteforce(gpu, n):
    """(n+1) % d == 0 (and % 2d == 0 for the MID layout's padding line): the
    reference reads past the index end there; every plain-counter
    backend must return the true suffix-rank interval instead."""
    rng = np.random.default_rng(n)
    text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n).tobytes()
    bf = util.BruteForce(text.decode())
    t = np.frombuffer(text, dtype=np.uint8)
    for k, d in ((2, 64), (1, 32), (2, 32)):
        idx = gpu.Index.build(text, k=k, d=d)
        for m in (2, 4, 12):
            if m > n:
                continue
            st = rng.integers(0, n - m + 1, size=64)
            q = np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                                rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=(32, m))])
            want = np.array([x for i in range(q.shape[0]) for x in bf.interval(q[i].tobytes())], dtype=np.uint32)
            for b in PLAIN:
                if not coop_supported(b, k, d):
                    continue
                assert np.array_equal(gpu.search_array(idx, q, b), want), (n, k, d, m, b)


@pytest.mark.parametrize("bases", [2, 8, 12])
@pytest.mark.parametrize("backend", ["task-mid", "task", "task-ac", "coop-mid",
                                     "coop"])
def test_ftab_jump_start_equals_oracle(gpu, oracle_mod, random_index, backend, bases):
    """The ftab replaces the first bases/K LF steps by a table built with the
    same LF steps: results must not change (reads shorter than the table keep
    the plain path)."""
    text, idxs = random_index
    gpu.set_ftab(bases)
    try:
        for k, d in ((2, 64), (1, 64), (2, 192)):
            if not coop_supported(backend, k, d):
                continue
            idx = idxs[(k, d)]
            ref_img = idx.alt_counters()[0].image() if backend in ALT else idx.image()
            for m, n in ((100, 6000), (150, 1500), (bases, 800), (2 * k, 300)):
                if m % k:
                    continue
                q = _reads(text, n, m, seed=m + 31 * k + bases)
                want, _ = oracle_mod.search(ref_img, q)
                got = gpu.search_array(idx, q, backend)
                assert np.array_equal(got, want), (backend, bases, k, d, m)
    finally:
        gpu.set_ftab(0)


@pytest.mark.parametrize("backend", ["task-mid", "task-ac", "coop-mid", "task"])
def test_long_reads_fused_limit_and_pack_fallback(gpu, oracle_mod, random_index, backend):
    """Fused packing keeps up to 16 code words per query in registers (256 bases
    at K=2, 256 at K=1); longer reads fall back to the pack kernel, which packs
    rows of any length in word chunks of 1 KiB of bases (whole rows below
    that).  Both sides of each limit, odd alignments (m % 4 != 0, m % 16 != 0)
    and reads of several thousand bases (the reference's GPU path takes any
    m % 4 == 0; round 4 stopped at 2559) must match."""
    text, idxs = random_index
    for k, d in ((2, 64), (1, 64)):
        idx = idxs[(k, d)]
        ref_img = idx.alt_counters()[0].image() if backend in ALT else idx.image()
        for m in (254, 256, 258, 300, 1000, 1022, 1024, 1026, 1040, 2558, 2560, 3001, 4096, 10000):
            if m % k:
                continue
            n = 1500 if m < 2000 else (300 if m < 5000 else 100)
            q = _reads(text, n, m, seed=m * 3 + k)
            want, _ = oracle_mod.search(ref_img, q)
            got = gpu.search_array(idx, q, backend)
            assert np.array_equal(got, want), (backend, k, m)


@pytest.mark.parametrize("n", [63, 127, 191, 255, 1023, 4095, 100, 129, 5000, 62, 125])
@pytest.mark.parametrize("tail", ["random", "T-run"])
def test_ac_tail_blocks(gpu, oracle_mod, n, tail):
    """The AltCounters searcher differs from the true rank only past the last
    real block: its sentinel counts the '$' rows of block E-1 as their stored
    code (a T-run at the end of the text puts the '$' rows of every BWT_s
    there).  The *-ac-mid backends must reproduce the AltCounters oracle.
    Where the reference reads past its own file -- (n+1) % d == 0
    or a step landing in the sentinel block, (n+1) % d >= d - K -- its result
    is undefined (the CPU oracle refuses it); there every AltCounters backend
    must stay in bounds (steps capped at (S+2)*d - 1, kfmi_device.h ac_clamp)
    and agree with the host search."""
    rng = np.random.default_rng(n + (7 if tail == "T-run" else 0))
    t = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n)
    if tail == "T-run":
        t[-min(n, 40):] = ord("T")
    text = t.tobytes()
    for k, d in ((2, 64), (1, 32), (2, 32), (2, 128)):
        idx = gpu.Index.build(text, k=k, d=d)
        ac200 = idx.alt_counters()[0]
        for m in (2, 4, 12):
            if m > n or m % k:
                continue
            st = rng.integers(0, n - m + 1, size=64)
            q = np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                                rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=(32, m)),
                                np.full((4, m), ord("T"), dtype=np.uint8), np.full((4, m), ord("A"), dtype=np.uint8)])
            try:
                want, _ = oracle_mod.search(ac200.image(), q)
                defined = True
            except ValueError:
                defined = False
                want = gpu.search_cpu_array(ac200, q, 2)
                assert int(want.max()) <= ((n + d) // d + 2) * d - 1
            for b in ACMID:
                if coop_supported(b, k, d):
                    assert np.array_equal(gpu.search_array(idx, q, b), want), (n, tail, k, d, m, b, defined)


@pytest.mark.parametrize("backend", ["coop", "coop-mid", "coop-ac", "coop-ac-mid"])
def test_coop_backends_equal_oracle(gpu, oracle_mod, random_index, backend, monkeypatch):
    """The coop kernel's staging rounds (each round decodes its requests'
    chunk addresses; the pre-addressed form measured neutral and was removed,
    DESIGN 5 "Coop issue") on every coop backend and geometry: the same results
    as the oracle, incl. partial last waves, reads with m % K != 0, the pack
    kernel (m > 256) and the ftab jump start."""
    text, idxs = random_index
    for k, d in ((2, 64), (1, 64), (1, 32), (1, 128), (2, 128), (2, 256), (2, 32)):
        idx = idxs[(k, d)]
        if not coop_supported(backend, k, d):
            continue
        ref_img = idx.alt_counters()[0].image() if backend in ALT else idx.image()
        lens = [(100, 20011), (150, 3001), (2 * k, 999), (300, 517)]
        if backend not in ALT:
            lens.append((101, 1203))
        for m, n in lens:
            q = _reads(text, n, m, seed=m * 13 + k)
            want, _ = oracle_mod.search(ref_img if m % k == 0 else idxs[(1, 64)].image(), q)
            got = gpu.search_array(idx, q, backend)
            assert np.array_equal(got, want), (backend, k, d, m)
        if d == 64:
            gpu.set_ftab(4 * k)
            q = _reads(text, 5003, 100, seed=19 + k)
            want, _ = oracle_mod.search(ref_img, q)
            got = gpu.search_array(idx, q, backend)
            gpu.set_ftab(0)
            assert np.array_equal(got, want), (backend, k, d, "ftab")


@pytest.mark.parametrize("split", ["1", "2", "4"])
@pytest.mark.parametrize("backend", ["task-mid", "task", "task-ac", "task-ac-mid"])
def test_split_gathers_equal_oracle(gpu, oracle_mod, random_index, backend, split, knobs):
    """Every fetch form on small indexes, by forcing the table-size class
    (kfmi_set_split_class = 1: under 2 GB, 2: 2-3.5 GB, 4: larger): the asm
    fetch in one group (class 1) or two (classes 2, 4) where it applies (K=2
    d=64, K=1 d=128), else the C++ fetch, in four 16-lane groups for class 4
    (and class 2 in the 8-word fused kernel).  The same results as the
    oracle, incl. partial last waves (n % 64 != 0), reads with m % K != 0
    (remainder table), fused and pack-kernel reads, and the ftab jump start;
    d = 192 has no split path (lf_stream) and must be unaffected."""
    text, idxs = random_index
    knobs.split(split)
    for k, d in ((2, 64), (1, 64), (1, 32), (1, 128), (2, 128), (2, 192)):
        idx = idxs[(k, d)]
        if not coop_supported(backend, k, d):
            continue
        ref_img = idx.alt_counters()[0].image() if backend in ALT else idx.image()
        lens = [(100, 20011), (150, 3001), (2 * k, 999), (300, 517)]
        if backend not in ALT:
            lens.append((101, 1203))
        for m, n in lens:
            q = _reads(text, n, m, seed=m * 11 + k)
            # m % K != 0: the true interval, i.e. the K = 1 oracle's
            want, _ = oracle_mod.search(ref_img if m % k == 0 else idxs[(1, 64)].image(), q)
            got = gpu.search_array(idx, q, backend)
            assert np.array_equal(got, want), (backend, k, d, m)
        if d == 64:
            gpu.set_ftab(4 * k)
            q = _reads(text, 5003, 100, seed=17 + k)
            want, _ = oracle_mod.search(ref_img, q)
            got = gpu.search_array(idx, q, backend)
            gpu.set_ftab(0)
            assert np.array_equal(got, want), (backend, k, d, "ftab")


@pytest.mark.parametrize("backend,k,d,bases", [("task-ac", 1, 64, 12), ("task-ac", 2, 64, 12), ("task", 1, 32, 10),
                                               ("task", 1, 64, 10), ("task-mid", 2, 64, 10), ("task-ac-mid", 1, 64, 10),
                                               ("coop-mid", 2, 64, 10), ("coop-ac-mid", 1, 64, 10),
                                               ("task", 2, 192, 8)])
def test_ftab_table_every_entry(gpu, random_index, backend, k, d, bases):
    """Every entry of a freshly built jump-start table, three builds: the
    bases-long read of each code searched with the table (one lookup, no step)
    equals the search without it.  The tables are built by lf_stream (DESIGN.md
    5a; the 3 Mbase K = 1 AltCounters case is test_ftab_lf_stream_k1_ac_table)."""
    text, idxs = random_index
    if (k, d) not in idxs:
        idxs[(k, d)] = gpu.Index.build(text, k=k, d=d)
    idx = idxs[(k, d)]
    codes = np.arange(4 ** bases, dtype=np.uint32)
    q = np.frombuffer(b"ACGT", np.uint8)[(codes[:, None] >> (2 * np.arange(bases - 1, -1, -1))[None, :]) & 3].copy()
    gpu.set_ftab(0)
    want = gpu.search_array(idx, q, backend)
    try:
        for build in range(3):
            idx.free_gpu()
            gpu.set_ftab(bases)
            got = gpu.search_array(idx, q, backend)
            gpu.set_ftab(0)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (backend, k, d, bases, build, int(bad.size), int(bad[0] // 2))
    finally:
        gpu.set_ftab(0)


def test_ftab_lf_stream_k1_ac_table(gpu, oracle_mod):
    """The round-5 intermittent table, at the size it showed on: a 3 Mbase
    random text, K = 1, d = 64, tag 201 (task-ac), 12-base table (4^12
    entries) built inside the library by lf_stream, four fresh builds, every
    entry equal to the C oracle's search of that 12-mer
    (fmIndexCPUBaseline-AltCounters.c:218-266).  The old load form (a 16-byte
    load at 8-byte alignment, consumed under a partial vmcnt wait) gave 15-69
    wrong entries in every build on the same code path (profiles/r06/
    ftab_var_r6*.log, var 1 / 15); load_words keeps it out."""
    rng = np.random.default_rng(2026)
    text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=3_000_001).tobytes()
    idx = gpu.Index.build(text, k=1, d=64)
    acimg = idx.alt_counters()[0].image()
    codes = np.arange(4 ** 12, dtype=np.uint32)
    q = np.frombuffer(b"ACGT", np.uint8)[(codes[:, None] >> (2 * np.arange(11, -1, -1))[None, :]) & 3].copy()
    want, _ = oracle_mod.search(acimg, q)
    try:
        for build in range(4):
            idx.free_gpu()
            gpu.set_ftab(12)
            got = gpu.search_array(idx, q, "task-ac")
            gpu.set_ftab(0)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (build, int(bad.size), int(bad[0] // 2), got[bad[0]], want[bad[0]])
    finally:
        gpu.set_ftab(0)
        idx.close()
