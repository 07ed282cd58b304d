"""K = 4 (the reference's K_STEPS is generic, genFMindex.c:29-56 and
fmIndexCPUBaseline.c:30-41; its GPU files stop at K = 2): the grouped-counter
backends task-grp / coop-grp (LAY_GRP).

Pins: the reference builder and CPU searcher compiled at K = 3, 4
(oracle/_ref/gfmi_{3,4}_64, cpu_{3,4}_64) against our builders and the C
restatement (CPU tests); the GPU backends against that restatement, against
the K = 2 results for the same reads (the interval of a read does not depend
on K), against brute-force suffix ranks at the B5 boundary, and through the
ftab, locate and streamed paths."""
import hashlib
import subprocess

import numpy as np
import pytest

import util

GRP = ("task-grp", "coop-grp")


def _text(n, seed, repeats=False):
    rng = np.random.default_rng(seed)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n)].copy()
    if repeats:
        for _ in range(20):
            a, b = rng.integers(0, n - 600, size=2)
            t[b:b + 500] = t[a:a + 500]
        t[-60:] = ord("T")
    return t


def _reads(t, n, m, seed):
    rng = np.random.default_rng(seed)
    st = rng.integers(0, t.size - m, size=n)
    return np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                           rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(n // 4, m)),
                           np.full((4, m), ord("T"), np.uint8), np.full((4, m), ord("A"), np.uint8)])


@pytest.mark.parametrize("k", [3, 4])
@pytest.mark.parametrize("repeats", [False, True])
def test_k34_builder_and_oracle_match_reference_binaries(kfmi_mod, oracle_mod, tmp_path, k, repeats):
    gfmi, cpu = oracle_mod.ref_binary("gfmi", k, 64), oracle_mod.ref_binary("cpu", k, 64)
    if not gfmi.exists() or not cpu.exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    n = 40_003
    t = _text(n, 10 * k + repeats, repeats)
    text = t.tobytes()
    (tmp_path / "ref.fa").write_bytes(b">x\n" + b"\n".join(text[i:i + 70] for i in range(0, n, 70)) + b"\n")
    subprocess.run([str(gfmi), "ref.fa", str(n)], cwd=tmp_path, check=True, capture_output=True, timeout=300)
    fn = tmp_path / f"ref.fa.{n}.64fmi{k}steps.fmi"
    ref = fn.read_bytes()
    ours = kfmi_mod.Index.build(text, k=k, d=64, gpu=False).image().tobytes()
    assert hashlib.md5(ours).hexdigest() == hashlib.md5(ref).hexdigest()
    for m in (12, 24, 100 if k == 4 else 102):
        q = _reads(t, 800, m, m)
        (tmp_path / "q.qry").write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in q))
        subprocess.run([str(cpu), str(fn), "q.qry", str(m), str(q.shape[0])], cwd=tmp_path, check=True,
                       capture_output=True, timeout=300)
        want = oracle_mod.read_results_file(str(fn) + ".res.cpu")
        got, _ = oracle_mod.search(ref, q)
        assert np.array_equal(got, want), (k, m)
        i2 = kfmi_mod.Index.build(text, k=2, d=64, gpu=False)
        assert np.array_equal(oracle_mod.search(i2.image(), q)[0], want)   # K-independent intervals


@pytest.fixture(scope="module")
def k4(kfmi_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    t = _text(500_003, 4, repeats=True)
    text = t.tobytes()
    return t, K.Index.build(text, k=4, d=64, gpu=True), K.Index.build(text, k=2, d=64, gpu=True)


@pytest.mark.gpu
@pytest.mark.parametrize("split", ["1", "4"])
@pytest.mark.parametrize("backend", GRP)
def test_grp_matches_oracle_and_k2(kfmi_mod, oracle_mod, k4, backend, split, knobs):
    """split 4: per-lane gathers as 4 exec-masked groups (the default for the
    96 GB GRP table at 3 Gbase; the coop kernel ignores it)."""
    K = kfmi_mod
    knobs.split(split)
    t, i4, i2 = k4
    for m, n in ((100, 20_000), (16, 4_000), (4, 2_000), (256, 1_000), (300, 1_000), (8, 500), (102, 1_001),
                 (150, 777)):
        q = _reads(t, n, m, m + 1)
        want, _ = oracle_mod.search(i4.image() if m % 4 == 0 else i2.image(), q)   # m % 4 = 2: remainder table
        got = K.search_array(i4, q, backend)
        assert np.array_equal(got, want), (backend, m, int(np.flatnonzero(got != want)[0]))
        assert np.array_equal(got, K.search_array(i2, q, "task-mid")), (backend, m)


@pytest.mark.gpu
def test_grp_rejects_other_k_and_takes_any_m(kfmi_mod, k4):
    K = kfmi_mod
    t, i4, i2 = k4
    q = _reads(t, 100, 100, 3)
    for backend, idx in (("task-mid", i4), ("coop", i4)):
        with pytest.raises(K.KfmiError) as e:
            K.search_array(idx, q, backend)
        assert e.value.code == 33, backend
    # the grouped backends take a K = 2 index too: its K = 4 index is derived on upload (DESIGN 5d')
    for backend in GRP:
        assert np.array_equal(K.search_array(i2, q, backend), K.search_array(i2, q, "task-mid")), backend
    # 102 % 4 = 2 (reference defect B6): the last 2 bases from the remainder
    # table (tests/test_remainder.py), the interval equals the K = 2 one
    q = _reads(t, 2000, 102, 1)
    for backend in GRP:
        assert np.array_equal(K.search_array(i4, q, backend), K.search_array(i2, q, "task-mid")), backend


@pytest.mark.gpu
@pytest.mark.parametrize("n", [63, 127, 255, 1023, 100])
def test_grp_b5_boundary_against_bruteforce(kfmi_mod, n):
    K = kfmi_mod
    rng = np.random.default_rng(n)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n)].copy()
    bf = util.BruteForce(t.tobytes().decode())
    idx = K.Index.build(t.tobytes(), k=4, d=64)
    for m in (4, 8, 12):
        if m > n:
            continue
        st = rng.integers(0, n - m + 1, size=48)
        q = np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                            np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=(32, m))]])
        want = np.array([x for i in range(q.shape[0]) for x in bf.interval(q[i].tobytes())], dtype=np.uint32)
        for b in GRP:
            assert np.array_equal(K.search_array(idx, q, b), want), (n, m, b)


@pytest.mark.gpu
@pytest.mark.parametrize("backend", GRP)
def test_grp_ftab_stream_locate(kfmi_mod, oracle_mod, k4, backend):
    K = kfmi_mod
    t, i4, _ = k4
    q = _reads(t, 6_000, 100, 77)
    want, _ = oracle_mod.search(i4.image(), q)
    for bases in (8, 12):
        K.set_ftab(bases)
        try:
            assert np.array_equal(K.search_array(i4, q, backend), want), bases
        finally:
            K.set_ftab(0)
    K.set_backend(backend)
    K.transfer_to_gpu(i4, None, None)
    for mode in ("1", "0"):
        import os
        os.environ["KFMI_STREAM_HOSTPACK"] = mode
        try:
            assert np.array_equal(K.search_stream(i4, q, chunk=1000), want), mode
        finally:
            os.environ.pop("KFMI_STREAM_HOSTPACK", None)
    K.load().kfmi_stream_release()
    i4.free_gpu()


@pytest.mark.gpu
def test_grp_locate_against_bruteforce(kfmi_mod):
    K = kfmi_mod
    t = _text(20_011, 8, repeats=True)
    text = t.tobytes()
    idx = K.Index.build(text, k=4, d=64, gpu=True, sa_rate=8)
    sa = util.suffix_array(text + b"$")
    q = _reads(t, 400, 12, 5)[:400]
    res, off, pos = K.locate_array(idx, q, backend="task-grp")
    for i in range(q.shape[0]):
        L, R = int(res[2 * i]), int(res[2 * i + 1])
        assert list(pos[off[i]:off[i + 1]]) == [int(x) for x in sa[L:R]], i


@pytest.mark.gpu
def test_k4_results_located_through_a_k2_companion(kfmi_mod):
    """The rows of [L, R) are suffix-array ranks, the same for every K of one
    text: K = 4 results (coop-grp) are located through a K = 2 index of the
    same text (the cooperative MID walk, one line per step) -- positions equal
    the brute-force suffix array and the K = 4 index's own (per-lane) walk."""
    K = kfmi_mod
    t = _text(50_021, 9, repeats=True)
    text = t.tobytes()
    sa = util.suffix_array(text + b"$")
    i4 = K.Index.build(text, k=4, d=64, gpu=True, sa_rate=8)
    i2 = K.Index.build(text, k=2, d=64, gpu=True, sa_rate=8)
    q = _reads(t, 3000, 100, 6)
    try:
        K.set_backend("coop-grp")
        qq, r = K.Queries.from_array(q), K.Results.alloc(q.shape[0])
        K.transfer_to_gpu(i4, qq, r)
        K.search(i4, qq, r)
        own = K.locate(i4, r)
        K.set_backend("task-mid")
        K.transfer_to_gpu(i2, None, None)
        loc = K.locate(i2, r)                    # K = 4 results, K = 2 walk
        K.transfer_to_cpu(r)
        res = r.array()
        off, pos = loc.offsets(), loc.positions()
        assert np.array_equal(off, own.offsets()) and np.array_equal(pos, own.positions())
        for i in range(q.shape[0]):
            L, R = int(res[2 * i]), int(res[2 * i + 1])
            assert [int(x) for x in pos[off[i]:off[i + 1]]] == [int(x) for x in sa[L:R]], i
        loc.close(); own.close(); qq.close(); r.close()
    finally:
        i4.free_gpu(); i2.free_gpu()
        i4.close(); i2.close()


@pytest.mark.gpu
def test_k4_index_under_the_implicit_default_backend(kfmi_mod, oracle_mod, tmp_path):
    """No KFMI_BACKEND, no kfmi_set_backend: a K = 4 index is uploaded for
    coop-grp (the default task-mid has no K = 4 geometry).  Fresh process, so
    the thread's backend is still the implicit one."""
    t = _text(100_003, 12)
    q = _reads(t, 2000, 100, 12)
    np.save(tmp_path / "q.npy", q)
    (tmp_path / "t.bin").write_bytes(t.tobytes())
    code = f"""
import sys, numpy as np
sys.path.insert(0, {str(util.PKG)!r})
import kstep_fmi as K
K.load(); K.set_device(0)
i4 = K.Index.build(open({str(tmp_path / "t.bin")!r}, "rb").read(), k=4, d=64)
q = np.load({str(tmp_path / "q.npy")!r})
np.save({str(tmp_path / "got.npy")!r}, K.search_array(i4, q))
print(K.get_backend())
"""
    env = {k: v for k, v in __import__("os").environ.items() if k != "KFMI_BACKEND"}
    p = subprocess.run([__import__("sys").executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    i4 = kfmi_mod.Index.build(t.tobytes(), k=4, d=64)
    want, _ = oracle_mod.search(i4.image(), q)
    assert np.array_equal(np.load(tmp_path / "got.npy"), want)
