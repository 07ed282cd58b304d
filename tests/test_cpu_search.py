"""searchIndexCPU (interface.h:30) from the product library
(csrc/host/cpu_search.c), host only -- no GPU needed:

* every golden index (tags 100/101/200/201, K in {1, 2}, d in {64, 192}, m in
  {1, 2, 12, 100, 150}) searched through kfmi_search_cpu equals the reference
  CPU searchers' result files (plain and AltCounters semantics);
* the reference's own driver (common/searchQueries.c) compiled WITHOUT -DCUDA
  and linked against libkstepfmi.so (oracle/Makefile searchQueries_cpu_dropin)
  calls it from every thread of its omp parallel region (the orphaned
  worksharing contract, searchQueries.c:84-95) and writes `.res.cpu` files
  byte-equal to the golden ones, at 1 and several threads;
* reads with m % K != 0 on plain indexes give the true suffix-array interval
  (brute force), AltCounters indexes reject them; (n+1) % d == 0 (B5) gives
  the true interval too;
* batch sizes (KFMI_CPU_BATCH) and thread counts do not change a result."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from util import GOLDEN, REPO, BruteForce, golden_cases, manifest, read_qry

CPU_DROPIN = REPO / "oracle" / "_ref" / "searchQueries_cpu_dropin"


def _golden_results(path) -> np.ndarray:
    from oracle import oracle
    return oracle.read_results_file(path)


CASES = list(golden_cases())


@pytest.mark.parametrize("case,key,k,d,tag,m,idx,qry,res", CASES,
                         ids=[f"{c[0]}-{c[1]}-t{c[4]}-m{c[5]}" for c in CASES])
def test_cpu_search_equals_reference_results(kfmi_mod, case, key, k, d, tag, m, idx, qry, res):
    I = kfmi_mod.Index.load(idx)
    got = kfmi_mod.search_cpu_array(I, read_qry(qry, m), nthreads=3)
    I.close()
    assert np.array_equal(got, _golden_results(res))


@pytest.mark.parametrize("key,tag,res_tag,m", [("k2_d64", 100, 100, 100), ("k2_d64", 200, 200, 100),
                                               ("k2_d64", 101, 100, 150), ("k2_d64", 201, 200, 12),
                                               ("k1_d64", 100, 100, 1), ("k1_d192", 200, 200, 150),
                                               ("k2_d192", 100, 100, 2)])
@pytest.mark.parametrize("threads", [1, 4])
def test_reference_cpu_driver_runs_on_engine(tmp_path, key, tag, res_tag, m, threads):
    if not CPU_DROPIN.exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    for case in ("textA", "textB"):
        c = manifest()[case]
        ent = c["indexes"][key]
        if f"{m}.{res_tag}" not in ent["results"]:
            continue
        idx = tmp_path / f"{case}.fmi"
        shutil.copy(GOLDEN / case / ent["files"][str(tag)]["file"], idx)
        qd = c["queries"][str(m)]
        shutil.copy(GOLDEN / case / qd["file"], tmp_path / "q.qry")
        env = dict(os.environ, OMP_NUM_THREADS=str(threads))
        p = subprocess.run([str(CPU_DROPIN), str(idx), str(tmp_path / "q.qry"), str(m), str(qd["num"])],
                           capture_output=True, text=True, env=env, timeout=120)
        assert p.returncode == 0, p.stdout + p.stderr
        assert "TIME:" in p.stdout
        want = (GOLDEN / case / ent["results"][f"{m}.{res_tag}"]["file"]).read_bytes()
        assert (tmp_path / f"{case}.fmi.res.cpu").read_bytes() == want, (case, key, tag, m)
        assert not (tmp_path / f"{case}.fmi.res.gpu").exists()


def test_cpu_driver_links_gnu_openmp_and_engine():
    if not CPU_DROPIN.exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    out = subprocess.run(["ldd", str(CPU_DROPIN)], capture_output=True, text=True).stdout
    assert "libkstepfmi.so" in out and "libgomp" in out and "not found" not in out
    nm = subprocess.run(["nm", "-D", str(REPO / "k-step_fm-index_amd" / "lib" / "libkstepfmi.so")],
                        capture_output=True, text=True).stdout
    assert " T searchIndexCPU" in nm and " T kfmi_search_cpu" in nm


def _random_case(n, seed):
    rng = np.random.default_rng(seed)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n)]
    return t, t.tobytes(), rng


def test_remainder_reads_are_true_intervals(kfmi_mod):
    """m % K != 0 at K = 2 and 4 (remainder table), text ends in an A-run so the
    x.A^j.$ suffixes matter; brute-force suffix ranks of T$."""
    t, text, rng = _random_case(3001, 7)
    text = text[:-4] + b"CAAA"
    t = np.frombuffer(text, np.uint8)
    bf = BruteForce(text.decode())
    for k in (2, 4):
        I = kfmi_mod.Index.build(text, k=k, d=64)
        for m in (1, 3, 5, 7, 13, 101):
            if m % k == 0:
                continue
            st = rng.integers(0, len(text) - m, size=150)
            q = np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                                np.frombuffer(text[-m:], np.uint8)[None, :],
                                rng.choice(np.frombuffer(b"ACGT", np.uint8), size=(50, m))])
            got = kfmi_mod.search_cpu_array(I, q, nthreads=2).reshape(-1, 2)
            want = np.array([bf.interval(r.tobytes()) for r in q], dtype=np.uint32)
            assert np.array_equal(got, want), (k, m)
        I.close()


def test_altcounters_reject_remainder_reads(kfmi_mod):
    t, text, rng = _random_case(2001, 8)
    I = kfmi_mod.Index.build(text, k=2, d=64)
    a200, a201 = I.alt_counters()
    q = t[:15].reshape(1, 15).copy()
    for A in (a200, a201):
        with pytest.raises(kfmi_mod.KfmiError) as ei:
            kfmi_mod.search_cpu_array(A, q)
        assert ei.value.code == 33
    for X in (a200, a201, I):
        X.close()


def test_b5_text_length_gives_true_intervals(kfmi_mod):
    """(n+1) % d == 0: R of the first step lies in block nentries, which the
    reference reads past its index (B5); the host search takes the end
    counters there -- the true interval, as the GPU layouts' padding entry."""
    n = 64 * 40 - 1
    t, text, rng = _random_case(n, 9)
    bf = BruteForce(text.decode())
    st = rng.integers(0, n - 10, size=200)
    q = t[st[:, None] + np.arange(10)[None, :]]
    for k in (1, 2):
        I = kfmi_mod.Index.build(text, k=k, d=64)
        got = kfmi_mod.search_cpu_array(I, q).reshape(-1, 2)
        assert np.array_equal(got, np.array([bf.interval(r.tobytes()) for r in q], dtype=np.uint32)), k
        I.close()


def test_batch_and_thread_counts_do_not_change_results(kfmi_mod, oracle_mod, monkeypatch):
    t, text, rng = _random_case(200_001, 10)
    I = kfmi_mod.Index.build(text, k=2, d=64)
    st = rng.integers(0, len(text) - 100, size=5003)                 # not a multiple of any batch
    q = np.concatenate([t[st[:, None] + np.arange(100)[None, :]],
                        rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(301, 100))])
    want, _ = oracle_mod.search(I.image(), q)
    for b in ("1", "7", "32", "256"):
        monkeypatch.setenv("KFMI_CPU_BATCH", b)
        for thr in (1, 3, 8):
            assert np.array_equal(kfmi_mod.search_cpu_array(I, q, nthreads=thr), want), (b, thr)
    I.close()


def test_cpu_search_argument_errors(kfmi_mod):
    t, text, rng = _random_case(1001, 11)
    I = kfmi_mod.Index.build(text, k=2, d=64)
    q = kfmi_mod.Queries.from_array(t[:20].reshape(2, 10).copy())
    r = kfmi_mod.Results.alloc(1)                       # fewer results than queries
    with pytest.raises(kfmi_mod.KfmiError) as ei:
        kfmi_mod.search_cpu(I, q, r)
    assert ei.value.code == 33
    # searchIndexCPU itself is void (interface.h:30): the status is kfmi_last_error
    L = kfmi_mod.load()
    L.searchIndexCPU(I.ptr, q.ptr, r.ptr)
    assert L.kfmi_last_error() == 33
    r.close()
    r = kfmi_mod.Results.alloc(2)
    L.searchIndexCPU(I.ptr, q.ptr, r.ptr)               # outside a parallel region: the calling thread
    assert L.kfmi_last_error() == 0
    assert np.array_equal(r.array(), kfmi_mod.search_cpu_array(I, t[:20].reshape(2, 10).copy()))
    for h in (q, r, I):
        h.close()


@pytest.mark.gpu
def test_cpu_search_on_a_device_resident_index(kfmi_mod):
    """An index built on the device without a host image: searchIndexCPU
    fetches its entries once (kfmi_host_entries, one thread of the team) and
    returns what the GPU backends return."""
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    t, text, rng = _random_case(300_001, 12)
    idx = K.Index.build(text, k=2, d=64, gpu=True, host_image=False)
    st = rng.integers(0, len(text) - 100, size=20_000)
    q = np.ascontiguousarray(t[st[:, None] + np.arange(100)[None, :]])
    want = K.search_array(idx, q, "task-mid")
    assert np.array_equal(K.search_cpu_array(idx, q, nthreads=4), want)
    idx.close()


def test_large_image_on_2mb_pages(kfmi_mod, oracle_mod, monkeypatch, tmp_path):
    """An index image of 64 MB or more is a 2 MB-aligned mapping advised to
    huge pages (kfmi_big_alloc; the host search's random LFs then walk 2 MB
    pages), KFMI_HUGEPAGES=0 a plain allocation; both search alike, survive a
    save / load round trip and are released by freeIndex."""
    import ctypes
    t, text, rng = _random_case(46_000_001, 13)          # 46M bases: a 69 MB tag-100 image
    q = t[rng.integers(0, len(text) - 100, size=3000)[:, None] + np.arange(100)]
    res = {}
    for hp in ("1", "0"):
        monkeypatch.setenv("KFMI_HUGEPAGES", hp)
        I = kfmi_mod.Index.build(text, k=2, d=64)
        img = I.image()
        assert img.nbytes >= 64 << 20
        addr = img.__array_interface__["data"][0]
        assert (addr % (2 << 20) == 0) == (hp == "1"), (hp, hex(addr))
        res[hp] = kfmi_mod.search_cpu_array(I, q, nthreads=4)
        I.save(tmp_path / f"i{hp}")                                   # the reference's file naming
        J = kfmi_mod.Index.load(next(tmp_path.glob(f"i{hp}.*fmi")))  # loadIndex allocates the same way
        assert np.array_equal(kfmi_mod.search_cpu_array(J, q, nthreads=2), res[hp])
        J.close()
        if hp == "1":
            want, _ = oracle_mod.search(img, q)
            assert np.array_equal(res[hp], want)
        del img
        I.close()
    assert np.array_equal(res["1"], res["0"])


@pytest.mark.parametrize("form", ["plain", "ac"])
def test_cpu_search_on_corrupt_counters_stays_in_image(kfmi_mod, oracle_mod, form):
    """searchIndexCPU (the product's host search) on a file whose counters are
    wrapped or oversized (0xFFFFFFFF, 2^31, random u32 on an eighth of the
    entries): a step landing past the last entry reads the padding entry's
    end counters (cs_lf), so the search returns instead of reading past the
    image -- the host side of the GPU kernels' LF cap."""
    K = kfmi_mod
    rng = np.random.default_rng(92)
    t = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=20_001)
    src = K.Index.build(t.tobytes(), k=2, d=64)
    img = np.array(src.image(), dtype=np.uint8, copy=True)
    src.close()
    h = oracle_mod.header(img)
    k, d, ne = h["steps"], h["chunk"], h["nentries"]
    nb = d // 32
    ew = 2 * nb * k + 4 ** k
    q = np.concatenate([t[rng.integers(0, t.size - 40, size=300)[:, None] + np.arange(40)],
                        rng.choice(np.frombuffer(b"ACGT", np.uint8), size=(100, 40))])
    for how in ("ones", "high", "random"):
        bad = img.copy()
        ent = bad[bad.size - 4 * ew * ne:].view(np.uint32).reshape(ne, ew)
        rows = rng.choice(ne, size=max(1, ne // 8), replace=False)
        vals = {"ones": 0xFFFFFFFF, "high": 0x80000000}.get(how)
        ent[rows, 2 * nb * k:] = (vals if vals is not None else
                                  rng.integers(0, 1 << 32, size=(rows.size, 4 ** k), dtype=np.uint64).astype(np.uint32))
        idx = K.Index.from_image(bad)
        if form == "ac":
            idx = idx.alt_counters()[0]
        got = K.search_cpu_array(idx, q, nthreads=2)
        assert got.shape == (2 * q.shape[0],)
        idx.close()
