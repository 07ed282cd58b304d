"""GPU parity at the configs' own scale (BASELINE configs #2-#5): the 3 Gbase
recipe text indexed on the device, searched by every
backend through the C ABI.

Pins (produced by the reference's own binaries,
/root/reference/src/genFMindex.c:457-543 and fmIndexCPUBaseline.c:157-292):
  * the GPU-built tag-100 index image           md5 38f85a87...
  * the q1M reads (random.Random(1))            md5 973c43bb...
  * every backend's q1M results file            md5 96148f99...
  * the q10M reads (random.Random(10))          md5 6a87831e...
  * the q10M results file (one backend's md5, every other backend equal)
                                                md5 cfa6bc65...
The 150 bp leg (config #5's read length) has no reference vector at this
scale: 200K sampled + 50K random/N/lowercase reads are checked against the C
restatement (oracle/fmi_oracle.c), plain and AltCounters semantics.

The text has n+1 = 3,000,000,001 rows, so every LF here crosses 2^31.
"""
import hashlib

import numpy as np
import pytest

import util
from test_gpu_parity import ALT, PLAIN

pytestmark = pytest.mark.gpu

N3G = 3_000_000_000


@pytest.fixture(scope="module")
def gpu(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    return kfmi_mod


@pytest.fixture(scope="module")
def g3(gpu):
    from kstep_fmi import synth
    text = synth.text_3g(N3G)
    idx = gpu.Index.build(text, k=2, d=64, gpu=True)
    yield text, idx
    idx.free_gpu()
    idx.close()


@pytest.fixture(scope="module")
def reads(g3, oracle_mod):
    """q1M, q10M (md5-pinned) and the 150 bp leg with its oracle results."""
    from kstep_fmi import synth
    text, idx = g3
    q1m = synth.gather_reads(text, synth.read_starts(N3G, 1_000_000, 100, seed=1), 100)
    q10m = synth.gather_reads(text, synth.read_starts(N3G, 10_000_000, 100, seed=10), 100)
    rng = np.random.default_rng(150)
    t = np.frombuffer(text, dtype=np.uint8)
    st = rng.integers(0, N3G - 150, size=200_000)
    q150 = np.concatenate([t[st[:, None] + np.arange(150)[None, :]],
                           rng.choice(np.frombuffer(b"ACGTNacgt", dtype=np.uint8), size=(50_000, 150))])
    want150, _ = oracle_mod.search(idx.image(), q150)
    i200, i201 = idx.alt_counters()
    i201.close()
    want150ac, _ = oracle_mod.search(i200.image(), q150)
    i200.close()
    return {"q1m": q1m, "q10m": q10m, "q150": q150, "want150": want150, "want150ac": want150ac, "res10m": {}}


def test_3g_index_md5_pinned(g3):
    """GPU builder output == the reference builder's 3 Gbase tag-100 file."""
    from kstep_fmi import synth
    _, idx = g3
    h = idx.header()
    assert h["bwtsize"] == N3G + 1 and h["bwtsize"] > 2 ** 31
    assert hashlib.md5(idx.image().tobytes()).hexdigest() == synth.MD5["ref3g.k2d64.fmi"]


def test_3g_reads_md5_pinned(reads):
    from kstep_fmi import synth
    assert synth.qry_md5(reads["q1m"]) == synth.MD5["q1M.qry"]
    assert synth.qry_md5(reads["q10m"]) == synth.MD5["q10M.qry"]


@pytest.mark.parametrize("backend", ("task-mid",) + tuple(b for b in PLAIN + ALT if b != "task-mid"))
def test_3g_backend_full_scale(gpu, g3, reads, backend, tmp_path):
    from kstep_fmi import synth
    _, idx = g3
    # q1M: every backend's own results file md5 (configs #2-#4 read count 1M)
    res = gpu.search_array(idx, reads["q1m"], backend)
    assert int(res.max()) > 2 ** 31                       # rows past 2^31 are exercised
    assert util.results_md5(gpu, res, tmp_path) == synth.MD5["res3g.q1M"], backend
    # q10M: the headline batch; md5 once, then bit-equality with it
    res = gpu.search_array(idx, reads["q10m"], backend)
    ref = reads["res10m"]
    if not ref:
        assert util.results_md5(gpu, res, tmp_path) == synth.MD5["res3g.q10M"], backend
        ref["res"] = res
    else:
        assert np.array_equal(res, ref["res"]), backend
    # 150 bp (config #5's read length): oracle restatement, plain or AC semantics
    want = reads["want150ac"] if backend in ALT else reads["want150"]
    got = gpu.search_array(idx, reads["q150"], backend)
    assert np.array_equal(got, want), (backend, int(np.flatnonzero(got != want)[0]))
    idx.free_gpu()


@pytest.mark.parametrize("split", ["", "1"])
def test_3g_kstep4_full_scale(gpu, g3, reads, split, tmp_path, knobs):
    """K = 4 on the same 3 Gbase text (LAY_GRP, 96 GB of lines, device-resident
    build): the same suffix-array intervals, so the q1M results file md5 and
    the q10M results equal the K = 2 pins; 150 bp (150 % 4 = 2 bases from the
    remainder table) equals the plain oracle.  task-grp runs with its default
    split-issue gathers ("") and with plain issue ("1")."""
    from kstep_fmi import synth
    text, idx2 = g3
    if split:
        knobs.split(split)
    idx2.free_gpu()
    i4 = gpu.Index.build(text, k=4, d=64, gpu=True, host_image=False)
    try:
        for backend in (("task-grp", "coop-grp") if not split else ("task-grp",)):
            res = gpu.search_array(i4, reads["q1m"], backend)
            assert util.results_md5(gpu, res, tmp_path) == synth.MD5["res3g.q1M"], backend
            res = gpu.search_array(i4, reads["q10m"], backend)
            if reads["res10m"]:
                assert np.array_equal(res, reads["res10m"]["res"]), backend
            else:
                assert util.results_md5(gpu, res, tmp_path) == synth.MD5["res3g.q10M"], backend
            got = gpu.search_array(i4, reads["q150"], backend)
            assert np.array_equal(got, reads["want150"]), (backend, int(np.flatnonzero(got != reads["want150"])[0]))
    finally:
        i4.free_gpu()
        i4.close()


def test_3g_config5_whole_batch(gpu, g3, oracle_mod):
    """Config #5's whole batch in one process: 80M x 150 bp reads (12 GB of
    ASCII, more than 2^32 bytes and 2^32 intervals' worth of offsets) on the
    3 Gbase index, through the reference's own handles laid out as config #5
    lays them out -- the index replicated on 8 members (KFMI_DEVICES; here the
    one card listed 8 times, so the replicas and slices are real but the card
    is shared) and the reads cut into 8 slices -- and through the streamed
    path on the same group.  Both equal, and an evenly spread 200 K-read sample
    equals the CPU oracle.  (The 8-GPU timing is the driver's SCALE run.)"""
    from kstep_fmi import synth
    text, idx = g3
    n = 80_000_000
    rng = np.random.default_rng(805)
    reads = synth.gather_reads(text, rng.integers(0, N3G - 150, size=n), 150)
    assert reads.nbytes > 2 ** 32
    sel = np.linspace(0, n - 1, 200_000).astype(np.int64)
    want, _ = oracle_mod.search(idx.image(), reads[sel])
    gpu.set_backend("task-mid")
    try:
        gpu.set_devices([0] * 8)
        q = gpu.Queries.from_array(reads)
        r = gpu.Results.alloc(n)
        gpu.transfer_to_gpu(idx, q, r)
        gpu.search(idx, q, r)
        gpu.transfer_to_cpu(r)
        res = r.array().copy()
        q.close()
        r.close()
        assert np.array_equal(res.reshape(-1, 2)[sel], want.reshape(-1, 2))
        streamed = gpu.search_stream(idx, reads)
        assert np.array_equal(streamed, res)
    finally:
        gpu.set_devices([])
        idx.free_gpu()
