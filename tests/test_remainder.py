"""Reads whose length is not a multiple of K (m % K = rem != 0).

The reference reads P[-1] there, so it defines no result.
Here the last rem bases of such a read are resolved by one lookup in a
remainder table (rem_tab_kernel: [L, R) of every rem-base string, from two
K-steps out of [0, n+1) and the text's last bases at row 0) and the K-steps
cover the rest: the result is the read's suffix-array interval, i.e. what the
K = 1 searcher returns.  Checked against the oracle on a K = 1 index of the
same text (fmIndexCPUBaseline.c:157-292 at K_STEPS=1, pinned by the golden
files) and against brute-force suffix ranks on small texts, for the fused and
the pack-kernel code paths, K = 2 and K = 4.  The AltCounters-semantics
backends keep rejecting such reads.
"""
import numpy as np
import pytest

import util

pytestmark = pytest.mark.gpu

PLAIN2 = ("task", "coop", "task-mid", "coop-mid")
GRP = ("task-grp", "coop-grp")
ALT = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")


@pytest.fixture(scope="module")
def gpu(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_device(0)
    return kfmi_mod


@pytest.fixture(scope="module")
def texts(kfmi_mod):
    rng = np.random.default_rng(77)
    text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=1_000_003).tobytes()
    K = kfmi_mod
    return text, {kd: K.Index.build(text, k=kd[0], d=kd[1]) for kd in [(1, 64), (2, 64), (2, 192), (4, 64)]}


def _reads(text, n, m, seed):
    rng = np.random.default_rng(seed)
    t = np.frombuffer(text, dtype=np.uint8)
    st = rng.integers(0, len(text) - m, size=n)
    samp = t[st[:, None] + np.arange(m)[None, :]]
    rnd = rng.choice(np.frombuffer(b"ACGTNacgt", dtype=np.uint8), size=(n // 4, m))
    # the read that ends the text (its remainder bases are the text's last ones)
    end = t[len(text) - m:][None, :]
    return np.ascontiguousarray(np.concatenate([samp, rnd, end]))


@pytest.mark.parametrize("fused", ["1", "0"])
def test_rem_matches_k1_oracle(gpu, oracle_mod, texts, fused, knobs):
    knobs.fused(fused)
    text, idx = texts
    img1 = idx[(1, 64)].image()
    cases = [((2, 64), PLAIN2, (1, 3, 5, 17, 99, 101, 151, 255, 257, 301, 1025, 2049, 4001)),
             ((2, 192), ("task-mid", "coop-mid"), (1, 33, 101)),
             ((4, 64), GRP, (1, 2, 3, 5, 6, 7, 98, 99, 101, 150, 151, 254, 258, 1023, 1026, 4097))]
    for kd, backends, ms in cases:
        for m in ms:
            q = _reads(text, 3000 if m < 1000 else 300, m, seed=m + kd[0])
            want, _ = oracle_mod.search(img1, q)
            for b in backends:
                got = gpu.search_array(idx[kd], q, b)
                assert np.array_equal(got, want), (kd, b, m, fused, int(np.flatnonzero(got != want)[0]))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 7, 63, 64, 127, 100])
@pytest.mark.parametrize("tail", ["random", "A-run", "CA", "T-run"])
def test_rem_small_texts_against_bruteforce(gpu, n, tail):
    """Tiny texts and text ends built to hit the x.A^j.$ suffixes the table
    subtracts (an A-run or 'CA' at the end of the text)."""
    rng = np.random.default_rng(n * 13 + len(tail))
    t = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n)
    end = {"random": b"", "A-run": b"AAAA", "CA": b"CA", "T-run": b"TTT"}[tail]
    if end:
        e = np.frombuffer(end, dtype=np.uint8)[-n:]
        t[n - len(e):] = e
    text = t.tobytes()
    bf = util.BruteForce(text.decode())
    for k, d, backends in ((2, 64, ("task-mid", "coop-mid", "task")), (2, 32, ("task-mid", "task")),
                           (4, 64, GRP)):
        if n + 1 < k:                     # the builders need n + 1 >= K rows
            continue
        idx = gpu.Index.build(text, k=k, d=d)
        for m in range(1, 8):
            if m % k == 0:
                continue
            allq = np.array(np.meshgrid(*[np.frombuffer(b"ACGT", dtype=np.uint8)] * min(m, 3)), dtype=np.uint8)
            allq = allq.reshape(min(m, 3), -1).T                              # every string of min(m,3) bases
            if m > 3:
                allq = np.concatenate([rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=(allq.shape[0], m - 3)),
                                       allq], axis=1)
            st = rng.integers(0, max(1, n - m + 1), size=16)
            parts = [allq]
            if m <= n:
                parts.append(t[st[:, None] + np.arange(m)[None, :]])
                parts.append(t[n - m:][None, :])
            q = np.ascontiguousarray(np.concatenate(parts).astype(np.uint8))
            want = np.array([x for i in range(q.shape[0]) for x in bf.interval(q[i].tobytes())], dtype=np.uint32)
            for b in backends:
                if b.startswith("coop") and d == 32:
                    continue
                got = gpu.search_array(idx, q, b)
                assert np.array_equal(got, want), (n, tail, k, d, m, b)
        idx.close()


def test_rem_rejected_by_altcounters_backends(gpu, texts):
    text, idx = texts
    q = _reads(text, 100, 101, seed=1)
    for b in ALT:
        with pytest.raises(gpu.KfmiError) as e:
            gpu.search_array(idx[(2, 64)], q, b)
        assert e.value.code == 33, b


def test_rem_block_count_and_groups(gpu, oracle_mod, texts):
    """count_blocks starts from the table too (no index line for the remainder);
    a device group of one card listed twice returns the same intervals."""
    text, idx = texts
    q = _reads(text, 5000, 99, seed=5)
    want, _ = oracle_mod.search(idx[(1, 64)].image(), q)
    gpu.set_backend("task-mid")
    qq = gpu.Queries.from_array(q)
    r = gpu.Results.alloc(q.shape[0])
    gpu.transfer_to_gpu(idx[(2, 64)], qq, r)
    blocks = gpu.count_blocks(idx[(2, 64)], qq)
    assert 49 * q.shape[0] <= blocks <= 2 * 49 * q.shape[0]
    qq.close()
    r.close()
    gpu.set_devices([0, 0])
    try:
        assert np.array_equal(gpu.search_array(idx[(2, 64)], q, "coop-mid"), want)
    finally:
        gpu.set_devices([])
