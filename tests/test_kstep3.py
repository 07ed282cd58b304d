"""K = 3 on the GPU (the reference's K_STEPS is generic, genFMindex.c:29-56 and
fmIndexCPUBaseline.c:30-41; its scripts sweep k in 1..4): the grouped-counter
layout at K = 3 (4 lines of 128 B per block: the 48 B of bit planes + 16 of the
64 counters), task-grp / coop-grp.  A K-step is 6 bits, so the code words hold
5 K-steps (30 bits): the pack kernel writes them directly, the fused packers
re-cut their 16-bases-per-word stream (recut30).

Pins: the CPU restatement at K = 3, itself pinned against the reference's
K = 3 builder and searcher (oracle/_ref/gfmi_3_64, cpu_3_64) by
tests/test_kstep4.py; the K = 1 oracle for read lengths that are not multiples
of 3 (remainder table); brute-force suffix arrays for locate."""
import os

import numpy as np
import pytest

import util

pytestmark = pytest.mark.gpu

GRP = ("task-grp", "coop-grp")


def _text(n, seed):
    rng = np.random.default_rng(seed)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n)].copy()
    for _ in range(20):
        a, b = rng.integers(0, n - 600, size=2)
        t[b:b + 500] = t[a:a + 500]
    t[-50:] = ord("T")
    return t


def _reads(t, n, m, seed):
    rng = np.random.default_rng(seed)
    st = rng.integers(0, t.size - m, size=n)
    return np.ascontiguousarray(np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                                                rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(n // 4, m)),
                                                np.full((4, m), ord("T"), np.uint8),
                                                np.full((4, m), ord("A"), np.uint8)]))


@pytest.fixture(scope="module")
def k3(kfmi_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    t = _text(400_009, 3)
    text = t.tobytes()
    return t, K.Index.build(text, k=3, d=64, gpu=True), K.Index.build(text, k=1, d=64, gpu=False)


def test_k3_gpu_builder_equals_host_builder(kfmi_mod, k3):
    t, i3, _ = k3
    host = kfmi_mod.Index.build(t.tobytes(), k=3, d=64, gpu=False)
    assert bytes(host.image()) == bytes(i3.image())


@pytest.mark.parametrize("split", ["1", "4"])
@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("backend", GRP)
def test_k3_matches_oracle(kfmi_mod, oracle_mod, k3, backend, fused, split, knobs):
    knobs.fused(fused)
    knobs.split(split)   # 4: exec-masked gather groups (task-grp; coop ignores it)
    K = kfmi_mod
    t, i3, i1 = k3
    for m, n in ((99, 20_000), (150, 4_000), (3, 500), (15, 2_000), (126, 2_000), (129, 2_000), (255, 1_000),
                 (300, 1_000), (100, 3_000), (101, 3_000), (1, 300), (2, 300), (256, 1_000),
                 (1020, 300), (1500, 300), (3001, 150),
                 # m % 16 == 0: 16-B aligned slices whose length is not (the
                 # last chunk of 1,040 / 1,056, chunk 3 of 4,128)
                 (1040, 200), (1056, 200), (4128, 100)):
        q = _reads(t, n, m, m + 3)
        want = oracle_mod.search(i3.image() if m % 3 == 0 else i1.image(), q)[0]
        got = K.search_array(i3, q, backend)
        assert np.array_equal(got, want), (backend, m, fused, int(np.flatnonzero(got != want)[0]))


@pytest.mark.parametrize("backend", GRP)
def test_k3_ftab_stream_device_parse(kfmi_mod, oracle_mod, k3, backend, tmp_path):
    K = kfmi_mod
    t, i3, i1 = k3
    q = _reads(t, 6_000, 99, 77)
    want, _ = oracle_mod.search(i3.image(), q)
    for bases in (3, 9, 12, 15):
        K.set_ftab(bases)
        try:
            assert np.array_equal(K.search_array(i3, q, backend), want), bases
        finally:
            K.set_ftab(0)
    # host-streamed search: K = 3 chunks always go as ASCII (packed in the kernel)
    K.set_backend(backend)
    K.transfer_to_gpu(i3, None, None)
    for mode in ("1", "2"):
        os.environ["KFMI_STREAM_HOSTPACK"] = mode
        try:
            assert np.array_equal(K.search_stream(i3, q, chunk=1000), want), mode
        finally:
            os.environ.pop("KFMI_STREAM_HOSTPACK", None)
    K.load().kfmi_stream_release()
    # reads parsed on the device, 240 bases (more code-word rows at K = 3 than the
    # parser allocates for 16 bases per word)
    q240 = _reads(t, 3_000, 240, 9)
    fn = tmp_path / "q.fa"
    fn.write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in q240))
    qd = K.Queries.load_gpu(fn, 240)
    r = K.Results.alloc(qd.num())
    K.transfer_to_gpu(i3, qd, r)
    K.search(i3, qd, r)
    K.transfer_to_cpu(r)
    assert np.array_equal(r.array(), oracle_mod.search(i3.image(), q240)[0])
    qd.close()
    r.close()
    i3.free_gpu()


def test_k3_locate_and_block_count(kfmi_mod, oracle_mod):
    K = kfmi_mod
    t = _text(20_011, 8)
    text = t.tobytes()
    idx = K.Index.build(text, k=3, d=64, gpu=True, sa_rate=8)
    sa = util.suffix_array(text + b"$")
    q = _reads(t, 400, 12, 5)[:400]
    for b in GRP:
        res, off, pos = K.locate_array(idx, q, backend=b)
        for i in range(q.shape[0]):
            L, R = int(res[2 * i]), int(res[2 * i + 1])
            assert list(pos[off[i]:off[i + 1]]) == [int(x) for x in sa[L:R]], (b, i)
    q = _reads(t, 2000, 99, 6)
    _, want = oracle_mod.search(idx.image(), q)
    K.set_backend("task-grp")
    qq = K.Queries.from_array(q)
    r = K.Results.alloc(q.shape[0])
    K.transfer_to_gpu(idx, qq, r)
    assert K.count_blocks(idx, qq) == want


def test_k3_other_backends_refuse(kfmi_mod, k3):
    K = kfmi_mod
    t, i3, _ = k3
    q = _reads(t, 100, 99, 1)
    for b in ("task-mid", "coop-mid", "task", "coop-ac"):
        with pytest.raises(K.KfmiError) as e:
            K.search_array(i3, q, b)
        assert e.value.code == 33, b
