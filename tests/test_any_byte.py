"""Reads holding every byte value.  The reference maps a base by its ASCII
bits 1-2 (base2index, fmIndexCPUBaseline.c:213-226: A/a=0 C/c=1 G/g=2 T/t=3,
N->2, anything else by those bits), so a read is any byte string; reads handed
over in memory (searchIndexGPU on a caller's buffer, not a FASTA file) can
hold NUL, '\\n' or bytes >= 0x80.  Every searcher must map them as the
restatement does (oracle/fmi_oracle.c code_of)."""
import numpy as np
import pytest

PLAIN = ("task", "coop", "task-mid", "coop-mid")
ALT = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")


def _case(k, m):
    rng = np.random.default_rng(256 + k * 1000 + m)
    t = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=30_001)
    all_bytes = np.arange(256, dtype=np.uint8)
    q = [rng.integers(0, 256, size=(300, m)).astype(np.uint8)]
    # every byte value at every position class of a K-mer, inside text-sampled reads
    st = rng.integers(0, t.size - m, size=256)
    s = t[st[:, None] + np.arange(m)[None, :]].copy()
    s[np.arange(256), rng.integers(0, m, size=256)] = all_bytes
    q.append(s)
    return t.tobytes(), np.ascontiguousarray(np.concatenate(q))


@pytest.mark.parametrize("k,m", [(1, 37), (2, 100), (2, 64)])
def test_any_byte_host(kfmi_mod, oracle_mod, k, m):
    K = kfmi_mod
    text, q = _case(k, m)
    idx = K.Index.build(text, k=k, d=64)
    acs = idx.alt_counters()
    try:
        want = oracle_mod.search(idx.image(), q)[0]
        assert np.array_equal(K.search_cpu_array(idx, q, 2), want)
        want_ac = oracle_mod.search(acs[0].image(), q)[0]
        for a in acs:
            assert np.array_equal(K.search_cpu_array(a, q, 2), want_ac)
    finally:
        for x in (idx,) + tuple(acs):
            x.close()


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", [(1, 37), (2, 100), (2, 64)])
def test_any_byte_gpu(kfmi_mod, oracle_mod, k, m):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    text, q = _case(k, m)
    idx = K.Index.build(text, k=k, d=64, gpu=True)
    acs = idx.alt_counters()
    try:
        want = oracle_mod.search(idx.image(), q)[0]
        want_ac = oracle_mod.search(acs[0].image(), q)[0]
        for b in PLAIN + ALT:
            try:
                got = K.search_array(idx, q, b)
            except K.KfmiError as e:
                assert e.code == 33, (b, e.code)   # a geometry the backend does not take
                continue
            assert np.array_equal(got, want_ac if b in ALT else want), (b, k, m)
    finally:
        for x in (idx,) + tuple(acs):
            x.close()
