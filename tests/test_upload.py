"""Query uploads (transferCPUtoGPU, interface.h:40): the ASCII upload (the
default) and the host-packed one (KFMI_UPLOAD=packed, K in {1, 2, 4}) leave
the same reads on the device -- the packed
upload's code words are what the pack kernel writes -- so every backend
returns the oracle's intervals either way: several upload chunks
(KFMI_UPLOAD_CHUNK) with partial ones, m % K != 0 (remainder row), reads past
the fused limit, ftab, block counts, device groups, K = 4."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PLAIN = ("task-mid", "coop-mid", "task", "coop")
ALT = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")


@pytest.fixture(scope="module")
def gpu(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    kfmi_mod.set_devices([])
    kfmi_mod.set_device(0)
    return kfmi_mod


@pytest.fixture(scope="module")
def data(gpu):
    rng = np.random.default_rng(77)
    text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=1_000_001).tobytes()
    idx = {kd: gpu.Index.build(text, k=kd[0], d=kd[1]) for kd in ((2, 64), (1, 64), (2, 128), (4, 64))}
    return text, idx


def _reads(text, n, m, seed):
    rng = np.random.default_rng(seed)
    t = np.frombuffer(text, dtype=np.uint8)
    st = rng.integers(0, len(text) - m, size=n)
    return np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                           rng.choice(np.frombuffer(b"ACGTNacgt", dtype=np.uint8), size=(n // 5, m))])


@pytest.mark.parametrize("backend", PLAIN + ALT)
def test_packed_upload_equals_oracle(gpu, oracle_mod, data, backend, monkeypatch):
    text, idx = data
    monkeypatch.setenv("KFMI_UPLOAD", "packed")
    monkeypatch.setenv("KFMI_UPLOAD_CHUNK", "4093")          # many chunks, the last one partial
    for kd in ((2, 64), (1, 64), (2, 128)):
        k = kd[0]
        I = idx[kd]
        ref = I.alt_counters()[0].image() if backend in ALT else I.image()
        lens = [(100, 20011), (2 * k, 999), (300, 517)]
        if backend not in ALT:
            lens += [(101, 1203), (7, 2001)]
        for m, n in lens:
            q = _reads(text, n, m, seed=m * 3 + k)
            want, _ = oracle_mod.search(ref if m % k == 0 else idx[(1, 64)].image(), q)
            try:
                got = gpu.search_array(I, q, backend)
            except gpu.KfmiError as e:
                assert e.code == 33 and backend.startswith("coop")   # geometry the coop kernel refuses
                break
            assert np.array_equal(got, want), (backend, kd, m)


def test_ascii_and_packed_uploads_agree(gpu, oracle_mod, data, monkeypatch):
    """The same handles re-transferred in either form, the ftab jump start and
    block counts on packed reads; a K = 1 then K = 2 index re-packs the reads."""
    text, idx = data
    q = _reads(text, 30011, 100, seed=5)
    want, blocks = oracle_mod.search(idx[(2, 64)].image(), q)
    Q = gpu.Queries.from_array(q)
    R = gpu.Results.alloc(q.shape[0])
    gpu.set_backend("task-mid")
    monkeypatch.setenv("KFMI_UPLOAD_CHUNK", "1000")
    assert gpu.upload_form(Q) == "none"
    for form in ("ascii", "packed", "ascii", "packed"):
        monkeypatch.setenv("KFMI_UPLOAD", form)
        for kd in ((1, 64), (2, 64)):
            gpu.transfer_to_gpu(idx[kd], Q, R)
            assert gpu.upload_form(Q) == form
            gpu.search(idx[kd], Q, R)
            gpu.transfer_to_cpu(R)
            w = want if kd == (2, 64) else oracle_mod.search(idx[kd].image(), q)[0]
            assert np.array_equal(R.array(), w), (form, kd)
        assert gpu.count_blocks(idx[(2, 64)], Q) == blocks, form
        gpu.set_ftab(8)
        gpu.search(idx[(2, 64)], Q, R)
        gpu.transfer_to_cpu(R)
        gpu.set_ftab(0)
        assert np.array_equal(R.array(), want), (form, "ftab")
    Q.close()
    R.close()


def test_packed_upload_k4_and_groups(gpu, oracle_mod, data, monkeypatch):
    text, idx = data
    monkeypatch.setenv("KFMI_UPLOAD", "packed")
    monkeypatch.setenv("KFMI_UPLOAD_CHUNK", "2048")
    q = _reads(text, 9001, 100, seed=9)
    want, _ = oracle_mod.search(idx[(2, 64)].image(), q)
    assert np.array_equal(gpu.search_array(idx[(4, 64)], q, "coop-grp"), want)
    q102 = _reads(text, 3001, 102, seed=10)                       # 102 % 4 = 2: remainder row
    assert np.array_equal(gpu.search_array(idx[(4, 64)], q102, "coop-grp"),
                          oracle_mod.search(idx[(1, 64)].image(), q102)[0])
    gpu.set_devices([0, 0, 0])                                      # every member packs its own slice
    try:
        assert np.array_equal(gpu.search_array(idx[(2, 64)], q, "task-mid"), want)
        Q = gpu.Queries.from_array(q)
        R = gpu.Results.alloc(q.shape[0])
        gpu.transfer_to_gpu(idx[(2, 64)], Q, R)
        assert gpu.upload_form(Q) == "packed"
        Q.close()
        R.close()
    finally:
        gpu.set_devices([])


def test_default_upload_is_ascii(gpu, oracle_mod, data, monkeypatch):
    """No KFMI_UPLOAD: the reads go up as ASCII (the reference's form) at any
    size; a 70 MB batch gives the same results as the packed upload and the
    oracle on a sample."""
    text, idx = data
    monkeypatch.delenv("KFMI_UPLOAD", raising=False)
    q = _reads(text, 583_333, 100, seed=11)                        # 70 MB with the random fifth
    Q = gpu.Queries.from_array(q)
    R = gpu.Results.alloc(q.shape[0])
    gpu.set_backend("task-mid")
    gpu.transfer_to_gpu(idx[(2, 64)], Q, R)
    assert gpu.upload_form(Q) == "ascii"
    gpu.search(idx[(2, 64)], Q, R)
    gpu.transfer_to_cpu(R)
    got = R.array().copy()
    Q.close()
    R.close()
    monkeypatch.setenv("KFMI_UPLOAD", "packed")
    assert np.array_equal(gpu.search_array(idx[(2, 64)], q, "task-mid"), got)
    s = np.arange(0, q.shape[0], 97)
    want, _ = oracle_mod.search(idx[(2, 64)].image(), q[s])
    assert np.array_equal(got.reshape(-1, 2)[s].ravel(), want)
