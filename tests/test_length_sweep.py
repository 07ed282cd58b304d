"""Read lengths across every code path that cuts a read into pieces: the fused
packers (whole rows staged in LDS, m <= 256), the pack kernel (whole rows up
to ~1 KiB, then word chunks of 1 KiB of bases per row, 16-B copies where a
slice is 16-B aligned), the remainder table (m % K bases), the host-packed
upload (KFMI_UPLOAD=packed) and the streamed search -- for K = 1, 2 on the
plain and AltCounters layouts and K = 3, 4 on the grouped one.

Every result is the read's suffix-array interval, so one oracle serves all:
the CPU restatement of fmIndexCPUBaseline.c:157-292 on the K = 1 index of the
same text (pinned by the golden files, tests/test_oracle.py).  On a random
text the AltCounters searchers (fmIndexCPUBaseline-AltCounters.c:145-310)
return the same intervals; they reject m % K != 0.
Lengths: both sides of every boundary above (16, 64, 256, 1,024, 2,048,
4,096 bases), multiples of 16 whose K = 3 slices are not (1,040, 1,056,
4,128), and seeded random ones up to 5,000."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PLAIN = ("task", "coop", "task-mid", "coop-mid")
ALT = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")
GRP = ("task-grp", "coop-grp")
# K = 1: the cooperative AltCounters kernels need 4 counters per half entry
# (CoopCfg::OK), so coop-ac takes K = 2 only
BACKENDS = {1: PLAIN + ("task-ac", "task-ac-mid", "coop-ac-mid"), 2: PLAIN + ALT, 3: GRP, 4: GRP}

LENGTHS = sorted({1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 1020,
                  1023, 1024, 1025, 1026, 1040, 1056, 2047, 2048, 2064, 3072, 4095, 4096, 4128}
                 | {int(x) for x in np.random.default_rng(4242).integers(6, 5000, size=8)})


@pytest.fixture(scope="module")
def sweep(kfmi_mod, oracle_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    rng = np.random.default_rng(2026)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=300_007)].copy()
    for _ in range(10):   # a few repeats: wide intervals deep into long reads
        a, b = rng.integers(0, t.size - 6000, size=2)
        t[b:b + 5000] = t[a:a + 5000]
    text = t.tobytes()
    idx = {k: K.Index.build(text, k=k, d=64) for k in (1, 2, 3, 4)}
    img1 = idx[1].image()
    cases = {}
    for m in LENGTHS:
        st = rng.integers(0, t.size - m, size=64)
        q = np.ascontiguousarray(np.concatenate([
            t[st[:, None] + np.arange(m)[None, :]],
            rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(16, m)),
            t[t.size - m:][None, :]]))          # the read that ends the text
        cases[m] = (q, oracle_mod.search(img1, q)[0])
    yield K, idx, cases
    for i in idx.values():
        i.close()


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_lengths_every_backend(sweep, k, fused, knobs):
    knobs.fused(fused)
    K, idx, cases = sweep
    for b in BACKENDS[k]:
        for m, (q, want) in cases.items():
            if b in ALT and m % k:
                continue
            got = K.search_array(idx[k], q, b)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (b, k, m, fused, int(bad[0]))


@pytest.mark.parametrize("k", [1, 2, 4])
def test_lengths_host_packed_upload(sweep, k, monkeypatch):
    monkeypatch.setenv("KFMI_UPLOAD", "packed")
    K, idx, cases = sweep
    for b in ("task-mid", "coop-mid") if k < 4 else GRP:
        for m, (q, want) in cases.items():
            got = K.search_array(idx[k], q, b)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (b, k, m, int(bad[0]))


@pytest.mark.parametrize("hostpack", ["0", "1"])
@pytest.mark.parametrize("k,backend", [(1, "task-mid"), (2, "task-mid"), (2, "coop"), (3, "coop-grp"),
                                       (4, "task-grp")])
def test_lengths_streamed(sweep, k, backend, hostpack, monkeypatch):
    monkeypatch.setenv("KFMI_STREAM_HOSTPACK", hostpack)
    K, idx, cases = sweep
    K.set_backend(backend)
    K.transfer_to_gpu(idx[k], None, None)
    for m, (q, want) in cases.items():
        got = K.search_stream(idx[k], q, chunk=32)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (backend, k, m, hostpack, int(bad[0]))
