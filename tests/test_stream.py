"""Streamed search from host memory (kfmi_search_stream): chunked
H2D / pack + LF / D2H overlap on a few HIP streams (KFMI_STREAM_SLOTS), with the reads packed on the
host (default) or on the device, must return exactly what the
resident-batch path (kfmi_search) and the CPU oracle return, for ragged chunk
sizes and for pinned and pageable host buffers."""
import numpy as np
import pytest

import util

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup(kfmi_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    rng = np.random.default_rng(77)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=300_001).tobytes()
    idx = K.Index.build(text, k=2, d=64, gpu=True)
    t = np.frombuffer(text, np.uint8)
    starts = rng.integers(0, len(text) - 100, size=7_000)
    reads = np.concatenate([t[starts[:, None] + np.arange(100)],
                            rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(3_007, 100))])
    return K, idx, reads


@pytest.mark.parametrize("hostpack", ["1", "0", "2", "3"])
@pytest.mark.parametrize("backend", ["task-mid", "coop-mid", "task", "coop-ac"])
@pytest.mark.parametrize("chunk", [0, 1_000, 4_099])
def test_stream_equals_batch_and_oracle(setup, oracle_mod, backend, chunk, hostpack, monkeypatch):
    """hostpack 1: code words packed on the host (qpack.c) and sent over PCIe;
    0: ASCII sent and packed on the device; 2 (default): chosen per chunk by
    the cost model; 3: alternating chunks (both kinds in one batch)."""
    K, idx, reads = setup
    monkeypatch.setenv("KFMI_STREAM_HOSTPACK", hostpack)
    want = K.search_array(idx, reads, backend)
    got = K.search_stream(idx, reads, chunk=chunk)
    assert np.array_equal(got, want)
    frac = K.load().kfmi_stream_hostpacked_fraction()
    if hostpack in ("0", "1"):
        assert frac == float(hostpack)
    elif hostpack == "3" and chunk:
        assert 0.0 < frac < 1.0
    if chunk == 1_000 and backend == "task-mid":
        ores, _ = oracle_mod.search(idx.image(), reads, 8)
        assert np.array_equal(got, ores)


@pytest.mark.parametrize("slots", ["2", "3", "8"])
@pytest.mark.parametrize("hostpack", ["3", "2"])
def test_stream_slot_counts(setup, hostpack, slots, monkeypatch):
    """Any number of chunks in flight (2..8 slots; default 6), also after a
    call with more slots left the extra ones idle."""
    K, idx, reads = setup
    monkeypatch.setenv("KFMI_STREAM_HOSTPACK", hostpack)
    want = K.search_array(idx, reads, "task-mid")
    monkeypatch.setenv("KFMI_STREAM_SLOTS", slots)
    for chunk in (997, 0):
        assert np.array_equal(K.search_stream(idx, reads, chunk=chunk), want), (slots, chunk)


@pytest.mark.parametrize("hostpack", ["1", "0", "2", "3"])
def test_stream_pinned_buffers(setup, hostpack, monkeypatch):
    K, idx, reads = setup
    monkeypatch.setenv("KFMI_STREAM_HOSTPACK", hostpack)
    K.set_backend("task-mid")
    K.transfer_to_gpu(idx, None, None)
    want = K.search_array(idx, reads)
    pin_in = K.pinned_empty(reads.shape, np.uint8)
    pin_in[:] = reads
    pin_out = K.pinned_empty((2 * reads.shape[0],), np.uint32)
    got = K.search_stream(idx, pin_in, out=pin_out, chunk=777)
    assert np.array_equal(got, want)
    # mixed: pinned in, pageable out
    assert np.array_equal(K.search_stream(idx, pin_in, chunk=2_048), want)
    assert K.last_timing()["total_ms"] > 0


@pytest.mark.parametrize("hostpack", ["1", "0", "2", "3"])
def test_stream_k1_and_150bp(kfmi_mod, oracle_mod, hostpack, monkeypatch):
    K = kfmi_mod
    monkeypatch.setenv("KFMI_STREAM_HOSTPACK", hostpack)
    K.set_device(0)
    rng = np.random.default_rng(5)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=50_000).tobytes()
    idx = K.Index.build(text, k=1, d=64, gpu=True)
    t = np.frombuffer(text, np.uint8)
    reads = t[rng.integers(0, len(text) - 150, size=2_000)[:, None] + np.arange(150)]
    K.set_backend("task-mid")
    K.transfer_to_gpu(idx, None, None)
    got = K.search_stream(idx, reads, chunk=300)
    ores, _ = oracle_mod.search(idx.image(), reads, 8)
    assert np.array_equal(got, ores)


def test_stream_errors(setup):
    K, idx, reads = setup
    K.set_backend("task-mid")
    K.transfer_to_gpu(idx, None, None)
    assert K.search_stream(idx, reads[:0]).size == 0
    odd = np.ascontiguousarray(reads[:10, :99])          # 99 % K != 0 (B6): the remainder table
    assert np.array_equal(K.search_stream(idx, odd), K.search_array(idx, odd, "task-mid"))
    K.set_backend("coop-ac")                             # AltCounters semantics: no result defined there
    K.transfer_to_gpu(idx, None, None)
    with pytest.raises(K.KfmiError) as e:
        K.search_stream(idx, odd)
    assert e.value.code == 33
    K.set_backend("task-mid")
    fresh = K.Index.build(b"ACGTACGTTGCA" * 50, k=2, d=64, gpu=False)
    with pytest.raises(K.KfmiError) as e:
        K.search_stream(fresh, reads[:10])
    assert e.value.code == 34
    K.load().kfmi_stream_release()


@pytest.mark.parametrize("hostpack", ["1", "0", "2", "3"])
@pytest.mark.parametrize("m", [2, 4, 16, 32, 34, 254, 256, 300, 1000, 1030, 3000, 6000])
def test_stream_read_lengths(kfmi_mod, hostpack, m, monkeypatch):
    """Every word-count class of the host packer (ceil(m/16) words, partial
    last word) and of the fused/unfused device paths, up to reads the pack
    kernel takes in several word chunks."""
    K = kfmi_mod
    monkeypatch.setenv("KFMI_STREAM_HOSTPACK", hostpack)
    K.set_device(0)
    rng = np.random.default_rng(m)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=20_000).tobytes()
    idx = K.Index.build(text, k=2, d=64, gpu=True)
    t = np.frombuffer(text, np.uint8)
    reads = np.concatenate([t[rng.integers(0, len(text) - m, size=700)[:, None] + np.arange(m)],
                            rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(77, m))])
    want = K.search_array(idx, reads, "task-mid")
    got = K.search_stream(idx, reads, chunk=256)
    assert np.array_equal(got, want)
    K.load().kfmi_stream_release()


def test_stream_does_not_block_other_calls(setup):
    """A long streamed search on device 0 holds only that device's stream pool:
    resident-batch searches from another thread on the same device complete
    while it runs (round-1 ADVICE: the pool lock used to be process-wide)."""
    import threading
    import time
    K, idx, reads = setup
    K.set_backend("task-mid")
    K.transfer_to_gpu(idx, None, None)
    big = np.ascontiguousarray(np.tile(reads, (300, 1)))          # 3M reads in 4096-read chunks
    want_big = np.tile(K.search_array(idx, reads), 300)
    K.transfer_to_gpu(idx, None, None)
    stream_out, done = {}, {}

    def streamer():
        K.set_device(0)
        K.set_backend("task-mid")
        stream_out["res"] = K.search_stream(idx, big, chunk=4096)
        done["stream"] = time.perf_counter()

    th = threading.Thread(target=streamer)
    th.start()
    time.sleep(0.01)
    small = K.search_array(idx, reads[:1000])
    done["search"] = time.perf_counter()
    th.join()
    assert np.array_equal(stream_out["res"], want_big)
    assert np.array_equal(small, want_big[:2000])
    assert done["search"] < done["stream"], "search waited for the whole streamed call"


def test_threads_with_different_ftab(setup, oracle_mod):
    """kfmi_set_ftab is per thread; tables are built once per (index, bases) and
    never freed while the index is on the device, so concurrent searches with
    different table sizes on one index stay exact (round-1 ADVICE)."""
    import threading
    K, idx, reads = setup
    want, _ = oracle_mod.search(idx.image(), reads, 8)
    K.set_backend("task-mid")
    K.transfer_to_gpu(idx, None, None)
    errs = []

    def worker(bases):
        try:
            K.set_device(0)
            K.set_backend("task-mid")
            K.set_ftab(bases)
            for _ in range(5):
                q = K.Queries.from_array(reads)
                r = K.Results.alloc(reads.shape[0])
                K.transfer_to_gpu(idx, q, r)
                K.search(idx, q, r)
                K.transfer_to_cpu(r)
                if not np.array_equal(r.array(), want):
                    errs.append(bases)
                q.close()
                r.close()
        except Exception as e:      # noqa: BLE001 -- reported below
            errs.append(repr(e))

    ths = [threading.Thread(target=worker, args=(b,)) for b in (0, 8, 10, 12)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs


@pytest.fixture(scope="module")
def rem_setup(kfmi_mod):
    """One text, its K = 1 image (the oracle's intervals are K-independent) and
    K = 2 / K = 4 indexes; reads of m % K != 0 with N and lowercase mixed in."""
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    rng = np.random.default_rng(151)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=200_003).tobytes()
    i1 = K.Index.build(text, k=1, d=64, gpu=False)
    idx = {2: K.Index.build(text, k=2, d=64, gpu=True), 4: K.Index.build(text, k=4, d=64, gpu=True, host_image=False)}
    return K, text, i1.image(), idx


@pytest.mark.parametrize("group", [[], [0, 0]])
@pytest.mark.parametrize("hostpack", ["1", "0", "2", "3"])
@pytest.mark.parametrize("k,backend", [(2, "task-mid"), (2, "task"), (2, "coop"), (4, "coop-grp")])
@pytest.mark.parametrize("m", [101, 150, 151])
def test_stream_remainder_reads(rem_setup, oracle_mod, k, backend, m, hostpack, group, monkeypatch):
    """m % K != 0 streamed: the last m % K bases of every read come
    from the remainder table -- host packing writes their codes as one more
    word row, ASCII chunks are packed in the kernel -- on one device and on a
    device group; results equal the K = 1 oracle (true suffix-array
    intervals) and the resident-batch search.  task and coop on the reference
    tag-101 layout take the line-local (NEIGHBOR) fetch paths at K = 2 d = 64
    (ADVICE r3)."""
    K, text, img1, idx = rem_setup
    monkeypatch.setenv("KFMI_STREAM_HOSTPACK", hostpack)
    rng = np.random.default_rng(m * 7 + k)
    t = np.frombuffer(text, np.uint8)
    reads = np.concatenate([t[rng.integers(0, len(text) - m, size=3_000)[:, None] + np.arange(m)],
                            rng.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(131, m))])
    # reads ending inside the text's first / last bases, and ones sharing the text's last bases
    reads[0] = t[len(text) - m:]
    reads[1, :] = t[:m]
    want, _ = oracle_mod.search(img1, reads, 8)
    try:
        K.set_devices(group)
        K.set_backend(backend)
        K.transfer_to_gpu(idx[k], None, None)
        got = K.search_stream(idx[k], reads, chunk=1_000)
        assert np.array_equal(got, want)
        assert np.array_equal(K.search_stream(idx[k], reads), want)
        if not group:
            assert np.array_equal(K.search_array(idx[k], reads, backend), want)
    finally:
        K.set_devices([])
        idx[k].free_gpu()
