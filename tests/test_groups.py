"""Device groups (kfmi_set_devices / KFMI_DEVICES): runtime multi-GPU behind
the reference's handles (SURVEY 8(b) device selection, 8(e) query slicing).
The index is replicated per member, queries and results are cut into
contiguous 64-read slices; results and locate output must equal the
single-device ones bit for bit.  On a one-GPU box the group lists device 0
several times (independent replicas and streams on one card), which runs
every line of the group path."""
import os
import subprocess
import sys

import numpy as np
import pytest

import util


def test_device_list_from_env_and_validation(kfmi_mod):
    code = ("import sys; sys.path[:0] = {paths!r}; import kstep_fmi as K; "
            "print(K.get_devices())").format(paths=[str(util.REPO), str(util.PKG)])
    env = dict(os.environ, KFMI_DEVICES="0, 1,2")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.stdout.strip() == "[0, 1, 2]", out.stderr
    K = kfmi_mod
    K.set_devices([])
    assert K.get_devices() == []
    with pytest.raises(K.KfmiError):
        K.set_devices([K.device_count() + 3])
    with pytest.raises(K.KfmiError):
        K.set_devices(list(range(17)))


@pytest.fixture(scope="module")
def setup(kfmi_mod):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_devices([])
    K.set_device(0)
    rng = np.random.default_rng(41)
    text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=200_001).tobytes()
    idx = K.Index.build(text, k=2, d=64, gpu=True, sa_rate=4)
    t = np.frombuffer(text, np.uint8)
    reads = np.concatenate([t[rng.integers(0, len(text) - 100, size=3_000)[:, None] + np.arange(100)],
                            rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(333, 100))])
    return K, idx, reads


def run_trio(K, idx, reads):
    q = K.Queries.from_array(reads)
    r = K.Results.alloc(reads.shape[0])
    K.transfer_to_gpu(idx, q, r)
    K.search(idx, q, r)
    K.transfer_to_cpu(r)
    return q, r, r.array().copy()


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["task-mid", "coop-mid", "task", "coop-ac", "task-ac-mid"])
@pytest.mark.parametrize("group", [[0, 0], [0, 0, 0]])
@pytest.mark.parametrize("num", [3_333, 130, 64, 1, 0])
def test_group_equals_single_device(setup, backend, group, num):
    K, idx, reads = setup
    sub = np.ascontiguousarray(reads[:num])
    K.set_backend(backend)
    K.set_devices([])
    q, r, want = run_trio(K, idx, sub)
    q.close(); r.close()
    try:
        K.set_devices(group)
        q, r, got = run_trio(K, idx, sub)
        assert np.array_equal(got, want)
        assert K.last_timing()["total_ms"] >= 0
        q.close(); r.close()
    finally:
        K.set_devices([])
        idx.free_gpu()


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["task-mid", "coop-mid", "task-ac"])
@pytest.mark.parametrize("group", [[0, 0], [0, 0, 0]])
def test_group_streamed_search_equals_single_device(setup, backend, group):
    """kfmi_search_stream on a device group: one slice per member, each
    streamed on its own replica from its own host thread."""
    K, idx, reads = setup
    K.set_backend(backend)
    K.set_devices([])
    _, _, want = run_trio(K, idx, reads)
    try:
        K.set_devices(group)
        K.transfer_to_gpu(idx, None, None)
        for num in (reads.shape[0], 130, 64, 1, 0):
            sub = np.ascontiguousarray(reads[:num])
            got = K.search_stream(idx, sub, chunk=257)
            assert np.array_equal(got, want[:2 * num]), (backend, group, num)
        K.set_ftab(8)                     # the caller's per-thread setting reaches the members
        try:
            assert np.array_equal(K.search_stream(idx, reads), want)
        finally:
            K.set_ftab(0)
    finally:
        K.set_devices([])
        idx.free_gpu()


@pytest.mark.gpu
def test_group_locate_and_mode_switch(setup):
    K, idx, reads = setup
    K.set_backend("task-mid")
    K.set_devices([])
    q, r, want = run_trio(K, idx, reads)
    loc1 = K.locate(idx, r)
    single_bytes = idx.device_bytes()
    blocks1 = K.count_blocks(idx, q)
    q.close(); r.close()
    try:
        K.set_devices([0, 0, 0])
        q, r, got = run_trio(K, idx, reads)
        assert np.array_equal(got, want)
        assert K.count_blocks(idx, q) == blocks1 > 0          # sum over the members' slices
        loc3 = K.locate(idx, r)
        assert np.array_equal(loc3.offsets(), loc1.offsets())
        assert np.array_equal(loc3.positions(), loc1.positions())
        assert idx.device_bytes() == 3 * single_bytes > 0   # three replicas
        # the same handles back in single-device mode
        K.set_devices([])
        K.transfer_to_gpu(idx, q, r)
        K.search(idx, q, r)
        K.transfer_to_cpu(r)
        assert np.array_equal(r.array(), want)
        q.close(); r.close()
    finally:
        K.set_devices([])
        idx.free_gpu()


@pytest.mark.gpu
def test_group_search_driver(tmp_path):
    """The reference's searchQueries flow, unmodified, over a group of three."""
    import shutil
    c = util.manifest()["textA"]
    ent = c["indexes"]["k2_d64"]
    shutil.copy(util.GOLDEN / "textA" / ent["files"]["101"]["file"], tmp_path / "idx.fmi")
    qd = c["queries"]["100"]
    shutil.copy(util.GOLDEN / "textA" / qd["file"], tmp_path / "q.qry")
    env = dict(os.environ, KFMI_BACKEND="task-mid", KFMI_DEVICES="0,0,0", KFMI_ITERS="2")
    p = subprocess.run([str(util.PKG / "bin" / "searchQueries"), "idx.fmi", "q.qry", "100", str(qd["num"])],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    want = (util.GOLDEN / "textA" / ent["results"]["100.100"]["file"]).read_bytes()
    assert (tmp_path / "idx.fmi.res.gpu").read_bytes() == want


@pytest.mark.gpu
def test_group_replication_breakdown(kfmi_mod):
    """A group's index replicas are built once (host upload + relayout on the
    first member) and fanned out device-to-device.  No wall-clock pass/fail
    here (bench.py reports the setup times, variants.group_replication): the
    test checks the replicas and that kfmi_last_timing splits the setup into
    its parts -- members' streams/events, the fan-out copies, the rest being
    the first member's upload -- as disjoint parts of the total."""
    K = kfmi_mod
    rng = np.random.default_rng(7)
    text = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=20_000_000, dtype=np.uint8)].tobytes()
    idx = K.Index.build(text, k=2, d=64, gpu=True)
    K.set_backend("task-mid")
    try:
        K.set_devices([])
        K.transfer_to_gpu(idx, None, None)
        single = idx.device_bytes()
        for group in ([0, 0], [0, 0, 0]):
            K.set_devices(group)
            idx.free_gpu()
            K.transfer_to_gpu(idx, None, None)
            t = K.last_timing()
            print(f"group {group}: setup {t['total_ms']:.2f} ms = members' streams/events {t['pack_ms']:.2f} + "
                  f"fan-out {t['lf_ms']:.2f} + first member's upload")
            assert idx.device_bytes() == len(group) * single > 0
            assert t["pack_ms"] >= 0 and t["lf_ms"] >= 0
            assert t["total_ms"] >= t["pack_ms"] + t["lf_ms"]
    finally:
        K.set_devices([])
        idx.free_gpu()
        idx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("group", [[0, 0], [0, 0, 0]])
def test_group_takes_device_parsed_queries(setup, tmp_path, group):
    """Reads parsed on the device (kfmi_load_queries_gpu) have no host copy: a
    device group gives every member its slice device to device from the
    parsing device, which keeps its copy -- the same handle then still works
    in single-device mode, and in group mode again."""
    K, idx, reads = setup
    path = tmp_path / "q.fa"
    n = 2_999                                     # not a multiple of 64: a short last slice
    path.write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in reads[:n]))
    K.set_backend("task-mid")
    want = K.search_array(idx, reads[:n])
    q = K.Queries.load_gpu(path, 100)
    r = K.Results.alloc(n)
    try:
        for devs in (group, [], group):
            K.set_devices(devs)
            K.transfer_to_gpu(idx, q, r)
            K.search(idx, q, r)
            K.transfer_to_cpu(r)
            assert np.array_equal(r.array(), want), devs
    finally:
        K.set_devices([])
        idx.free_gpu()
        q.close()
        r.close()


@pytest.mark.gpu
def test_two_physical_devices(setup, tmp_path):
    """A group over two different GPUs: peer access, hipMemcpyPeerAsync replica
    fan-out, device-to-device read slices, streamed search and block counts
    across devices -- and the caller's current device left as it was (every
    entry point restores it).  Needs two GPUs (the driver's one-GPU boxes skip
    it; the same-device branches are covered by the tests above)."""
    K, idx, reads = setup
    if K.device_count() < 2:
        pytest.skip("one GPU visible: the cross-device branch needs two")
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")

    def current():
        d = ctypes.c_int(-1)
        assert hip.hipGetDevice(ctypes.byref(d)) == 0
        return d.value

    assert hip.hipSetDevice(1) == 0
    K.set_backend("task-mid")
    K.set_devices([])
    want = K.search_array(idx, reads)
    assert current() == 1
    path = tmp_path / "q.fa"
    path.write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in reads))
    try:
        K.set_devices([0, 1])
        q, r, got = run_trio(K, idx, reads)
        assert np.array_equal(got, want)
        assert current() == 1
        assert K.count_blocks(idx, q) > 0
        assert np.array_equal(K.search_stream(idx, reads), want)
        q.close(); r.close()
        qd = K.Queries.load_gpu(path, 100)            # parsed on device 0, sliced to device 1 over xGMI
        rd = K.Results.alloc(reads.shape[0])
        K.transfer_to_gpu(idx, qd, rd)
        K.search(idx, qd, rd)
        K.transfer_to_cpu(rd)
        assert np.array_equal(rd.array(), want)
        qd.close(); rd.close()
        assert current() == 1
    finally:
        K.set_devices([])
        idx.free_gpu()
        hip.hipSetDevice(0)
