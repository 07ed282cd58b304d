"""AltCounters files back to plain counters (kfmi_transform_plain), and the
AltCounters-semantics MID128 backends on AltCounters files.

The reference's -AC searchers take only the tfmiAC output (tag 200 / 201,
transformIndexAlternateCounters.c:387-479: half the counters per entry and a
sentinel entry).  kfmi_transform_plain recovers the tag-100 file from it byte
for byte -- pinned on the golden files the reference tools wrote
(tests/golden: every case's .ac / .interleaving.ac against its .fmi), on
seeded random indexes (K 1-4, d 32-192, on and off the B5 boundary) and on
the 'ref'-mode indexes whose last block holds a '$' row two D_s share.  On
the GPU, task-ac-mid / coop-ac-mid then take a tag-200/201 file directly and
return what the reference AltCounters searcher (the oracle's restatement,
fmIndexCPUBaseline-AltCounters.c:145-310) returns on that file; with
KFMI_STRICT_TAG=1 (the reference's tag rule) tag 201 is the file they ask for."""
import os
import subprocess

import numpy as np
import pytest

import util
from util import GOLDEN, manifest

ACGT = np.frombuffer(b"ACGT", np.uint8)


def _golden():
    for case, c in sorted(manifest().items()):
        for key, ent in sorted(c["indexes"].items()):
            if "200" in ent["files"]:
                yield case, key


@pytest.mark.parametrize("case,key", list(_golden()))
def test_plain_from_golden_ac_files(kfmi_mod, case, key):
    files = manifest()[case]["indexes"][key]["files"]
    want = (GOLDEN / case / files["100"]["file"]).read_bytes()
    for tag in ("200", "201"):
        a = kfmi_mod.Index.load(GOLDEN / case / files[tag]["file"])
        p = a.plain()
        assert bytes(p.image()) == want, (case, key, tag)
        p.close()
        a.close()


def test_plain_round_trip_random(kfmi_mod):
    K = kfmi_mod
    rng = np.random.default_rng(31)
    for _ in range(120):
        k = int(rng.choice([1, 2, 3, 4]))
        d = int(rng.choice([32, 64, 128, 192])) if k <= 2 else 64
        n = int(rng.choice([d - 1, 2 * d - 1, d, int(rng.integers(2 * k + 1, 4000))]))
        n = max(n, 2 * k + 1)
        if rng.random() < 0.5:
            t = ACGT[rng.integers(0, 4, size=n)]
        else:
            t = np.repeat(ACGT[rng.integers(0, 4, size=n)], rng.integers(1, 30, size=n))[:n]
        idx = K.Index.build(t.tobytes(), k=k, d=d)
        for a in idx.alt_counters():
            p = a.plain()
            assert bytes(p.image()) == bytes(idx.image()), (k, d, n, a.header()["tag"])
            p.close()
            a.close()
        idx.close()


def test_plain_round_trip_shared_dollar_rows(kfmi_mod):
    from test_alphabet import dup_dollar_last_block_indexes
    K = kfmi_mod
    K.set_alphabet("ref")
    try:
        for t, k, idx in dup_dollar_last_block_indexes(K):
            for a in idx.alt_counters():
                p = a.plain()
                assert bytes(p.image()) == bytes(idx.image()), (k, idx.header()["dollar_pos"])
                p.close()
            idx.close()
    finally:
        K.set_alphabet(None)


def test_plain_refuses_other_tags(kfmi_mod):
    idx = kfmi_mod.Index.build(b"ACGTTGCAACGTAGGT" * 8, k=2, d=64)
    with pytest.raises(kfmi_mod.KfmiError) as e:
        idx.plain()
    assert e.value.code == 200
    idx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["task-ac-mid", "coop-ac-mid"])
@pytest.mark.parametrize("k,d", [(2, 64), (1, 64), (2, 192), (1, 32), (2, 128)])
def test_ac_mid_backends_take_ac_files(kfmi_mod, oracle_mod, backend, k, d):
    K = kfmi_mod
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    if backend.startswith("coop") and (2 * (d // 32) * k) % 4:
        pytest.skip("the cooperative kernel stages 16-byte chunks of planes (K = 1, d = 32 has 8 bytes)")
    K.set_device(0)
    rng = np.random.default_rng(k * 1000 + d)
    n = 200_003
    t = ACGT[rng.integers(0, 4, size=n)].copy()
    t[-40:] = ord("T")            # '$' rows of every BWT_s in the last block: the AC tail matters
    text = t.tobytes()
    idx = K.Index.build(text, k=k, d=d)
    st = rng.integers(0, n - 100, size=20_000)
    q = np.concatenate([t[st[:, None] + np.arange(100)[None, :]], np.full((8, 100), ord("T"), np.uint8),
                        rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(2000, 100))])
    for a in idx.alt_counters():
        want, _ = oracle_mod.search(a.image(), q)
        assert np.array_equal(K.search_array(a, q, backend), want), (backend, k, d, a.header()["tag"])
        a.close()
    idx.close()


@pytest.mark.gpu
def test_reference_driver_strict_tag_ac_mid(tmp_path):
    """The reference's driver (oracle/_ref/searchQueries_dropin) with
    KFMI_STRICT_TAG=1 and task-ac-mid: loadIndex asks for tag 201 (the
    reference's rule for an AltCounters searcher), and the engine searches it."""
    dropin = util.REPO / "oracle" / "_ref" / "searchQueries_dropin"
    if not dropin.exists():
        pytest.fail("oracle/_ref/searchQueries_dropin missing on the GPU box")
    c = manifest()["textA"]
    ent = c["indexes"]["k2_d64"]
    qd = c["queries"]["100"]
    for tag, ok in (("201", True), ("101", False)):
        idx = tmp_path / f"i{tag}.fmi"
        idx.write_bytes((GOLDEN / "textA" / ent["files"][tag]["file"]).read_bytes())
        p = subprocess.run([str(dropin), str(idx), str(GOLDEN / "textA" / qd["file"]), "100", str(qd["num"])],
                           capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, KFMI_BACKEND="task-ac-mid", KFMI_STRICT_TAG="1"))
        assert (p.returncode == 0) == ok, p.stdout + p.stderr
        if ok:
            want = (GOLDEN / "textA" / ent["results"]["100.200"]["file"]).read_bytes()
            assert (tmp_path / f"i{tag}.fmi.res.gpu").read_bytes() == want
