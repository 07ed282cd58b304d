"""Builders on real-FASTA alphabets (KFMI_ALPHABET / kfmi_set_alphabet).

The reference builder takes any byte: readRef copies lines verbatim
(common/common.c:42-76, header lines and 255-byte fgets pieces included),
divbwt64 sorts raw bytes (genFMindex.c:482) and counters / bit planes go
through base2index (N -> G, lowercase -> uppercase, :71-84).  For K >= 2 its LF
walk (generateOthersBWTs :327-400) only counts 'A'/'C'/'G'/'T', so on such a
text it leaves rows of BWT_1.. unwritten -- uninitialised malloc memory.
tests/golden/alpha holds the reference tools' own output on an hg38-style
multi-FASTA (N runs, soft-masked and IUPAC letters, a second record's header,
a 300-byte line), built under MALLOC_PERTURB_ for K >= 2 (make_golden_alpha.py);
the "ref" mode must reproduce every file byte for byte (fill byte = perturb ^
0xff) and every searcher result, from both builders.
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import util
from test_gpu_parity import coop_supported

ALPHA = util.GOLDEN / "alpha"


def man():
    return json.loads((ALPHA / "alpha.json").read_text())


class _Ref(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint64), ("p", ctypes.c_void_p)]


def load_ref_text(K, n):
    L = K.load()
    ref = ctypes.c_void_p()
    assert L.loadRef(str(ALPHA / "ref.fa").encode(), n, ctypes.byref(ref)) == 0
    r = _Ref.from_address(ref.value)
    text = ctypes.string_at(r.p, r.size)
    L.freeReference(ctypes.byref(ref), None)
    return text


@pytest.fixture
def ref_mode(kfmi_mod, monkeypatch):
    monkeypatch.delenv("KFMI_REF_FILL", raising=False)
    kfmi_mod.set_alphabet("ref")
    yield kfmi_mod
    kfmi_mod.set_alphabet(None)


def builds():
    return sorted(man()["indexes"].items())


def test_loadref_ref_mode_is_readref(ref_mode):
    K = ref_mode
    m = man()
    text = load_ref_text(K, m["n"])
    assert hashlib.md5(text).hexdigest() == m["text_md5"]
    assert b">chr2 second record" in text                 # header lines are part of the text
    assert b"N" * 300 in text and b"n" * 50 in text


@pytest.mark.parametrize("key,ent", builds())
def test_host_builder_ref_mode_equals_reference(ref_mode, monkeypatch, key, ent):
    K = ref_mode
    text = load_ref_text(K, man()["n"])
    if ent["fill"] is not None:
        monkeypatch.setenv("KFMI_REF_FILL", str(ent["fill"]))
    idx = K.Index.build(text, k=ent["k"], d=ent["d"], gpu=False)
    assert hashlib.md5(idx.image().tobytes()).hexdigest() == ent["md5"]["100"]
    if "101" in ent["files"]:
        i101 = idx.interleave()
        i200, i201 = idx.alt_counters()
        for tag, ix in (("101", i101), ("200", i200), ("201", i201)):
            assert hashlib.md5(ix.image().tobytes()).hexdigest() == ent["md5"][tag], tag


def test_reference_output_depends_on_uninitialised_memory():
    """The K = 2 reference index differs between MALLOC_PERTURB_ values: its
    output is not a function of the text (recorded, not assumed)."""
    ix = man()["indexes"]
    assert ix["k2_d64_p85"]["md5"]["100"] != ix["k2_d64_p170"]["md5"]["100"]


@pytest.mark.parametrize("key,ent", builds())
def test_oracle_on_reference_indexes(oracle_mod, key, ent):
    """The CPU restatement reproduces the reference searchers on these indexes
    (counts that are consistent per block, LF that is not a bijection)."""
    for rk, r in sorted(ent["results"].items()):
        m, tag = (int(x) for x in rk.split("."))
        if str(tag) not in ent["files"]:
            continue
        img = np.fromfile(ALPHA / ent["files"][str(tag)]["file"], dtype=np.uint8)
        reads = util.read_qry(ALPHA / man()["queries"][str(m)]["file"], m)
        got, _ = oracle_mod.search(img, reads)
        want = np.array((ALPHA / r["file"]).read_bytes().split()[1:], dtype=np.uint32)
        assert np.array_equal(got, want), (key, rk)


def test_modes_agree_on_acgt_text(kfmi_mod):
    K = kfmi_mod
    rng = np.random.default_rng(3)
    text = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=20_011)].tobytes()
    md5s = set()
    try:
        for mode in ("acgt", "map", "ref"):
            K.set_alphabet(mode)
            for k in (1, 2):
                md5s.add((k, hashlib.md5(K.Index.build(text, k=k, d=64).image().tobytes()).hexdigest()))
    finally:
        K.set_alphabet(None)
    assert len(md5s) == 2


def test_map_mode_is_the_mapped_text(kfmi_mod):
    K = kfmi_mod
    text = (ALPHA / "ref.fa").read_bytes().split(b"\n", 1)[1].replace(b"\n", b"")   # any bytes
    mapped = bytes(b"ACGT"[K.load().base2index(x)] for x in text)
    try:
        K.set_alphabet("map")
        a = K.Index.build(text, k=2, d=64).image()
        K.set_alphabet("acgt")
        b = K.Index.build(mapped, k=2, d=64).image()
        with pytest.raises(K.KfmiError) as e:
            K.Index.build(text, k=2, d=64)
        assert e.value.code == 8                          # KFMI_E_BUILDING_BWT: non-ACGT in "acgt"
    finally:
        K.set_alphabet(None)
    assert np.array_equal(a, b)


def test_set_alphabet_rejects_unknown(kfmi_mod):
    with pytest.raises(kfmi_mod.KfmiError):
        kfmi_mod.set_alphabet("iupac")


# ---------------------------------------------------------------- GPU -------

@pytest.mark.gpu
@pytest.mark.parametrize("key,ent", builds())
def test_gpu_builder_ref_mode_equals_reference(ref_mode, monkeypatch, key, ent):
    K = ref_mode
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    text = load_ref_text(K, man()["n"])
    if ent["fill"] is not None:
        monkeypatch.setenv("KFMI_REF_FILL", str(ent["fill"]))
    idx = K.Index.build(text, k=ent["k"], d=ent["d"], gpu=True)
    assert hashlib.md5(idx.image().tobytes()).hexdigest() == ent["md5"]["100"]
    idx2 = K.Index.build(text, k=ent["k"], d=ent["d"], gpu=True, sa_rate=4)   # with SA samples
    assert np.array_equal(idx2.image(), idx.image())


PLAIN = ("task", "coop", "task-mid", "coop-mid", "task-packed", "coop-packed")
AC = ("task-ac", "coop-ac", "task-ac128", "coop-ac128", "task-ac-mid", "coop-ac-mid")


@pytest.mark.gpu
@pytest.mark.parametrize("key,ent", builds())
def test_gpu_search_on_reference_indexes(ref_mode, monkeypatch, key, ent):
    """Every backend on the reference-built indexes of the alpha text equals
    the reference's CPU searchers (plain: cpu_*, AltCounters: cpuac_*).  The
    index is the committed reference file, or -- where only its md5 is
    committed -- the host builder's md5-equal rebuild."""
    K = ref_mode
    K.set_device(0)
    if "100" in ent["files"]:
        idx = K.Index.load(ALPHA / ent["files"]["100"]["file"])
    else:
        if ent["fill"] is not None:
            monkeypatch.setenv("KFMI_REF_FILL", str(ent["fill"]))
        idx = K.Index.build(load_ref_text(K, man()["n"]), k=ent["k"], d=ent["d"], gpu=False)
        assert hashlib.md5(idx.image().tobytes()).hexdigest() == ent["md5"]["100"]
    for rk, r in sorted(ent["results"].items()):
        m, tag = (int(x) for x in rk.split("."))
        reads = util.read_qry(ALPHA / man()["queries"][str(m)]["file"], m)
        want = np.array((ALPHA / r["file"]).read_bytes().split()[1:], dtype=np.uint32)
        backends = (PLAIN if ent["k"] <= 2 else ("coop-grp", "task-grp")) if tag == 100 else AC
        for be in backends:
            if not coop_supported(be, ent["k"], ent["d"]):
                continue                                   # geometry the cooperative kernel rejects (code 33)
            got = K.search_array(idx, reads, be)
            assert np.array_equal(got, want), (key, rk, be)
    idx.close()
