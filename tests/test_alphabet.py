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

import ref_fill
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


def ref_build(K, text, ent, gpu):
    """The 'ref'-mode build of `text` as the reference tool wrote it: the
    product's image (its defined fill) with the unvisited rows patched to the
    golden's fill byte (tests/ref_fill.py); the product index itself when no
    patch applies."""
    idx = K.Index.build(text, k=ent["k"], d=ent["d"], gpu=gpu)
    if ent["fill"] is None or ent["k"] < 2:
        return idx
    img = ref_fill.patch(idx.image(), text, ref_fill.full_sa(K, text, ent["k"], ent["d"]), ent["fill"])
    idx.close()
    return K.Index.from_image(img)


@pytest.fixture
def ref_mode(kfmi_mod):
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
def test_host_builder_ref_mode_equals_reference(ref_mode, key, ent):
    K = ref_mode
    text = load_ref_text(K, man()["n"])
    idx = ref_build(K, text, ent, gpu=False)
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
def test_gpu_builder_ref_mode_equals_reference(ref_mode, key, ent):
    K = ref_mode
    if K.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    K.set_device(0)
    text = load_ref_text(K, man()["n"])
    idx = ref_build(K, text, ent, gpu=True)
    assert hashlib.md5(idx.image().tobytes()).hexdigest() == ent["md5"]["100"]
    # the GPU builder's own image (its defined fill) equals the host builder's,
    # with SA samples too
    plain = K.Index.build(text, k=ent["k"], d=ent["d"], gpu=True)
    idx2 = K.Index.build(text, k=ent["k"], d=ent["d"], gpu=True, sa_rate=4)
    assert np.array_equal(idx2.image(), plain.image())
    assert np.array_equal(plain.image(), K.Index.build(text, k=ent["k"], d=ent["d"], gpu=False).image())


PLAIN = ("task", "coop", "task-mid", "coop-mid")
AC = ("task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid")


@pytest.mark.gpu
@pytest.mark.parametrize("key,ent", builds())
def test_gpu_search_on_reference_indexes(ref_mode, key, ent):
    """Every backend on the reference-built indexes of the alpha text equals
    the reference's CPU searchers (plain: cpu_*, AltCounters: cpuac_*).  The
    index is the committed reference file, or -- where only its md5 is
    committed -- the host builder's md5-equal rebuild."""
    K = ref_mode
    K.set_device(0)
    if "100" in ent["files"]:
        idx = K.Index.load(ALPHA / ent["files"]["100"]["file"])
    else:
        idx = ref_build(K, load_ref_text(K, man()["n"]), ent, gpu=False)
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
        if tag == 100 and ent["k"] == 2 and ent["d"] == 64:
            # the grouped-counter backends take a K = 2 file through the device
            # derivation (DESIGN.md 5d'), which needs an LF_K that is a
            # permutation: this text's N runs make the reference walk's BWT_1
            # not one, so the derivation refuses (KFMI_E_BUILDING_FMI) instead
            # of searching a wrong K = 4 index
            for be in ("coop-grp", "task-grp"):
                with pytest.raises(K.KfmiError) as e:
                    K.search_array(idx, reads, be)
                assert e.value.code == 9, (key, rk, be, e.value.code)
    idx.close()


def dup_dollar_indexes(K, want=6):
    """'ref'-mode indexes whose dollarPositionBWT repeats a row: a text with
    non-ACGT bytes makes the reference's LF walk revisit rows (genFMindex.c
    :347-400), and two D_s on one row are excluded once by its counters but
    discounted once per s by its searchers (fmIndexCPUBaseline.c:252-256).
    Seeded search over small N-rich texts, K = 2, 3, 4, d = 64; each returned
    index has a duplicate, and together they put one in block 0 and in a
    later block."""
    out, blocks = [], set()
    rng = np.random.default_rng(2024)
    alpha = np.frombuffer(b"ACGTN", np.uint8)
    for _ in range(20000):
        n = int(rng.integers(150, 2500))
        t = alpha[rng.choice(5, size=n, p=rng.dirichlet(np.ones(5)))].tobytes()
        for k in (2, 3, 4):
            try:
                idx = K.Index.build(t, k=k, d=64)
            except K.KfmiError:
                continue
            dp = idx.header()["dollar_pos"]
            dups = {p for p in dp if dp.count(p) > 1}
            if dups and (len(out) < want // 2 or any(p // 64 not in blocks for p in dups)):
                blocks |= {p // 64 for p in dups}
                out.append((t, k, idx))
            else:
                idx.close()
        if len(out) >= want and len(blocks) > 1:
            break
    assert len(out) >= want and len(blocks) > 1, (len(out), blocks)
    return out


def _all_reads(t, k, rng):
    """Every 2K-mer and 4-mer over ACGT, plus substrings of the text (N kept)."""
    import itertools
    rows = [np.frombuffer(bytes(p), np.uint8) for m in (2 * k, 4 * k if k < 3 else k)
            for p in itertools.product(b"ACGT", repeat=m)]
    tt = np.frombuffer(t, np.uint8)
    out = {}
    for r in rows:
        out.setdefault(r.size, []).append(r)
    for m in (k, 2 * k, 3 * k, 6 * k):
        st = rng.integers(0, len(t) - m, size=300)
        out.setdefault(m, []).extend(tt[st[:, None] + np.arange(m)[None, :]])
    return {m: np.stack(v) for m, v in out.items()}


def test_cpu_search_on_duplicate_dollar_rows(ref_mode, oracle_mod):
    """searchIndexCPU equals the reference searchers (the oracle restates
    them) on indexes with a repeated '$' row, every tag."""
    K = ref_mode
    rng = np.random.default_rng(5)
    for t, k, idx in dup_dollar_indexes(K):
        i101 = idx.interleave()
        i200, i201 = idx.alt_counters()
        for m, q in _all_reads(t, k, rng).items():
            for tagged, img in ((idx, idx), (i101, idx), (i200, i200), (i201, i200)):
                want, _ = oracle_mod.search(img.image(), q)
                assert np.array_equal(K.search_cpu_array(tagged, q, 2), want), (k, m, tagged.header()["tag"])
        for x in (idx, i101, i200, i201):
            x.close()


def dup_dollar_last_block_indexes(K):
    """'ref'-mode indexes with (n+1) % 64 == 0 and a '$' row two D_s share in
    the last block: the R end of the first K-step lands one block past the
    end (B5), where every searcher of this build takes the end counters.
    Texts replayed from a recorded seeded search (rng 77: draws 1613 and 3512,
    n = 127 and 575; K = 4 and K = 2, 3, 4)."""
    rng = np.random.default_rng(77)
    alpha = np.frombuffer(b"ACGTN", np.uint8)
    out = []
    for it in range(3513):
        n = 64 * int(rng.integers(2, 40)) - 1
        t = alpha[rng.choice(5, size=n, p=rng.dirichlet(np.ones(5)))].tobytes()
        for k in {1613: (4,), 3512: (2, 3, 4)}.get(it, ()):
            idx = K.Index.build(t, k=k, d=64)
            dp = idx.header()["dollar_pos"]
            assert (n + 1) % 64 == 0 and any(dp.count(p) > 1 and p // 64 == (n + 1) // 64 - 1 for p in dp), (it, k, dp)
            out.append((t, k, idx))
    return out


def _end_counters(idx):
    """What a padding entry past the last block holds (the GPU layouts store
    one, kfmi_search.hip end_counters): per code, the last entry's counter plus
    the code's rows in the last block, less each distinct '$' row of that block
    with that dollarBase once -- the next entry the builder would write (its
    counters exclude a row once however many D_s share it).
    Read from the tag-100 image: 24 + 8K header bytes, then entries of
    2 * NB * K plane words (plane s*2NB + t*NB + w, row p at bit 31 - p of
    word w) and NC counters."""
    h = idx.header()
    k, nb, nc, ne = h["steps"], h["chunk"] // 32, h["ncounters"], h["nentries"]
    ew = 2 * nb * k + nc
    ent = np.frombuffer(bytes(idx.image()[24 + 8 * k:]), np.uint32)[:ne * ew].reshape(ne, ew)
    last = ent[-1]
    rows = np.arange(32 * nb)
    codes = np.zeros(rows.size, np.int64)
    for s in range(k):
        b0 = (last[s * 2 * nb + rows // 32] >> (31 - rows % 32).astype(np.uint32)) & 1
        b1 = (last[s * 2 * nb + nb + rows // 32] >> (31 - rows % 32).astype(np.uint32)) & 1
        codes |= (b0.astype(np.int64) | (b1.astype(np.int64) << 1)) << (2 * s)
    end = last[2 * nb * k:].astype(np.int64) + np.bincount(codes, minlength=nc)
    lastblk = ne - 1
    seen = set()
    for p, c in zip(h["dollar_pos"], h["dollar_base"]):
        if p // (32 * nb) == lastblk and p not in seen:
            end[c] -= 1
        seen.add(p)
    return ent[0, 2 * nb * k:].astype(np.int64), end


def test_cpu_search_end_counters_on_shared_dollar_rows(ref_mode):
    """past the last block (B5) the host search and the GPU layouts
    disagreed when two D_s share a row of the last block (the host discounted
    it per s; INTER's line-local step once; the stored padding entries per s,
    which MID's backward steps then corrected a second time).  Every searcher
    now reads the same padding entry: the end counters with each '$' row
    excluded once.  One K-step of every K-mer from [0, n+1) gives
    [C0[c], end[c]); on the GPU every backend equals the host search
    (test_gpu_end_counters_equal_cpu_search_on_duplicate_dollar_rows)."""
    import itertools
    K = ref_mode
    for t, k, idx in dup_dollar_last_block_indexes(K):
        c0, end = _end_counters(idx)
        q = np.stack([np.frombuffer(bytes(p), np.uint8) for p in itertools.product(b"ACGT", repeat=k)])
        # itertools order = code order: first base in the high digit, last base at bits 0-1
        for tagged in (idx, idx.interleave()):
            iv = K.search_cpu_array(tagged, q, 1).reshape(-1, 2).astype(np.int64)
            assert np.array_equal(iv[:, 0], c0) and np.array_equal(iv[:, 1], end), (k, idx.header()["dollar_pos"])
        idx.close()


def padded_image(idx):
    """The tag-100 image with one more entry: the padding block every GPU
    layout appends (end counters, zero planes = rows of code 0), so that the
    oracle -- the reference's searcher restated -- never reads past its index
    where the reference would (B5)."""
    h = idx.header()
    k, nb = h["steps"], h["chunk"] // 32
    img = np.array(idx.image())
    pad = np.zeros(2 * nb * k + h["ncounters"], np.uint32)
    pad[2 * nb * k:] = _end_counters(idx)[1].astype(np.uint32)
    hdr = img[:24].view(np.uint32).copy()
    hdr[4] += 1
    return np.concatenate([hdr.view(np.uint8), img[24:], pad.view(np.uint8)])


def test_cpu_search_past_the_end_is_the_padding_entry(ref_mode, oracle_mod):
    """On 'ref'-mode indexes with (n+1) % 64 == 0 and shared '$' rows in the
    last block, searchIndexCPU equals the oracle run on the image plus the
    GPU layouts' padding entry: steps can land past n+1 there (the walk is
    not a permutation), where the padding block's rows read as code 0."""
    K = ref_mode
    rng = np.random.default_rng(8)
    for t, k, idx in dup_dollar_last_block_indexes(K):
        img = padded_image(idx)
        for m, q in _all_reads(t, k, rng).items():
            want, _ = oracle_mod.search(img, q)
            for tagged in (idx, idx.interleave()):
                assert np.array_equal(K.search_cpu_array(tagged, q, 1), want), (k, m, tagged.header()["tag"])
        idx.close()


@pytest.mark.gpu
def test_gpu_end_counters_equal_cpu_search_on_duplicate_dollar_rows(ref_mode):
    """The same last-block indexes: every plain GPU backend equals
    searchIndexCPU (the reference reads past its file there, B5, so the
    product's host search is the check), on all K-mers and text substrings."""
    K = ref_mode
    K.set_device(0)
    rng = np.random.default_rng(8)
    for t, k, idx in dup_dollar_last_block_indexes(K):
        for m, q in _all_reads(t, k, rng).items():
            want = K.search_cpu_array(idx, q, 1)
            for be in (PLAIN if k == 2 else ("coop-grp", "task-grp")):
                if not coop_supported(be, k, 64):
                    continue
                assert np.array_equal(K.search_array(idx, q, be), want), (k, m, be, idx.header()["dollar_pos"])
        idx.close()


@pytest.mark.gpu
def test_gpu_search_on_duplicate_dollar_rows(ref_mode, oracle_mod):
    """Every backend on indexes with a repeated '$' row equals the reference
    searchers: the line-local step from block b-1 discounts each '$' row of
    b-1 once (as the builder's counters), and the steps whose direction
    differs from the semantics' own (MID lines backward where the reference
    steps forward; MIDAC, task-ac/coop-ac from b-1, forward where the
    AltCounters searcher steps backward) are corrected by the duplicate count
    (kfmi_device.h dollar_dup)."""
    K = ref_mode
    K.set_device(0)
    rng = np.random.default_rng(6)
    for t, k, idx in dup_dollar_indexes(K):
        img200 = idx.alt_counters()[0].image()
        for m, q in _all_reads(t, k, rng).items():
            want, _ = oracle_mod.search(idx.image(), q)
            want_ac, _ = oracle_mod.search(img200, q)
            backends = (PLAIN + AC) if k == 2 else ("coop-grp", "task-grp")
            for be in backends:
                if not coop_supported(be, k, 64):
                    continue
                got = K.search_array(idx, q, be)
                assert np.array_equal(got, want_ac if be in AC else want), (k, m, be, idx.header()["dollar_pos"])
        idx.close()
