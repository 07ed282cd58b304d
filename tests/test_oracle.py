"""The oracle (oracle/fmi_oracle.c) pinned against the reference's own outputs.

Every expected result here was written by the reference CPU searchers
(fmIndexCPUBaseline.c / -AltCounters.c, compiled by oracle/Makefile) and is
committed under tests/golden/ (see tests/golden/make_golden.py).
"""
import hashlib

import numpy as np
import pytest

import util
from util import GOLDEN, golden_cases, manifest, read_qry

CASES = list(golden_cases())


@pytest.mark.parametrize("case,key,k,d,tag,m,idx,qry,res", CASES,
                         ids=[f"{c[0]}-{c[1]}-t{c[4]}-m{c[5]}" for c in CASES])
def test_oracle_matches_reference_results(oracle_mod, case, key, k, d, tag, m, idx, qry, res):
    img = np.fromfile(idx, dtype=np.uint8)
    q = read_qry(qry, m)
    got, blocks = oracle_mod.search(img, q, nthreads=4)
    want = oracle_mod.read_results_file(res)
    assert np.array_equal(got, want)
    assert q.shape[0] * (m // k) <= blocks <= 2 * q.shape[0] * (m // k)


def test_fixture_md5s():
    for case, c in manifest().items():
        for ent in c["indexes"].values():
            for f in ent["files"].values():
                assert hashlib.md5((GOLDEN / case / f["file"]).read_bytes()).hexdigest() == f["md5"]
            for r in ent["results"].values():
                assert hashlib.md5((GOLDEN / case / r["file"]).read_bytes()).hexdigest() == r["md5"]


@pytest.mark.parametrize("case", sorted(manifest()))
def test_plain_results_are_suffix_ranks(oracle_mod, case):
    """Independent check: plain-counter results equal brute-force suffix ranks
    of T$ (the AC layout differs only by the sentinel quirk, textB)."""
    c = manifest()[case]
    text = util.read_fasta_text(GOLDEN / case / "ref.fa")
    bf = util.BruteForce(text)
    for m, qd in c["queries"].items():
        q = read_qry(GOLDEN / case / qd["file"], int(m))
        ent = c["indexes"]["k1_d64"]
        res = oracle_mod.read_results_file(GOLDEN / case / ent["results"][f"{m}.100"]["file"])
        for i in range(q.shape[0]):
            assert (int(res[2 * i]), int(res[2 * i + 1])) == bf.interval(q[i].tobytes()), (case, m, i)


def test_ac_quirk_is_real():
    """textB puts the '$' rows in the last block: the reference AC searcher
    differs from the plain one there, and the oracle reproduces both."""
    c = manifest()["textB"]["indexes"]["k2_d64"]["results"]
    a = (GOLDEN / "textB" / c["12.100"]["file"]).read_bytes()
    b = (GOLDEN / "textB" / c["12.200"]["file"]).read_bytes()
    assert a != b


def test_oracle_rejects_bad_input(oracle_mod):
    img = np.fromfile(GOLDEN / "textA" / "k2_d64.100.fmi", dtype=np.uint8)
    with pytest.raises(ValueError):
        oracle_mod.search(img, np.zeros((3, 5), dtype=np.uint8))   # m % K != 0
    with pytest.raises(ValueError):
        oracle_mod.search(img[:30], np.zeros((3, 4), dtype=np.uint8))


def test_oracle_refuses_reads_past_the_index(kfmi_mod, oracle_mod):
    """(n+1) % d == 0: the first step's R lies in block nentries, which the
    reference reads past its file.  The restatement refuses
    instead of reading past its image; the same reads one entry further
    (padding with the end counters, tests/test_alphabet.py padded_image) and
    every text length off the boundary are answered."""
    rng = np.random.default_rng(5)
    for n, d in ((63, 64), (959, 32), (1023, 64), (191, 192)):
        text = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n).tobytes()
        for k in (1, 2):
            idx = kfmi_mod.Index.build(text, k=k, d=d)
            q = np.frombuffer(text[:4 * k], np.uint8).reshape(1, -1).copy()
            with pytest.raises(ValueError, match="past the index"):
                oracle_mod.search(idx.image(), q)
            idx.close()
        text1 = text + b"A"
        idx = kfmi_mod.Index.build(text1, k=2, d=d)
        want = util.BruteForce(text1.decode()).interval(text1[:8])
        assert tuple(oracle_mod.search(idx.image(), np.frombuffer(text1[:8], np.uint8).reshape(1, -1))[0]) == want
        idx.close()
