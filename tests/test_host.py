"""Host-side (no GPU) tests of libkstepfmi.so: ABI exports, file formats,
transforms and the host index builder -- each pinned bit-exactly against
files written by the reference's own tools (tests/golden, make_golden.py)."""
import hashlib
import re
import subprocess

import numpy as np
import pytest

import util
from util import GOLDEN, REPO, manifest, read_qry

HEADER = REPO / "include" / "kstep_fmi.h"


def declared_functions():
    src = HEADER.read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", src)
    skip = {"if", "defined", "extern", "enum"}
    return sorted({n for n in names if n not in skip})


def test_library_exports_every_declared_symbol(kfmi_mod):
    lib = kfmi_mod.load()
    names = declared_functions()
    assert len(names) >= 40
    out = subprocess.run(["nm", "-D", "--defined-only", str(kfmi_mod.LIB_PATH)],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        getattr(lib, n)   # resolvable through ctypes
    # the reference's never-defined entry points are not exported;
    # searchIndexCPU (interface.h:30) is, as the host search the reference's CPU
    # driver calls (csrc/host/cpu_search.c, tests/test_cpu_search.py) -- never a
    # fallback of the GPU entry points, which fail without a device
    for n in ("searchIndex", "errorIndex"):
        assert n not in exported
    assert "searchIndexCPU" in exported


def test_error_strings(kfmi_mod):
    lib = kfmi_mod.load()
    assert lib.errorCommon(0) == b"No error"
    assert b"tfmiBMP" in lib.errorCommon(101)
    assert b"interleaving.ac" in lib.errorCommon(201)


def test_base2index(kfmi_mod):
    lib = kfmi_mod.load()
    for ch, code in zip(b"ACGTNacgtn$", [0, 1, 2, 3, 2, 0, 1, 2, 3, 2, 3]):
        assert lib.base2index(ch) == code == util.code_of(ch)


def _golden_index_files():
    for case, c in sorted(manifest().items()):
        for key, ent in sorted(c["indexes"].items()):
            yield case, key, ent


@pytest.mark.parametrize("case,key,ent", list(_golden_index_files()),
                         ids=[f"{a}-{b}" for a, b, _ in _golden_index_files()])
def test_load_and_transforms_bit_exact(kfmi_mod, tmp_path, case, key, ent):
    files = {int(t): GOLDEN / case / f["file"] for t, f in ent["files"].items()}
    idx = kfmi_mod.Index.load(files[100])
    h = idx.header()
    assert (h["tag"], h["steps"], h["chunk"]) == (100, ent["k"], ent["d"])
    assert idx.image().tobytes() == files[100].read_bytes()
    i101 = idx.interleave()
    assert i101.image().tobytes() == files[101].read_bytes()
    i200, i201 = idx.alt_counters()
    assert i200.image().tobytes() == files[200].read_bytes()
    assert i201.image().tobytes() == files[201].read_bytes()
    # file names follow the reference tools
    base = tmp_path / "x.fmi"
    i101.save(base)
    i200.save(base)
    i201.save(base)
    assert (tmp_path / "x.fmi.interleaving").read_bytes() == files[101].read_bytes()
    assert (tmp_path / "x.fmi.ac").read_bytes() == files[200].read_bytes()
    assert (tmp_path / "x.fmi.interleaving.ac").read_bytes() == files[201].read_bytes()
    # strict loader: the reference's tag check and error code
    with pytest.raises(kfmi_mod.KfmiError) as e:
        kfmi_mod.Index.load(files[100], required_tag=101)
    assert e.value.code == 101


@pytest.mark.parametrize("case", sorted(manifest()))
def test_host_builder_matches_reference_builder(kfmi_mod, tmp_path, case):
    c = manifest()[case]
    text = util.read_fasta_text(GOLDEN / case / "ref.fa").encode()
    for key, ent in c["indexes"].items():
        idx = kfmi_mod.Index.build(text, k=ent["k"], d=ent["d"], gpu=False)
        got = hashlib.md5(idx.image().tobytes()).hexdigest()
        assert got == ent["files"]["100"]["md5"], (case, key)
    # naming of genFMindex.c:162
    idx.save(tmp_path / "ref.fa")
    assert (tmp_path / f"ref.fa.{len(text)}.{ent['d']}fmi{ent['k']}steps.fmi").exists()


def test_builder_rejects_non_acgt(kfmi_mod):
    with pytest.raises(kfmi_mod.KfmiError):
        kfmi_mod.Index.build(b"ACGTNACGT", k=2, d=64)


def test_query_loader_and_results_writer(kfmi_mod, tmp_path):
    c = manifest()["textA"]
    qfile = GOLDEN / "textA" / c["queries"]["100"]["file"]
    n = c["queries"]["100"]["num"]
    q = kfmi_mod.Queries.load(qfile, 100, n)
    q.close()
    with pytest.raises(kfmi_mod.KfmiError):
        kfmi_mod.Queries.load(qfile, 99, n)          # wrong read length
    with pytest.raises(kfmi_mod.KfmiError):
        kfmi_mod.Queries.load(qfile, 100, n + 1)     # not enough reads
    # results file format of common.c:201-220, byte for byte
    ref = GOLDEN / "textA" / c["indexes"]["k2_d64"]["results"]["100.100"]["file"]
    r = kfmi_mod.Results.alloc(n)
    arr = r.array()
    from oracle import oracle
    arr[:] = oracle.read_results_file(ref)
    r.save(tmp_path / "out")
    assert (tmp_path / "out.res.gpu").read_bytes() == ref.read_bytes()


def test_sais_against_bruteforce(kfmi_mod):
    rng = np.random.default_rng(7)
    for n in [1, 2, 3, 10, 100, 1000, 5000]:
        for alph in ("ACGT", "AC", "A"):
            t = "".join(rng.choice(list(alph), size=n))
            idx = kfmi_mod.Index.build(t.encode(), k=1, d=32)
            img = idx.image()
            # rebuild through the oracle-independent path: rank of every 1-mer
            bf = util.BruteForce(t)
            from oracle import oracle
            for p in ("A", "C", "G", "T"):
                res, _ = oracle.search(img, np.frombuffer(p.encode(), dtype=np.uint8).reshape(1, 1))
                assert (int(res[0]), int(res[1])) == bf.interval(p.encode()), (n, alph, p)


def test_gpu_entry_points_fail_without_a_device(kfmi_mod):
    """No CPU fallback behind the GPU entry points: on a host without a HIP
    device they return KFMI_E_NO_DEVICE (30) and write no results, even though
    the library also carries searchIndexCPU."""
    if kfmi_mod.device_count() > 0:
        pytest.skip("a HIP device is visible")
    rng = np.random.default_rng(3)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=5001)]
    idx = kfmi_mod.Index.build(t.tobytes(), k=2, d=64)
    q = kfmi_mod.Queries.from_array(t[:1000].reshape(10, 100).copy())
    r = kfmi_mod.Results.alloc(10)
    with pytest.raises(kfmi_mod.KfmiError) as ei:
        kfmi_mod.transfer_to_gpu(idx, q, r)
    assert ei.value.code == 30
    with pytest.raises(kfmi_mod.KfmiError):
        kfmi_mod.search(idx, q, r)
    assert not r.array().any()
    assert kfmi_mod.upload_form(q) == "none"          # nothing went up, in either form
    for h in (q, r, idx):
        h.close()
