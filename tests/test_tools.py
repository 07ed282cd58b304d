"""The engine's command-line tools with the reference's CLIs and file names:
gfmi (generateIndex.c), tfmiBMP / tfmiAC (transform*.c), searchQueries
(searchQueries.c).  Outputs compared byte-for-byte with the reference tools'
files committed in tests/golden."""
import os
import shutil
import subprocess

import pytest

from util import GOLDEN, PKG, manifest

BIN = PKG / "bin"


def run(args, cwd, env=None):
    e = dict(os.environ, **(env or {}))
    p = subprocess.run([str(a) for a in args], cwd=cwd, capture_output=True, text=True, env=e, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


@pytest.mark.parametrize("case", ["textA", "textB", "textD"])
def test_gfmi_and_transforms_match_reference_files(tmp_path, case):
    c = manifest()[case]
    shutil.copy(GOLDEN / case / "ref.fa", tmp_path / "ref.fa")
    for key, ent in c["indexes"].items():
        k, d = ent["k"], ent["d"]
        run([BIN / "gfmi", "ref.fa", c["n"]], tmp_path, {"KFMI_K": str(k), "KFMI_D": str(d), "KFMI_BUILD_GPU": "0"})
        base = tmp_path / f"ref.fa.{c['n']}.{d}fmi{k}steps.fmi"
        run([BIN / "tfmiBMP", base.name], tmp_path)
        run([BIN / "tfmiAC", base.name], tmp_path)
        for tag, suffix in ((100, ""), (101, ".interleaving"), (200, ".ac"), (201, ".interleaving.ac")):
            got = (tmp_path / (base.name + suffix)).read_bytes()
            assert got == (GOLDEN / case / ent["files"][str(tag)]["file"]).read_bytes(), (case, key, tag)
        # saveRef copy (common.c:119-130): "<ref>.<n>.fa"
        assert (tmp_path / f"ref.fa.{c['n']}.fa").exists()


def test_tools_report_reference_errors(tmp_path):
    p = subprocess.run([str(BIN / "tfmiBMP"), str(GOLDEN / "textA" / "k2_d64.101.fmi")],
                       capture_output=True, text=True)
    assert p.returncode != 0 and "gfmiBaseLine" in p.stderr     # wants a tag-100 input
    p = subprocess.run([str(BIN / "gfmi"), str(tmp_path / "missing.fa"), "10"], capture_output=True, text=True)
    assert p.returncode != 0 and "reference file" in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("backend,tag,res_tag", [("task-mid", 100, 100), ("task", 101, 100), ("coop-ac", 201, 200), ("task-ac-mid", 201, 200)])
def test_search_driver(tmp_path, backend, tag, res_tag):
    c = manifest()["textA"]
    ent = c["indexes"]["k2_d64"]
    shutil.copy(GOLDEN / "textA" / ent["files"][str(tag)]["file"], tmp_path / "idx.fmi")
    qd = c["queries"]["100"]
    shutil.copy(GOLDEN / "textA" / qd["file"], tmp_path / "q.qry")
    out = run([BIN / "searchQueries", "idx.fmi", "q.qry", 100, qd["num"]], tmp_path,
              {"KFMI_BACKEND": backend, "KFMI_ITERS": "3"})
    assert f"BACKEND: {backend}" in out and "TIME:" in out
    want = (GOLDEN / "textA" / ent["results"][f"100.{res_tag}"]["file"]).read_bytes()
    assert (tmp_path / "idx.fmi.res.gpu").read_bytes() == want


@pytest.mark.gpu
def test_gfmi_sa_and_search_driver_locate(tmp_path):
    """CLI locate path (extension): gfmi with KFMI_SA_RATE writes <index>.sa,
    searchQueries with KFMI_SA_FILE writes <index>.pos.gpu; every position
    must start an occurrence of its read and the counts must equal R - L."""
    import numpy as np
    import util
    c = manifest()["textA"]
    shutil.copy(GOLDEN / "textA" / "ref.fa", tmp_path / "ref.fa")
    n = c["n"]
    run([BIN / "gfmi", "ref.fa", n], tmp_path, {"KFMI_SA_RATE": "4"})
    idx = tmp_path / f"ref.fa.{n}.64fmi2steps.fmi"
    assert (tmp_path / (idx.name + ".sa")).exists()
    qd = c["queries"]["12"]
    shutil.copy(GOLDEN / "textA" / qd["file"], tmp_path / "q.qry")
    out = run([BIN / "searchQueries", idx.name, "q.qry", 12, qd["num"]], tmp_path,
              {"KFMI_BACKEND": "task-mid", "KFMI_ITERS": "1", "KFMI_SA_FILE": idx.name + ".sa"})
    assert "LOCATE:" in out
    text = util.read_fasta_text(GOLDEN / "textA" / "ref.fa")
    reads = util.read_qry(tmp_path / "q.qry", 12)
    res = [ln.split() for ln in (tmp_path / (idx.name + ".res.gpu")).read_text().splitlines()[1:]]
    lines = (tmp_path / (idx.name + ".pos.gpu")).read_text().splitlines()
    assert len(lines) == len(reads) == len(res)
    for rd, (L, R), ln in zip(reads, res, lines):
        f = [int(x) for x in ln.split()]
        assert f[0] == int(R) - int(L) == len(f) - 1
        want = bytes(b"ACGT"[util.code_of(ch)] for ch in rd.tobytes()).decode()
        for p in f[1:]:
            assert text[p:p + 12] == want
