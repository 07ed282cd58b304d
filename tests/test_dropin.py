"""Drop-in proof: the reference's own driver (common/searchQueries.c, compiled
unmodified with -DCUDA by oracle/Makefile) linked against libkstepfmi.so in
place of the reference's .c/.cu backends, run on a golden index, writes the
same results the reference CPU searcher wrote."""
import os
import shutil
import subprocess

import pytest

from util import GOLDEN, REPO, manifest

DROPIN = REPO / "oracle" / "_ref" / "searchQueries_dropin"


def test_dropin_links_against_engine():
    if not DROPIN.exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    out = subprocess.run(["ldd", str(DROPIN)], capture_output=True, text=True).stdout
    assert "libkstepfmi.so" in out and "not found" not in out


@pytest.mark.gpu
@pytest.mark.parametrize("backend,tag,res_tag", [("task", 101, 100), ("coop", 101, 100), ("task-packed", 100, 100),
                                                 ("task-ac", 201, 200), ("coop-ac", 201, 200)])
def test_reference_driver_runs_on_engine(tmp_path, backend, tag, res_tag):
    if not DROPIN.exists():
        pytest.fail("oracle/_ref/searchQueries_dropin missing on the GPU box")
    c = manifest()["textA"]
    ent = c["indexes"]["k2_d64"]
    idx = tmp_path / "index.fmi"
    shutil.copy(GOLDEN / "textA" / ent["files"][str(tag)]["file"], idx)
    qd = c["queries"]["100"]
    shutil.copy(GOLDEN / "textA" / qd["file"], tmp_path / "q.qry")
    env = dict(os.environ, KFMI_BACKEND=backend, KFMI_STRICT_TAG="1" if tag in (101, 201) else "0")
    p = subprocess.run([str(DROPIN), str(idx), str(tmp_path / "q.qry"), "100", str(qd["num"])],
                       capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "TIME:" in p.stdout
    want = (GOLDEN / "textA" / ent["results"][f"100.{res_tag}"]["file"]).read_bytes()
    assert (tmp_path / "index.fmi.res.gpu").read_bytes() == want
