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
@pytest.mark.parametrize("backend,tag,res_tag", [("task", 101, 100), ("coop", 101, 100), ("task-mid", 100, 100),
                                                 ("task-ac", 201, 200), ("coop-ac", 201, 200),
                                                 # the K = 2 file on the K = 4 layout (derived on upload, DESIGN 5d')
                                                 ("coop-grp", 101, 100), ("task-grp", 100, 100)])
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


@pytest.mark.gpu
def test_reference_driver_on_a_k4_index(oracle_mod, tmp_path):
    """The unmodified driver on a K = 4 .fmi written by the reference's own
    builder (oracle/_ref/gfmi_4_64), no backend chosen: the engine uploads it
    for coop-grp; the .res.gpu equals the reference K = 4 CPU searcher's
    .res.cpu (oracle/_ref/cpu_4_64) byte for byte."""
    import numpy as np
    gfmi, cpu = oracle_mod.ref_binary("gfmi", 4, 64), oracle_mod.ref_binary("cpu", 4, 64)
    if not DROPIN.exists() or not gfmi.exists() or not cpu.exists():
        pytest.fail("oracle/_ref binaries missing on the GPU box")
    n = 60_001
    rng = np.random.default_rng(44)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n)]
    text = t.tobytes()
    (tmp_path / "ref.fa").write_bytes(b">x\n" + b"\n".join(text[i:i + 70] for i in range(0, n, 70)) + b"\n")
    subprocess.run([str(gfmi), "ref.fa", str(n)], cwd=tmp_path, check=True, capture_output=True, timeout=300)
    fn = tmp_path / f"ref.fa.{n}.64fmi4steps.fmi"
    st = rng.integers(0, n - 100, size=3000)
    q = np.concatenate([t[st[:, None] + np.arange(100)[None, :]],
                        rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(500, 100))])
    (tmp_path / "q.qry").write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in q))
    subprocess.run([str(cpu), str(fn), "q.qry", "100", str(q.shape[0])], cwd=tmp_path, check=True,
                   capture_output=True, timeout=300)
    env = {k: v for k, v in os.environ.items() if k not in ("KFMI_BACKEND", "KFMI_STRICT_TAG")}
    p = subprocess.run([str(DROPIN), str(fn), "q.qry", "100", str(q.shape[0])], cwd=tmp_path,
                       capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert (tmp_path / (fn.name + ".res.gpu")).read_bytes() == (tmp_path / (fn.name + ".res.cpu")).read_bytes()
