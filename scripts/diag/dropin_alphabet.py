"""Real-FASTA ('ref' alphabet) worlds through the reference's own searcher and
its driver on this library: tests/test_alphabet_worlds.py's multi-FASTA files
(N runs, soft-masked stretches, IUPAC letters, 30-400-byte lines), indexed by
the reference's builder (oracle/_ref/gfmi_K_d under MALLOC_PERTURB_, thread
cache off) and, at K <= 2, its transforms; then for every tag the reference's
cpu / cpuac searcher and searchQueries_cpu_dropin (with --gpu,
searchQueries_dropin on a random GPU backend) write their results files from
the same index file and queries, which must be byte-identical wherever the
restatement (oracle/) says the reference is defined.

usage: python3 scripts/diag/dropin_alphabet.py SECONDS [--gpu]"""
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import dropin_degenerate as D  # noqa: E402

sys.path.insert(0, str(D.REPO / "tests"))
from test_alphabet_worlds import world as alpha_world  # noqa: E402

K = D.K
oracle = D.oracle


def run_world(w, gpu):
    k, d, fasta, n, pert = alpha_world(w)
    rng = np.random.default_rng(870_000 + w)
    checked = []
    with tempfile.TemporaryDirectory() as td:
        tp = Path(td)
        (tp / "ref.fa").write_bytes(fasta)
        env = {x: v for x, v in os.environ.items() if x != "MALLOC_PERTURB_"}
        if pert is not None:
            env["MALLOC_PERTURB_"] = str(pert)
            env["GLIBC_TUNABLES"] = "glibc.malloc.tcache_count=0"
        run = lambda *a: subprocess.run([str(x) for x in a], cwd=tp, check=True, capture_output=True,  # noqa: E731
                                        timeout=120, env=env)
        run(D.REF / f"gfmi_{k}_{d}", "ref.fa", n)
        fn = f"ref.fa.{n}.{d}fmi{k}steps.fmi"
        if k <= 2:
            run(D.REF / f"tfmiBMP_{k}_{d}", fn)
            run(D.REF / f"tfmiAC_{k}_{d}", fn)
        m = k * int(rng.integers(1, 60 // k + 1))
        q = np.ascontiguousarray(rng.choice(np.frombuffer(b"ACGTNacgtRY", np.uint8), size=(int(rng.integers(1, 300)), m)))
        (tp / "q.qry").write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in q))
        want = {}
        for tag in ((100, 101, 200, 201) if k <= 2 else (100,)):
            base = 200 if tag >= 200 else 100
            img = np.fromfile(tp / (fn + D.TAGS[base]), dtype=np.uint8)
            if not D.defined(img, q):
                continue
            if base not in want:
                dd = tp / f"ref{base}"
                dd.mkdir()
                shutil.copy(tp / (fn + D.TAGS[base]), dd)
                subprocess.run([str(D.REF / f"{'cpuac' if base == 200 else 'cpu'}_{k}_{d}"), fn + D.TAGS[base],
                                str(tp / "q.qry"), str(m), str(q.shape[0])], cwd=dd, check=True,
                               capture_output=True, timeout=120, env=dict(os.environ, OMP_NUM_THREADS="1"))
                want[base] = (dd / (fn + D.TAGS[base] + ".res.cpu")).read_bytes()
            if gpu:
                pool = ("coop-grp", "task-grp") if k > 2 else (D.ALT if tag >= 200 else D.PLAIN)
                backend = str(rng.choice(pool))
                binary, suffix, e2 = D.REF / "searchQueries_dropin", ".res.gpu", {"KFMI_BACKEND": backend}
            else:
                backend = "cpu"
                binary, suffix, e2 = D.REF / "searchQueries_cpu_dropin", ".res.cpu", {"OMP_NUM_THREADS": "2"}
            od = tp / f"ours{tag}"
            od.mkdir()
            shutil.copy(tp / (fn + D.TAGS[tag]), od)
            p = subprocess.run([str(binary), fn + D.TAGS[tag], str(tp / "q.qry"), str(m), str(q.shape[0])], cwd=od,
                               capture_output=True, text=True, timeout=120, env=dict(os.environ, **e2))
            if p.returncode != 0:
                raise RuntimeError(f"world {w}: driver failed ({backend}, tag {tag}): {p.stdout[-300:]} {p.stderr[-300:]}")
            checked.append((tag, backend, (od / (fn + D.TAGS[tag] + suffix)).read_bytes() == want[base]))
    return k, d, n, m, checked


def main():
    limit = float(sys.argv[1]) if len(sys.argv) > 1 else 120
    gpu = "--gpu" in sys.argv
    if gpu:
        K.set_device(0)
    t0 = time.time()
    w = files = bad = 0
    while time.time() - t0 < limit:
        k, d, n, m, checked = run_world(w, gpu)
        for tag, b, same in checked:
            files += 1
            if not same:
                bad += 1
                print(f"MISMATCH world {w}: K={k} d={d} n={n} m={m} tag={tag} {b}", flush=True)
        w += 1
        if w % 25 == 0:
            print(f"{w} worlds, {files} files compared, {bad} bad, {time.time() - t0:.0f}s", flush=True)
    print(f"done: {w} worlds, {files} files compared, {bad} bad", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
