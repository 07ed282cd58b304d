"""Degenerate texts through the reference's own driver and searchers.

tests/test_dropin_worlds.py with the texts it does not draw: homopolymers of
each letter, two- and three-letter texts, short periods, long runs at the end,
tiny texts (n from 2K+2), reads of 1..400 bases and reads longer than the
text (up to 1,022 bases: the reference's loadQueries cuts longer lines, B11).
For every tag: the reference's builder and transforms write the files
(oracle/_ref gfmi / tfmiBMP / tfmiAC), its own searcher (cpu / cpuac) writes
the results, and the reference driver compiled against libkstepfmi.so
(searchQueries_cpu_dropin; with --gpu, searchQueries_dropin on a random GPU
backend that takes the tag) must write the same bytes -- wherever the
restatement (oracle/) says the reference is defined; elsewhere the reference
may fault and nothing is compared.

usage: python3 scripts/diag/dropin_degenerate.py SECONDS [--gpu]"""
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "k-step_fm-index_amd"))
sys.path.insert(0, str(REPO))
import kstep_fmi as K  # noqa: E402
from oracle import oracle  # noqa: E402

REF = REPO / "oracle" / "_ref"
GEOMS = [(1, 64), (2, 64), (1, 192), (2, 192), (3, 64), (4, 64)]
TAGS = {100: "", 101: ".interleaving", 200: ".ac", 201: ".interleaving.ac"}
PLAIN = ("task", "coop", "task-mid", "coop-mid")
ALT = ("task-ac", "task-ac-mid", "coop-ac-mid")
ACGT = np.frombuffer(b"ACGT", np.uint8)


def text(rng, n):
    kind = int(rng.integers(0, 7))
    if kind == 0:
        t = np.full(n, ACGT[rng.integers(0, 4)], np.uint8)
    elif kind == 1:
        t = ACGT[rng.choice(4, size=2, replace=False)][rng.integers(0, 2, size=n)]
    elif kind == 2:
        t = ACGT[rng.choice(4, size=3, replace=False)][rng.integers(0, 3, size=n)]
    elif kind == 3:
        t = np.resize(ACGT[rng.integers(0, 4, size=int(rng.integers(1, 8)))], n)
    elif kind == 4:
        t = ACGT[rng.integers(0, 4, size=n)]
        t[-int(rng.integers(1, n + 1)):] = ACGT[rng.integers(0, 4)]
    elif kind == 5:
        t = np.full(n, ACGT[rng.integers(0, 4)], np.uint8)
        t[rng.integers(0, n, size=int(rng.integers(1, 4)))] = ACGT[rng.integers(0, 4)]
    else:
        t = np.repeat(ACGT[rng.integers(0, 4, size=n)], rng.integers(1, 300, size=n))[:n]
    return np.ascontiguousarray(t, np.uint8), kind


def reads(rng, t, m, nq):
    n = t.size
    parts = [np.full((2, m), t[-1], np.uint8), rng.choice(ACGT, size=(max(1, nq // 4), m))]
    for c in ACGT:
        parts.append(np.full((1, m), c, np.uint8))
    if m <= n:
        st = rng.integers(0, n - m + 1, size=nq)
        parts.append(t[st[:, None] + np.arange(m)[None, :]])
        parts.append(t[n - m:][None, :])
    return np.ascontiguousarray(np.concatenate(parts))


def defined(img, q):
    try:
        oracle.search(img, q)
        return True
    except ValueError:
        return False


def run_world(w, gpu):
    rng = np.random.default_rng(810_000 + w)
    k, d = GEOMS[int(rng.integers(0, len(GEOMS)))]
    n = int(rng.integers(2 * k + 2, 40)) if rng.random() < 0.25 else int(rng.integers(40, 3000))
    t, kind = text(rng, n)
    m = k * int(rng.integers(1, 400 // k + 1))
    if rng.random() < 0.1:   # longer than the text (the reference cuts reads of 1,023+ bases: B11)
        m = min(k * ((n + k) // k + int(rng.integers(0, 3))), 1022 // k * k)
    q = reads(rng, t, m, int(rng.integers(1, 300)))
    idx = K.Index.build(t.tobytes(), k=k, d=d)
    imgs = {100: idx.image()}
    acs = ()
    if k <= 2:
        acs = idx.alt_counters()
        imgs[200] = acs[0].image()
    ok = {tag: defined(imgs[200 if tag >= 200 else 100], q) for tag in ((100, 101, 200, 201) if k <= 2 else (100,))}
    for x in (idx,) + tuple(acs):
        x.close()
    checked = []
    if not any(ok.values()):
        return k, d, n, kind, m, checked
    with tempfile.TemporaryDirectory() as td:
        tp = Path(td)
        (tp / "ref.fa").write_bytes(b">w\n" + b"\n".join(t.tobytes()[j:j + 70] for j in range(0, n, 70)) + b"\n")
        run = lambda *a: subprocess.run([str(x) for x in a], cwd=tp, check=True, capture_output=True,  # noqa: E731
                                        timeout=120)
        run(REF / f"gfmi_{k}_{d}", "ref.fa", n)
        fn = f"ref.fa.{n}.{d}fmi{k}steps.fmi"
        if k <= 2:
            run(REF / f"tfmiBMP_{k}_{d}", fn)
            run(REF / f"tfmiAC_{k}_{d}", fn)
        (tp / "q.qry").write_bytes(b"".join(b">r\n" + r.tobytes() + b"\n" for r in q))
        want = {}
        for tag, good in ok.items():
            if not good:
                continue
            base = 200 if tag >= 200 else 100
            if base not in want:
                dd = tp / f"ref{base}"
                dd.mkdir()
                shutil.copy(tp / (fn + TAGS[base]), dd)
                subprocess.run([str(REF / f"{'cpuac' if base == 200 else 'cpu'}_{k}_{d}"), fn + TAGS[base],
                                str(tp / "q.qry"), str(m), str(q.shape[0])], cwd=dd, check=True,
                               capture_output=True, timeout=120, env=dict(os.environ, OMP_NUM_THREADS="1"))
                want[base] = (dd / (fn + TAGS[base] + ".res.cpu")).read_bytes()
            if gpu:
                pool = ("coop-grp", "task-grp") if k > 2 else (ALT if tag >= 200 else PLAIN)
                backend = str(rng.choice(pool))
                binary, suffix, env = REF / "searchQueries_dropin", ".res.gpu", {"KFMI_BACKEND": backend}
            else:
                backend = "cpu"
                binary, suffix, env = REF / "searchQueries_cpu_dropin", ".res.cpu", {"OMP_NUM_THREADS": "2"}
            od = tp / f"ours{tag}"
            od.mkdir()
            shutil.copy(tp / (fn + TAGS[tag]), od)
            p = subprocess.run([str(binary), fn + TAGS[tag], str(tp / "q.qry"), str(m), str(q.shape[0])], cwd=od,
                               capture_output=True, text=True, timeout=120, env=dict(os.environ, **env))
            if p.returncode != 0:   # every backend in the pools takes these geometries
                raise RuntimeError(f"world {w}: driver failed ({backend}, tag {tag}): {p.stdout[-300:]} {p.stderr[-300:]}")
            got = (od / (fn + TAGS[tag] + suffix)).read_bytes()
            checked.append((tag, backend, got == want[base]))
    return k, d, n, kind, m, checked


def main():
    limit = float(sys.argv[1]) if len(sys.argv) > 1 else 120
    gpu = "--gpu" in sys.argv
    if gpu:
        K.set_device(0)
    t0 = time.time()
    w = searches = bad = undefined = 0
    while time.time() - t0 < limit:
        k, d, n, kind, m, checked = run_world(w, gpu)
        if not checked:
            undefined += 1
        for tag, backend, same in checked:
            searches += 1
            if not same:
                bad += 1
                print(f"MISMATCH world {w}: K={k} d={d} n={n} kind={kind} m={m} tag={tag} {backend}", flush=True)
        w += 1
        if w % 25 == 0:
            print(f"{w} worlds, {searches} files compared, {bad} bad, {undefined} wholly undefined, "
                  f"{time.time() - t0:.0f}s", flush=True)
    print(f"done: {w} worlds, {searches} files compared, {bad} bad, {undefined} wholly undefined", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
