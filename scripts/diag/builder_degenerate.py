"""Degenerate texts (scripts/diag/dropin_degenerate.py's generator) through
the builders: the reference's gfmi / tfmiBMP / tfmiAC files against this
build's host builder (and with --gpu the GPU builder) and transforms, byte for
byte, for as long as it is given.

usage: python3 scripts/diag/builder_degenerate.py SECONDS [--gpu]"""
import hashlib
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import dropin_degenerate as D  # noqa: E402

K = D.K


def ref_files(tp, k, d, text):
    n = len(text)
    (tp / "ref.fa").write_bytes(b">w\n" + b"\n".join(text[j:j + 70] for j in range(0, n, 70)) + b"\n")
    run = lambda *a: subprocess.run([str(x) for x in a], cwd=tp, check=True, capture_output=True,  # noqa: E731
                                    timeout=120)
    run(D.REF / f"gfmi_{k}_{d}", "ref.fa", n)
    fn = f"ref.fa.{n}.{d}fmi{k}steps.fmi"
    out = {100: (tp / fn).read_bytes()}
    if k <= 2:
        run(D.REF / f"tfmiBMP_{k}_{d}", fn)
        run(D.REF / f"tfmiAC_{k}_{d}", fn)
        for tag in (101, 200, 201):
            out[tag] = (tp / (fn + D.TAGS[tag])).read_bytes()
    return out


def md5(b):
    return hashlib.md5(bytes(b)).hexdigest()


def main():
    limit = float(sys.argv[1]) if len(sys.argv) > 1 else 120
    gpu = "--gpu" in sys.argv
    if gpu:
        K.set_device(0)
    t0 = time.time()
    w = files = bad = 0
    while time.time() - t0 < limit:
        rng = np.random.default_rng(820_000 + w)
        k, d = D.GEOMS[int(rng.integers(0, len(D.GEOMS)))]
        n = int(rng.integers(2 * k + 2, 40)) if rng.random() < 0.3 else int(rng.integers(40, 6000))
        t, kind = D.text(rng, n)
        text = t.tobytes()
        with tempfile.TemporaryDirectory() as td:
            want = ref_files(Path(td), k, d, text)
        idx = K.Index.build(text, k=k, d=d, gpu=gpu)
        got = {100: idx.image()}
        extra = []
        if k <= 2:
            i101 = idx.interleave()
            a200, a201 = idx.alt_counters()
            got.update({101: i101.image(), 200: a200.image(), 201: a201.image()})
            extra = [i101, a200, a201]
        for tag, img in got.items():
            files += 1
            if md5(img) != md5(want[tag]):
                bad += 1
                print(f"MISMATCH world {w}: K={k} d={d} n={n} kind={kind} tag={tag}", flush=True)
        for x in [idx] + extra:
            x.close()
        w += 1
        if w % 50 == 0:
            print(f"{w} worlds, {files} files, {bad} bad, {time.time() - t0:.0f}s", flush=True)
    print(f"done: {w} worlds, {files} files, {bad} bad ({'GPU' if gpu else 'host'} builder)", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
