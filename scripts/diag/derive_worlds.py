"""Device derivation (kfmi_derive_index_gpu: a K = 1 file to K = 2, a K = 2
file to K = 4) on degenerate texts (scripts/diag/dropin_degenerate.py's
generator: homopolymers, two and three letters, short periods, runs at the
end, texts of a few bases) and uniform ones up to 2 Mbase, against the index
the host builder (byte-equal to the reference's gfmi) makes from the text.

usage: python3 scripts/diag/derive_worlds.py SECONDS"""
import hashlib
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import dropin_degenerate as D  # noqa: E402

K = D.K


def md5(b):
    return hashlib.md5(bytes(b)).hexdigest()


def main():
    limit = float(sys.argv[1]) if len(sys.argv) > 1 else 120
    K.set_device(0)
    t0 = time.time()
    w = bad = 0
    while time.time() - t0 < limit:
        rng = np.random.default_rng(840_000 + w)
        kin = int(rng.integers(1, 3))
        r = rng.random()
        n = int(rng.integers(8, 40)) if r < 0.25 else int(rng.integers(40, 20_000)) if r < 0.9 else \
            int(rng.integers(20_000, 2_000_000))
        if rng.random() < 0.3:
            t = D.ACGT[rng.integers(0, 4, size=n)].copy()
            kind = "uniform"
        else:
            t, kind = D.text(rng, n)
        text = t.tobytes()
        src = K.Index.build(text, k=kin, d=64, gpu=bool(rng.integers(0, 2)))
        g = src.derive(2 * kin, host_image=True)
        want = K.Index.build(text, k=2 * kin, d=64)
        if md5(g.image()) != md5(want.image()):
            bad += 1
            print(f"MISMATCH world {w}: n={n} kind={kind} K {kin} -> {2 * kin}", flush=True)
        for x in (src, g, want):
            x.close()
        w += 1
        if w % 50 == 0:
            print(f"{w} derivations, {bad} bad, {time.time() - t0:.0f}s", flush=True)
    print(f"done: {w} derivations, {bad} bad", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
