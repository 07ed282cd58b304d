"""Search on degenerate texts (scripts/diag/dropin_degenerate.py's
generator: homopolymers of each letter, two and three letters, short periods,
runs at the end, texts of a few bases) with any read length -- m % K != 0
through the remainder table -- and a random ftab, against brute-force suffix
ranks: the host search, and with --gpu every plain GPU backend the geometry
takes (K 1-4; the grouped layout at K 3, 4 and from K = 2 by derivation);
at K <= 2 also the AltCounters files through the host search and every
AltCounters backend, against the restatement (oracle/) where the reference
is defined and the host search where it is not.

usage: python3 scripts/diag/search_degenerate.py SECONDS [--gpu]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import dropin_degenerate as D  # noqa: E402

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests"))
import util  # noqa: E402
from test_random_worlds import ALT, GRP, PLAIN, _takes  # noqa: E402
from oracle import oracle  # noqa: E402

K = D.K


def run_world(w, gpu):
    """[(searcher, first differing read or None)] for world w."""
    rng = np.random.default_rng(860_000 + w)
    k = int(rng.choice([1, 2, 2, 3, 4]))
    d = 64 if k > 2 else int(rng.choice([32, 64, 128, 192]))
    n = int(rng.integers(2 * k + 2, 40)) if rng.random() < 0.25 else int(rng.integers(40, 4000))
    t, kind = D.text(rng, n)
    m = int(rng.integers(1, 120))
    q = D.reads(rng, t, m, int(rng.integers(1, 200)))
    bf = util.BruteForce(t.tobytes().decode())
    want = np.array([x for r in q for x in bf.interval(r.tobytes())], dtype=np.uint32)
    idx = K.Index.build(t.tobytes(), k=k, d=d, gpu=gpu and bool(rng.integers(0, 2)))
    got = {"host": K.search_cpu_array(idx, q, 2)}
    if gpu:
        bases = k * int(rng.integers(0, 8 // k + 1))
        K.set_ftab(bases if m % k == 0 else 0)
        try:
            for b in PLAIN + GRP:
                if _takes(b, k, d, n):
                    got[b] = K.search_array(idx, q, b)
        finally:
            K.set_ftab(0)
    wants = {b: want for b in got}
    if k <= 2 and m % k == 0:   # AltCounters semantics: the restatement where defined, else the host search
        acs = idx.alt_counters()
        try:
            try:
                want_ac = oracle.search(acs[0].image(), q)[0]
            except ValueError:
                want_ac = K.search_cpu_array(acs[0], q, 2)
            got["host-ac"] = K.search_cpu_array(acs[1], q, 2)
            wants["host-ac"] = want_ac
            if gpu:
                for b in ALT:
                    if _takes(b, k, d, n):
                        got[b] = K.search_array(idx, q, b)
                        wants[b] = want_ac
        finally:
            for x in acs:
                x.close()
    idx.close()
    out = []
    for b, g in got.items():
        diff = np.flatnonzero(g != wants[b])
        out.append((b, None if diff.size == 0 else
                    f"K={k} d={d} n={n} kind={kind} m={m} read {int(diff[0]) // 2}"))
    return out


def main():
    limit = float(sys.argv[1]) if len(sys.argv) > 1 else 120
    gpu = "--gpu" in sys.argv
    if gpu:
        K.set_device(0)
    t0 = time.time()
    w = calls = bad = 0
    while time.time() - t0 < limit:
        for b, what in run_world(w, gpu):
            calls += 1
            if what:
                bad += 1
                print(f"MISMATCH world {w}: {b}: {what}", flush=True)
        w += 1
        if w % 50 == 0:
            print(f"{w} worlds, {calls} searches, {bad} bad, {time.time() - t0:.0f}s", flush=True)
    print(f"done: {w} worlds, {calls} searches, {bad} bad", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
