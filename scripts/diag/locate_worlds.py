"""Locate on degenerate texts (scripts/diag/dropin_degenerate.py's generator:
homopolymers -- one interval holding most rows, LF walks to a sample as long
as the rate allows -- two and three letters, short periods, runs at the end,
texts of a few bases) and uniform ones: K 1, 2, d 64 or 192, the SA sampled
at a random power-of-two rate by the host or GPU builder, max_occ 0 or small,
every plain and AltCounters task backend; positions against the suffix array
the host builder keeps at rate 1.

usage: python3 scripts/diag/locate_worlds.py SECONDS"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
import dropin_degenerate as D  # noqa: E402

K = D.K
BACKENDS = ("task", "task-mid", "coop-mid", "task-ac", "task-ac-mid")


def main():
    limit = float(sys.argv[1]) if len(sys.argv) > 1 else 120
    K.set_device(0)
    t0 = time.time()
    w = calls = bad = 0
    while time.time() - t0 < limit:
        rng = np.random.default_rng(850_000 + w)
        k = int(rng.integers(1, 3))
        d = int(rng.choice([64, 192]))
        n = int(rng.integers(2 * k + 2, 40)) if rng.random() < 0.2 else int(rng.integers(40, 30_000))
        t, kind = D.text(rng, n)
        text = t.tobytes()
        rate = int(rng.choice([1, 2, 4, 8, 16, 32, 64]))
        full = K.Index.build(text, k=k, d=d, sa_rate=1)
        sa = np.array(full.sa()[1], dtype=np.int64)
        full.close()
        idx = K.Index.build(text, k=k, d=d, gpu=bool(rng.integers(0, 2)), sa_rate=rate)
        m = k * int(rng.integers(1, 40 // k + 1))
        if m > n:
            m = k
        st = rng.integers(0, n - m + 1, size=int(rng.integers(1, 500)))
        q = np.ascontiguousarray(np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                                                 rng.choice(D.ACGT, size=(8, m)), np.full((2, m), t[-1], np.uint8)]))
        max_occ = int(rng.choice([0, 0, 1, 3, 100]))
        for b in BACKENDS:
            calls += 1
            res, off, pos = K.locate_array(idx, q, b, max_occ)
            L = res[0::2].astype(np.int64)
            R = res[1::2].astype(np.int64)
            w_pos, w_off = [], [0]
            for lo, hi in zip(L, R):
                hi = min(hi, n + 1)   # rows past n+1 hold no suffix (AltCounters intervals reach them)
                hi = min(hi, lo + max_occ) if max_occ else hi
                seg = sa[lo:hi] if hi > lo else sa[:0]
                w_pos.append(seg)
                w_off.append(w_off[-1] + seg.size)
            want = np.concatenate(w_pos).astype(np.uint32) if w_pos else np.zeros(0, np.uint32)
            if not (np.array_equal(off, np.array(w_off, np.uint64)) and np.array_equal(pos, want)):
                bad += 1
                print(f"MISMATCH world {w}: K={k} d={d} n={n} kind={kind} rate={rate} max_occ={max_occ} {b}",
                      flush=True)
        idx.close()
        w += 1
        if w % 25 == 0:
            print(f"{w} worlds, {calls} locates, {bad} bad, {time.time() - t0:.0f}s", flush=True)
    print(f"done: {w} worlds, {calls} locates, {bad} bad", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
