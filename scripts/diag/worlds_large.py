"""The random worlds of tests/test_random_worlds.py at larger scale: texts of
10 kbase to 1.5 Mbase (runs, tandem repeats, copied segments, two letters),
up to 20,000 reads of 1-400 bases; every GPU backend the geometry takes
against the CPU oracle (brute-force suffix ranks where the plain reference
is undefined, B5; the host search where the AltCounters one is).  Runs until the time limit; prints every mismatch."""
import sys, time, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import util
import kstep_fmi as K
from oracle import oracle
from test_random_worlds import PLAIN, ALT, GRP, _takes, ACGT

K.set_device(0)
limit = float(sys.argv[1]) if len(sys.argv) > 1 else 200
t0 = time.time(); w = 0; calls = 0; bad = 0
while time.time() - t0 < limit:
    rng = np.random.default_rng(700_000 + w)
    w += 1
    n = int(rng.integers(10_000, 1_500_000))
    kind = int(rng.integers(0, 4))
    if kind == 0:
        t = ACGT[rng.integers(0, 4, size=n)].copy()
    elif kind == 1:
        t = np.repeat(ACGT[rng.integers(0, 4, size=n)], rng.integers(1, 60, size=n))[:n].copy()
    elif kind == 2:
        t = ACGT[rng.integers(0, 4, size=n)].copy()
        for _ in range(200):
            ln = int(rng.integers(50, 5000)); a, b = rng.integers(0, n - ln, size=2)
            t[b:b + ln] = t[a:a + ln]
    else:
        t = ACGT[rng.integers(0, 4, size=2)][rng.integers(0, 2, size=n)].copy()
    k = int(rng.choice([1, 2, 2, 3, 4]))
    d = 64 if k > 2 else int(rng.choice([32, 64, 128, 192, 448, 960]))
    m = int(rng.integers(1, 401))
    nq = int(rng.integers(1, 20_000))
    st = rng.integers(0, n - m + 1, size=nq)
    q = np.ascontiguousarray(np.concatenate([t[st[:, None] + np.arange(m)[None, :]],
                                             rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(nq // 8 + 1, m))]))
    text = t.tobytes()
    idx = K.Index.build(text, k=k, d=d, gpu=bool(rng.integers(0, 2)) if k <= 4 else False)
    i1 = K.Index.build(text, k=1, d=64)
    b5 = (n + 1) % d == 0 or (n + 1) % 64 == 0
    if b5:
        bf = util.BruteForce(text.decode())
        want = np.array([x for r in q for x in bf.interval(r.tobytes())], dtype=np.uint32)
    else:
        want = oracle.search(i1.image(), q)[0]
    want_ac = None
    acs = ()
    if k <= 2 and m % k == 0:
        acs = idx.alt_counters()
        try:
            want_ac = oracle.search(acs[0].image(), q)[0]
        except ValueError:   # reads past the reference's file: undefined; agree with the host search
            want_ac = K.search_cpu_array(acs[0], q, 4)
    for b in PLAIN + ALT + GRP:
        if not _takes(b, k, d, n) or (b in ALT and (m % k or want_ac is None)):
            continue
        calls += 1
        got = K.search_array(idx, q, b)
        wv = want_ac if b in ALT else want
        if not np.array_equal(got, wv):
            bad += 1
            j = int(np.flatnonzero(got != wv)[0]) // 2
            print(f"MISMATCH world {w - 1} n={n} k={k} d={d} m={m} kind={kind} {b}: read {j} got {got[2*j:2*j+2]} want {wv[2*j:2*j+2]}", flush=True)
    for x in (idx, i1) + tuple(acs):
        x.close()
    if w % 10 == 0:
        print(f"{w} worlds, {calls} searches, {bad} bad, {time.time() - t0:.0f}s", flush=True)
print(f"done: {w} worlds, {calls} searches, {bad} bad", flush=True)
