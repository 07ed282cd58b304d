"""Intermittent-result hunt: every backend x K in {1, 2} x d in {64, 128, 192,
448, 960} x ftab {0, 8, 12}, many batches with re-uploads, each call against
the oracle; prints every mismatching call, then a per-(backend, K, d) tally."""
import sys, time, collections, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import kstep_fmi as K
from oracle import oracle
K.set_device(0)
rng = np.random.default_rng(7)
text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=2_000_003).tobytes()
t = np.frombuffer(text, np.uint8)
geoms = [(1, 64), (2, 64), (1, 128), (2, 128), (1, 192), (2, 192), (2, 448), (2, 960), (1, 448)]
idxs = {g: K.Index.build(text, k=g[0], d=g[1]) for g in geoms}
img = {g: i.image() for g, i in idxs.items()}
ac = {g: i.alt_counters()[0].image() for g, i in idxs.items()}
BACK = ["task", "coop", "task-mid", "coop-mid", "task-ac", "coop-ac", "task-ac-mid", "coop-ac-mid"]
def coop_ok(b, k, d):
    if not b.startswith("coop"):
        return True
    bmw = 2 * (d // 32) * k
    if b == "coop-ac":
        return k == 2 and bmw % 4 == 0
    if b == "coop":
        return bmw % 4 == 0 and (bmw + 4 ** k) % 4 == 0
    return bmw % 4 == 0
calls = collections.Counter(); bad = collections.Counter()
t0 = time.time(); it = 0
limit = float(sys.argv[1]) if len(sys.argv) > 1 else 150
while time.time() - t0 < limit:
    it += 1
    g = geoms[it % len(geoms)]
    k, d = g
    b = BACK[(it // len(geoms)) % len(BACK)]
    if not coop_ok(b, k, d):
        continue
    ft = int(rng.choice([0, 8, 12])) if k == 1 else int(rng.choice([0, 8, 12]))
    m = 100
    st = rng.integers(0, len(text) - m, size=4000)
    q = np.concatenate([t[st[:, None] + np.arange(m)[None, :]], rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(500, m))])
    K.set_ftab(ft)
    try:
        got = K.search_array(idxs[g], q, b)
    except K.KfmiError as e:
        K.set_ftab(0)
        continue
    K.set_ftab(0)
    want = oracle.search(ac[g] if "ac" in b else img[g], q)[0]
    key = (b, k, d, ft)
    calls[key] += 1
    nb = int(np.sum(got != want))
    if nb:
        bad[key] += 1
        j = int(np.flatnonzero(got != want)[0]) // 2
        print(f"MISMATCH it={it} {key}: {nb} ends; read {j} got {got[2*j:2*j+2]} want {want[2*j:2*j+2]}", flush=True)
    if it % 13 == 0:
        idxs[g].free_gpu()
    if it % 500 == 0:
        print(f"it {it} {time.time()-t0:.0f}s calls {sum(calls.values())} bad {sum(bad.values())}", flush=True)
print("tally (backend, K, d, ftab): bad / calls", flush=True)
for key in sorted(calls):
    if bad[key]:
        print(" ", key, bad[key], "/", calls[key])
print(f"done: {sum(calls.values())} calls, {sum(bad.values())} bad", flush=True)
