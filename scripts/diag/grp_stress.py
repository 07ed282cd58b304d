"""Intermittent-result hunt on the grouped-counter layout: task-grp / coop-grp at
K = 3 and 4 (and a K = 2 file derived on upload), ftab 0 / 4 / 8 / 12 bases,
read lengths with and without remainders, re-uploads; oracle = the K = 1
restatement (the reads' suffix-array intervals)."""
import sys, time, collections, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import kstep_fmi as K
from oracle import oracle
K.set_device(0)
rng = np.random.default_rng(9)
text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=2_000_003).tobytes()
t = np.frombuffer(text, np.uint8)
idxs = {3: K.Index.build(text, k=3, d=64, gpu=True), 4: K.Index.build(text, k=4, d=64, gpu=True),
        2: K.Index.build(text, k=2, d=64)}
img1 = K.Index.build(text, k=1, d=64).image()
calls = collections.Counter(); bad = collections.Counter()
t0 = time.time(); it = 0
while time.time() - t0 < float(sys.argv[1]) if len(sys.argv) > 1 else 120:
    it += 1
    k = [3, 4, 2][it % 3]
    b = ["task-grp", "coop-grp"][(it // 3) % 2]
    m = int(rng.choice([96, 99, 100, 101, 150, 151, 33]))
    ft = int(rng.choice([0, 4, 8, 12]))
    st = rng.integers(0, len(text) - m, size=4000)
    q = np.concatenate([t[st[:, None] + np.arange(m)[None, :]], rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=(400, m))])
    K.set_ftab(ft)
    got = K.search_array(idxs[k], q, b)
    K.set_ftab(0)
    want = oracle.search(img1, q)[0]
    key = (b, k, ft)
    calls[key] += 1
    if np.any(got != want):
        bad[key] += 1
        j = int(np.flatnonzero(got != want)[0]) // 2
        print(f"MISMATCH it={it} {key} m={m}: read {j} got {got[2*j:2*j+2]} want {want[2*j:2*j+2]}", flush=True)
    if it % 17 == 0:
        idxs[k].free_gpu()
print({str(k): (bad[k], v) for k, v in sorted(calls.items())})
print(f"done: {sum(calls.values())} calls, {sum(bad.values())} bad", flush=True)
