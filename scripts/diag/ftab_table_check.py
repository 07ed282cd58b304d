"""Is the ftab table (task-ac, K=1, d=64, 12 bases) built wrong sometimes, or
is the search step wrong?  (a) all 4^12 12-mers searched with ftab 12 (the
table itself) vs without ftab, over several fresh builds; (b) the stress
batches with ftab 0 for task-ac."""
import sys, time, itertools, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import os
from pathlib import Path
import kstep_fmi as K
if os.environ.get("KFMI_DIAG_LIB"):   # an A/B library build (scripts/diag/oldpkg)
    K.LIB_PATH = Path(os.environ["KFMI_DIAG_LIB"])
from oracle import oracle
print("library", K.LIB_PATH, flush=True)
K.set_device(0)
rng = np.random.default_rng(2026)
text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=3_000_001).tobytes()
t = np.frombuffer(text, np.uint8)
idx = K.Index.build(text, k=1, d=64)
acimg = idx.alt_counters()[0].image()
codes = np.arange(4 ** 12, dtype=np.uint32)
q12 = np.frombuffer(b"ACGT", np.uint8)[((codes[:, None] >> (2 * np.arange(11, -1, -1))[None, :]) & 3)].copy()
K.set_ftab(0)
base = K.search_array(idx, q12, "task-ac")
want = oracle.search(acimg, q12)[0]
print("no-ftab 12-mers vs oracle mismatches:", int(np.sum(base != want)), flush=True)
for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    idx.free_gpu()
    K.set_ftab(12)
    got = K.search_array(idx, q12, "task-ac")
    K.set_ftab(0)
    bad = np.flatnonzero(got != want)
    print(f"build {trial}: table entries wrong: {len(set((bad // 2).tolist()))}", flush=True)
    for b in bad[:4]:
        j = b // 2
        print("   code", j, q12[j].tobytes(), "got", got[2*j:2*j+2], "want", want[2*j:2*j+2], flush=True)
def reads(n, m, seed):
    r = np.random.default_rng(seed)
    st = r.integers(0, len(text) - m, size=n)
    return np.concatenate([t[st[:, None] + np.arange(m)[None, :]], r.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(n // 4, m))])
K.set_ftab(0)
nb = 0
t0 = time.time()
calls = 0
while time.time() - t0 < 60:
    calls += 1
    q = reads(6000, 100, 10_000 + calls)
    got = K.search_array(idx, q, "task-ac")
    w = oracle.search(acimg, q)[0]
    if np.any(got != w):
        nb += 1
        b = np.flatnonzero(got != w)[0]
        print("no-ftab MISMATCH call", calls, "read", b // 2, got[b - b % 2:b - b % 2 + 2], w[b - b % 2:b - b % 2 + 2], flush=True)
    if calls % 10 == 0:
        idx.free_gpu()
print(f"no-ftab task-ac: {calls} calls, {nb} with mismatches", flush=True)
