"""Stress the configuration of the one intermittent mismatch seen in session P
(test_ftab_jump_start_equals_oracle[task-ac-12]: task-ac, ftab 12, K=1, d=64,
m=100): many batches, re-uploads, interleaved backends and table sizes."""
import sys, time, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import kstep_fmi as K
from oracle import oracle
K.set_device(0)
rng = np.random.default_rng(2026)
text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=3_000_001).tobytes()
t = np.frombuffer(text, np.uint8)
def reads(n, m, seed):
    r = np.random.default_rng(seed)
    st = r.integers(0, len(text) - m, size=n)
    return np.concatenate([t[st[:, None] + np.arange(m)[None, :]], r.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(n // 4, m))])
idxs = {(1, 64): K.Index.build(text, k=1, d=64), (2, 64): K.Index.build(text, k=2, d=64)}
acimg = {kd: i.alt_counters()[0].image() for kd, i in idxs.items()}
t0 = time.time()
total = bad_calls = 0
it = 0
while time.time() - t0 < float(sys.argv[1]) if len(sys.argv) > 1 else 120:
    it += 1
    kd = (1, 64) if it % 3 else (2, 64)
    idx = idxs[kd]
    bases = int(rng.choice([2, 8, 12, 12, 12, 11]))
    if bases % kd[0]:
        bases = 12
    m = int(rng.choice([100, 150, 100]))
    q = reads(6000, m, it)
    b = str(rng.choice(["task-ac", "task-ac", "task", "task-mid", "coop-ac-mid"]))
    K.set_ftab(bases)
    want = oracle.search(acimg[kd] if "ac" in b else idx.image(), q)[0]
    got = K.search_array(idx, q, b)
    K.set_ftab(0)
    total += 1
    nb = int(np.sum(got != want))
    if nb:
        bad_calls += 1
        bad = np.flatnonzero(got != want)
        j = bad[0] // 2
        print(f"MISMATCH it={it} {b} kd={kd} ftab={bases} m={m}: {nb} ends in {len(set(bad // 2))} reads; read {j} got {got[2*j:2*j+2]} want {want[2*j:2*j+2]}", flush=True)
    if it % 7 == 0:
        idx.free_gpu()
    if it % 25 == 0:
        print(f"it {it}: {total} calls, {bad_calls} with mismatches, {time.time()-t0:.0f}s", flush=True)
print(f"done: {total} calls, {bad_calls} with mismatches", flush=True)
