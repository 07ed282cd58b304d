"""Locate walks (lf_row -> lf_stream) on the K = 1, d = 64 index under the
AltCounters layout (task-ac) and the plain ones, many batches, positions
against the suffix array (from the host builder's full samples, rate 1)."""
import sys, time, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import kstep_fmi as K
K.set_device(0)
rng = np.random.default_rng(2026)
n = 3_000_001
text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=n).tobytes()
t = np.frombuffer(text, np.uint8)
full = K.Index.build(text, k=1, d=64, sa_rate=1)
sa = np.array(full.sa()[1], dtype=np.uint32)
idx = K.Index.build(text, k=1, d=64, gpu=True, sa_rate=32)
t0 = time.time(); calls = bad = 0
limit = float(sys.argv[1]) if len(sys.argv) > 1 else 90
while time.time() - t0 < limit:
    calls += 1
    b = ["task-ac", "task", "task-mid", "task-ac-mid"][calls % 4]
    st = rng.integers(0, n - 30, size=20000)
    q = t[st[:, None] + np.arange(30)[None, :]]
    res, off, pos = K.locate_array(idx, q, b)
    L = res[0::2].astype(np.int64); R = res[1::2].astype(np.int64)
    want = np.concatenate([sa[l:r] for l, r in zip(L, R)]) if len(L) else np.zeros(0, np.uint32)
    if pos.size != want.size or np.any(pos != want):
        bad += 1
        nb = int(np.sum(pos != want)) if pos.size == want.size else -1
        print("MISMATCH call", calls, b, nb, flush=True)
    if calls % 11 == 0:
        idx.free_gpu()
print(f"locate: {calls} calls, {bad} bad", flush=True)
