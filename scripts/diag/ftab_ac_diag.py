"""Diagnose test_ftab_jump_start_equals_oracle[task-ac-12] (K=1, d=64, m=100)."""
import sys, numpy as np
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
idx = K.Index.build(text, k=1, d=64)
a200 = idx.alt_counters()[0]
q = reads(6000, 100, 100 + 31 + 12)
want, _ = oracle.search(a200.image(), q)
for trial in range(3):
    for bases in (0, 12, 8, 11, 12):
        K.set_ftab(bases)
        got = K.search_array(idx, q, "task-ac")
        bad = np.flatnonzero(got != want)
        print("trial", trial, "ftab", bases, "mismatches", bad.size, flush=True)
        if bad.size:
            for b in bad[:6]:
                j = b // 2
                print("  read", j, "end", b % 2, "got", got[b], "want", want[b], "read", q[j].tobytes()[-14:], flush=True)
    # another index object: fresh upload, fresh ftab
    idx.free_gpu()
K.set_ftab(0)
for b in ("task-mid", "task", "coop-ac-mid", "task-ac-mid"):
    K.set_ftab(12)
    got = K.search_array(idx, q, b)
    w = want if "ac" in b else oracle.search(idx.image(), q)[0]
    print(b, "ftab12 mismatches", int(np.sum(got != w)), flush=True)
K.set_ftab(0)
