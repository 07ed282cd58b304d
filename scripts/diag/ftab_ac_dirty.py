"""test_ftab_jump_start_equals_oracle[task-ac-12] after dirtying device memory:
fill and free most of the card with a byte pattern, then search."""
import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import torch
import kstep_fmi as K
from oracle import oracle
pat = int(sys.argv[1], 0) if len(sys.argv) > 1 else 0xFF
bufs = []
for _ in range(40):   # 40 x 4 GiB = 160 GiB of the pattern
    b = torch.empty(4 << 30, dtype=torch.uint8, device="cuda:0")
    b.fill_(pat)
    bufs.append(b)
torch.cuda.synchronize()
del bufs
torch.cuda.empty_cache()
K.set_device(0)
rng = np.random.default_rng(2026)
text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=3_000_001).tobytes()
t = np.frombuffer(text, np.uint8)
def reads(n, m, seed):
    r = np.random.default_rng(seed)
    st = r.integers(0, len(text) - m, size=n)
    return np.concatenate([t[st[:, None] + np.arange(m)[None, :]], r.choice(np.frombuffer(b"ACGTNacgt", np.uint8), size=(n // 4, m))])
for k, d in ((1, 64), (2, 64), (2, 192)):
    idx = K.Index.build(text, k=k, d=d)
    a200 = idx.alt_counters()[0]
    for bases in (0, 2, 8, 12):
        for m in (100, 150, max(bases, k)):
            if m % k:
                continue
            q = reads(3000, m, m + 31 * k + bases)
            want_ac, _ = oracle.search(a200.image(), q)
            want, _ = oracle.search(idx.image(), q)
            K.set_ftab(bases)
            for b in ("task-ac", "task", "task-mid", "coop", "coop-mid",
                      "task-ac-mid", "coop-ac-mid"):
                if b.startswith("coop") and (2 * (d // 32) * k) % 4:
                    continue
                try:
                    got = K.search_array(idx, q, b)
                except K.KfmiError as e:
                    print("refused", b, k, d, e.code)
                    continue
                w = want_ac if "ac" in b else want
                nb = int(np.sum(got != w))
                if nb:
                    bad = np.flatnonzero(got != w)
                    j = bad[0] // 2
                    print(f"MISMATCH {b} k={k} d={d} ftab={bases} m={m}: {nb} ends; first read {j} got {got[2*j:2*j+2]} want {w[2*j:2*j+2]} tail {q[j].tobytes()[-14:]}", flush=True)
            K.set_ftab(0)
    idx.close()
print("done pattern", hex(pat), flush=True)
