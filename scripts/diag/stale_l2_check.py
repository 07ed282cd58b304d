"""After a device copy is freed and re-made, does the first kernel that reads
it see stale data?  Loop: free the handle's device copy (index lines + a
134 MB ftab table), search all 4^12 12-mers WITHOUT ftab (the search kernel is
the first reader of the re-uploaded lines), then with ftab 12; both against
the oracle."""
import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import kstep_fmi as K
from oracle import oracle
K.set_device(0)
rng = np.random.default_rng(2026)
text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=3_000_001).tobytes()
idx = K.Index.build(text, k=1, d=64)
acimg = idx.alt_counters()[0].image()
codes = np.arange(4 ** 12, dtype=np.uint32)
q12 = np.frombuffer(b"ACGT", np.uint8)[((codes[:, None] >> (2 * np.arange(11, -1, -1))[None, :]) & 3)].copy()
want = oracle.search(acimg, q12)[0]
backend = sys.argv[2] if len(sys.argv) > 2 else "task-ac"
for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    idx.free_gpu()
    K.set_ftab(0)
    a = K.search_array(idx, q12, backend)
    K.set_ftab(12)
    b = K.search_array(idx, q12, backend)
    K.set_ftab(0)
    print(f"{backend} trial {trial}: no-ftab wrong {int(np.sum(a != want))}, ftab12 wrong {int(np.sum(b != want))}", flush=True)
