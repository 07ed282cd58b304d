"""Repeated device derivations (derive_codes_kernel: one lf_stream per row)
against the index built from the text, byte for byte."""
import sys, time, hashlib, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "k-step_fm-index_amd"); sys.path.insert(0, ".")
import kstep_fmi as K
K.set_device(0)
rng = np.random.default_rng(11)
text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=3_000_001).tobytes()
src = {1: K.Index.build(text, k=1, d=64), 2: K.Index.build(text, k=2, d=64)}
want = {2: hashlib.md5(bytes(src[2].image())).hexdigest(),
        4: hashlib.md5(bytes(K.Index.build(text, k=4, d=64).image())).hexdigest()}
t0 = time.time(); n = bad = 0
while time.time() - t0 < float(sys.argv[1]) if len(sys.argv) > 1 else 90:
    kin = 1 + (n % 2)
    g = src[kin].derive(2 * kin, host_image=True)
    h = hashlib.md5(bytes(g.image())).hexdigest()
    g.close()
    n += 1
    if h != want[2 * kin]:
        bad += 1
        print("MISMATCH derive", kin, "->", 2 * kin, "iteration", n, flush=True)
print(f"derive: {n} derivations, {bad} differ", flush=True)
