"""Round-6 ftab experiment: the K=1, d=64 AltCounters jump-start table built
inside the library by lf_stream variants (KFMI_FTAB_DIAG, kfmi_kernels.h
ftab_diag_kernel), every 12-mer entry checked against the C oracle.  The
variant kernels existed only for the experiment (commit "ftab root cause:
in-library lf_stream variants"); they are gone from the library, which now
ignores KFMI_FTAB_DIAG -- every row of this script then times the product's
lf_stream build.  Logs: profiles/r06/ftab_var_r6[a-e].log.
  0 task step (fetch_block + lf_from_block, the round-5 build)
  1 lf_stream as is (the round-5 failing build; from r6e on, the fixed one)
  2 lf_stream + s_waitcnt vmcnt(0) after each end's loads
  3 lf_stream with volatile 4-byte plane loads (no merged 16-B load)
  4 lf_stream, entries walked in reverse grid order
  5 lf_stream with agent-scope (sc1) loads
  6 lf_stream and the dword step side by side, first difference recorded
  7 lf_stream with 16-byte-aligned loads only
 10 both ends' loads in one asm block, registers copied after each partial wait
 12 lf_stream with a compiler barrier between the 8-byte plane loads
 13 lf_stream's loads, one full vmcnt(0) before any use
 14 lf_stream, R's step before L's
 15 the old load form (merged 16-byte load at 8-byte alignment), control
"""
import os, sys, time, numpy as np
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
t0 = time.time()
want = oracle.search(acimg, q12)[0].reshape(-1, 2)
print(f"oracle table {time.time() - t0:.1f}s", flush=True)
builds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
order = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 3, 4, 5, 6, 7, 1]
for var in order:
    os.environ["KFMI_FTAB_DIAG"] = str(var)
    tot = 0
    for b in range(builds):
        idx.free_gpu()
        K.set_ftab(12)
        got = K.search_array(idx, q12, "task-ac").reshape(-1, 2)
        K.set_ftab(0)
        if var == 6:   # records of the first step where lf_stream != the dword-load step
            recs = np.flatnonzero(got[:, 0] & 0x80000000)
            r = got[recs, 0].astype(np.int64)
            f = {"t": (r >> 26) & 15, "end(1=R)": (r >> 25) & 1, "e": (r >> 24) & 1, "c": (r >> 22) & 3,
                 "b%16": (r >> 18) & 15, "o": (r >> 12) & 63, "sameblk": (r >> 11) & 1,
                 "diff": ((r & 0xFF) ^ 0x80) - 0x80}
            print(f"var 6 build {b}: {recs.size} entries with a step where lf_stream != dword step", flush=True)
            for k, a in f.items():
                u, n = np.unique(a, return_counts=True)
                print(f"   {k}: {dict(zip(u.tolist(), n.tolist()))}", flush=True)
            tot += recs.size
            continue
        if var == 10:   # VGPR copies after the partial waits vs the registers after vmcnt(0)
            recs = np.flatnonzero(got[:, 0] & 0x80000000)
            r = got[recs, 0].astype(np.int64)
            f = {"t": (r >> 26) & 15, "mask(1 Lpl,2 Rpl,4 Lc,8 Rc)": (r >> 22) & 15, "bR%16": (r >> 18) & 15,
                 "bL%16": (r >> 14) & 15, "sameblk": (r >> 13) & 1, "oR": r & 63}
            plain = np.setdiff1d(np.arange(len(got)), recs)
            wrong = int(np.sum(np.any(got[plain] != want[plain], axis=1)))
            print(f"var 10 build {b}: {recs.size} entries with a register changed after its partial wait; "
                  f"{wrong} other entries wrong", flush=True)
            for k, a in f.items():
                u, n = np.unique(a, return_counts=True)
                print(f"   {k}: {dict(zip(u.tolist(), n.tolist()))}", flush=True)
            tot += recs.size
            continue
        bad = np.flatnonzero(np.any(got != want, axis=1))
        tot += bad.size
        msg = f"var {var} build {b}: wrong entries {bad.size}"
        if bad.size:
            dl = got[bad, 0].astype(np.int64) - want[bad, 0]
            dr = got[bad, 1].astype(np.int64) - want[bad, 1]
            wg = bad // 256
            msg += (f"; dL {dict(zip(*np.unique(dl, return_counts=True)))} dR {dict(zip(*np.unique(dr, return_counts=True)))}"
                    f"; workgroups min {wg.min()} med {int(np.median(wg))} max {wg.max()} of 65536"
                    f"; lanes {sorted(set((bad % 64).tolist()))[:12]}; first {[(int(j), q12[j].tobytes().decode(), got[j].tolist(), want[j].tolist()) for j in bad[:3]]}")
        print(msg, flush=True)
    print(f"== var {var}: {tot} wrong entries in {builds} builds", flush=True)
