"""Every grid-stride loop of the library iterating many times at test sizes.

The grid-stride launches (device FASTA rows `fa_rows`, the ftab build, locate's
row fill and both locate walks, the in-place index interleave) take more than
one trip round their loop only past 2^32 work-items -- more than 16 GB of reads
or positions, sizes no test reaches.  KFMI_MAX_GRID caps their grids (a test
knob, kfmi_grid.h): with 1-3 workgroups every loop runs hundreds of
iterations.  The same script runs with and without the cap and every output
(device-parsed reads searched, ftab searches, remainder reads, locate offsets
and positions, per backend) must be bit-equal, and equal to the CPU oracle.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import util

pytestmark = pytest.mark.gpu

CHILD = r"""
import hashlib, json, os, sys, tempfile
sys.path[:0] = %(paths)r
import numpy as np
import kstep_fmi as K
from oracle import oracle

K.load()
K.set_device(0)
rng = np.random.default_rng(2024)
text = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=300_007)]
idx = K.Index.build(text.tobytes(), k=2, d=64, gpu=True, sa_rate=8)
img = idx.image()
out = {}

def h(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()

# 1. device FASTA parse (fa_rows grid-stride) of 120 K reads, searched
st = rng.integers(0, text.size - 100, size=120_000)
reads = text[st[:, None] + np.arange(100)[None, :]]
want, _ = oracle.search(img, reads)
with tempfile.TemporaryDirectory() as td:
    fn = os.path.join(td, "q.fa")
    with open(fn, "wb") as f:
        f.write(b"".join(b">r%%d\r\n" %% i + r.tobytes() + b"\n" for i, r in enumerate(reads)))
    K.set_backend("task-mid")
    q = K.Queries.load_gpu(fn, 100)
    r = K.Results.alloc(reads.shape[0])
    K.transfer_to_gpu(idx, q, r)
    K.search(idx, q, r)
    K.transfer_to_cpu(r)
    out["device_parse"] = h(r.array())
    out["device_parse_ok"] = bool(np.array_equal(r.array(), want))
    q.close(); r.close()

# 2. ftab jump start (ftab_build_kernel grid-stride, 4^10 entries), two layouts;
#    "task" also runs the in-place interleave of the uploaded tag-100 entries
for be in ("task", "task-mid", "coop-mid"):
    K.set_ftab(10)
    got = K.search_array(idx, reads[:20_000], be)
    K.set_ftab(0)
    out["ftab_" + be] = h(got)
    out["ftab_ok_" + be] = bool(np.array_equal(got, want[:40_000]))

# 3. reads with m %% K != 0 (remainder table) on the same index; the oracle
#    restates the reference, which needs m %% K == 0: its K = 1 image pins them
r101 = text[st[:5_000, None] + np.arange(101)[None, :]]
i1 = K.Index.build(text.tobytes(), k=1, d=64, gpu=False)
w101, _ = oracle.search(i1.image(), r101)
got = K.search_array(idx, r101, "task-mid")
out["rem101"] = h(got)
out["rem101_ok"] = bool(np.array_equal(got, w101))

# 4. locate (row fill grid-stride + per-lane and cooperative walks), short reads
#    so that intervals hold many rows
short = text[st[:30_000, None] + np.arange(6)[None, :]]
for be, coop in (("task-mid", "1"), ("task-mid", "0"), ("task", "0")):
    os.environ["KFMI_LOCATE_COOP"] = coop
    K.set_backend(be)
    qq = K.Queries.from_array(short)
    rr = K.Results.alloc(short.shape[0])
    K.transfer_to_gpu(idx, qq, rr)
    K.search(idx, qq, rr)
    K.transfer_to_cpu(rr)
    loc = K.locate(idx, rr, 0)
    off, pos = loc.offsets(), loc.positions()
    res = rr.array().reshape(-1, 2)
    ok = bool(np.array_equal(np.diff(off), (res[:, 1] - res[:, 0]).astype(np.uint64)))
    pick = np.arange(0, short.shape[0], 97)
    for i in pick:
        p = pos[off[i]:off[i + 1]].astype(np.int64)
        ok = ok and bool((text[p[:, None] + np.arange(6)[None, :]] == short[i]).all()) and len(set(p)) == p.size
    out["locate_%%s_%%s" %% (be, coop)] = h(off) + h(pos)
    out["locate_ok_%%s_%%s" %% (be, coop)] = ok
    out["locate_total_%%s_%%s" %% (be, coop)] = int(loc.total())
    loc.close(); qq.close(); rr.close()
print(json.dumps(out))
"""


def _run(cap):
    env = dict(os.environ)
    env.pop("KFMI_MAX_GRID", None)
    if cap:
        env["KFMI_MAX_GRID"] = str(cap)
    code = CHILD % {"paths": [str(util.REPO), str(util.PKG)]}
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_grid_stride_loops_capped_equal_uncapped(kfmi_mod):
    if kfmi_mod.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    free = _run(0)
    for cap in (1, 3):
        capped = _run(cap)
        assert capped == free, {k: (free[k], capped.get(k)) for k in free if capped.get(k) != free[k]}
    for k, v in free.items():
        if "_ok" in k:
            assert v is True, k
    assert free["locate_total_task-mid_1"] > 30_000          # intervals of many rows
