"""bench.py's cpu_baseline legs on a small case (no GPU): the reference's own
CPU searcher (oracle/_ref/cpu_<K>_<d>, built from /root/reference sources) run
through its file interface agrees with the oracle restatement."""
import numpy as np
import pytest

import bench
from oracle import oracle


@pytest.mark.parametrize("k", [1, 2])
def test_reference_cpu_baseline_matches_oracle(kfmi_mod, k):
    if not (oracle.REF_DIR / f"cpu_{k}_64").exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    rng = np.random.default_rng(k)
    text = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=200_001).tobytes()
    idx = kfmi_mod.Index.build(text, k=k, d=64)
    t = np.frombuffer(text, dtype=np.uint8)
    reads = t[rng.integers(0, len(t) - 100, size=3000)[:, None] + np.arange(100)]
    want, _ = oracle.search(idx.image(), reads)
    out = bench.cpu_reference_baseline(idx, reads, 2000, k, 64, 2, want)
    assert out is not None and out["kind"] == "reference" and out["parity_with_gpu"]
    assert out["value"] > 0
