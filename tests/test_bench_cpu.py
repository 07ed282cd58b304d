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
    assert out["value"] > 0 and out["threads"] == 2 and out["cores"] == min(2, bench.cpu_effective())


def test_cpu_product_rows_equal_oracle(kfmi_mod):
    """bench.cpu_product_rows: the library's searchIndexCPU timed on a sample,
    equal to the oracle's results at every thread count."""
    rng = np.random.default_rng(9)
    t = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=100_001)
    idx = kfmi_mod.Index.build(t.tobytes(), k=2, d=64)
    reads = t[rng.integers(0, len(t) - 100, size=2000)[:, None] + np.arange(100)]
    want, _ = oracle.search(idx.image(), reads)
    rows = bench.cpu_product_rows(idx, reads, want, [1, 3])
    assert [r["threads"] for r in rows] == [1, 3] and all(r["equal_gpu"] and r["value"] > 0 for r in rows)
    assert [r["cores"] for r in rows] == [1, min(3, bench.cpu_effective())]


def test_cores_never_exceed_usable_cpus(monkeypatch):
    """cpu_baseline.cores is the CPUs a run actually had: the
    thread count capped by the affinity mask and the cgroup quota -- 256
    threads on a box with a 16-CPU quota report cores 16, threads 256."""
    monkeypatch.setattr(bench, "cpu_threads", lambda: 256)
    monkeypatch.setattr(bench, "cpu_quota", lambda: 16.0)
    assert bench.cpu_effective() == 16
    assert bench.baseline_thread_counts() == [256, 16]
    assert [bench.cores_used(t) for t in (256, 16, 4, 1)] == [16, 16, 4, 1]
    monkeypatch.setattr(bench, "cpu_quota", lambda: None)      # no quota: the affinity mask bounds it
    assert bench.cores_used(512) == 256 and bench.cores_used(8) == 8


def test_real_quota_bounds_cores():
    """Whatever this host's cgroup grants: every reported core count is at
    most the quota when one exists."""
    q = bench.cpu_quota()
    for t in bench.baseline_thread_counts():
        c = bench.cores_used(t)
        assert 1 <= c <= t and c <= bench.cpu_threads()
        if q:
            assert c <= max(1, int(round(q)))


def test_variant_roofline_and_pmc_file(tmp_path, monkeypatch):
    """A variant row's roofline: 36 B x distinct blocks over its LF time against
    8 TB/s, plus its fabric read requests when the committed PMC file
    (scripts/traffic_variants.py output) was taken on the same config."""
    import argparse
    import json
    a = argparse.Namespace(queries=10_000_000, ref_size=3_000_000_000, qlen=100, d=64, k=2)
    pmc = {"config": {"queries": 10_000_000, "ref_size": 3_000_000_000, "qlen": 100, "d": 64},
           "source": "x.csv", "backends": {"coop@k2": {"rdreq_per_launch": 582_000_000, "tcc_req_per_launch": 672_000_000,
                                                      "kernel_ms_under_pmc": 10.9}}}
    fn = tmp_path / "tv.json"
    fn.write_text(json.dumps(pmc))
    monkeypatch.setattr(bench, "VARIANTS_PMC", fn)
    got = bench.load_variants_pmc(a.queries, a.ref_size, a.qlen, a.d)
    assert got == pmc
    r = bench.variant_roofline(578_600_000, 36, 10.9, a, "coop", got, 56.0)
    assert r["bytes_per_launch"] == 578_600_000 * 36
    assert abs(r["frac"] - 578_600_000 * 36 / 10.9e-3 / 8e12) < 1e-4
    assert r["line_requests_per_query"] == 58.2 and "line_request_frac" not in r
    assert r["traffic"] == 582_000_000 * 128                 # one 128-B request per random L2 miss
    # fabric line bytes are labelled as such, never as an HBM fraction
    assert abs(r["l2_fabric_line_bytes_vs_8TBs_incl_ic_hits"] - 582e6 * 128 / 10.9e-3 / 8e12) < 1e-4
    assert not any("hbm" in k.lower() for k in r)
    assert "fabric_read_requests_per_launch" not in bench.variant_roofline(1, 36, 1.0, a, "task", got, 56.0)
    a.queries = 1_000_000                                # another config: the file does not apply
    assert bench.load_variants_pmc(a.queries, a.ref_size, a.qlen, a.d) is None
    # config #5's pass (150 bp) is its own file, keyed by its own shape
    assert bench.load_variants_pmc(10_000_000, 3_000_000_000, 150, 64, fn) is None


def test_traffic_variants_parser(tmp_path):
    """scripts/traffic_variants.py cuts the LF launches of a PMC pass into the
    order file's runs and checks each run's kernel against its backend."""
    import csv
    import json
    import subprocess
    import sys
    from util import REPO
    order = {"queries": 1000, "ref_size": 5000, "qlen": 100, "d": 64,
             "order": [{"backend": "task-mid", "k": 2, "launches": 3, "warmup": 1, "lf_ms_hip_events": 1.0,
                        "distinct_blocks": 5},
                       {"backend": "coop-grp", "k": 4, "launches": 2, "warmup": 1, "lf_ms_hip_events": 0.5,
                        "distinct_blocks": 4}]}
    (tmp_path / "order.json").write_text(json.dumps(order))
    names = ["void kfmi::task_kernel<kfmi::Geo<2, 2, 3>, 1, 8, 8>(kfmi::IdxArgs)"] * 3 + \
            ["void kfmi::coop_kernel<kfmi::Geo<4, 2, 6>, 8>(kfmi::IdxArgs)"] * 2
    with open(tmp_path / "p.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value",
                                          "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for i, n in enumerate(names):
            for cn, v in (("TCC_EA0_RDREQ_sum", 100 + i), ("TCC_REQ_sum", 200 + i)):
                w.writerow({"Dispatch_Id": 10 + i, "Kernel_Name": n, "Grid_Size": 1024, "Counter_Name": cn,
                            "Counter_Value": v, "Start_Timestamp": 0, "End_Timestamp": 1_000_000})
        w.writerow({"Dispatch_Id": 99, "Kernel_Name": "void kfmi::build_mid_kernel<2, 2>()", "Grid_Size": 1024,
                    "Counter_Name": "TCC_EA0_RDREQ_sum", "Counter_Value": 1, "Start_Timestamp": 0, "End_Timestamp": 1})
    p = subprocess.run([sys.executable, str(REPO / "scripts" / "traffic_variants.py"), str(tmp_path / "p.csv"),
                        str(tmp_path / "order.json"), "--source", "t"], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    out = json.loads(p.stdout)
    assert out["backends"]["task-mid@k2"]["rdreq_per_launch"] == 101      # median of launches 2, 3 (101, 102)
    assert out["backends"]["coop-grp@k4"]["rdreq_per_launch"] == 104 and out["backends"]["coop-grp@k4"]["launches_timed"] == 1


def test_probe_rows_and_best_of_runs():
    """gather_probe output: only the main table's rows count (the 4 MB / 200 MB
    tables the tool probes afterwards are dropped), and repeated runs keep each
    kind's fastest row -- the ceiling is the max over repeats."""
    import json
    want = int(0.2e9) & ~127

    def out(rate_a, rate_b):
        return "\n".join([json.dumps({"table_bytes": want}),
                          json.dumps({"kind": "chain1", "line_B": 128, "Glines_s": rate_a}),
                          "not json",
                          json.dumps({"kind": "indep", "line_B": 64, "Glines_s": rate_b}),
                          json.dumps({"table_bytes": 4 << 20}),
                          json.dumps({"kind": "indep", "line_B": 64, "Glines_s": 172.0})])
    t1, r1 = bench.probe_rows(out(54.1, 54.3), "0.2")
    t2, r2 = bench.probe_rows(out(54.9, 53.9), "0.2")
    assert t1 == t2 == want and len(r1) == len(r2) == 2
    best = {(r["kind"], r["line_B"]): r["Glines_s"] for r in bench.best_of_runs([r1, r2])}
    assert best == {("chain1", 128): 54.9, ("indep", 64): 54.3}
    assert bench.probe_rows(out(1, 1), "3") == (None, [])


def test_replay_requests_from_committed_counts():
    """Replay request rates: a mode the PMC pass counted uses its count, the
    others the median of the counted modes; the best mode is the fastest rate."""
    replay = [{"unroll": 1, "groups": 1, "ms": 10.0}, {"unroll": 4, "groups": 2, "ms": 9.5},
              {"unroll": 8, "groups": 2, "ms": 9.0}]
    pmc = {"rdreq_per_launch": {"u1g1": 540_000_000, "u4g2": 538_000_000, "u0g2": 539_000_000}}
    rp = bench.replay_requests(replay, pmc)
    assert rp["requests"] == {"u1g1": 540_000_000, "u4g2": 538_000_000, "u8g2": 539_000_000}
    assert rp["G_requests_per_s"]["u1g1"] == 54.0 and rp["best_mode"] == "u8g2"
    assert rp["best_G_requests_per_s"] == round(539e6 / 9.0e-3 / 1e9, 2)
    assert bench.replay_requests(None, pmc) is None and bench.replay_requests(replay, {}) is None


def test_committed_traffic_profile_carries_replay_counts():
    import json
    tr = json.loads((bench.ROOT / "profiles" / "traffic.json").read_text())
    assert tr["backend"] == "task-mid" and tr["rdreq_per_launch"] > 0
    c = tr["replay"]["rdreq_per_launch"]
    # every replay mode re-issues the kernel's lines plus its trace stream
    assert all(v > tr["rdreq_per_launch"] for v in c.values())


def test_committed_traffic_is_the_guides_fetch_size_recipe():
    """roofline.traffic: FETCH_SIZE (KB) x 1024 x 2 (gfx950 tallies a 128-B
    request at 64 B), consistent with the request-size pass: every request of
    the LF kernel is 128 B, so the bytes equal TCC_EA0_RDREQ x 128 within 0.1 %."""
    import json
    tr = json.loads((bench.ROOT / "profiles" / "traffic.json").read_text())
    b = tr["fetch_size_corrected_bytes_per_launch"]
    assert b == round(tr["fetch_size_kb_per_launch"] * 2048)
    sz = tr["request_sizes_per_launch"]
    assert sz["TCC_EA0_RDREQ_128B"] / sz["TCC_EA0_RDREQ"] > 0.9999
    assert abs(b - sz["TCC_EA0_RDREQ"] * 128) / b < 1e-3
    assert abs(sz["TCC_EA0_RDREQ"] - tr["rdreq_per_launch"]) / tr["rdreq_per_launch"] < 1e-3
