"""The committed PMC figures (profiles/traffic*.json, tools/pmc_traffic.py / pmc_mhap.py) are
keyed to the workload and the kernel sources they were taken on, and bench.py /
bench_mhap.py report `traffic: null` for any other pair.  These checks fail when a kernel
source changes without new counter passes, so a bench line never prices a kernel with
another build's bytes, and never silently drops them either."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def test_overlapincore_traffic_matches_sources_and_workloads(monkeypatch):
    import bench
    monkeypatch.delenv("CANU_C4_PLAN", raising=False)
    # the default line and the configs4-rank side line exactly as bench.py runs them
    for argv, cls in ((["--steps", "1"], bench.Configs2),
                      (["--workload", "configs4-rank", "--steps", "1", "--warmup", "1",
                        "--no-cpu-baseline", "--no-side"], bench.Configs4Rank)):
        job = cls(bench.parse_args(argv), 0, 1, None)
        traffic, note = bench.load_traffic(job, 1)
        assert traffic, note
        assert traffic["_method"]["src_sha"] == bench.source_hash()
        assert traffic["k_extend"]["hbm_bytes_per_launch"] > 0


def test_overlapincore_traffic_unused_at_n_gt_1():
    import bench
    job = bench.Configs2(bench.parse_args([]), 0, 2, None)
    traffic, note = bench.load_traffic(job, 2)
    assert traffic == {} and "N > 1" in note


def test_mhap_traffic_matches_sources_and_workload():
    import bench_mhap
    args = bench_mhap.parse_args(["--steps", "1", "--warmup", "1", "--no-cpu-baseline"])
    t, note = bench_mhap.load_pmc(args, 1)
    assert t is not None, note
    assert t["_method"]["src_sha"] == bench_mhap.mhap_source_hash()
