"""bench.py / bench_mhap.py --gpus N: the launch decision (canu_amd/launch.py), on CPU.

`python bench.py --gpus N` with no launcher must start N ranks itself (a child
torch.distributed.run, decided before anything touches the GPU), and every rank must
refuse a world that differs from N.  The end-to-end case runs a 2-rank gloo world of a tiny
script that uses the same helpers, so the spawn path itself is exercised here.
"""
from __future__ import annotations

import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from canu_amd import launch  # noqa: E402


def test_needs_spawn_decision():
    assert launch.needs_spawn(2, {})
    assert launch.needs_spawn(8, {"RANK": "0"})            # a stray RANK is no launcher
    assert not launch.needs_spawn(1, {})
    assert not launch.needs_spawn(None, {})
    assert not launch.needs_spawn(8, {"WORLD_SIZE": "8"})  # already under torch.distributed.run


def test_spawn_command_shape():
    cmd = launch.spawn_command(4, "/x/bench.py", ["--gpus", "4", "--steps", "2"], 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--master-port=29512" in cmd
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "4", "--steps", "2"]


def test_world_mismatch_is_an_error(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert launch.world_from_env(2) == (1, 2, 1)
    assert launch.world_from_env(None) == (1, 2, 1)
    with pytest.raises(SystemExit):
        launch.world_from_env(8)


def test_bench_args_defaults_per_workload():
    import bench
    a = bench.parse_args([])
    assert (a.gpus, a.reads, a.read_len, a.coverage, a.seed) == (None, 50_000, 10_000, 25.0, 1)
    b = bench.parse_args(["--workload", "configs4-rank", "--gpus", "2"])
    assert (b.gpus, b.reads, b.read_len, b.coverage, b.seed) == (2, 500_000, 12_000, 15.0, 5)


def test_cpu_share_reads_quota():
    import bench
    s = bench.cpu_share()
    assert s["usable"] >= 1 and s["usable"] <= (os.cpu_count() or 1)
    if s["quota_cpus"] is not None:
        assert s["usable"] <= max(1, int(s["quota_cpus"]))


def test_spawn_two_ranks_end_to_end(tmp_path):
    """`script --gpus 2` with no launcher prints a 2-rank world from rank 0 (gloo, CPU)."""
    script = tmp_path / "tiny.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {ROOT!r})
        from canu_amd import launch
        n = int(sys.argv[sys.argv.index('--gpus') + 1])
        if launch.needs_spawn(n):
            sys.exit(launch.spawn_ranks(n, os.path.abspath(__file__), sys.argv[1:]))
        rank, world, _ = launch.world_from_env(n)
        import torch.distributed as dist
        dist.init_process_group('gloo')
        assert dist.get_world_size() == n
        if rank == 0:
            print('WORLD', dist.get_world_size(), flush=True)
        dist.destroy_process_group()
    """))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cp = subprocess.run([sys.executable, str(script), "--gpus", "2"], capture_output=True,
                        text=True, env=env, timeout=240)
    assert cp.returncode == 0, cp.stderr[-2000:]
    assert "WORLD 2" in cp.stdout
