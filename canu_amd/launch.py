"""One process per GPU for the bench scripts: `--gpus N` without an external launcher.

The driver runs `python bench.py --gpus N ...` (and, for N > 1, sometimes the same line under
`torch.distributed.run`).  When no launcher set WORLD_SIZE and N > 1, the script is started
again as N ranks by `torch.distributed.run` in a CHILD process (no exec: this process has
not touched the GPU and never does), and the parent exits with the launcher's status.
Every rank then checks that the world it joined has exactly N ranks.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def needs_spawn(n_gpus: int | None, env=None) -> bool:
    """True when this process must start N ranks itself: --gpus N > 1 and no launcher."""
    env = os.environ if env is None else env
    return n_gpus is not None and n_gpus > 1 and "WORLD_SIZE" not in env


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_command(n_gpus: int, script: str, argv: list[str], port: int) -> list[str]:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n_gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            script, *argv]


def spawn_ranks(n_gpus: int, script: str, argv: list[str]) -> int:
    """Run `script argv` as n_gpus ranks (torch.distributed.run, 127.0.0.1 rendezvous) in a
    child process; returns its exit status."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on these hosts
    cmd = spawn_command(n_gpus, script, argv, free_port())
    return subprocess.call(cmd, env=env)


def world_from_env(n_gpus: int | None) -> tuple[int, int, int]:
    """(rank, world, local_rank) from the launcher's environment; a world that differs from
    an explicit --gpus N is an error, not a silent 1-GPU run."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if n_gpus is not None and world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but the launcher started a world of {world} ranks")
    return rank, world, local
