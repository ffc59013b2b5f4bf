"""`--gpus N` for the bench scripts: one child process per rank.

The driver may run `python bench.py --gpus N` directly instead of through
torch.distributed.run.  Then the parent, BEFORE any GPU call (it never imports
torch), starts N children of the same script with the rank environment
torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE,
LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), waits for them and exits
with the first failing status.  It never replaces itself (no exec): the
children are ordinary subprocesses.  Under torch.distributed.run (WORLD_SIZE
set) the world size must equal --gpus, else the run fails loudly instead of
measuring the wrong number of GPUs.

The reference's own shape is a spawn pool over np.array_split chunks
(dgen_os/python/dgen_model.py:312-328); here one rank is one GPU.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence, Tuple


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def rank_envs(n: int, port: int, base: Optional[Dict[str, str]] = None) -> List[Dict[str, str]]:
    """The N rank environments (torch.distributed.run's variables, one node)."""
    base = dict(os.environ if base is None else base)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this host driver
    out = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                  "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(port)})
        out.append(e)
    return out


def launch_plan(n: int, script: str, argv: Sequence[str], port: Optional[int] = None,
                base: Optional[Dict[str, str]] = None) -> List[Tuple[List[str], Dict[str, str]]]:
    """(command, environment) of every rank child."""
    port = free_port() if port is None else int(port)
    cmd = [sys.executable, "-u", os.path.abspath(script), *argv]
    return [(list(cmd), e) for e in rank_envs(n, port, base)]


def check_world(gpus: int) -> Optional[int]:
    """None: this process is a rank (or the single-GPU run) and goes on.
    An int: the status to exit with (a world-size mismatch)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != int(gpus):
        print(f"error: --gpus {gpus} but WORLD_SIZE={ws}: launch one rank per GPU "
              f"(torch.distributed.run --nproc-per-node {gpus}) or drop WORLD_SIZE", file=sys.stderr, flush=True)
        return 2
    return None


def run_ranks(plan: List[Tuple[List[str], Dict[str, str]]], poll_s: float = 0.2) -> int:
    """Start every rank, wait; on the first failure end the others (their own
    process groups, by PID) and return that status."""
    procs = [subprocess.Popen(cmd, env=env, start_new_session=True) for cmd, env in plan]
    status = 0
    try:
        live = set(range(len(procs)))
        while live:
            for i in sorted(live):
                rc = procs[i].poll()
                if rc is None:
                    continue
                live.discard(i)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"error: rank {i} exited with {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for j in live:
                        _stop(procs[j])
            if live:
                time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            _stop(p)
        raise
    return status


def _stop(p: subprocess.Popen) -> None:
    if p.poll() is not None:
        return
    try:
        os.killpg(p.pid, signal.SIGTERM)
    except (ProcessLookupError, PermissionError):
        return
    try:
        p.wait(timeout=20)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            pass


def maybe_launch(gpus: int, script: str, argv: Sequence[str]) -> Optional[int]:
    """Call first thing in main(), before torch is imported.  Returns None
    when this process should run the benchmark itself, else the exit status
    of the N-rank launch (or of a world-size mismatch)."""
    bad = check_world(gpus)
    if bad is not None:
        return bad
    if os.environ.get("WORLD_SIZE") is not None or int(gpus) <= 1:
        return None
    return run_ranks(launch_plan(int(gpus), script, argv))
