"""One process per GPU from a plain ``python bench.py --gpus N`` (no torchrun needed).

The reference runs one env per OS process (SB3 ``SubprocVecEnv``, simulator/CTDECattleHerder.py:91-97).
Here the unit of a process is a whole GPU's worth of envs: ``spawn_ranks`` starts N copies of a script
with the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) set,
before the parent has touched the GPU, and returns the first non-zero exit status.  If one rank dies
the others are stopped (they would otherwise wait in the rendezvous), by their exact PIDs.

This module must not import torch: the parent never initialises HIP.
"""
import os
import socket
import subprocess
import sys
import time


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank, world, port, base=None):
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
    return env


def spawn_ranks(n, script, argv, timeout=None):
    """Run ``python script *argv`` as ranks 0..n-1 of one node; returns the exit status for the parent."""
    port = free_port()
    procs = [subprocess.Popen([sys.executable, script, *argv], env=rank_env(r, n, port)) for r in range(n)]
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                print(f"launch: ranks did not finish within {timeout} s", file=sys.stderr)
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc
