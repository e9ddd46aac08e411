"""Diagnostics: step time vs. how the flocking parity (step_counter_A mod 2) is spread over the
workgroups' envs.  'sync': every env flocks on the same steps (the state after a common reset);
'alt': consecutive envs alternate (4 of 8 per workgroup flock each step)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402


def run(kind, steps=400):
    b = HerdBatch(4096, 4, 16)
    b.reset()
    d, i = b.get_state_raw()
    E = 4096
    ints = i.reshape(10, E)
    if kind == "alt":
        ints[2] = np.arange(E) % 2
    elif kind == "rand":
        ints[2] = np.random.default_rng(0).integers(0, 2, E)
    b.set_state_raw(d, ints.reshape(-1))
    for _ in range(20):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    b.close()
    print(f"{kind}: {dt * 1e6:.2f} us/step  {4096 / dt / 1e6:.1f} M env-steps/s")


for k in ("sync", "alt", "rand", "sync"):
    run(k)
