"""Diagnostics: the device PPO collection (DeviceRolloutBuffer.collect, C4, T = 32) launched eagerly from the host
vs captured once into a HIP graph and replayed -- how much of a collection step is host launch overhead."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402
from cattleherd.policy import DevicePolicy  # noqa: E402
from cattleherd.rollout import DeviceRolloutBuffer  # noqa: E402

E, n, m, T = 4096, 4, 16, 32
d = np.load(os.path.join(ROOT, "tests", "golden", "policy_ctde_v16_6.npz"))
sd = {k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k}
actor, critic = DevicePolicy.sb3_actor(sd, clip=False), DevicePolicy.sb3_critic(sd)
b = HerdBatch(E, n, m)
b.reset()
rb = DeviceRolloutBuffer(b, T, act_dim=48)
log_std = torch.full((48,), -1.0, device=b.device)
for _ in range(2):
    rb.collect(actor, critic, log_std, seed=1)
torch.cuda.synchronize()
reps = 5
t0 = time.perf_counter()
for i in range(reps):
    rb.collect(actor, critic, log_std, seed=2 + i)
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / reps / T * 1e6
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(side):
    with torch.cuda.graph(g, stream=side):
        rb.collect(actor, critic, log_std, seed=7)
torch.cuda.current_stream().wait_stream(side)
g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(reps):
    g.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t0) / reps / T * 1e6
print(f"PPO collection at C4: eager {eager:.1f} us/step ({E / eager:.1f} M env-steps/s), "
      f"graph replay {graph:.1f} us/step ({E / graph:.1f} M env-steps/s)", flush=True)
