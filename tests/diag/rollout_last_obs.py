"""Diagnostic: after DeviceRolloutBuffer.collect, is the env's obs buffer the obs after the last step, and is
rb.value V(that obs)?  (A twin batch replays the stored actions.)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "rl-cattle-herding_amd"))
from cattleherd.env import HerdBatch  # noqa: E402
from cattleherd.policy import DevicePolicy  # noqa: E402
from cattleherd.rollout import DeviceRolloutBuffer  # noqa: E402

E, n, m, T = 512, 4, 16, int(sys.argv[1]) if len(sys.argv) > 1 else 5
sc = 4800 - 30 + (np.arange(E) % 60)


def make():
    bb = HerdBatch(E, n, m, mode="ctde", curriculum_level=2, compat=True)
    bb.reset()
    bb.set_state({"step_counter": sc})
    return bb


b = make()
A = 4 * n
actor = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, A], seed=1), "tanh", None)
critic = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 1], seed=2), "tanh", None)
log_std = torch.full((A,), -1.0, device=b.device)
rb = DeviceRolloutBuffer(b, T)
rb.collect(actor, critic, log_std, seed=123)
torch.cuda.synchronize()
b2 = make()
for t in range(T):
    same = torch.equal(b2.obs.view(E, -1), rb.obs[t])
    b2.step(rb.actions[t].clamp(-1.0, 1.0).view(E, n, 4), autoreset=True, terminal_obs=True)
    print("t", t, "obs[t] equal", same)
d = (b.obs.view(E, -1) - b2.obs.view(E, -1)).abs()
print("final obs: max diff", float(d.max()), "envs differing", int((d.max(1).values > 0).sum()))
bad = (d > 0).nonzero()
print("first differing (env, col):", bad[:12].tolist())
v = critic.forward(b.obs.view(E, -1))[:, 0]
vr = critic.reference(b2.obs.view(E, -1))[:, 0]
print("rb.value vs V(b.obs) max", float((rb.value[:, 0] - v).abs().max()), "vs torch V(b2.obs)", float((rb.value[:, 0] - vr).abs().max()))
vb = critic.forward_batch(b)[:, 0]
vprev = critic.forward(rb.obs[T - 1])[:, 0]
print("rb.value vs forward_batch(b)", float((rb.value[:, 0] - vb).abs().max()), "vs V(obs[T-1])",
      float((rb.value[:, 0] - vprev).abs().max()), "forward_batch vs forward", float((vb - v).abs().max()))
print("envs where rb.value != V(b.obs):", int(((rb.value[:, 0] - v).abs() > 1e-5).sum()), "of", E)
