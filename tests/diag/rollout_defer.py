"""Diagnostic: native ch_rollout_collect (deferred truncation bootstrap) vs the Python step loop (immediate):
per-step reward differences."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "rl-cattle-herding_amd"))
from cattleherd.env import HerdBatch  # noqa: E402
from cattleherd.policy import DevicePolicy  # noqa: E402
from cattleherd.rollout import DeviceRolloutBuffer  # noqa: E402

E, T, n, m = 256, int(sys.argv[1]) if len(sys.argv) > 1 else 24, 4, 16
sc = 4800 - 12 + (np.arange(E) % 24)
out = []
for native in (True, False):
    b = HerdBatch(E, n, m, mode="ctde", curriculum_level=2)
    b.reset()
    b.set_state({"step_counter": sc})
    actor = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 4 * n], seed=1), "tanh", None)
    critic = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 1], seed=2), "tanh", None)
    rb = DeviceRolloutBuffer(b, T)
    log_std = torch.full((4 * n,), -1.0, device=b.device)
    (rb.collect if native else rb.collect_steps)(actor, critic, log_std, seed=9)
    torch.cuda.synchronize()
    out.append((rb.rewards.cpu().numpy(), rb.episode_starts.cpu().numpy()))
    b.close()
(rn, esn), (rp, esp) = out
print("episode starts equal:", np.array_equal(esn, esp), "resets per step:", esn.sum(1).astype(int).tolist())
for t in range(T):
    d = rn[t] != rp[t]
    if d.any():
        idx = np.nonzero(d)[0]
        print(f"t {t}: {d.sum()} envs differ, e.g. env {idx[:4].tolist()} native {rn[t, idx[:4]]} python {rp[t, idx[:4]]}")
print("done")
