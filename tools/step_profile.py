"""Diagnostics: per-window step time over a long random-action rollout (4096 x (4,16) CTDE f64),
with the share of envs flocking and the resets per window."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402

b = HerdBatch(4096, 4, 16)
b.reset()
W = 100
for w in range(24):
    resets = torch.zeros((), dtype=torch.int64, device=b.device)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(W):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / W
    st = b.get_state()
    flk = ((st["step_counter_A"] + 1) % 2 == 0).mean()
    print(f"steps {w * W:5d}-{(w + 1) * W:5d}: {dt * 1e6:6.2f} us/step | next-step flocking share {flk:.2f} | "
          f"episode mean {st['episode'].mean():.2f} | n mean {st['n'].mean():.2f} | level mean {st['level'].mean():.2f}")
b.close()
