"""Diagnostics: the policy forward (ch_policy_forward / ch_mlp_forward) alone, for rocprofv3 and timing.

usage: python tools/mlp_probe.py [reps]            # model-v16-6 actor on a 4096-env CTDE batch
       python tools/mlp_probe.py sweep             # forward time vs rows (dense inputs, ch_mlp_forward)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402
from cattleherd.policy import DevicePolicy  # noqa: E402


def actor():
    d = np.load(os.path.join(ROOT, "tests", "golden", "policy_ctde_v16_6.npz"))
    return DevicePolicy.sb3_actor({k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k})


def timed(fn, k=200):
    for _ in range(10):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(k):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / k * 1000.0


def main():
    a = actor()
    if len(sys.argv) > 1 and sys.argv[1] == "sweep":
        for rows in (16, 256, 1024, 4096, 16384, 65536):
            x = torch.randn(rows, 1032, device="cuda") * 0.1
            y = torch.empty(rows, 48, device="cuda")
            print(f"rows {rows}: dense 1032-wide forward {timed(lambda: a.forward(x, y)):.2f} us", flush=True)
        return
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    b = HerdBatch(4096, 4, 16)
    b.reset()
    y = torch.empty(4096, 48, device=b.device)
    print(f"batch forward (live width 344): {timed(lambda: a.forward_batch(b, y), reps):.2f} us", flush=True)


if __name__ == "__main__":
    main()
