"""Diagnostics: the RLlib-shaped per-agent forward (86 -> 256 -> 256 -> 8 and -> 1) on a configs[4] batch (4096 x
(4, 32): 16384 agent rows), timed alone and with the k_mlp2 phase clocks of wave 0 of every workgroup.  The row
tiles per workgroup come from CH_MLP_RT (read once per process: run one process per setting).

  CH_MLP_RT=4 python tools/mlp_marl_probe.py
  python tools/mlp_marl_probe.py --ctde      # the SB3 actor (model-v16-6) on 8192 CTDE envs: the PPO forward's kernel
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd import _lib  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402
from cattleherd.policy import DevicePolicy  # noqa: E402


def timed(fn, k=100):
    for _ in range(5):
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
    rt = int(os.environ.get("CH_MLP_RT", "0") or 0)
    ctde = "--ctde" in sys.argv
    if ctde:
        b = HerdBatch(8192, 4, 16, mode="ctde")
        b.reset()
        d = np.load(os.path.join(ROOT, "tests", "golden", "policy_ctde_v16_6.npz"))
        sd = {k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k}
        pol = DevicePolicy.sb3_actor(sd, clip=False, cache_packed=True)
        val = DevicePolicy.sb3_critic(sd, cache_packed=True)
        rows, na, flops_row = 8192, 48, 2.0 * (344 * 128 + 128 * 128 + 128 * 48)
    else:
        b = HerdBatch(4096, 4, 32, mode="marl")
        b.reset()
        pol = DevicePolicy(DevicePolicy.random_layers([86, 256, 256, 8], seed=1), "tanh", None, cache_packed=True)
        val = DevicePolicy(DevicePolicy.random_layers([86, 256, 256, 1], seed=2), "tanh", None, cache_packed=True)
        rows, na, flops_row = 4096 * 4, 8, 2.0 * (86 * 256 + 256 * 256 + 256 * 8)
    yp = torch.empty(rows, na, device=b.device)
    yv = torch.empty(rows, 1, device=b.device)
    out = {"net": "ctde actor" if ctde else "marl policy", "rt_env": rt, "policy_us": timed(lambda: pol.forward_batch(b, yp)),
           "value_us": timed(lambda: val.forward_batch(b, yv))}
    # phase clocks of one policy forward (wave 0 of each workgroup, cycles from its start)
    lib = _lib.lib()
    lib.ch__set_mlp_tstamp.argtypes = [ctypes.c_void_p]
    ts = torch.zeros(rows * 16, dtype=torch.int64, device=b.device)
    lib.ch__set_mlp_tstamp(ctypes.c_void_p(ts.data_ptr()))
    pol.forward_batch(b, yp)
    torch.cuda.synchronize()
    lib.ch__set_mlp_tstamp(None)
    t = ts.view(-1, 16).cpu().numpy().astype(np.float64)
    t = t[t[:, 0] > 0]
    d = t[:, :13] - t[:, :1]
    names = ["start", "w issued", "x issued", "x stored", "staged", "L0 loop", "L0 done", "L1 loop", "L1 done",
             "L2 loop", "end", "L0 stored", "L1 stored"]
    out["workgroups"] = int(len(t))
    out["phases_mean"] = {nm: float(np.mean(d[:, i])) for i, nm in enumerate(names)}
    out["phases_max"] = {nm: float(np.max(d[:, i])) for i, nm in enumerate(names)}
    flops = rows * flops_row
    out["policy_tflops"] = flops / (out["policy_us"] * 1e-6) / 1e12
    print(json.dumps(out), flush=True)
    b.close()


if __name__ == "__main__":
    main()
