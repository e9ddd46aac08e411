"""ch_rollout_collect at 4096 CTDE envs on each collection path (0 default, 8 never fused, 4 fused step + actor):
random nets and the trained model-v16-6 actor / critic; prints errors and buffer equality against path 8.

  python tools/fused_probe.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))


def run(path, nets, T=6, E=4096, act_dim=16):
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    from cattleherd.rollout import DeviceRolloutBuffer
    L = _lib.lib()
    L.ch__rollout_fused_steps.restype = ctypes.c_int64
    b = HerdBatch(E, 4, 16, mode="ctde", curriculum_level=2)
    b.reset()
    b.set_state({"step_counter": 4800 - T // 2 + (np.arange(E) % T)})
    assert L.ch__set_rollout_path(b.handle, ctypes.c_int32(path)) == 0
    g, blk, lds, kv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
    L.ch__geometry(b.handle, ctypes.byref(g), ctypes.byref(blk), ctypes.byref(lds), ctypes.byref(kv))
    print(f"geometry G {g.value} block {blk.value} lds {lds.value} kernel {kv.value}", flush=True)
    rb = DeviceRolloutBuffer(b, T, act_dim=act_dim)
    log_std = torch.full((act_dim,), -1.0, device=b.device)
    try:
        rb.collect(*nets, log_std, seed=9)
        torch.cuda.synchronize()
        out = {k: getattr(rb, k).cpu() for k in ("obs", "actions", "rewards", "values", "log_probs", "returns")}
        print(f"path {path}: ok, fused steps {L.ch__rollout_fused_steps(b.handle)}", flush=True)
    except Exception as e:   # noqa: BLE001 (a probe: report and go on)
        print(f"path {path}: {type(e).__name__}: {e}", flush=True)
        out = None
    b.close()
    return out


def main():
    import torch
    from cattleherd.policy import DevicePolicy
    rnd = (DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 16], seed=1), "tanh", None),
           DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 1], seed=2), "tanh", None))
    d = np.load(os.path.join(ROOT, "tests", "golden", "policy_ctde_v16_6.npz"))
    sd = {k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k}
    sb3 = (DevicePolicy.sb3_actor(sd, clip=False), DevicePolicy.sb3_critic(sd))
    for name, nets, ad in (("random", rnd, 16), ("sb3", sb3, 48)):
        res = {p: run(p, nets, act_dim=ad) for p in (0, 8, 4)}
        if res[8] is not None and res[4] is not None:
            print(name, "fused == unfused:", {k: bool(torch.equal(res[8][k], res[4][k])) for k in res[8]}, flush=True)


if __name__ == "__main__":
    main()
