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


def trace(T=3):
    """k_mlp2 phase clocks (ch__set_mlp_tstamp) of the fused forward: the last fused step of a T-step collection,
    wave 0 of every workgroup, cycles from the forward's start; beside them the separate actor forward's."""
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceRolloutBuffer
    L = _lib.lib()
    L.ch__set_mlp_tstamp.argtypes = [ctypes.c_void_p]
    d = np.load(os.path.join(ROOT, "tests", "golden", "policy_ctde_v16_6.npz"))
    sd = {k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k}
    actor, critic = DevicePolicy.sb3_actor(sd, clip=False), DevicePolicy.sb3_critic(sd)
    b = HerdBatch(4096, 4, 16, mode="ctde")
    b.reset()
    for _ in range(300):
        b.step(None, random_actions=True, autoreset=True, terminal_obs=False)
    ts = torch.zeros(2 * 256 * 16, dtype=torch.int64, device=b.device)
    names = ["start", "w issued", "x issued", "x stored", "staged", "L0 loop", "L0 done", "L1 loop", "L1 done",
             "L2 loop", "end"]
    rb = DeviceRolloutBuffer(b, T, act_dim=48)
    log_std = torch.full((48,), -1.0, device=b.device)
    for path in (4, 4, 8):
        assert L.ch__set_rollout_path(b.handle, ctypes.c_int32(path)) == 0
        if path == 8:   # the separate actor forward alone on the same observations
            y = torch.empty(4096, 48, device=b.device)
            L.ch__set_mlp_tstamp(ctypes.c_void_p(ts.data_ptr()))
            actor.forward_batch(b, y)
        else:
            L.ch__set_mlp_tstamp(ctypes.c_void_p(ts.data_ptr()))
            rb.collect(actor, critic, log_std, seed=3)
        torch.cuda.synchronize()
        L.ch__set_mlp_tstamp(None)
        tv = ts.view(2, 256, 16)[1 if path == 4 else 0].cpu().numpy().astype(np.float64)
        t = tv[:, :11]
        dd = t - t[:, :1]
        print("fused" if path == 4 else "separate", " ".join(f"{nm} {np.mean(dd[:, i]):.0f}/{np.max(dd[:, i]):.0f}"
                                                      for i, nm in enumerate(names)), flush=True)
        if path == 4:   # wall clock (100 MHz) of the fused kernel's workgroups: start, barrier, end
            w = tv[:, 13:16] * 0.01   # us
            w0 = w[:, 0].min()
            print(f"  wall us: WG start q50/max {np.median(w[:, 0] - w0):.2f}/{np.max(w[:, 0] - w0):.2f} | step part "
                  f"mean/max {np.mean(w[:, 1] - w[:, 0]):.2f}/{np.max(w[:, 1] - w[:, 0]):.2f} | barrier at q50/max "
                  f"{np.median(w[:, 1] - w0):.2f}/{np.max(w[:, 1] - w0):.2f} | forward mean/max "
                  f"{np.mean(w[:, 2] - w[:, 1]):.2f}/{np.max(w[:, 2] - w[:, 1]):.2f} | end q50/max "
                  f"{np.median(w[:, 2] - w0):.2f}/{np.max(w[:, 2] - w0):.2f}", flush=True)
            bar = w[:, 1] - w0
            late = bar > np.median(bar) + 5
            cyc = dd[:, 10]
            print(f"  late-barrier WGs {int(late.sum())}: forward wall {np.mean((w[:, 2] - w[:, 1])[late]) if late.any() else 0:.2f} "
                  f"us vs {np.mean((w[:, 2] - w[:, 1])[~late]):.2f} | forward cycles {np.mean(cyc[late]) if late.any() else 0:.0f} "
                  f"vs {np.mean(cyc[~late]):.0f} | barrier-time quantiles " +
                  " ".join(f"{q}:{np.quantile(bar, q / 100):.1f}" for q in (10, 25, 50, 75, 90, 99)), flush=True)
            print("  first 32 WGs (barrier us, forward us):", [(round(float(bar[i]), 1), round(float(w[i, 2] - w[i, 1]), 1))
                                                              for i in range(32)], flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "trace":
        return trace()
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
