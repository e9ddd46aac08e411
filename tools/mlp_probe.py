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
    if len(sys.argv) > 1 and sys.argv[1] == "trace":
        return trace()
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


def trace():
    """k_mlp2 phase clocks (ch__set_mlp_tstamp): wave 0 of every workgroup, cycles from its start."""
    import ctypes
    from cattleherd import _lib
    a = actor()
    b = HerdBatch(4096, 4, 16)
    b.reset()
    y = torch.empty(4096, 48, device=b.device)
    ts = torch.zeros(256 * 16, dtype=torch.int64, device=b.device)
    lib = _lib.lib()
    lib.ch__set_mlp_tstamp.argtypes = [ctypes.c_void_p]
    for _ in range(20):
        a.forward_batch(b, y)
    for rep in range(4):
        packed = rep % 2 == 0
        a._net.packed = a._packed.data_ptr() if packed else None
        lib.ch__set_mlp_tstamp(ctypes.c_void_p(ts.data_ptr()))
        a.forward_batch(b, y)
        torch.cuda.synchronize()
        t = ts.view(256, 16).cpu().numpy().astype(np.float64)[:, :11]
        d = t - t[:, :1]
        names = ["start", "x issued", "w issued", "x stored", "staged", "L0 loop", "L0 done", "L1 loop", "L1 done",
                 "L2 loop", "end"]
        print("rep", rep, "packed" if packed else "raw", " ".join(f"{nm} {np.mean(d[:, i]):.0f}/{np.max(d[:, i]):.0f}" for i, nm in enumerate(names)),
              flush=True)
    lib.ch__set_mlp_tstamp(None)
    for packed in (True, False):
        a._net.packed = a._packed.data_ptr() if packed else None
        print(f"forward (timed, {'packed' if packed else 'raw'} weights): {timed(lambda: a.forward_batch(b, y)):.2f} us",
              flush=True)
    a._net.packed = a._packed.data_ptr()


if __name__ == "__main__":
    main()
