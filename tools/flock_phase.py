"""The flock phase of the step kernel on its own (SURVEY §8(d) "flock kernel"):
per-launch time of k_step2 with the drone chain, task and observation phases skipped
(ch__set_phase_mask 1|4|8 = 13: staging, cattle integration, the alpha / shepherd / predator / gamma terms
and the velocity update remain), against everything skipped (15) and the full step (0), at several
batch sizes.  Flock-phase bytes per flocking env-update: SURVEY §8(d) B_flock = 24 M + 8 N (read the
herd's positions and velocities and the drones' positions, write the velocities); half the envs flock
in a step (every second step_counter_A).

  python tools/flock_phase.py                 # table (JSON lines)
  python tools/flock_phase.py --only 13 --envs 262144 --launches 50   # one configuration
  python tools/flock_phase.py --envs 262144 --state-out /tmp/s.npz        # warmed-up state, then under rocprofv3:
  python tools/flock_phase.py --only 13 --envs 262144 --state-in /tmp/s.npz --launches 50   # every launch flock-only
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))


def run(E, n, m, mode, mask, launches, warm=40, state_in=None, state_out=None):
    """Per-launch us of the step kernel under phase mask `mask`.  state_out: run the full-step warm-up, save the
    state (np.savez) and stop; state_in: start from such a state with the mask set before the first launch, so
    that every step-kernel launch of the process is a masked one (a clean counter record under rocprofv3)."""
    import numpy as np
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    b = HerdBatch(E, n, m, mode=mode)
    b.reset()
    if state_in:
        d = np.load(state_in)
        b.set_state({k: d[k] for k in d.files})
        _lib.lib().ch__set_phase_mask(b.handle, ctypes.c_int32(mask))
    else:
        for _ in range(warm):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        if state_out:
            torch.cuda.synchronize()
            np.savez(state_out, **b.get_state())
            b.close()
            return None
        _lib.lib().ch__set_phase_mask(b.handle, ctypes.c_int32(mask))
    for _ in range(4):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(launches):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / launches * 1000.0
    b.close()
    return us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", type=int, default=None)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--launches", type=int, default=100)
    ap.add_argument("--mode", default="ctde")
    ap.add_argument("--drones", type=int, default=4)
    ap.add_argument("--cattle", type=int, default=16)
    ap.add_argument("--state-out", default=None, help="save the warmed-up state here and exit")
    ap.add_argument("--state-in", default=None, help="start from a saved state, every launch masked")
    a = ap.parse_args()
    n, m = a.drones, a.cattle
    if a.state_out:
        run(a.envs, n, m, a.mode, 0, 0, state_out=a.state_out)
        return
    if a.only is not None:
        print(json.dumps({"envs": a.envs, "mask": a.only, "state_in": a.state_in,
                          "us": run(a.envs, n, m, a.mode, a.only, a.launches, state_in=a.state_in)}))
        return
    for E in (4096, 65536, 262144):
        t = {mask: run(E, n, m, a.mode, mask, a.launches if E <= 65536 else 30) for mask in (0, 13, 15)}
        flock_us = t[13] - t[15]
        b_flock = (24 * m + 8 * n) * E / 2
        print(json.dumps({"envs": E, "mode": a.mode, "drones": n, "cattle": m, "full_us": t[0], "flock_only_us": t[13],
                          "skeleton_us": t[15], "flock_phase_us": flock_us, "flock_bytes": b_flock,
                          "flock_gbs": b_flock / (flock_us * 1e-6) / 1e9 if flock_us > 0 else None}), flush=True)


if __name__ == "__main__":
    main()
