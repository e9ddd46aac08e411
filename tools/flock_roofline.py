"""Compute roofline of the flock phase (north_star N1): useful fp64 FLOP per launch over the
flock phase's time, against the fp64 vector FMA peak, with its HBM fraction beside it.

The flock phase's time is the step kernel with the drone chain, task and observation phases masked off
(ch__set_phase_mask 13: staging, cattle integration, the alpha / shepherd / predator / gamma terms, the velocity
update) minus the skeleton with the flock masked off too (mask 15), over the same launches from the same burnt-in
state (tools/flock_phase.py).  The work is counted from that state on the host: every env whose step_counter_A is
odd flocks in the next launch (BaseAviary.py:454, every second step); in a flocking env the cheap pass tests all
M(M-1)/2 cow pairs, the full alpha evaluation runs on the pairs inside the bump's support (|z| <= 1.2, the queue),
the shepherd / predator term on every (cow, live drone) pair (all within the 999 + 2 m sensing range), gamma and the
velocity update on every cow.  FLOP per unit (~31 FLOP + 2 sqrt + 1 cos per cow pair, ~60 FLOP +
3 sqrt + 1 cos per cow-drone pair; sqrt and cos counted as one FLOP each, the convention that undercounts):
    cheap pair test 5, full alpha pair 34, cow-drone pair 64, gamma + velocity update + speed clip per cow 28.
Bytes: SURVEY.md 8(d) B_flock = 24 M + 8 N per flocking env.  Peak: 78.6 TFLOP/s fp64 vector FMA (wave64 FMA in 4
cycles per SIMD = 32 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz); ridge 78.6 / 8 TB/s = 9.8 FLOP/B.  The flock carries
~16-17 useful FLOP/B by this count (~28 by SURVEY's, which folds in the transcendental costs), so it is compute-side of
the ridge: the north_star's 40 % of HBM would need ~2/3 of the fp64 FMA peak in useful FLOP, and the compute roofline is
the one it is held to.

  python tools/flock_roofline.py --out profiles/counters        # C4, C5 and 262144 x (4, 16)
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))

PEAK_TFLOPS = 78.6
HBM_GBS = 8000.0
FLOP = {"cheap_pair": 5, "alpha_pair": 34, "cow_drone_pair": 64, "cow": 28}


def work(s, n_cfg):
    """FLOP and bytes of the next launch's flock phase from a state dict (HerdBatch.get_state)."""
    pos = s["cow_pos"]                                  # [E, M, 2]
    E, M = pos.shape[:2]
    flock = (s["step_counter_A"] + 1) % 2 == 0          # the launch increments it first (BaseAviary.py:367, 454)
    iu = np.triu_indices(M, 1)
    inr = np.zeros(E, np.int64)
    for e0 in range(0, E, 8192):                        # the queue: pairs inside the bump's support
        p = pos[e0:e0 + 8192]
        d = p[:, iu[0], :] - p[:, iu[1], :]
        inr[e0:e0 + 8192] = ((d ** 2).sum(-1) <= 1.44 * (1 + 1e-9)).sum(1)
    nd = np.minimum(s["n"], n_cfg)
    P = M * (M - 1) // 2
    f = flock.astype(np.float64)
    flop = (f * (P * FLOP["cheap_pair"] + inr * FLOP["alpha_pair"] + M * nd * FLOP["cow_drone_pair"] +
                 M * FLOP["cow"])).sum()
    byts = (f * (24 * M + 8 * nd)).sum()
    return {"flocking_envs": int(flock.sum()), "alpha_pairs": int((f * inr).sum()),
            "cow_drone_pairs": int((f * M * nd).sum()), "cheap_pairs": int(f.sum() * P), "pairs_per_flocking_env":
            float(inr[flock].mean()) if flock.any() else 0.0, "flop": float(flop), "bytes": float(byts)}


def measure(mode, E, n, m, launches, warm, reps=5):
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    b = HerdBatch(E, n, m, mode=mode)
    b.reset()
    for _ in range(warm):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    s0 = b.get_state()
    L = _lib.lib()
    res = {0: [], 13: [], 15: []}
    # masks interleaved over `reps` rounds, each round back-to-back launches from the same state under one event
    # pair; the median per mask (one slow round -- a clock ramp, a neighbour's job -- does not move the difference)
    for _ in range(reps):
        for mask in (0, 13, 15):
            b.set_state(s0)
            L.ch__set_phase_mask(b.handle, ctypes.c_int32(mask))
            b.step(random_actions=True, autoreset=True, terminal_obs=False)   # (rewrites the obs blocks in full)
            b.set_state(s0)
            s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s_ev.record()
            for _ in range(launches):
                b.step(random_actions=True, autoreset=True, terminal_obs=False)
            e_ev.record()
            torch.cuda.synchronize()
            res[mask].append(s_ev.elapsed_time(e_ev) * 1000.0 / launches)
    # the work of the same launches, counted from the state each one starts from (the sequence is deterministic:
    # Philox draws keyed by the env state)
    b.set_state(s0)
    L.ch__set_phase_mask(b.handle, ctypes.c_int32(13))
    ws = []
    for _ in range(launches):
        torch.cuda.synchronize()
        ws.append(work(b.get_state(), n))
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    L.ch__set_phase_mask(b.handle, ctypes.c_int32(0))
    b.close()
    spread = {k: [float(min(v)), float(max(v))] for k, v in res.items()}
    res = {k: (float(np.median(v)), None) for k, v in res.items()}
    flock_us = res[13][0] - res[15][0]
    flop = float(np.mean([w["flop"] for w in ws]))
    byts = float(np.mean([w["bytes"] for w in ws]))
    tflops = flop / (flock_us * 1e-6) / 1e12
    gbs = byts / (flock_us * 1e-6) / 1e9
    return {"mode": mode, "envs": E, "drones": n, "cattle": m, "launches": launches,
            "full_step_us": res[0][0], "flock_only_us": res[13][0], "skeleton_us": res[15][0], "flock_phase_us": flock_us,
            "min_max_us": {"full": spread[0], "flock_only": spread[13], "skeleton": spread[15]}, "reps": reps,
            "flocking_envs_per_launch": float(np.mean([w["flocking_envs"] for w in ws])),
            "alpha_pairs_per_launch": float(np.mean([w["alpha_pairs"] for w in ws])),
            "cow_drone_pairs_per_launch": float(np.mean([w["cow_drone_pairs"] for w in ws])),
            "cheap_pairs_per_launch": float(np.mean([w["cheap_pairs"] for w in ws])),
            "alpha_pairs_per_flocking_env": float(np.mean([w["pairs_per_flocking_env"] for w in ws])),
            "useful_flop_per_launch": flop, "achieved_tflops": tflops, "frac_of_fp64_peak": tflops / PEAK_TFLOPS,
            "flock_bytes_per_launch": byts, "achieved_gbs": gbs, "frac_of_hbm": gbs / HBM_GBS,
            "flop_per_byte": flop / byts if byts else None}


def main():
    from cattleherd._lib import code_object_hash
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "counters"))
    ap.add_argument("--configs", default="c4,c5,big")
    a = ap.parse_args()
    cfgs = {"c4": ("ctde", 4096, 4, 16, 40, 300), "c5": ("marl", 4096, 4, 32, 40, 300),
            "big": ("ctde", 262144, 4, 16, 10, 60)}
    recs = []
    for name in a.configs.split(","):
        mode, E, n, m, launches, warm = cfgs[name]
        r = measure(mode, E, n, m, launches, warm)
        r["config"] = name
        print(json.dumps(r), flush=True)
        recs.append(r)
    out = {"code_object": code_object_hash(), "records": recs, "flop_model": FLOP, "peak_tflops": PEAK_TFLOPS,
           "note": "flock phase = launch time under phase mask 13 (flock only) minus mask 15 (skeleton), per launch, "
                   "from one burnt-in state, median of `reps` interleaved rounds (flock_only_us is the masked launch "
                   "itself, an upper bound on the phase); useful FLOP counted on the host from the state each launch starts from "
                   "(tools/flock_roofline.py docstring); peak = fp64 vector FMA rate; ridge 9.8 FLOP/B; the flock carries "
                   "~16.5 FLOP/B, so 40 % of HBM would need ~2/3 of the fp64 FMA peak in useful FLOP"}
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "flock_roofline.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
