#!/usr/bin/env python3
"""Benchmark: env-steps/s of the batched cattle-herding env on N MI355X (BASELINE.json metric).

A "step" = one env.step() of every env on the GPU (reference: BaseAviary.step,
sb3_envs/BaseAviary.py:335-465) = one launch of the fused HIP step kernel over device-resident
state, with synthetic Philox random actions drawn in the kernel and SB3-style auto-reset.
Workload (default, BASELINE configs[3] per GPU): 4096 envs/GPU x (4 drones, 16 cattle), CTDE
(12, 86) observations.  Multi-GPU: one process per GPU (torchrun), envs sharded by env_id_offset,
no per-step exchange; one RCCL all-reduce of the metric vector closes the rollout.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))

WORKLOADS = {
    # name: (mode, envs/GPU, drones, cattle, compat, description)
    "c4": ("ctde", 4096, 4, 16, True, "BASELINE configs[3]: 4096 envs/GPU x (4 drones, 16 cattle), CTDE obs (12,86), "
                                      "random-action rollout with auto-reset"),
    "c2": ("ctde", 1024, 2, 8, True, "BASELINE configs[1]: 1024 envs x (2 drones, 8 cattle), CTDE, random actions"),
    # configs[2] is a training run: NaN-safe rewards (compat = 0), else every 2-drone reward is NaN
    "c3": ("ctde", 4096, 2, 8, False, "BASELINE configs[2]: 4096 envs x (2 drones, 8 cattle), CTDE, NaN-safe rewards "
                                      "(compat=0, the PPO training configuration)"),
    "c5": ("marl", 4096, 4, 32, True, "BASELINE configs[4]: 4096 envs x (4 drones, 32 cattle), MARL per-agent obs (4,86)"),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F32_PEAK_TFLOPS = 157.3   # f32-input MFMA: 64 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz (dense)
POLICY_GOLDEN = os.path.join(ROOT, "tests", "golden", "policy_ctde_v16_6.npz")
# the reference's trained RLlib PPO weights (simulator/policy_weights.pkl, read data-only into this fixture by
# tests/golden/make_policy_marl_golden.py)
POLICY_MARL_GOLDEN = os.path.join(ROOT, "tests", "golden", "policy_marl_rllib.npz")
PROFILES = os.path.join(ROOT, "profiles")


def algorithmic_bytes(mode, n, m, rows, real_bytes, eval_metrics=True):
    """HBM bytes one env-step moves with this SoA layout (DESIGN.md "Roofline"), everything the kernel reads
    and writes counted once: the carried state, its Euler-angle cache and per-env flags, the evaluation
    accumulators and the outputs."""
    drone = 26 * real_bytes * 2 * n                   # state read + write (22 components + the cached link frame)
    euler = 3 * real_bytes * 2 * n                    # Euler angles of the stored attitude, read + written
    evald = 8 * 2 * n if eval_metrics else 0          # update_evaluation_metrics' per-drone distance, read + written
    tags = 2 * 2 + 8 * 2                              # stale flags (2 x u8) and the obs-buffer tag, read + written
    actions = 16 * n                                  # drawn actions written to actions_out
    cattle = (4 * real_bytes + 2 * real_bytes + real_bytes) * m   # read pos+vel, write pos, vel every 2nd step
    env = 2 * (9 * 4 + 2 * real_bytes)                # env scalars read + write
    metrics = 2 * 7 * 8                               # per-env metric accumulators read + write
    # observation: the entries a step changes in each live row -- own state (10), two nearest drones
    # (4), min(m, 16) cattle offsets (2 each); the constant-zero bytes of the [rows][86] block persist
    # in the caller's buffer and are not rewritten (ch_api.cpp obs_zero_ptr, DESIGN.md "Observations")
    obs = n * (10 + 4 + 2 * min(m, 16)) * 4
    k = 1 if mode == "ctde" else n
    flags = 4 * k + 2 * k + n + 1                     # reward, terminated, truncated, agent_active, reset flag
    return drone + euler + evald + tags + actions + cattle + env + metrics + obs + flags


def survey_bytes(mode, n, m, rows):
    """SURVEY.md 8(d)'s reference byte model (fp32 SoA, minimal carried state, the full observation block):
    B_step = 16N (actions) + 176N (drone R/W) + 32M (cattle R/W) + 64 (env scalars R/W) + 344R (obs) + 6K."""
    k = 1 if mode == "ctde" else n
    return 16 * n + 176 * n + 32 * m + 64 + 344 * rows + 6 * k


COUNTERS = os.path.join(PROFILES, "counters")


def counter_record(name):
    """The committed counter record profiles/counters/<name>.json (tools/counter_record.py, tools/flock_roofline.py)
    if it was measured on the code object this process runs (cattleherd._lib.code_object_hash), else ({}, reason)."""
    from cattleherd._lib import code_object_hash
    path = os.path.join(COUNTERS, f"{name}.json")
    if not os.path.exists(path):
        return {}, f"no record {os.path.relpath(path, ROOT)}"
    with open(path) as fh:
        d = json.load(fh)
    have = code_object_hash()
    if d.get("code_object") != have:
        return {}, f"{os.path.relpath(path, ROOT)} is of code object {d.get('code_object')}, this library is {have}"
    d["source"] = os.path.relpath(path, ROOT)
    return d, None


def valu_issue(d, dtype, kern_us):
    """Compute-side view of the step kernel from its counter record: VALU wave-instructions per launch (PMC
    SQ_INSTS_VALU) priced at their issue cost on a SIMD (wave64: 4 cycles fp64, 2 fp32; the MI355X guide's constants
    table) over all SIMDs (256 CUs x 4) at 2.4 GHz for this launch time."""
    if "sq_insts_valu" not in d:
        return None
    cyc = 4 if dtype == "f64" else 2
    simd_cycles = 256 * 4 * kern_us * 1e-6 * 2.4e9
    return {"valu_insts_per_launch": d["sq_insts_valu"], "salu_insts_per_launch": d.get("sq_insts_salu"),
            "lds_insts_per_launch": d.get("sq_insts_lds"),
            "issue_cycles_per_inst": cyc, "issue_frac": d["sq_insts_valu"] * cyc / simd_cycles,
            "active_frac": (d["sq_active_inst_valu"] * 4 / simd_cycles) if "sq_active_inst_valu" in d else None,
            "source": d.get("source"),
            "note": "issue_frac = VALU issue cycles / SIMD cycles (upper bound: counts every VALU op at the wide rate); "
                    "active_frac from SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves)"}


def kernel_name(b, multi=False):
    """Which step kernel the handle launches (internal diagnostics entry point); `multi`: ch_step_n's k_step2_multi
    (at most 512 threads per workgroup)."""
    import ctypes
    from cattleherd import _lib
    g, blk, lds, kv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
    _lib.lib().ch__geometry(b.handle, ctypes.byref(g), ctypes.byref(blk), ctypes.byref(lds), ctypes.byref(kv))
    if kv.value == 2 and multi:
        return (f"ch::k_step2_multi (every workgroup steps its envs back to back; {g.value} envs/workgroup, "
                f"{min(blk.value, 512)} threads, {lds.value} B LDS)")
    if kv.value == 2:
        return f"ch::k_step2 (drone wave + cow waves; {g.value} envs/workgroup, {blk.value} threads, {lds.value} B LDS)"
    return "ch::k_env (team per env)"


def policy_rollout(b, n, steps, warmup):
    """Rollout with the reference's trained CTDE actor (model-v16-6, f32 MFMA forward) choosing every
    action: env-steps/s of forward + step, and the forward alone against the f32 MFMA peak."""
    import numpy as np
    import torch
    from cattleherd.policy import DevicePolicy
    d = np.load(POLICY_GOLDEN)
    # the trained model's weights are frozen: packed once (cache_packed)
    actor = DevicePolicy.sb3_actor({k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k},
                                   cache_packed=True)
    E = b.n_envs
    stream = torch.cuda.current_stream()
    b.reset()
    for _ in range(warmup):
        b.step_policy(actor)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        b.step_policy(actor)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    nk = min(200, steps)
    s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    y = torch.empty((E, actor.dims[-1]), dtype=torch.float32, device=b.device)
    s_ev.record(stream)
    for _ in range(nk):
        actor.forward_batch(b, y)
    e_ev.record(stream)
    torch.cuda.synchronize()
    fwd_us = s_ev.elapsed_time(e_ev) / nk * 1000.0
    # multiplied work: the live input width n*86 of layer 1 (the zero tail is skipped), layers 2-3 in full
    d0 = actor.dims
    flops = 2.0 * E * (n * 86 * d0[1] + sum(d0[i] * d0[i + 1] for i in range(1, len(d0) - 1)))
    tf = flops / (fwd_us * 1e-6) / 1e12
    out = {"env_steps_per_s": E * steps / dt, "ms_per_step": dt / steps * 1000.0,
           "policy": "SB3 MlpPolicy actor 1032-128-128-48 tanh (model-v16-6), deterministic, f32",
           "forward_us": fwd_us,
           "roofline": {"bound": "mfma", "achieved": tf, "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": tf / MFMA_F32_PEAK_TFLOPS, "flops_per_forward": flops}}
    out["ppo_rollout"] = ppo_rollout(b, d)
    # the packed actor-critic reads the observation once, but each workgroup still streams both heads' weights
    # for its 16 rows, which is what the forward waits on: measured slower, reported beside it
    out["ppo_rollout_fused_nets"] = ppo_rollout(b, d, fused=True)
    # the actor forward in the step kernel's workgroups (k_step2_actor, ch_rollout_collect path bit 2), the critic
    # alone after it
    out["ppo_rollout_fused_step"] = ppo_rollout(b, d, fused_step=True)
    return out


PPO_BURN_IN = 300


def burn_in(b, steps=PPO_BURN_IN):
    """Reset, then random-action steps with auto-reset before a timed collection: a training run's rollouts see the
    envs' episode phases spread by their resets (half of them flocking on any step, BaseAviary.py:454), not the
    lock-step phases of a batch that has just been reset (every env flocking on the same steps)."""
    b.reset()
    for _ in range(steps):
        b.step(None, random_actions=True, autoreset=True, terminal_obs=False)


def ppo_rollout(b, d, T=32, fused=False, fused_step=False, reps=5):
    """SB3 collect_rollouts on the device (cattleherd.rollout): per step the actor and critic forwards (fused=True:
    one launch of the two heads packed as one net, DevicePolicy.sb3_actor_critic, bit-identical to the separate
    nets), Gaussian sample / log-prob / buffer store (with the previous step's reward bootstrap), env step with
    auto-reset and terminal obs, V(terminal obs); then GAE.  env-steps/s of one whole T-step collection (the median
    of `reps`, after one untimed collection).  fused_step: the actor forward in the step kernel (k_step2_actor)."""
    import numpy as np
    import torch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceRolloutBuffer
    sd = {k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k}
    actor = DevicePolicy.sb3_actor(sd, clip=False)
    critic = DevicePolicy.sb3_critic(sd)
    nets = (DevicePolicy.sb3_actor_critic(sd), None) if fused else (actor, critic)
    log_std = torch.full((actor.dims[-1],), -1.0, device=b.device)   # log_std_init (CTDECattleHerder.py:122)
    rb = DeviceRolloutBuffer(b, T, act_dim=actor.dims[-1])
    import ctypes
    from cattleherd import _lib
    L = _lib.lib()
    L.ch__rollout_fused_steps.restype = ctypes.c_int64
    # set or clear only the fused-actor bits (2: fused, 3: never fused); the copy / store-kernel bits the
    # environment chose for this handle stay, and the original value is restored after the leg
    path0 = L.ch__get_rollout_path(b.handle)
    L.ch__set_rollout_path(b.handle, ctypes.c_int32((path0 & 3) | (4 if fused_step else 8)))
    burn_in(b)
    rb.collect(*nets, log_std, seed=1)
    torch.cuda.synchronize()
    f0 = L.ch__rollout_fused_steps(b.handle)
    dts = []
    for r in range(reps):   # the median of `reps` collections, each from where the previous one left the envs
        t0 = time.perf_counter()
        rb.collect(*nets, log_std, seed=2 + r)
        torch.cuda.synchronize()
        dts.append(time.perf_counter() - t0)
    dt = float(np.median(dts))
    nf = (L.ch__rollout_fused_steps(b.handle) - f0) // reps
    L.ch__set_rollout_path(b.handle, ctypes.c_int32(path0))
    out = {"env_steps_per_s": b.n_envs * T / dt, "ms_per_step": dt / T * 1000.0, "n_steps": T,
           "burn_in": PPO_BURN_IN, "reps": reps, "min_max_ms_per_step": [min(dts) / T * 1e3, max(dts) / T * 1e3],
           "policy": ("actor + critic fused (one forward per step)" if fused else "actor and critic separately") +
                     (", actor forward in the step kernel (k_step2_actor)" if fused_step else ""),
           "fused_steps": int(nf),
           "buffer_GB": sum(t.numel() * 4 for t in (rb.obs, rb.actions)) / 1e9}
    del rb
    return out


def ppo_train_iteration(b, T=32, batch_size=64, n_envs_ref=24):
    """configs[2] end to end: one PPO training iteration of the CTDE driver (CTDECattleHerder.py:107-127) on the device
    -- the collection (cattleherd.rollout, T steps of every env) then the update (cattleherd.ppo.PPOUpdate: SB3 PPO.train
    with the driver's hyper-parameters, n_epochs 10 over the whole buffer, Adam, clip_grad_norm; each 32 minibatch steps
    one captured HIP graph) -- on a fresh SB3 MlpPolicy (pi/vf 128-128 tanh, log_std -1, torch's default init).  The
    update's cost per env-step is n_epochs / batch_size SGD steps whatever n_steps is, so T < the driver's 2048 changes
    the rate only by the collection's per-iteration constants.  Two minibatch sizes: the driver's 64, and 64 x E / 24
    (the driver's 24 envs' rows per minibatch per env).  Timed: the second iteration (the first captures the graphs)."""
    import torch
    from cattleherd.ppo import PPOUpdate, SB3ActorCritic
    from cattleherd.rollout import DeviceRolloutBuffer
    out = {}
    E = b.n_envs
    for name, bs in (("driver_batch", batch_size), ("batch_scaled_with_envs", int(round(batch_size * E / n_envs_ref)))):
        model = SB3ActorCritic(obs_dim=b.obs_rows * 86, act_dim=48, device=b.device, seed=0)
        actor, critic, log_std = model.device_nets()
        rb = DeviceRolloutBuffer(b, T, act_dim=48)
        upd = PPOUpdate(model, batch_size=bs)
        burn_in(b)
        rb.collect(actor, critic, log_std, seed=1)
        upd.train(rb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rb.collect(actor, critic, log_std, seed=2)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        steps = upd.train(rb)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[name] = {"env_steps_per_s": E * T / (t2 - t0), "collect_env_steps_per_s": E * T / (t1 - t0),
                     "collect_s": t1 - t0, "update_s": t2 - t1, "update_share": (t2 - t1) / (t2 - t0),
                     "batch_size": bs, "sgd_steps": steps, "us_per_sgd_step": (t2 - t1) / steps * 1e6,
                     "rows": E * T, "n_steps": T, "n_epochs": upd.n_epochs}
        del rb, upd, model
        torch.cuda.empty_cache()
    out["note"] = ("one PPO iteration = device collection of T steps x E envs + SB3 PPO.train over that buffer "
                   "(lr 3e-4, n_epochs 10, clip 0.1, ent 0.1, vf 0.7, max_grad_norm 0.5, CTDECattleHerder.py:107-127); "
                   "SB3 semantics restated (parity unpinned); the reference's published SB3 time/fps is 93-269 "
                   "(24 CPU envs, SURVEY 6)")
    return out


def marl_ppo_rollout(b, T=32):
    """configs[4]'s training use: RLlib PPO sampling with one shared policy over every agent (DTDECattleHerder.py:
    62-97; the RLlib default model, 86 -> 256 -> 256 -> 8 tanh = DiagGaussian mean and log_std, and a separate value
    branch 86 -> 256 -> 256 -> 1, with the reference's trained weights simulator/policy_weights.pkl) on the device
    (cattleherd.rollout.DeviceMarlRolloutBuffer): per
    step the two forwards (f32 MFMA), the per-agent sample / log-prob / store, the env step with the wrapper's
    drop-out; then per-agent GAE.  env-steps/s (and agent-steps/s) of one whole T-step collection after an untimed
    one."""
    import torch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceMarlRolloutBuffer
    import numpy as np
    d = np.load(POLICY_MARL_GOLDEN)
    w = {k.replace("__", "."): d[k] for k in d.files if "__" in k}
    policy = DevicePolicy.rllib_policy(w, cache_packed=True)
    value = DevicePolicy.rllib_value(w, cache_packed=True)
    rb = DeviceMarlRolloutBuffer(b, T)
    burn_in(b)
    rb.collect(policy, value, seed=1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rb.collect(policy, value, seed=2)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"env_steps_per_s": b.n_envs * T / dt, "agent_steps_per_s": b.n_envs * b.num_drones * T / dt,
           "ms_per_step": dt / T * 1000.0, "n_steps": T, "burn_in": PPO_BURN_IN,
           "policy": "RLlib default model 86-256-256-8 (mean, log_std) + value 86-256-256-1, tanh, f32, the reference's "
                     "trained weights (simulator/policy_weights.pkl)",
           "gae": "per agent, gamma 0.99, lambda 1.0 (RLlib PPO default)",
           "buffer_GB": sum(t.numel() * t.element_size() for t in (rb.obs, rb.actions)) / 1e9}
    del rb
    return out


def near_herd_leg(b, n, m, reps=8, steps=100, burn=10, seed=11, multi=False):
    """configs[4] at training conditions: the headline's random actions drive the drones away from the herd (the
    steady state is ~96 % truncated agent-steps with every cow-drone pair beyond the predator range, where the
    shepherd term takes its far-drone closed form).  Here, `reps` times, every env's drones are put 0.6-1.4 m from a
    random cow of their herd (set_state, untimed), `burn` untimed steps run, then `steps` timed steps: the flock's
    near-drone shepherd and predator terms and the task's non-truncated paths run as in training.  Reports the rate
    and, from each window's first state, the share of cow-drone pairs within 1 m (mu < 1) and 1.1 m (predator).
    `multi` (the headline ran ch_step_n): each window also runs from the same state through ch_step_n -- one plain
    step after the state restore, then one k_step2_multi launch of the rest -- and that is the reported rate, with
    the single-launch one beside it."""
    import numpy as np
    import torch
    rng = np.random.default_rng(seed)
    E = b.n_envs
    times, times_n, near1, pred, ends, trunc, steps_done = [], [], [], [], 0.0, 0.0, 0.0
    for _ in range(reps):
        s = b.get_state()
        cows = s["cow_pos"][:, :m]
        pick = rng.integers(0, m, (E, n))
        ang = rng.uniform(-np.pi, np.pi, (E, n))
        rad = rng.uniform(0.6, 1.4, (E, n))
        c = np.take_along_axis(cows, pick[..., None].repeat(2, -1), 1)
        dp = s["drone_pos"].copy()
        dp[:, :, 0] = c[..., 0] + rad * np.cos(ang)
        dp[:, :, 1] = c[..., 1] + rad * np.sin(ang)
        b.set_state({"drone_pos": dp})
        for _ in range(burn):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        g = b.get_state()
        d = np.linalg.norm(g["cow_pos"][:, None, :m, :] - g["drone_pos"][:, :n, None, :2], axis=-1)
        live = np.arange(n)[None, :, None] < g["n"][:, None, None]
        near1.append(float((d[np.broadcast_to(live, d.shape)] < 1.0).mean()))
        pred.append(float((d[np.broadcast_to(live, d.shape)] <= 1.1).mean()))
        s0 = b.get_state_raw() if multi else None
        b.metrics(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        mv = b.metrics(reset=True)
        ends += mv[1]; trunc += mv[5]; steps_done += mv[0]
        if multi:   # the same window from the same state through ch_step_n (the headline's form)
            b.set_state_raw(*s0)
            b.step_n(1, random_actions=True)   # (set_state rewrote the observation blocks: one plain step)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b.step_n(steps - 1, random_actions=True)
            torch.cuda.synchronize()
            times_n.append((time.perf_counter() - t0) * steps / (steps - 1))
            b.metrics(reset=True)
    dt = float(np.sum(times))
    out = {"env_steps_per_s": E * steps * reps / dt, "us_per_step": dt / (steps * reps) * 1e6}
    if multi:
        dn = float(np.sum(times_n))
        out = {"env_steps_per_s": E * steps * reps / dn, "us_per_step": dn / (steps * reps) * 1e6,
               "launch": "ch_step_n (k_step2_multi), the same windows from the same states as the single-launch figure",
               "single_launch": out}
    return {**out,
            "windows": reps, "steps_per_window": steps, "untimed_steps_after_placement": burn,
            "cow_drone_pairs_within_1m": float(np.mean(near1)), "cow_drone_pairs_within_1.1m": float(np.mean(pred)),
            "episode_ends": ends, "truncated_agent_step_fraction": trunc / max(steps_done * n, 1.0),
            "note": "drones re-placed 0.6-1.4 m from a random cow of their herd before each window (untimed)"}


def marl_vec_rollout(n, m, E, steps, warmup, burn_in):
    """configs[4] through the batched RLlib multi-agent surface (cattleherd.marl_vec_env): random actions,
    the wrapper semantics and in-launch resets; env-steps/s of the zero-copy tensor path (one launch plus the
    output views per step, terminal observations requested), and of the dict path (per-env agent dicts built on
    the host from one copy of the outputs) on a few steps."""
    import torch
    from cattleherd.marl_vec_env import CattleHerdMultiAgentVecEnv
    venv = CattleHerdMultiAgentVecEnv(E, {"num_drones": n, "num_cattle": m, "min_drones": n, "max_drones": n})
    venv.reset()
    g = torch.Generator(device=venv.batch.device).manual_seed(0)
    acts = [torch.rand((E, n, 4), generator=g, device=venv.batch.device) * 2 - 1 for _ in range(8)]
    for t in range(burn_in + warmup):
        venv.step_tensors(acts[t % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ended = 0
    for t in range(steps):
        out = venv.step_tensors(acts[t % 8])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ended = int(out["all_done"].sum())
    nd = min(steps, 10)
    venv.refresh_agents()
    host = [a.cpu().numpy() for a in acts]
    t1 = time.perf_counter()
    for t in range(nd):
        venv.step(host[t % 8])
    dd = time.perf_counter() - t1
    venv.close()
    return {"tensor_env_steps_per_s": E * steps / dt, "tensor_ms_per_step": dt / steps * 1e3,
            "dict_env_steps_per_s": E * nd / dd, "dict_ms_per_step": dd / nd * 1e3, "dict_steps": nd,
            "ended_last_step": ended,
            "note": "tensor path: ch_step with terminal observations + the reset/agent-mask views; dict path: "
                    "RLlibMultiAgentWrapper-style dicts for every env built on the host"}


def host_surfaces(steps):
    """The drop-in host surfaces at full size, numpy in and out (what the reference's drivers see):
    sb3_vecenv -- cattleherd.vec_env.CattleHerdVecEnv at configs[3]'s per-GPU size (4096 x (4, 16)), the
    ``vec_env_cls`` swap for CTDECattleHerder.py's SubprocVecEnv: numpy actions in, step, ch_outputs_to_host
    (pinned), SB3 infos; marl_vec_env_dict -- cattleherd.marl_vec_env.CattleHerdMultiAgentVecEnv.step at
    configs[4] (4096 x (4, 32)): RLlibMultiAgentWrapper-style dicts for every env."""
    import numpy as np
    import torch
    from cattleherd.marl_vec_env import CattleHerdMultiAgentVecEnv
    from cattleherd.vec_env import CattleHerdVecEnv
    out = {}
    rng = np.random.default_rng(0)
    E = 4096
    venv = CattleHerdVecEnv(E, num_drones=4, num_cattle=16)
    venv.reset()
    acts = [rng.uniform(-1, 1, (E, 4, 4)).astype(np.float32) for _ in range(4)]
    for t in range(300):   # burn-in: auto-resets at their steady-state rate
        venv.step(acts[t % 4])
    k = max(20, min(steps, 100))
    ended = 0
    t0 = time.perf_counter()
    for t in range(k):
        _, _, dones, _ = venv.step(acts[t % 4])
        ended += int(dones.sum())
    dt = time.perf_counter() - t0
    venv.close()
    out["sb3_vecenv"] = {"env_steps_per_s": E * k / dt, "ms_per_step": dt / k * 1e3, "steps": k, "episodes_ended": ended,
                         "config": "4096 envs x (4 drones, 16 cattle), CTDE, numpy actions (E, 4, 4)",
                         "note": "VecEnv.step: action H2D, one launch (terminal observations on), one ch_outputs_to_host "
                                 "(live obs rows, reward, flags, ended envs compacted on the device) into pinned buffers, "
                                 "SB3 infos with terminal_observation / TimeLimit.truncated / Monitor episode"}
    mv = CattleHerdMultiAgentVecEnv(E, {"num_drones": 4, "num_cattle": 32, "min_drones": 4, "max_drones": 4})
    mv.reset()
    g = torch.Generator(device=mv.batch.device).manual_seed(0)
    dev_acts = torch.rand((E, 4, 4), generator=g, device=mv.batch.device) * 2 - 1
    for _ in range(200):
        mv.step_tensors(dev_acts)
    mv.refresh_agents()
    host_acts = [rng.uniform(-1, 1, (E, 4, 4)).astype(np.float32) for _ in range(4)]
    for t in range(3):
        mv.step(host_acts[t % 4])
    kd = 10
    t0 = time.perf_counter()
    for t in range(kd):
        mv.step(host_acts[t % 4])
    dt = time.perf_counter() - t0
    mv.close()
    out["marl_vec_env_dict"] = {"env_steps_per_s": E * kd / dt, "agent_steps_per_s": 4 * E * kd / dt,
                                "ms_per_step": dt / kd * 1e3, "steps": kd,
                                "config": "4096 envs x (4 drones, 32 cattle), MARL wrapper semantics, numpy actions",
                                "note": "CattleHerdMultiAgentVecEnv.step: one launch, one ch_outputs_to_host, obs / "
                                        "rewards / dones / truncs / infos dicts keyed agent_i + __all__ for every env"}
    return out


def cpu_baseline(mode, n, m, seconds=12.0):
    """The CPU oracle (scalar fp64 C port, OpenMP one env per thread) on a bounded sample, on every
    core this process may use: OMP_NUM_THREADS when the pool sets it (16 per GPU on the MI355X
    boxes), else the CPU affinity mask.  os.cpu_count() is reported beside it: on the GPU box it is
    the whole machine, of which one GPU's job gets a share."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from cattleherd._lib import spawn_table
    table = spawn_table(m)
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = int(omp) if omp.isdigit() and int(omp) > 0 else affinity
    threads = max(1, min(threads, affinity))
    E = threads * 4
    secs, steps = O.batch_rollout(0 if mode == "ctde" else 1, n, m, table, E=E, T=20, threads=threads)
    T = max(20, int(seconds / max(secs, 1e-6) * 20))
    secs, steps = O.batch_rollout(0 if mode == "ctde" else 1, n, m, table, E=E, T=T, threads=threads)
    return {"value": steps / secs, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "affinity_cpus": affinity, "omp_num_threads": omp or None,
            "sample": f"{E} envs x {T} random-action steps ({steps} env-steps, {secs:.1f} s) of the fp64 C oracle, "
                      f"{threads} OpenMP threads (one env per thread iteration)"}


def launch_check(args):
    """--launch-check: the multi-rank plumbing alone (no GPU): process group over ``--backend``, world
    size, per-rank env ranges, the metric all-reduce and the max-over-ranks time."""
    from cattleherd import distributed as D
    rank, world, _ = D.world_info()
    D.init(args.backend)
    import torch.distributed as dist
    seen = dist.get_world_size() if dist.is_initialized() else 1
    if seen != args.gpus:
        print(f"bench: --gpus {args.gpus} but the process group has {seen} ranks", file=sys.stderr)
        sys.exit(3)
    E = args.envs or WORKLOADS[args.workload][1]
    lo = D.env_offset(rank, E)
    mv, t = D.reduce_rollout([float(rank + 1)] * 8, 0.5 + rank, device="cpu")
    ranks = D.gather_rank_info(D.rank_device_info(use_gpu=False))
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": seen, "backend": args.backend,
                          "env_ranges": [[D.env_offset(r, E), D.env_offset(r, E) + E] for r in range(seen)],
                          "metric_sum": float(mv[0]), "max_time": t, "rank0_range": [lo, lo + E],
                          "ranks": ranks, "distinct_devices": D.distinct_devices(ranks)}), flush=True)
    D.shutdown()
    if not D.distinct_devices(ranks):
        print("bench: two ranks would drive the same device slot", file=sys.stderr)
        sys.exit(4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--envs", type=int, default=None, help="override envs per GPU")
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    ap.add_argument("--physics", default="pyb", choices=["pyb", "dyn", "pyb_gnd", "pyb_drag", "pyb_dw", "pyb_gnd_drag_dw"],
                    help="Physics variant (BaseAviary.py:420-450); the headline is the reference default pyb")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--policy", action="store_true",
                    help="also time a rollout driven by the on-device SB3 policy (model-v16-6 weights, CTDE only)")
    ap.add_argument("--train", action="store_true",
                    help="CTDE: also time one PPO training iteration (device collection + SB3 PPO update, configs[2])")
    ap.add_argument("--steps-per-launch", type=int, default=-1,
                    help="timed steps per ch_step_n call (k_step2_multi: every workgroup steps its envs back to back "
                         "in one launch); -1 (default) = all timed steps in one call; 1 = one ch_step launch per step")
    ap.add_argument("--counter-probe", type=int, default=0,
                    help="(tools/counter_record.py --multi) after the burn-in, 10 ch_step_n calls of this many steps "
                         "each, nothing else; no JSON line")
    ap.add_argument("--graph", type=int, default=0,
                    help="steps per captured HIP graph in the timed loop (0 = one host launch per step)")
    ap.add_argument("--backend", default="nccl", help="process-group backend (nccl = RCCL over xGMI)")
    ap.add_argument("--burn-in", type=int, default=1200,
                    help="untimed random-action steps before the warmup, so the timed steps start from the "
                         "steady-state spread of episode phases (auto-resets at their long-run rate); 1200 = the "
                         "level-7 CTDE episode cap (80 s at 15 steps/s)")
    ap.add_argument("--marl-vec", action="store_true",
                    help="MARL workloads: also time the batched multi-agent surface (tensor and dict paths)")
    ap.add_argument("--launch-check", action="store_true",
                    help="run only the multi-rank plumbing (process group, env ranges, all-reduce); no GPU")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the legs after the headline (terminal observations, host surfaces): counter passes")
    args = ap.parse_args()

    # --gpus N from a plain `python bench.py`: one child process per GPU, started before this
    # process touches the GPU (cattleherd.launch imports no torch)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from cattleherd.launch import spawn_ranks
        sys.exit(spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    if args.launch_check:
        return launch_check(args)

    import torch
    import torch.distributed as dist
    from cattleherd import distributed as D
    from cattleherd.env import HerdBatch
    rank, world, local = D.world_info()
    if world > 1:
        D.init(args.backend, device_index=local)   # RCCL over xGMI; one process per GPU
        world = dist.get_world_size()
    torch.cuda.set_device(local if world > 1 else 0)
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but the process group has {world} ranks", file=sys.stderr)
        sys.exit(3)

    mode, E, n, m, compat, desc = WORKLOADS[args.workload]
    if args.envs:
        E = args.envs
    b = HerdBatch(E, n, m, mode=mode, precision=args.precision, env_id_offset=D.env_offset(rank, E),
                  physics=args.physics, compat=compat)
    print(f"bench: rank {rank}/{world} device {torch.cuda.current_device()} envs "
          f"[{D.env_offset(rank, E)}, {D.env_offset(rank, E) + E})", file=sys.stderr, flush=True)
    # every rank's device (index, PCI address), gathered to rank 0 into the JSON line: a multi-GPU line proves
    # from its own content that N ranks stepped N distinct devices (exit 4 otherwise)
    ranks = D.gather_rank_info(D.rank_device_info(use_gpu=True))
    if not D.distinct_devices(ranks):
        print(f"bench: ranks share a device: {ranks}", file=sys.stderr)
        sys.exit(4)
    stream = torch.cuda.current_stream()

    # end of a rollout (SURVEY §8(d) "host sync at the end"): device reduction of the per-env metric
    # rows, the RCCL all-reduce over xGMI (the rollout's only collective), one 64-byte copy to pinned
    # memory and the stream sync
    mbuf = torch.zeros(8, dtype=torch.float64, device=b.device)
    mhost = torch.zeros(8, dtype=torch.float64).pin_memory()

    def end_of_rollout():
        b.metrics_device(reset=True, out=mbuf)
        if world > 1:
            dist.all_reduce(mbuf)
        mhost.copy_(mbuf, non_blocking=True)
        stream.synchronize()
        return mhost.numpy().copy()

    b.reset()
    # burn-in (untimed, before the warmup): the envs leave the common starting point, so the timed steps see
    # episode phases -- and auto-resets -- at their steady-state spread rather than K steps of fresh episodes
    for _ in range(args.burn_in):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    if args.counter_probe:   # the multi-step kernel's counter passes: equal dispatches of a known step count
        for _ in range(10):
            b.step_n(args.counter_probe, random_actions=True)
        torch.cuda.synchronize()
        b.close()
        D.shutdown()
        return
    # steps per ch_step_n call: -1 (default) = every timed step in one call; 1 = one ch_step launch per step
    spl = args.steps if args.steps_per_launch < 0 else max(1, args.steps_per_launch)
    if spl > 1:
        b.step_n(max(args.warmup, 1), random_actions=True)   # (also uploads the multi-step kernel's parameters)
    else:
        for _ in range(args.warmup):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
    # the timed loop: K steps as whole graph replays of `chunk` steps (plus single launches for the rest)
    chunk = args.graph if args.graph > 0 and args.steps >= args.graph and spl == 1 else 0
    graph = b.capture_rollout(chunk) if chunk else None
    end_of_rollout()   # warm: reduction kernel, pinned copy, first collective; zeroes the metric rows
    b.sync()

    def run(k):
        done = 0
        if spl > 1:   # ch_step_n: each workgroup steps its envs back to back inside one launch
            while done < k:
                n = min(spl, k - done)
                b.step_n(n, random_actions=True)
                done += n
            return
        if graph is not None:
            while done + chunk <= k:
                graph.replay()
                done += chunk
        while done < k:
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
            done += 1

    # the timed region: exactly K steps of every env, bracketed by barrier + device sync on both sides (SURVEY
    # 8(d): E*T / wall, auto-reset included, host sync at the end)
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    D.barrier()
    dt = time.perf_counter() - t0
    _, dt = D.reduce_rollout([0.0], dt, device=b.device)   # max over ranks
    b.sync()   # raises if a step kernel recorded a device error (hand-off timeout)

    # the end of the rollout, after the timed steps: the device metric reduction of those K steps, the RCCL
    # all-reduce over the ranks (the run's only collective; the path has no per-step exchange), the pinned copy
    torch.cuda.synchronize()
    te = time.perf_counter()
    mv = end_of_rollout()
    rollout_end_us = (time.perf_counter() - te) * 1e6

    # live per-launch kernel timing with HIP events on the launch stream (roofline): one event pair
    # around nk back-to-back launches (an event between every two launches would break the queue's
    # back-to-back dispatch and add its own packet time to every sample)
    nk = min(200, args.steps)
    s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_ev.record(stream)
    if spl > 1:
        b.step_n(nk, random_actions=True)   # one k_step2_multi launch of nk steps
    else:
        for _ in range(nk):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
    e_ev.record(stream)
    torch.cuda.synchronize()
    kern_us = s_ev.elapsed_time(e_ev) / nk * 1000.0   # per step
    rb = 8 if args.precision == "f64" else 4
    bytes_step = algorithmic_bytes(mode, n, m, b.obs_rows, rb)
    survey_step = survey_bytes(mode, n, m, b.obs_rows)
    if args.physics != "pyb":
        bytes_step += 2 * 7 * rb * n   # carried last_clipped_action + rpy_rates, read and written
    achieved = bytes_step * E / (kern_us * 1e-6) / 1e9
    achieved_survey = survey_step * E / (kern_us * 1e-6) / 1e9
    default_cfg = E == WORKLOADS[args.workload][1] and args.physics == "pyb"
    from cattleherd import _lib as _L
    multi_ran = spl > 1 and _L.lib().ch__multi_steps(b.handle) > 0   # (other geometries: one launch per step)
    # the counter record of the kernel the headline ran (the multi-step kernel's per step, tools/counter_record.py --multi)
    rec_name = f"{args.workload}_{args.precision}" + ("_multi" if multi_ran else "")
    rec, rec_why = counter_record(rec_name) if default_cfg else ({}, "not a default workload")
    traffic = rec.get("traffic_bytes_per_launch")
    kname = kernel_name(b, multi=multi_ran)
    # the same kernel with SB3's terminal observations requested (the synced reset path: the headline's sync-free
    # one does not write info["terminal_observation"])
    term_leg = None
    if not args.no_extras:
        nt = min(200, args.steps)
        for _ in range(10):
            b.step(random_actions=True, autoreset=True, terminal_obs=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(nt):
            b.step(random_actions=True, autoreset=True, terminal_obs=True)
        torch.cuda.synchronize()
        dt1 = time.perf_counter() - t1
        term_leg = {"env_steps_per_s": E * world * nt / dt1, "ms_per_step": dt1 / nt * 1e3, "steps": nt,
                    "note": "ch_step with terminal_obs (SB3 info['terminal_observation'] written for every auto-reset): "
                            "the VecEnv / rollout-buffer path; the headline value is the sync-free path without it"}
    # the same random-action rollout with one ch_step launch per step (the form an SB3 / RLlib caller steps in: a
    # policy between two steps), beside the headline's ch_step_n form
    single_leg = None
    if not args.no_extras or spl > 1:
        ns = min(2000, args.steps)
        for _ in range(5):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        torch.cuda.synchronize()
        D.barrier()
        t2 = time.perf_counter()
        for _ in range(ns):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        torch.cuda.synchronize()
        D.barrier()
        dt2 = time.perf_counter() - t2
        _, dt2 = D.reduce_rollout([0.0], dt2, device=b.device)
        s_ev.record(stream)
        for _ in range(nk):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        e_ev.record(stream)
        torch.cuda.synchronize()
        single_leg = {"env_steps_per_s": E * world * ns / dt2, "ms_per_step": dt2 / ns * 1e3, "steps": ns,
                      "kernel": kernel_name(b), "kernel_us": s_ev.elapsed_time(e_ev) / nk * 1000.0,
                      "note": "one ch_step launch per step (k_step2): the grid of every step waits for its slowest "
                              "workgroup and the next launch"}
    wg = rec.get("wg_trace") or {}

    out = None
    if rank == 0:
        value = E * world * args.steps / dt
        out = {
            "metric": "env-steps/sec (agent-steps/sec) at 4096 envs/GPU, 1/2/4/8 MI355X",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1000.0, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.precision, "agent_steps_per_s": value * n,
            "data": "synthetic: Philox4x32 random VEL actions in-kernel, spawn table from config/cattle_positions.yaml; "
                    f"envs burnt in for {args.burn_in} untimed steps before the warmup (steady-state episode phases, "
                    "auto-resets inside the timed steps at their long-run rate); headline without SB3 terminal "
                    "observations (terminal_obs=False, the sync-free auto-reset path), the terminal-observation path in "
                    "terminal_obs_leg",
            "launch": (f"ch_step_n, {spl} steps per call: every workgroup steps its envs back to back in one "
                       f"k_step2_multi launch (bit-identical to ch_step launches, tests/test_gpu_runtime.py)" if multi_ran else
                       f"ch_step_n, {spl} steps per call, one launch per step (no multi-step kernel for this geometry)"
                       if spl > 1 else
                       f"HIP graph of {chunk} steps per replay" if graph is not None else "one host launch per step"),
            "ranks": ranks,   # each rank's device index and PCI address (distinct, checked above)
            "rollout_end_us": rollout_end_us,
            "config": {"workload": desc, "envs_per_gpu": E, "num_drones": n, "num_cattle": m, "mode": mode,
                       "physics": args.physics,
                       "parallelism": f"env-sharded x{world} (no per-step collective)"},
            # The kernel moves a few MB per launch and is bound by the latency of its dependent fp64 chains (the drone
            # wave's action -> PID -> 4 substeps -> bookkeeping), not by HBM or VALU throughput: the
            # HBM fraction is reported against 8 TB/s as the north_star asks, the chain/workgroup cycles beside it.
            "roofline": {"bound": "latency", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": rec.get("source") or rec_why, "code_object": rec.get("code_object"),
                         "algorithmic_bytes_per_launch": bytes_step * E,
                         "kernel": kname, "kernel_us": kern_us, "bytes_per_env_step": bytes_step,
                         "traffic_over_algorithmic": (traffic / (bytes_step * E)) if traffic else None,
                         "latency": ({"chain_cycles": wg.get("chain_cycles_q50"), "wg_cycles_q50": wg.get("wg_cycles_q50"),
                                      "wg_cycles_max": wg.get("wg_cycles_max"), "chain_over_wg": wg.get("chain_over_wg"),
                                      "post_chain_cycles": wg.get("post_chain_cycles"),
                                      "source": "tools/wg_trace.py --json (per-workgroup shader-clock phase stamps)"}
                                     if wg else None),
                         "byte_model": "this layout: f64 state, Euler cache, eval accumulators, flags, the obs "
                                       "entries a step changes (bench.py algorithmic_bytes)"},
            "roofline_survey": {"bound": "hbm", "achieved": achieved_survey, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": achieved_survey / HBM_PEAK_GBS, "bytes_per_env_step": survey_step,
                                "algorithmic_bytes_per_launch": survey_step * E, "kernel_us": kern_us,
                                "byte_model": "SURVEY.md 8(d): fp32 SoA, minimal carried state, full obs block"},
            "valu": valu_issue(rec, args.precision, kern_us) if rec else None,
            "terminal_obs_leg": term_leg,
            "single_launch_leg": single_leg,
            "rollout_metrics": {"episodes": mv[1], "mean_return": (mv[2] / mv[1]) if mv[1] else None,
                                "nan_rewards": mv[6], "terminated": mv[4], "truncated": mv[5], "env_steps": mv[0],
                                # what the timed steps were: truncation flags per (agent-)step and episode ends in the
                                # window (MARL: the wrapper's __all__ ignores truncation, marl_wrapper.py:113-117, so
                                # truncated envs keep stepping -- the steady state under random actions)
                                "truncated_fraction": mv[5] / max(mv[0] * (n if mode == "marl" else 1), 1.0),
                                "episode_ends_in_window": mv[1]},
        }
        fr, fr_why = counter_record("flock_roofline")
        out["flock_roofline"] = fr.get("records") and {k: fr[k] for k in ("records", "flop_model", "peak_tflops", "note",
                                                                         "source") if k in fr} or fr_why
        if args.policy and mode == "ctde":
            out["policy_rollout"] = policy_rollout(b, n, args.steps, args.warmup)
        if args.train and mode == "ctde":
            out["ppo_train_iteration"] = ppo_train_iteration(b)
        if args.policy and mode == "marl":
            out["marl_ppo_rollout"] = marl_ppo_rollout(b)
        if mode == "marl" and not args.no_extras:
            out["near_herd_leg"] = near_herd_leg(b, n, m, multi=multi_ran)
        if args.marl_vec and mode == "marl":
            b.close()
            out["marl_vec_env"] = marl_vec_rollout(n, m, E, args.steps, args.warmup, args.burn_in)
        if not args.no_extras and world == 1:
            out["host_surfaces"] = host_surfaces(args.steps)
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(mode, n, m, args.cpu_seconds)
        elif world == 1:
            out["cpu_baseline"] = None
    b.close()
    D.shutdown()
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
