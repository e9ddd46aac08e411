"""Golden vectors for the DTDE policy (RLlib half): the reference's trained RLlib PPO weights
(``simulator/policy_weights.pkl``, written by ``simulator/test.py:19-30`` from ``algo.get_weights()``) evaluated by
plain torch float32 on CPU.

The pickle is read WITHOUT unpickling: ``extract_trace.load_data_only`` walks its opcode stream and accepts only
containers, scalars, ``collections.OrderedDict()`` and the numpy array reconstruction globals (the file names no
other global).  It holds the default RLlib PPO RLModule (new API stack, ``vf_share_layers=False``):

* ``encoder.actor_encoder.net.mlp.{0,2}``: Linear(86, 256) tanh Linear(256, 256) tanh;
* ``pi.net.mlp.0``: Linear(256, 8) = DiagGaussian inputs (mean[4], log_std[4]), with ``pi.log_std_clip_param_const``
  (20) -- RLlib's MLP head clamps the log_std half to [-20, 20] when ``clip_log_std`` is set, which PPO's catalog
  does for a DiagGaussian head;
* ``encoder.critic_encoder.net.mlp.{0,2}`` + ``vf.net.mlp.0``: the same encoder shape and Linear(256, 1).

(RLlib is not installed here, so those module semantics are restated from its published design: parity
unpinned beyond these weights and the plain-torch forward below.)

Inputs: per-agent MARL observations (86,) of oracle rollouts -- 6 drones x 8 cattle (the configuration
``test.py:13`` restores), 4 x 32 (configs[4]) and 3 x 8 -- driven by random VEL actions and, for the 6 x 8 case,
closed loop by the trained policy's deterministic action clip(mean, -1, 1).  Writes
``tests/golden/policy_marl_rllib.npz``: the weight arrays, ``obs`` [R, 86], ``logits`` [R, 8] (pi output, log_std
half clamped), ``values`` [R].  Run here (the reference is only in this container):
    python tests/golden/make_policy_marl_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PKL = "/root/reference/gym_pybullet_drones/simulator/policy_weights.pkl"
OUT = os.path.join(HERE, "policy_marl_rllib.npz")


def load_weights(path=PKL):
    sys.path.insert(0, HERE)
    from extract_trace import load_data_only
    d = load_data_only(path)
    return {k: np.ascontiguousarray(v) for k, v in d.items()}


def forward(sd, x):
    """pi logits (log_std half clamped) and values, float32 torch on CPU."""
    t = {k: torch.tensor(v) for k, v in sd.items()}
    with torch.no_grad():
        h = torch.tanh(x @ t["encoder.actor_encoder.net.mlp.0.weight"].t() + t["encoder.actor_encoder.net.mlp.0.bias"])
        h = torch.tanh(h @ t["encoder.actor_encoder.net.mlp.2.weight"].t() + t["encoder.actor_encoder.net.mlp.2.bias"])
        lg = h @ t["pi.net.mlp.0.weight"].t() + t["pi.net.mlp.0.bias"]
        c = float(t["pi.log_std_clip_param_const"][0])
        mean, log_std = lg.chunk(2, dim=-1)
        lg = torch.cat([mean, log_std.clamp(-c, c)], -1)
        v = torch.tanh(x @ t["encoder.critic_encoder.net.mlp.0.weight"].t() + t["encoder.critic_encoder.net.mlp.0.bias"])
        v = torch.tanh(v @ t["encoder.critic_encoder.net.mlp.2.weight"].t() + t["encoder.critic_encoder.net.mlp.2.bias"])
        val = (v @ t["vf.net.mlp.0.weight"].t() + t["vf.net.mlp.0.bias"])[:, 0]
    return lg, val


def main():
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rl-cattle-herding_amd")]
    import oracle as O
    from cattleherd._lib import spawn_table
    sd = load_weights()
    obs = []
    for n, m, env_id, steps, closed in ((6, 8, 0, 30, False), (6, 8, 1, 60, True), (4, 32, 2, 20, False),
                                        (3, 8, 3, 10, False)):
        env = O.Env(1, n, m, spawn_table(m), env_id=env_id, start_level=3)
        o = env.reset()
        for t in range(steps):
            live = o[:env.st.n]
            obs.extend(np.asarray(live, np.float32))
            if closed:
                lg, _ = forward(sd, torch.tensor(np.asarray(live, np.float32)))
                a = lg[:, :4].clamp(-1.0, 1.0).numpy()
            else:
                a = env.random_actions(t)
            o, *_ = env.step(a, autoreset=True)
    x = torch.tensor(np.stack(obs))
    lg, val = forward(sd, x)
    arrays = {k.replace(".", "__"): v for k, v in sd.items()}
    np.savez_compressed(OUT, obs=x.numpy(), logits=lg.numpy(), values=val.numpy(), **arrays)
    print(OUT, x.shape[0], "rows; log_std range", float(lg[:, 4:].min()), float(lg[:, 4:].max()))


if __name__ == "__main__":
    main()
