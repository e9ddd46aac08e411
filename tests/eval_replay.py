"""Replay of tests/golden/eval_ctde.npz (the reference's evaluation logger over a stub-physics rollout,
make_golden.py gen_eval) through the Gymnasium CattleAviary with ``is_evaluating`` set, the batch
state injected before every step; shared by the CPU (oracle-backed FakeBatch) and GPU tests."""
import numpy as np

from helpers import close, load, stack, state_at

_SKIP = ("m", "ctor_level", "episode_len")


def replay(env):
    """Steps env through the fixture; returns (fixture, evaluation_data dict, per-step device distances)."""
    d = load("eval_ctde.npz")
    env.is_evaluating = True
    env.reset()
    resets = set(d["reset_at"].tolist())
    dist = []
    for t in range(len(d["action"])):
        s = state_at(d, "state_", t)
        env.batch.set_state({k: v for k, v in stack([s]).items() if k not in _SKIP})
        env.batch.invalidate_obs()
        env._sync_counts()
        env._tracker.set_step_start(env.batch.get_state())
        _, _, te, tr, _ = env.step(d["action"][t])
        dist.append(env.batch.eval_distances()[0].copy())
        if t in resets:
            assert te or tr, t
            env.reset()
    return d, env.eval_system.evaluation_data(), np.array(dist)


def check(d, ev, rtol=1e-9):
    """The evaluation_data dict against the reference's, field by field."""
    n_ep = len(d["ev_num_drones"])
    assert len(ev["num_drones"]) == n_ep and list(ev["num_drones"]) == d["ev_num_drones"].tolist()
    assert close(ev["time_taken"], d["ev_time_taken"], 1e-15, 0)[0]
    assert close(ev["effectiveness"], d["ev_effectiveness"], 1e-12, 0)[0]
    assert close(np.array([np.array(x) for x in ev["distances"]]), d["ev_distances"], rtol, 1e-12)[0]
    assert [len(x) for x in ev["time_per_step"]] == d["ev_steps_per_episode"].tolist()
    flat = lambda key: [row for ep in ev[key] for row in ep]  # noqa: E731
    assert close(flat("time_per_step"), d["ev_time_per_step"], 1e-15, 0)[0]
    assert close(flat("effectiveness_per_step"), d["ev_effectiveness_per_step"], 1e-12, 0)[0]
    assert close(np.array([np.array(r) for r in flat("distances_per_step")]), d["ev_distances_per_step"], rtol,
                 1e-12)[0]
    for key in ("drone_poses", "cattle_poses", "drone_vel", "cattle_vel"):
        assert close(np.array(flat(f"{key}_per_step")), d[f"ev_{key}_per_step"], 1e-9, 1e-12)[0], key
