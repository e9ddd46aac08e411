"""CPU tests of the evaluation logging against the reference's own evaluator output
(tests/golden/eval_ctde.npz, make_golden.py gen_eval: BaseAviary.update_evaluation_metrics and
evaluation_episode_trigger, sb3_envs/BaseAviary.py:1406-1450, utils/evaluation.py:5-94):
the oracle's per-drone distance accumulator, and the Gymnasium CattleAviary + Evaluator over the
oracle-backed FakeBatch producing the reference's evaluation_data.pkl contents."""
import numpy as np
import pytest

from eval_replay import check, replay
from fake_batch import FakeBatch
from helpers import close, load, state_at


def test_oracle_distance_accumulator_matches_reference(spawn16):
    """och_step's eval_dist in lockstep over the fixture equals the reference's final episode distances
    (its 2-vector has the value in both components)."""
    import oracle as O
    d = load("eval_ctde.npz")
    s0 = state_at(d, "state_", 0)
    env = O.Env(0, int(s0["n"]), int(s0["m"]), spawn16, start_level=int(s0["ctor_level"]))
    env.reset()
    ends = []
    for t in range(len(d["action"])):
        env.set_state(dict(state_at(d, "state_", t), eval_dist=env.get_state()["eval_dist"]))
        env.step(d["action"][t], autoreset=False)
        if t in set(d["reset_at"].tolist()):
            ends.append(env.get_state()["eval_dist"][:int(s0["n"])].copy())
            env.reset()
    full = [k for k, L in enumerate(d["ev_steps_per_episode"]) if L > 0]
    assert len(ends) == len(full)
    for k, e in zip(full, ends):
        assert close(e, d["ev_distances"][k][:, 0], 1e-9, 1e-12)[0]
        assert np.array_equal(d["ev_distances"][k][:, 0], d["ev_distances"][k][:, 1])


@pytest.fixture
def patched(monkeypatch):
    import importlib
    ca = importlib.import_module("gym_pybullet_drones.sb3_envs.CattleAviary")
    monkeypatch.setattr(ca, "HerdBatch", FakeBatch)
    return ca


def test_cattle_aviary_evaluation_data_matches_reference(patched, tmp_path):
    """The Gymnasium env with is_evaluating over the oracle: the evaluation_data dict equals the
    reference's (episode entries incl. the doubled time-out trigger, per-step rows incl. the time-out
    step landing in the next episode, aliased distance rows); save_evaluation_data writes it."""
    d = load("eval_ctde.npz")
    s0 = state_at(d, "state_", 0)
    env = patched.CattleAviary(num_drones=int(s0["n"]), num_cattle=int(s0["m"]), curriculum_level=int(d["level"]))
    d, ev, _ = replay(env)
    check(d, ev)
    path = tmp_path / "evaluation_data.pkl"
    env.evaluation_save(str(path))
    assert path.stat().st_size > 0


def _tracker_state(drone_xyz, cow_xy):
    drone = np.asarray(drone_xyz, np.float64)[None]
    cows = np.asarray(cow_xy, np.float64)[None]
    return {"drone_pos": drone, "drone_vel": np.zeros_like(drone), "cow_pos": cows, "cow_vel": np.zeros_like(cows)}


@pytest.mark.parametrize("case,drones,want", [
    ("clean time-out", [[0, 0, 0.45], [1.75, 0, 0.45], [3.5, 0, 0.45]], 2),
    ("altitude loss", [[0, 0, 0.80], [1.75, 0, 0.45], [3.5, 0, 0.45]], 0),
    ("collision", [[0, 0, 0.45], [0.1, 0, 0.45], [3.5, 0, 0.45]], 0),
    ("isolated drone", [[0, 0, 0.45], [1.75, 0, 0.45], [30, 0, 0.45]], 0),
    ("mission boundary", [[40, 0, 0.45], [41.75, 0, 0.45], [43.5, 0, 0.45]], 0),
])
def test_time_out_trigger_only_when_no_failure_truncation(case, drones, want):
    """_computeTruncated returns at its first failure condition (CattleAviary.py:513-542), so the time-out
    branch and its evaluation_episode_trigger (545-548) run only when none holds: a failure on the
    time-out step logs no episode entry."""
    from cattleherd.evaluation import EvalTracker, Evaluator, failure_truncation
    cows = [[2.0, 8.0], [3.0, 9.0], [1.0, 9.5], [2.5, 10.0]]
    s = _tracker_state(drones, cows)
    assert failure_truncation(s, 0, 3) == (want == 0), case
    ev = Evaluator()
    tr = EvalTracker(ev)
    tr.on_reset(s, 3)
    tr.after_step(s, np.zeros(3), 3, 4, step_counter_before=4804, ctrl_freq=60, episode_len_sec=80)
    assert len(ev.total_time_taken) == want, case
    assert len(ev.curr_time) == 1   # the step itself is logged either way (update_evaluation_metrics)
