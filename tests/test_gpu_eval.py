"""GPU test of the evaluation logging against the reference's own evaluator output
(tests/golden/eval_ctde.npz; BaseAviary.py:1406-1450, utils/evaluation.py:5-94): the Gymnasium
CattleAviary with is_evaluating over the HIP batch, the per-drone distances accumulated in the step
kernel (ch_get_eval), the evaluation_data dict field by field."""
import pytest

from eval_replay import check, replay
from helpers import load, state_at

pytestmark = pytest.mark.gpu


def test_cattle_aviary_evaluation_data_matches_reference_on_gpu():
    from gym_pybullet_drones.sb3_envs.CattleAviary import CattleAviary
    d = load("eval_ctde.npz")
    s0 = state_at(d, "state_", 0)
    env = CattleAviary(num_drones=int(s0["n"]), num_cattle=int(s0["m"]), curriculum_level=int(d["level"]))
    d, ev, dist = replay(env)
    check(d, ev)
    assert dist.shape == (len(d["action"]), int(s0["n"]))
    env.close()
