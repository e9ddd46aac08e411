"""GPU test of seed-exact resets: the Gymnasium CattleAviary with ``reference_rng_seed`` reproduces, bit
for bit, the reset states the reference produces after ``random.seed(s); np.random.seed(s)``
(tests/golden/reset_seeded.npz, make_golden.py gen_reset_seeded): NUM_DRONES, drone start positions,
cattle spawn positions and velocities, spawn index -- across resets separated by different numbers of
steps (the reference's unused drift noise, BaseAviary.py:1373, moves the NumPy stream every flocking step).
The host replays the draws (cattleherd/seeded.py) and ch_reset_with injects them."""
import numpy as np
import pytest

from helpers import load

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("si", [0, 1])
def test_seeded_resets_match_reference_bit_for_bit(si):
    from gym_pybullet_drones.sb3_envs.CattleAviary import CattleAviary
    d = load("reset_seeded.npz")
    seed = int(d["seeds"][si])
    env = CattleAviary(num_drones=12, num_cattle=16, reference_rng_seed=seed)
    rng = np.random.default_rng(5)
    for k, steps in enumerate(d["schedule"]):
        env.reset()
        s = env.batch.get_state()
        n = int(d[f"s{si}_n"][k])
        assert int(s["n"][0]) == n == env.NUM_DRONES, (seed, k)
        assert np.array_equal(s["cow_vel"][0, :16], d[f"s{si}_cow_vel"][k]), (seed, k)
        assert np.array_equal(s["cow_pos"][0, :16], d[f"s{si}_cow_pos"][k]), (seed, k)
        assert np.array_equal(s["drone_pos"][0, :n], d[f"s{si}_drone_pos"][k][:n]), (seed, k)
        assert int(s["spawn_index"][0]) == int(d[f"s{si}_spawn_index"][k]), (seed, k)
        assert int(s["step_counter_A"][0]) == 0
        for _ in range(int(steps)):
            env.step(rng.uniform(-1, 1, (12, 4)).astype(np.float32))
        assert env.step_counter_A == int(steps)
    env.close()
