"""CPU test of the seed-exact reset replay (cattleherd.seeded) against the reference's own draws under
seeded global RNGs (tests/golden/reset_seeded.npz, make_golden.py gen_reset_seeded: BaseAviary.py:242,
307, 617, 631, 1366, 1373): NUM_DRONES and the cattle spawn velocities of every reset, bit for bit."""
import numpy as np

from helpers import load


def test_replay_reproduces_reference_reset_draws():
    from cattleherd.seeded import ReferenceResetRNG
    d = load("reset_seeded.npz")
    for si, seed in enumerate(d["seeds"]):
        rng = ReferenceResetRNG(int(seed), 4, 12, 16)   # CTDE level 7: 4..12 drones (curriculum_learning.py:172-193)
        assert rng.ctor_num_drones == int(d[f"s{si}_ctor_n"])
        for k in range(len(d["schedule"])):
            n, vel = rng.reset(int(d[f"s{si}_scA_before"][k]))
            assert n == int(d[f"s{si}_n"][k]), (seed, k)
            assert np.array_equal(vel, d[f"s{si}_cow_vel"][k]), (seed, k)
