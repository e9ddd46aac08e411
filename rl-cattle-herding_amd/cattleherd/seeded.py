"""Seed-exact resets: the reference env's own random draws, replayed on the host.

The reference draws from the process-global generators and never seeds them (BaseAviary.reset ignores
``seed``).  A run is reproducible only if the caller seeds them first -- ``random.seed(s);
np.random.seed(s)`` before constructing the env.  ``ReferenceResetRNG(s, ...)`` replays what such an env
draws, in its order:

* construction: NUM_DRONES = random.randint(min, max) (sb3_envs/BaseAviary.py:242), then _housekeeping's
  per-cow draws;
* per cow spawned (the first min(M, 16), BaseAviary.py:611): a yaw np.pi * (2 np.random.rand() - 1) (617,
  only orients the cube) and a velocity angle the same way (631); velocity = 0.2 (cos, sin) (632);
* per flocking step (every second step_counter_A, BaseAviary.py:454-455): drift noise
  np.random.normal(0, 0.02, (M, 2)) (1373), preceded once per env lifetime by
  np.random.uniform(-0.1, 0.1, (M, 2)) (1366).  The noise is never used, but it moves the stream, so a
  reset's draws depend on how many flocking steps the previous episodes took;
* reset: NUM_DRONES = random.randint(min, max) (307), then the per-cow draws.

``reset(step_counter_A)`` takes the number of steps of the episode that ends (its step_counter_A) and
returns (NUM_DRONES, cow velocities [M, 2]) for ``HerdBatch.reset(num_drones=..., cow_vel=...)``
(ch_reset_with).  The velocities are computed here with NumPy, exactly as the reference does, so the
injected reset state is bit-identical to the reference's.
"""
import random

import numpy as np

MAX_VEL_CATTLE = 0.2   # BaseAviary.py:579
SPAWN_COWS = 16        # cows per scenario in config/cattle_positions.yaml


class ReferenceResetRNG:
    def __init__(self, seed, min_drones, max_drones, num_cattle):
        self.py = random.Random(seed)
        self.np = np.random.RandomState(seed)
        self.min_drones, self.max_drones, self.m = int(min_drones), int(max_drones), int(num_cattle)
        self._drift = False
        self.ctor_num_drones = self.py.randint(self.min_drones, self.max_drones)   # __init__ (242)
        self._cows()                                                                # __init__'s _housekeeping

    def _cows(self):
        vel = np.zeros((self.m, 2), np.float64)
        for j in range(min(self.m, SPAWN_COWS)):
            np.pi * (2 * self.np.rand() - 1)                  # yaw (617)
            a = np.pi * (2 * self.np.rand() - 1)              # velocity angle (631)
            vel[j] = (MAX_VEL_CATTLE * np.array([np.cos(a), np.sin(a), 0.0]))[:2]
        return vel

    def flocking_steps(self, k):
        for _ in range(int(k)):
            if not self._drift:
                self.np.uniform(-0.1, 0.1, size=(self.m, 2))   # 1366
                self._drift = True
            self.np.normal(0, 0.02, size=(self.m, 2))          # 1373

    def reset(self, step_counter_A=0):
        """Draws of the reset that follows an episode of ``step_counter_A`` steps."""
        self.flocking_steps(int(step_counter_A) // 2)
        n = self.py.randint(self.min_drones, self.max_drones)
        return n, self._cows()
