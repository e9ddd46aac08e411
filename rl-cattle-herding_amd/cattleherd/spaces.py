"""Action / observation spaces and enums matching the reference's (utils/enums.py,
BaseRLAviary._actionSpace/_observationSpace at sb3_envs/BaseRLAviary.py:106-133, 243-267,
BaseMARLAviary.py:106-130, 241-248).

Uses gymnasium.spaces.Box when gymnasium is importable (SB3 / RLlib need it); otherwise a minimal
Box with the same attributes, so the adapters import in environments without gymnasium.
"""
from enum import Enum

import numpy as np

try:  # pragma: no cover - gymnasium is not installed in the build container
    from gymnasium import spaces as _gspaces
    Box = _gspaces.Box
except Exception:  # noqa: BLE001
    class Box:
        """Stand-in for gymnasium.spaces.Box (low, high, shape, dtype, sample, contains)."""

        def __init__(self, low, high, shape=None, dtype=np.float32):
            low = np.asarray(low, dtype=dtype)
            high = np.asarray(high, dtype=dtype)
            if shape is not None:
                low = np.broadcast_to(low, shape).copy()
                high = np.broadcast_to(high, shape).copy()
            self.low, self.high, self.dtype = low, high, np.dtype(dtype)
            self.shape = low.shape

        def sample(self, rng=None):
            rng = rng or np.random.default_rng()
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.shape}, {self.dtype})"

# enums: same member names and values as the reference's utils/enums.py, plus DYN_RK4 (the RK4 integrator
# option of include/cattleherd.h CH_PHYS_DYN_RK4, not a reference member)
DroneModel = Enum("DroneModel", [("CF2X", "cf2x"), ("CF2P", "cf2p"), ("RACE", "racer")])
Physics = Enum("Physics", [("PYB", "pyb"), ("DYN", "dyn"), ("PYB_GND", "pyb_gnd"), ("PYB_DRAG", "pyb_drag"),
                           ("PYB_DW", "pyb_dw"), ("PYB_GND_DRAG_DW", "pyb_gnd_drag_dw"), ("DYN_RK4", "dyn_rk4")])
ImageType = Enum("ImageType", [("RGB", 0), ("DEP", 1), ("SEG", 2), ("BW", 3)])
ActionType = Enum("ActionType", [("RPM", "rpm"), ("PID", "pid"), ("VEL", "vel"), ("ONE_D_RPM", "one_d_rpm"),
                                 ("ONE_D_PID", "one_d_pid")])
ObservationType = Enum("ObservationType", [("KIN", "kin"), ("RGB", "rgb"), ("COKIN", "cokin")])

OBS_WIDTH = 86           # 10 + 4*2 + 16*2 + 9*4 (BaseRLAviary.py:262)
GLOBAL_MAX_NUM_DRONES = 12

# curriculum_learning.py:10-194: (min_num_drones, max_num_drones, episode_length seconds) per level -- the one
# host copy of the table the adapters read (the kernels carry the full level table, ch_device.h kLevels)
CURRICULUM = {0: (3, 3, 40), 1: (4, 4, 40), 2: (4, 4, 40), 3: (4, 4, 40), 4: (4, 4, 80), 5: (4, 4, 40),
              6: (4, 12, 80), 7: (4, 12, 80)}
DEFAULT_LEVEL = {"ctde": 7, "marl": 0}   # CattleAviary.py:62 / MARLCattleAviary.py:62


def ctde_action_space(n):
    return Box(low=-np.ones((n, 4)), high=np.ones((n, 4)), dtype=np.float32)


def ctde_observation_space():
    return Box(low=np.full((GLOBAL_MAX_NUM_DRONES, OBS_WIDTH), -np.inf, np.float32),
               high=np.full((GLOBAL_MAX_NUM_DRONES, OBS_WIDTH), np.inf, np.float32), dtype=np.float32)


def agent_action_space():
    return Box(low=-np.ones(4), high=np.ones(4), dtype=np.float32)


def agent_observation_space():
    return Box(low=np.full(OBS_WIDTH, -np.inf, np.float32), high=np.full(OBS_WIDTH, np.inf, np.float32),
               dtype=np.float32)


def check_supported(drone_model, physics, obs, act):
    """The HIP path implements the reference's COKIN/VEL configuration (CattleAviary.py:15-27) under every Physics."""
    def val(x):
        return getattr(x, "value", x)
    if val(drone_model) not in ("cf2x", "cf2p"):
        raise ValueError("[ERROR] in BaseRLAviary.__init()__, no controller is available for the specified drone_model")
    if val(physics) not in ("pyb", "dyn", "pyb_gnd", "pyb_drag", "pyb_dw", "pyb_gnd_drag_dw", "dyn_rk4"):
        raise ValueError(f"physics={val(physics)!r} is not a Physics member (utils/enums.py:13-21)")
    if val(obs) != "cokin":
        raise ValueError("[ERROR] in BaseRLAviary._observationSpace()")
    if val(act) != "vel":
        raise NotImplementedError(f"act={val(act)!r}: only ActionType.VEL is on the HIP path (DESIGN.md scope)")
