"""cattleherd — MI355X-native batched cattle-herding environment (HIP kernels behind a C ABI).

``HerdBatch`` (cattleherd.env) is the device-resident batch of environments; adapters with the
reference's Gymnasium / SB3 VecEnv / RLlib interfaces live in ``cattleherd.vec_env`` and in the
drop-in ``gym_pybullet_drones`` package next to this one.
"""
from ._lib import ChError, EXPORTS, METRIC_NAMES, lib, spawn_table  # noqa: F401

__all__ = ["HerdBatch", "ChError", "lib", "spawn_table"]


def __getattr__(name):
    if name == "HerdBatch":
        from .env import HerdBatch
        return HerdBatch
    raise AttributeError(name)
