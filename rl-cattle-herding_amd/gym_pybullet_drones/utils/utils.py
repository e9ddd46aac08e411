"""Helpers the reference's drivers import from ``gym_pybullet_drones.utils.utils``.

``CTDECattleHerder.py:42`` takes ``sync`` and ``str2bool``; ``DTDECattleHerder.py:12`` and
``DTDEModelPlayback.py:12`` take ``str2bool``.  Restated from the reference's ``utils/utils.py:10-53``
(same arguments, return values and errors); the 2-vector helpers below them (``utils.py:57-134``) are
used by ``flockUtils.py``, whose arithmetic the HIP kernels and the oracle restate, and are kept here
so ``import gym_pybullet_drones.utils.utils as utils`` works for any caller.
"""
import argparse
import math
import time

import numpy as np

_TRUE = frozenset(("yes", "true", "t", "y", "1"))
_FALSE = frozenset(("no", "false", "f", "n", "0"))


def sync(i, start_time, timestep):
    """Sleep so that iteration ``i`` of a loop stepping every ``timestep`` s does not run ahead of the
    wall clock started at ``start_time``.  Checked on every iteration when ``timestep`` > 0.04 s, else on
    every ``int(1 / (24 timestep))``-th (reference ``utils.py:10-29``)."""
    if timestep > .04 or i % int(1 / (24 * timestep)) == 0:
        behind = i * timestep - (time.time() - start_time)
        if behind > 0:
            time.sleep(behind)


def str2bool(val):
    """argparse ``type=`` for booleans: a bool passes through, yes/true/t/y/1 and no/false/f/n/0 (any case)
    map to True/False, anything else raises ``argparse.ArgumentTypeError`` (reference ``utils.py:33-54``)."""
    if isinstance(val, bool):
        return val
    v = val.lower()
    if v in _TRUE:
        return True
    if v in _FALSE:
        return False
    raise argparse.ArgumentTypeError("[ERROR] in str2bool(), a Boolean value is expected")


def unit_vector(vector):
    """``v / (1 + ‖v‖)`` (reference ``utils.py:57, 133``; the name is the reference's)."""
    return np.array(vector) / (1 + np.linalg.norm(vector))


def randrange(a, b):
    """A uniform draw in [a, b) from NumPy's global generator (reference ``utils.py:60-62``)."""
    return a + np.random.random() * (b - a)


def norm2(vector):
    """Squared norm of the first two components (reference ``utils.py:80-82``)."""
    return vector[0] * vector[0] + vector[1] * vector[1]


def norm(vector):
    """Norm of the first two components (reference ``utils.py:75-77``)."""
    return math.sqrt(vector[0] ** 2 + vector[1] ** 2)


def dist2(a, b):
    return norm2(a - b)


def dist(a, b):
    return norm(a - b)


def normalize(vector, pre_computed=None):
    """``vector / ‖vector‖``, or zeros(2) below 1e-13 (reference ``utils.py:107-121``)."""
    n = norm(vector) if pre_computed is None else pre_computed
    if n < 1e-13:
        return np.zeros(2)
    return np.array(vector) / n


def truncate(vector, max_length):
    """Scale ``vector`` down to ``max_length`` if it is longer (reference ``utils.py:124-130``)."""
    n = norm(vector)
    return normalize(vector, pre_computed=n) * max_length if n > max_length else vector
