"""CPU: the measurement tools' host-side counting and the committed search records they produced.

* ``tools/flock_roofline.work`` -- the per-launch work the flock roofline divides by (flocking envs, cheap-pass pairs,
  alpha pairs inside the bump's support, cow-drone pairs, FLOP and bytes) on a hand-built state.
* ``tests/golden/trace_policy_search.json`` -- the closed-loop search over the reference's shipped checkpoints for the
  policy that drove the real-PyBullet trace (``make_trace_policy_search.py``): a negative result, kept
  as data, whose shape the a5 pin relies on (the drone rigid body is pinned by action inversion instead).
"""
import importlib.util
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _flock_roofline():
    spec = importlib.util.spec_from_file_location("flock_roofline", os.path.join(ROOT, "tools", "flock_roofline.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_flock_roofline_work_counts():
    fr = _flock_roofline()
    E, M, N = 3, 4, 4
    pos = np.zeros((E, M, 2))
    # env 0: cows 0.5 m apart on a line -> pairs within 1.2 m: (0,1) (1,2) (2,3) (0,2 at 1.0 m) (1,3 at 1.0 m) = 5
    pos[0, :, 0] = [0.0, 0.5, 1.0, 1.5]
    # env 1: cows 10 m apart -> none in range; env 2: same as env 0 but it does not flock this launch
    pos[1, :, 0] = [0.0, 10.0, 20.0, 30.0]
    pos[2] = pos[0]
    s = {"cow_pos": pos, "step_counter_A": np.array([1, 3, 2]), "n": np.array([4, 2, 4])}
    w = fr.work(s, N)
    assert w["flocking_envs"] == 2                      # step_counter_A + 1 even: envs 0 and 1
    assert w["alpha_pairs"] == 5 and w["cheap_pairs"] == 2 * 6
    assert w["cow_drone_pairs"] == M * 4 + M * 2        # the live drones of each flocking env
    P, F = M * (M - 1) // 2, fr.FLOP
    flop = (P * F["cheap_pair"] + 5 * F["alpha_pair"] + M * 4 * F["cow_drone_pair"] + M * F["cow"]) + \
           (P * F["cheap_pair"] + 0 * F["alpha_pair"] + M * 2 * F["cow_drone_pair"] + M * F["cow"])
    assert w["flop"] == flop
    assert w["bytes"] == (24 * M + 8 * 4) + (24 * M + 8 * 2)


def test_trace_policy_search_record_is_negative():
    with open(os.path.join(ROOT, "tests", "golden", "trace_policy_search.json")) as fh:
        d = json.load(fh)
    cand = [r for r in d["records"] if "seg0" in r]
    assert d["checkpoints"] == len(d["records"]) and d["candidates_3x86"] == len(cand) > 0
    assert all(r["input_width"] == 258 for r in cand)
    assert not d["any_first_step_match"]
    # every 3-drone actor misses the first step's drone velocities by more than their size
    assert min(r["seg0"]["first_step_dv_rel"] for r in cand) > 1.0
