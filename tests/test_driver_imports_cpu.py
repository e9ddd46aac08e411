"""The reference's drivers import unchanged with ``rl-cattle-herding_amd/`` first on ``sys.path``.

``tests/golden/driver_imports.json`` lists every ``gym_pybullet_drones.*`` import of
``simulator/CTDECattleHerder.py``, ``DTDECattleHerder.py``, ``DTDEModelPlayback.py`` and ``test.py`` (made by
``tests/golden/make_driver_imports.py`` with ``ast``).  Each one is resolved in a fresh interpreter whose path
holds only the repo package (no reference checkout: the GPU box has none), then again with a reference checkout
behind it when one is present, where the package's overlay ``__path__`` must still pick the repo's modules for
everything the repo defines.  (VERDICT r5 "What's missing" 1; reference ``CTDECattleHerder.py:40-43``,
``DTDECattleHerder.py:11-13``, ``utils/utils.py:10-53``.)
"""
import argparse
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rl-cattle-herding_amd")
REF = "/root/reference"
FIXTURE = os.path.join(ROOT, "tests", "golden", "driver_imports.json")

_PROBE = r"""
import importlib, json, sys
rows = json.loads(sys.argv[1])
out = []
for r in rows:
    m = importlib.import_module(r["module"])
    missing = [n for n in r["names"] if not hasattr(m, n)]
    out.append({"module": r["module"], "file": getattr(m, "__file__", None), "missing": missing})
print(json.dumps(out))
"""


def _rows():
    with open(FIXTURE) as f:
        return json.load(f)["imports"]


def _resolve(pythonpath):
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(pythonpath))
    r = subprocess.run([sys.executable, "-c", _PROBE, json.dumps(_rows())], env=env, cwd="/",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_fixture_covers_the_drivers():
    rows = _rows()
    drivers = {r["driver"] for r in rows}
    assert {"CTDECattleHerder.py", "DTDECattleHerder.py", "DTDEModelPlayback.py"} <= drivers
    mods = {r["module"] for r in rows}
    for m in ("gym_pybullet_drones.utils.Logger", "gym_pybullet_drones.utils.utils",
              "gym_pybullet_drones.sb3_envs.CattleAviary", "gym_pybullet_drones.rllib_envs.marl_wrapper"):
        assert m in mods


def test_driver_imports_resolve_from_repo_alone():
    for r in _resolve([PKG]):
        assert not r["missing"], r
        assert r["file"].startswith(PKG), r


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "gym_pybullet_drones")), reason="no reference checkout")
def test_driver_imports_resolve_from_repo_ahead_of_reference():
    for r in _resolve([PKG, REF]):
        assert not r["missing"], r
        assert r["file"].startswith(PKG), r
    # the overlay reaches the reference for what the repo does not define
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([PKG, REF]))
    code = ("import gym_pybullet_drones.control as c, gym_pybullet_drones.utils.utils as u; "
            "print(list(c.__path__)[0]); print(u.__file__)")
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd="/", capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    ctl, utl = r.stdout.split()
    assert ctl.startswith(REF) and utl.startswith(PKG)


def test_str2bool_and_sync_semantics():
    sys.path.insert(0, PKG)
    from gym_pybullet_drones.utils.utils import str2bool, sync
    for v in ("yes", "TRUE", "t", "Y", "1", True):
        assert str2bool(v) is True
    for v in ("no", "False", "f", "N", "0", False):
        assert str2bool(v) is False
    with pytest.raises(argparse.ArgumentTypeError):
        str2bool("maybe")
    # iteration 3 of a 0.05 s loop started now must not return before 0.15 s have passed
    t0 = time.time()
    sync(3, t0, 0.05)
    assert time.time() - t0 >= 0.149
    # a loop that is already behind does not sleep
    t1 = time.time()
    sync(1, t1 - 10.0, 0.05)
    assert time.time() - t1 < 0.05


def test_logger_log_save_and_csv(tmp_path):
    sys.path.insert(0, PKG)
    import numpy as np
    from gym_pybullet_drones.utils.Logger import Logger
    lg = Logger(logging_freq_hz=60, output_folder=str(tmp_path / "res"), num_drones=2)
    st = np.arange(20, dtype=float)
    for k in range(3):
        lg.log(drone=0, timestamp=k / 60, state=st + k, control=np.zeros(12))
        lg.log(drone=1, timestamp=k / 60, state=-st - k, control=np.ones(12))
    # the reference's reordering (Logger.py:117): pos, vel (10:13), rpy (7:10), ang vel + rpm (13:20)
    want = np.hstack([st[0:3], st[10:13], st[7:10], st[13:20]])
    assert np.array_equal(lg.states[0, :, 0], want)
    assert lg.timestamps.shape[1] == 3 and np.array_equal(lg.controls[1, :, 2], np.ones(12))
    lg.save()
    lg.save_as_csv(comment="t")
    files = os.listdir(tmp_path / "res")
    assert any(f.endswith(".npy") for f in files)
    d = [f for f in files if f.startswith("save-flight-t-")][0]
    csvs = os.listdir(tmp_path / "res" / d)
    assert len(csvs) == 2 * (12 + 3 + 4 + 4)
    x0 = np.loadtxt(tmp_path / "res" / d / "x0.csv", delimiter=",")
    assert np.array_equal(x0[:, 1], lg.states[0, 0, :])
