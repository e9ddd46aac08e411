"""Stub modules that let the reference's own Python import and run in THIS container.

Generator-side only (used by ``make_golden.py``; never imported by tests, smoke() or bench.py,
and never shipped to the GPU box as code that runs there).

The reference (``/root/reference/gym_pybullet_drones``) imports ``pybullet``, ``pybullet_data``,
``gymnasium`` and ``ray`` — none is installed here (plain ``ModuleNotFoundError``; nothing was
refused).  We insert tiny stand-ins into ``sys.modules``:

* ``gymnasium``: ``Env``, ``spaces.Box``, ``envs.registration.register`` — pure containers.
* ``ray.rllib.env.MultiAgentEnv`` — empty base class.
* ``pybullet``: the quaternion helpers restated from pybullet.c
  (``getQuaternionFromEuler`` / ``getEulerFromQuaternion`` / ``getMatrixFromQuaternion``) and a
  rigid-body world that models what ``p.stepSimulation`` does to the bodies the reference loads:
  drones = one btMultiBody base (m, diag J from cf2x.urdf) with link forces at the prop offsets,
  default damping ``-m v (k + k|v|)``, gyroscopic term, semi-implicit Euler + exponential-map
  quaternion update; cattle cubes = frictionless constant-velocity xy bodies (the behaviour the
  recorded trace ``evaluation_data.pkl`` pins to 3.6e-15).  This physics model is OURS (Bullet is
  not available, so it is "parity unpinned"); the golden vectors therefore pin everything the
  reference computes AROUND the physics — PID, flocking, observations, rewards, termination,
  truncation, curriculum and reset bookkeeping — with this model in the loop.

The physics switches mirror ``ch_config`` in ``include/cattleherd.h`` so the oracle and the HIP
path can be run under exactly the same model.
"""
import math
import sys
import types

import numpy as np

REF_ROOT = "/root/reference"

# Physics-model switches (defaults = the product defaults, see DESIGN.md "Physics model").
PHYS = {
    "damping": 0.04,          # btMultiBody default linear/angular damping (k1 = k2)
    "torque_world": True,     # applyExternalTorque(LINK_FRAME) treated as world frame (Bullet multibody path)
    "gyro": True,             # btMultiBody::m_useGyroTerm default
    # LINK_FRAME forces / torques on a drone's links rotate by the link transform Bullet cached at the previous
    # stepSimulation's forward kinematics (the attitude one substep old), refreshed early only by
    # getLinkStates(computeForwardKinematics=1); pinned by the real-PyBullet trace (make_trace_inverse.py)
    "link_lag": True,
}

# --------------------------------------------------------------------------------------
# pybullet.c quaternion conventions (x, y, z, w)
# --------------------------------------------------------------------------------------

def getQuaternionFromEuler(rpy):
    phi, the, psi = rpy[0] / 2.0, rpy[1] / 2.0, rpy[2] / 2.0
    q = [math.sin(phi) * math.cos(the) * math.cos(psi) - math.cos(phi) * math.sin(the) * math.sin(psi),
         math.cos(phi) * math.sin(the) * math.cos(psi) + math.sin(phi) * math.cos(the) * math.sin(psi),
         math.cos(phi) * math.cos(the) * math.sin(psi) - math.sin(phi) * math.sin(the) * math.cos(psi),
         math.cos(phi) * math.cos(the) * math.cos(psi) + math.sin(phi) * math.sin(the) * math.sin(psi)]
    n = math.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    return tuple(c / n for c in q)


def getEulerFromQuaternion(q):
    x, y, z, w = float(q[0]), float(q[1]), float(q[2]), float(q[3])
    sqx, sqy, sqz, squ = x * x, y * y, z * z, w * w
    sarg = -2.0 * (x * z - w * y)
    if sarg <= -0.99999:
        return (0.0, -0.5 * math.pi, 2.0 * math.atan2(x, -y))
    if sarg >= 0.99999:
        return (0.0, 0.5 * math.pi, 2.0 * math.atan2(-x, y))
    return (math.atan2(2.0 * (y * z + w * x), squ - sqx - sqy + sqz),
            math.asin(sarg),
            math.atan2(2.0 * (x * y + w * z), squ + sqx - sqy - sqz))


def getMatrixFromQuaternion(q):
    x, y, z, w = float(q[0]), float(q[1]), float(q[2]), float(q[3])
    d = x * x + y * y + z * z + w * w
    s = 2.0 / d
    xs, ys, zs = x * s, y * s, z * s
    wx, wy, wz = w * xs, w * ys, w * zs
    xx, xy, xz = x * xs, x * ys, x * zs
    yy, yz, zz = y * ys, y * zs, z * zs
    return (1.0 - (yy + zz), xy - wz, xz + wy,
            xy + wz, 1.0 - (xx + zz), yz - wx,
            xz - wy, yz + wx, 1.0 - (xx + yy))


def quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return (aw * bx + ax * bw + ay * bz - az * by,
            aw * by + ay * bw + az * bx - ax * bz,
            aw * bz + az * bw + ax * by - ay * bx,
            aw * bw - ax * bx - ay * by - az * bz)


# --------------------------------------------------------------------------------------
# Rigid-body world
# --------------------------------------------------------------------------------------

CF2X_MASS = 0.027
CF2X_J = (1.4e-5, 1.4e-5, 2.17e-5)
PROP_OFFSETS = ((0.028, -0.028, 0.0), (-0.028, -0.028, 0.0), (-0.028, 0.028, 0.0), (0.028, 0.028, 0.0))


class _Body:
    def __init__(self, kind, pos, quat):
        self.kind = kind
        self.pos = [float(c) for c in pos]
        self.quat = [float(c) for c in quat]
        self.vel = [0.0, 0.0, 0.0]
        self.angv = [0.0, 0.0, 0.0]
        self.force = [0.0, 0.0, 0.0]      # world frame, at COM
        self.torque = [0.0, 0.0, 0.0]     # world frame
        self.cached = list(self.quat)     # the links' cached world transform (attitude part), set by loadURDF


class _World:
    def __init__(self):
        self.reset()

    def reset(self):
        self.bodies = {}
        self.next_id = 0
        self.dt = 1.0 / 240.0
        self.g = 9.8

    def add(self, kind, pos, quat):
        bid = self.next_id
        self.next_id += 1
        self.bodies[bid] = _Body(kind, pos, quat)
        return bid


WORLD = _World()


def _R(q):
    m = getMatrixFromQuaternion(q)
    return np.array(m, dtype=np.float64).reshape(3, 3)


def _step_drone(b, dt, g):
    b.cached = list(b.quat)   # stepSimulation's forward kinematics, before the integration
    R = _R(b.quat)
    m = CF2X_MASS
    J = np.array(CF2X_J)
    v = np.array(b.vel)
    w = np.array(b.angv)
    F = np.array(b.force) + np.array([0.0, 0.0, -m * g])
    tau_w = np.array(b.torque)
    k = PHYS["damping"]
    if k != 0.0:
        F = F - m * v * (k + k * math.sqrt(v @ v))
    wb = R.T @ w
    tb = R.T @ tau_w
    if k != 0.0:
        tb = tb - J * wb * (k + k * math.sqrt(wb @ wb))
    if PHYS["gyro"]:
        tb = tb - np.cross(wb, J * wb)
    alpha_w = R @ (tb / J)
    v = v + (F / m) * dt
    w = w + alpha_w * dt
    p = np.array(b.pos) + v * dt
    # exponential-map quaternion update (btMultiBody::stepPositionsMultiDof, base body)
    fang = math.sqrt(w @ w)
    if fang * dt > 0.5 * (0.5 * math.pi):
        fang = 0.5 * (0.5 * math.pi) / dt
    if fang < 0.001:
        axis = w * (0.5 * dt - (dt * dt * dt) * 0.020833333333 * fang * fang)
    else:
        axis = w * (math.sin(0.5 * fang * dt) / fang)
    dq = (axis[0], axis[1], axis[2], math.cos(fang * dt * 0.5))
    q = quat_mul(dq, b.quat)
    n = math.sqrt(sum(c * c for c in q))
    b.quat = [c / n for c in q]
    b.pos = list(p)
    b.vel = list(v)
    b.angv = list(w)


def _step_world():
    dt, g = WORLD.dt, WORLD.g
    for b in WORLD.bodies.values():
        if b.kind == "drone":
            _step_drone(b, dt, g)
        elif b.kind == "cow":
            b.pos[0] += b.vel[0] * dt
            b.pos[1] += b.vel[1] * dt
        b.force = [0.0, 0.0, 0.0]
        b.torque = [0.0, 0.0, 0.0]


def _make_pybullet():
    p = types.ModuleType("pybullet")
    p.DIRECT, p.GUI = 2, 1
    p.LINK_FRAME, p.WORLD_FRAME = 1, 2
    p.URDF_USE_INERTIA_FROM_FILE = 2
    p.GEOM_SPHERE = 2
    p.ER_TINY_RENDERER = 0
    p.ER_SEGMENTATION_MASK_OBJECT_AND_LINKINDEX = 0
    p.ER_NO_SEGMENTATION_MASK = 0
    p.connect = lambda *a, **k: 0
    p.disconnect = lambda *a, **k: None
    p.setGravity = lambda x, y, z, **k: setattr(WORLD, "g", -float(z))
    p.setRealTimeSimulation = lambda *a, **k: None
    p.setTimeStep = lambda dt, **k: setattr(WORLD, "dt", float(dt))
    p.setAdditionalSearchPath = lambda *a, **k: None
    p.resetSimulation = lambda **k: WORLD.reset()
    p.getQuaternionFromEuler = getQuaternionFromEuler
    p.getEulerFromQuaternion = getEulerFromQuaternion
    p.getMatrixFromQuaternion = getMatrixFromQuaternion
    p.createVisualShape = lambda *a, **k: -1

    def createMultiBody(**k):
        return WORLD.add("marker", k.get("basePosition", [0, 0, 0]), [0, 0, 0, 1])
    p.createMultiBody = createMultiBody

    def loadURDF(fname, basePosition=(0, 0, 0), baseOrientation=(0, 0, 0, 1), **k):
        f = str(fname)
        if f.endswith("plane.urdf"):
            kind = "plane"
        elif "cube" in f:
            kind = "cow"
        else:
            kind = "drone"
        return WORLD.add(kind, basePosition, baseOrientation)
    p.loadURDF = loadURDF

    def getBasePositionAndOrientation(bid, **k):
        b = WORLD.bodies[int(bid)]
        return tuple(b.pos), tuple(b.quat)
    p.getBasePositionAndOrientation = getBasePositionAndOrientation

    def getBaseVelocity(bid, **k):
        b = WORLD.bodies[int(bid)]
        return tuple(b.vel), tuple(b.angv)
    p.getBaseVelocity = getBaseVelocity

    def resetBaseVelocity(bid, linearVelocity=None, angularVelocity=None, **k):
        b = WORLD.bodies[int(bid)]
        if linearVelocity is not None:
            b.vel = [float(c) for c in linearVelocity]
        if angularVelocity is not None:
            b.angv = [float(c) for c in angularVelocity]
    p.resetBaseVelocity = resetBaseVelocity

    def resetBasePositionAndOrientation(bid, pos, quat, **k):
        b = WORLD.bodies[int(bid)]
        b.pos = [float(c) for c in pos]
        b.quat = [float(c) for c in quat]
    p.resetBasePositionAndOrientation = resetBasePositionAndOrientation

    def applyExternalForce(bid, link, forceObj, posObj, flags, **k):
        b = WORLD.bodies[int(bid)]
        R = _R(b.quat)
        Rf = _R(b.cached) if (PHYS["link_lag"] and link >= 0) else R
        f = Rf @ np.array(forceObj, dtype=np.float64)         # link frame == base frame (fixed joints)
        if 0 <= link <= 3:
            r = R @ np.array(PROP_OFFSETS[link])
        else:
            r = np.zeros(3)
        t = np.cross(r, f)
        for i in range(3):
            b.force[i] += f[i]
            b.torque[i] += t[i]
    p.applyExternalForce = applyExternalForce

    def applyExternalTorque(bid, link, torqueObj, flags, **k):
        b = WORLD.bodies[int(bid)]
        t = np.array(torqueObj, dtype=np.float64)
        if PHYS["link_lag"] and link >= 0:
            t = _R(b.cached) @ t
        elif not PHYS["torque_world"]:
            t = _R(b.quat) @ t
        for i in range(3):
            b.torque[i] += t[i]
    p.applyExternalTorque = applyExternalTorque

    def getLinkStates(bid, linkIndices, computeLinkVelocity=0, computeForwardKinematics=0, **k):
        # linkWorldPosition (entry 0) = the link's centre of mass: the prop offsets of cf2x.urdf
        # (links 0-3, inertial origins at +-0.028) or the base origin (link 4)
        b = WORLD.bodies[int(bid)]
        R = _R(b.quat)
        if computeForwardKinematics:
            b.cached = list(b.quat)
        out = []
        for li in linkIndices:
            off = PROP_OFFSETS[li] if 0 <= li <= 3 else (0.0, 0.0, 0.0)
            pos = tuple(np.array(b.pos) + R @ np.array(off))
            out.append((pos, tuple(b.quat), (0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0), pos, tuple(b.quat),
                        tuple(b.vel), tuple(b.angv)))
        return out
    p.getLinkStates = getLinkStates
    p.stepSimulation = lambda **k: _step_world()
    p.changeDynamics = lambda *a, **k: None
    return p


def install():
    """Insert the stub modules and make the reference package importable (read-only)."""
    if "pybullet" in sys.modules and getattr(sys.modules["pybullet"], "_is_stub", False):
        return
    p = _make_pybullet()
    p._is_stub = True
    sys.modules["pybullet"] = p
    pd = types.ModuleType("pybullet_data")
    pd.getDataPath = lambda: "/nonexistent"
    sys.modules["pybullet_data"] = pd

    gym = types.ModuleType("gymnasium")

    class Env:
        pass
    gym.Env = Env
    spaces = types.ModuleType("gymnasium.spaces")

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low = np.asarray(low, dtype=dtype)
            self.high = np.asarray(high, dtype=dtype)
            self.shape = self.low.shape if shape is None else tuple(shape)
            self.dtype = dtype
    spaces.Box = Box
    gym.spaces = spaces
    envs = types.ModuleType("gymnasium.envs")
    reg = types.ModuleType("gymnasium.envs.registration")
    reg.register = lambda **k: None
    envs.registration = reg
    gym.envs = envs
    sys.modules.update({"gymnasium": gym, "gymnasium.spaces": spaces,
                        "gymnasium.envs": envs, "gymnasium.envs.registration": reg})

    ray = types.ModuleType("ray")
    rllib = types.ModuleType("ray.rllib")
    renv = types.ModuleType("ray.rllib.env")

    class MultiAgentEnv:
        def __init__(self, *a, **k):
            pass
    renv.MultiAgentEnv = MultiAgentEnv
    ray.rllib = rllib
    rllib.env = renv
    sys.modules.update({"ray": ray, "ray.rllib": rllib, "ray.rllib.env": renv})

    # Namespace package pointing at the read-only reference (skips its gymnasium registrations).
    pkg = types.ModuleType("gym_pybullet_drones")
    pkg.__path__ = [REF_ROOT + "/gym_pybullet_drones"]
    sys.modules["gym_pybullet_drones"] = pkg
    for sub in ("sb3_envs", "rllib_envs", "utils", "control"):
        m = types.ModuleType("gym_pybullet_drones." + sub)
        m.__path__ = [REF_ROOT + "/gym_pybullet_drones/" + sub]
        sys.modules["gym_pybullet_drones." + sub] = m
    import pkg_resources
    _orig = pkg_resources.resource_filename

    def resource_filename(pkgname, res):
        if pkgname == "gym_pybullet_drones":
            return REF_ROOT + "/gym_pybullet_drones/" + res
        return _orig(pkgname, res)
    pkg_resources.resource_filename = resource_filename
