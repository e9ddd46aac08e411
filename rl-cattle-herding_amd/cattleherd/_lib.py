"""ctypes binding of libcattleherd.so (C ABI in include/cattleherd.h).

The product path has no CPU fallback: if the HIP library is missing or no device is visible,
``lib()`` / ``HerdBatch`` raise.
"""
import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CH_LIB_PATH") or os.path.join(_PKG, "libcattleherd.so")  # override: A/B diagnostics

CH_OK, CH_ERR_INVALID, CH_ERR_DEVICE, CH_ERR_NOMEM, CH_ERR_UNSUPPORTED = 0, -1, -2, -3, -4
CH_MODE_CTDE, CH_MODE_MARL = 0, 1
CH_PREC_F64, CH_PREC_F32 = 0, 1
CH_STEP_AUTORESET, CH_STEP_RANDOM_ACTIONS = 0x1, 0x2
METRIC_NAMES = ("steps", "episodes", "return_sum", "length_sum", "terminated", "truncated", "nan_rewards",
                "effectiveness_sum")
ABI_VERSION = 6
# Physics enum (utils/enums.py:13-21, include/cattleherd.h CH_PHYS_*)
PHYSICS = {"pyb": 0, "dyn": 1, "pyb_gnd": 2, "pyb_drag": 3, "pyb_dw": 4, "pyb_gnd_drag_dw": 5, "dyn_rk4": 6}

# every symbol include/cattleherd.h declares
EXPORTS = ("ch_default_config", "ch_create", "ch_destroy", "ch_last_error", "ch_shape", "ch_reset", "ch_reset_with",
           "ch_step", "ch_step_n",
           "ch_state_size", "ch_get_state", "ch_set_state", "ch_metrics", "ch_metrics_device", "ch_sync",
           "ch_get_eval", "ch_builtin_spawn_table", "ch_rollout_store", "ch_rollout_post", "ch_rollout_gae", "ch_rollout_collect",
           "ch_spawn_table", "ch_mlp_forward", "ch_mlp_forward_masked", "ch_policy_forward", "ch_mlp_packed_size",
           "ch_mlp_pack", "ch_outputs_to_host", "ch_marl_rollout_collect")
CH_ACT_NONE, CH_ACT_TANH, CH_ACT_RELU = 0, 1, 2


class ChConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("mode", ctypes.c_int32), ("num_drones", ctypes.c_int32),
                ("num_cattle", ctypes.c_int32), ("min_drones", ctypes.c_int32), ("max_drones", ctypes.c_int32),
                ("curriculum_level", ctypes.c_int32), ("ctrl_freq", ctypes.c_int32), ("pyb_freq", ctypes.c_int32),
                ("compat", ctypes.c_int32), ("precision", ctypes.c_int32), ("torque_world", ctypes.c_int32),
                ("gyro", ctypes.c_int32), ("marl_wrapper", ctypes.c_int32), ("damping", ctypes.c_double), ("seed", ctypes.c_uint64),
                ("env_id_offset", ctypes.c_int64), ("spawn_table", ctypes.POINTER(ctypes.c_double)),
                ("spawn_scenarios", ctypes.c_int32), ("spawn_cows", ctypes.c_int32), ("physics", ctypes.c_int32),
                ("eval_metrics", ctypes.c_int32), ("link_lag", ctypes.c_int32)]


class ChStepIO(ctypes.Structure):
    _fields_ = [("actions", ctypes.c_void_p), ("actions_out", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("reward", ctypes.c_void_p), ("terminated", ctypes.c_void_p), ("truncated", ctypes.c_void_p),
                ("terminal_obs", ctypes.c_void_p), ("agent_active", ctypes.c_void_p),
                ("reset_happened", ctypes.c_void_p), ("flags", ctypes.c_uint32), ("_pad", ctypes.c_uint32),
                ("episode_stats", ctypes.c_void_p)]


class ChHostOut(ctypes.Structure):
    _fields_ = [("obs", ctypes.c_void_p), ("reward", ctypes.c_void_p), ("terminated", ctypes.c_void_p),
                ("truncated", ctypes.c_void_p), ("reset_happened", ctypes.c_void_p), ("agent_active", ctypes.c_void_p),
                ("ended_count", ctypes.c_int64), ("ended_env", ctypes.c_void_p), ("ended_obs", ctypes.c_void_p),
                ("ended_stats", ctypes.c_void_p)]


class ChMlp(ctypes.Structure):
    _fields_ = [("n_layers", ctypes.c_int32), ("dims", ctypes.c_int32 * 5), ("weight", ctypes.c_void_p * 4),
                ("bias", ctypes.c_void_p * 4), ("hidden_act", ctypes.c_int32), ("clip", ctypes.c_int32),
                ("lo", ctypes.c_float), ("hi", ctypes.c_float), ("packed", ctypes.c_void_p),
                ("split_out", ctypes.c_int32 * 4), ("split_in", ctypes.c_int32 * 4)]


class ChError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libcattleherd error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """Load libcattleherd.so; raises if it is missing (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    P = ctypes.POINTER
    L.ch_default_config.argtypes = [P(ChConfig), i32, i32, i32]
    L.ch_create.argtypes = [P(ChConfig), i64, i32, P(vp)]
    L.ch_destroy.argtypes = [vp]
    L.ch_last_error.argtypes = [vp]
    L.ch_last_error.restype = ctypes.c_char_p
    L.ch_shape.argtypes = [vp, P(i64), P(i32), P(i32), P(i32)]
    L.ch_reset.argtypes = [vp, vp, vp, vp]
    L.ch_reset_with.argtypes = [vp, vp, vp, vp, vp, vp]
    L.ch_step.argtypes = [vp, P(ChStepIO), vp]
    if hasattr(L, "ch_step_n"):   # (an older library, e.g. an A/B baseline loaded through CH_LIB_PATH, lacks it)
        L.ch_step_n.argtypes = [vp, P(ChStepIO), i32, vp]
        L.ch__multi_steps.argtypes = [vp]
        L.ch__multi_steps.restype = i64
    L.ch_state_size.argtypes = [vp, P(i64), P(i64)]
    L.ch_get_state.argtypes = [vp, vp, vp, vp]
    L.ch_set_state.argtypes = [vp, vp, vp, vp]
    L.ch_metrics.argtypes = [vp, vp, i32, vp]
    L.ch_metrics_device.argtypes = [vp, vp, i32, vp]
    L.ch_sync.argtypes = [vp, vp]
    L.ch_get_eval.argtypes = [vp, vp, vp]
    L.ch_builtin_spawn_table.argtypes = [vp, P(i32), P(i32)]
    L.ch_spawn_table.argtypes = [i32, vp, P(i32), P(i32)]
    L.ch_mlp_forward.argtypes = [P(ChMlp), vp, i64, vp, vp]
    L.ch_mlp_forward_masked.argtypes = [P(ChMlp), vp, i64, vp, vp, vp]
    L.ch_policy_forward.argtypes = [vp, P(ChMlp), vp, vp, vp]
    L.ch_mlp_packed_size.argtypes = [P(ChMlp)]
    L.ch_mlp_pack.argtypes = [P(ChMlp), vp, vp]
    L.ch_outputs_to_host.argtypes = [vp, P(ChStepIO), P(ChHostOut), vp]
    for name in EXPORTS:
        if name not in ("ch_last_error",) and (name != "ch_step_n" or hasattr(L, name)):
            getattr(L, name).restype = ctypes.c_int
    L.ch_mlp_packed_size.restype = ctypes.c_int64
    _lib = L
    return L


def check(rc, handle=None):
    if rc != CH_OK:
        msg = lib().ch_last_error(handle)
        raise ChError(rc, msg.decode() if msg else "")
    return rc


def default_config(mode, num_drones, num_cattle):
    c = ChConfig()
    check(lib().ch_default_config(ctypes.byref(c), mode, num_drones, num_cattle))
    return c


def code_object_hash(path=None):
    """sha256 (hex, first 16 digits) of the device code in libcattleherd.so: the ``.hip_fatbin`` ELF section
    that holds the gfx950 code objects.  Host-side code and build paths do not enter it, so a rebuild of the same
    kernel sources with the same compiler and flags gives the same hash.  bench.py accepts a committed counter
    record (profiles/counters/) only for the code object it was measured on."""
    import hashlib
    import struct
    with open(path or LIB_PATH, "rb") as fh:
        data = fh.read()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise ValueError("not an ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    sec = [struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stro = sec[shstrndx][4]
    for name, _typ, _flags, _addr, off, size in sec:
        end = data.index(b"\0", stro + name)
        if data[stro + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    raise ValueError("no .hip_fatbin section")


def spawn_table(cows):
    """The spawn table ch_create uses by default (numpy float64 [100, max(cows,16), 2])."""
    import numpy as np
    s, c = ctypes.c_int32(), ctypes.c_int32()
    check(lib().ch_spawn_table(cows, None, ctypes.byref(s), ctypes.byref(c)))
    out = np.zeros((s.value, c.value, 2), np.float64)
    check(lib().ch_spawn_table(cows, out.ctypes.data, None, None))
    return out
