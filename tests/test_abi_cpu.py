"""CPU tests: the C-ABI library loads, exports every symbol include/cattleherd.h declares, and its
host-only entry points behave (no GPU needed)."""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "cattleherd.h")).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(ch_\w+)\(", src, re.M)))


def test_library_exports_header_symbols():
    from cattleherd import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.EXPORTS)


def test_default_config_and_struct_layout():
    from cattleherd import _lib
    c = _lib.default_config(_lib.CH_MODE_CTDE, 12, 16)
    assert c.abi_version == _lib.ABI_VERSION and c.ctrl_freq == 60 and c.pyb_freq == 240
    assert c.compat == 1 and c.damping == 0.04 and c.min_drones == -1
    assert ctypes.sizeof(_lib.ChStepIO) == 9 * 8 + 8 + 8


def test_builtin_spawn_table_is_the_reference_yaml(spawn16):
    from cattleherd import _lib
    t = _lib.spawn_table(16)
    assert t.shape == (100, 16, 2)
    assert np.array_equal(t, spawn16)
    t32 = _lib.spawn_table(32)
    assert t32.shape == (100, 32, 2) and np.array_equal(t32[:, :16], spawn16)
    d = np.linalg.norm(t32[:, 16:, None] - t32[:, None], axis=-1)   # extra cows vs all cows
    d[:, np.arange(16), 16 + np.arange(16)] = 9
    assert d.min() >= 0.75   # the generator's 0.8 spacing (cattle_spawn.py:12), relaxed at most 5 %


def test_create_without_gpu_fails_loudly():
    """No CPU fallback: ch_create reports a device error when no HIP device is visible."""
    import torch
    if torch.cuda.is_available():
        return
    from cattleherd import _lib
    c = _lib.default_config(0, 4, 16)
    h = ctypes.c_void_p()
    rc = _lib.lib().ch_create(ctypes.byref(c), 8, 0, ctypes.byref(h))
    assert rc == _lib.CH_ERR_DEVICE
    assert b"no HIP device" in _lib.lib().ch_last_error(None)


def test_invalid_configs_rejected():
    from cattleherd import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    c = _lib.default_config(0, 13, 16)
    assert L.ch_create(ctypes.byref(c), 8, 0, ctypes.byref(h)) == _lib.CH_ERR_INVALID
    c = _lib.default_config(0, 4, 16)
    c.pyb_freq = 250
    assert L.ch_create(ctypes.byref(c), 8, 0, ctypes.byref(h)) == _lib.CH_ERR_INVALID
    assert b"pyb_freq is not divisible" in L.ch_last_error(None)
    c = _lib.default_config(0, 1, 4)
    assert L.ch_create(ctypes.byref(c), 8, 0, ctypes.byref(h)) == _lib.CH_ERR_UNSUPPORTED


def test_physics_field_default_and_range():
    """ch_config.physics (CH_PHYS_*, utils/enums.py:13-21): PYB by default, out-of-range rejected
    before any device call."""
    from cattleherd import _lib
    L = _lib.lib()
    c = _lib.ChConfig()
    c.physics = 7
    assert L.ch_default_config(ctypes.byref(c), 0, 4, 16) == 0
    assert c.physics == _lib.PHYSICS["pyb"] == 0
    assert _lib.ChConfig.physics.offset == _lib.ChConfig.spawn_cows.offset + 4
    assert _lib.ChConfig.eval_metrics.offset == _lib.ChConfig.physics.offset + 4 and c.eval_metrics == 1
    assert ctypes.sizeof(_lib.ChConfig) % 8 == 0
    h = ctypes.c_void_p()
    for bad in (-1, 7):
        c.physics = bad
        assert L.ch_create(ctypes.byref(c), 8, 0, ctypes.byref(h)) == _lib.CH_ERR_INVALID
        assert b"physics" in L.ch_last_error(None)


def test_mlp_packed_size_is_the_operand_layout():
    """ch_mlp_packed_size (host only): per layer ceil(N / 16) tiles x K pairs of 32 padded to a multiple of 4 x
    512 floats (two halves of 64 lanes x 4); invalid nets report -1."""
    from cattleherd import _lib
    L = _lib.lib()
    net = _lib.ChMlp()
    net.n_layers = 3
    for i, d in enumerate((1032, 128, 128, 48)):
        net.dims[i] = d
    pairs = lambda k: (((k + 31) // 32) + 3) // 4 * 4  # noqa: E731
    want = 8 * pairs(1032) * 512 + 8 * pairs(128) * 512 + 3 * pairs(128) * 512
    assert L.ch_mlp_packed_size(ctypes.byref(net)) == want
    net.dims[1] = 300
    assert L.ch_mlp_packed_size(ctypes.byref(net)) == -1
