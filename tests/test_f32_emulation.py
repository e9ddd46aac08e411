"""The f32 mode's precision policy, checked on the host (tools/f32_emu.py): the drone path evaluated with numpy
float32 / float64 per piece from oracle states reproduces the oracle bit for bit in all-f64, misses 1e-4 relative
on the body rates in all-f32 (the pre-round-4 kernel: 2.5e-4 measured on the GPU, profiles/r04/zj/f32_probe_before.log),
and holds it with the pieces ch_device.h carries in f64 since round 4 (8.0e-5 measured on the GPU,
profiles/r04/zk/f32_probe3.log; the GPU test is test_gpu_parity.py::test_f32_throughput_mode_error_budget)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_f32_policy_body_rates_within_1e4_relative():
    import f32_emu
    d = f32_emu.draw(E=96)
    pols = f32_emu.policies()
    assert f32_emu.errors(pols["all f64"], d) == (0.0, 0.0)
    assert f32_emu.errors(pols["all f32 (before round 4)"], d)[1] > 1e-4
    assert f32_emu.errors(pols["kernel (round 4)"], d)[1] < 1e-4
