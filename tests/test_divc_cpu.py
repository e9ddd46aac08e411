"""The corrected-quotient division the step kernels use for constant and loop-invariant divisors
(ch_device.h divc) must equal IEEE division bit for bit: tools/div_check.c replays it on the host
(fp64 fma) for every divisor the kernels pass and for random divisors, including +-0, inf and NaN."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_divc_matches_ieee_division(tmp_path):
    exe = tmp_path / "div_check"
    subprocess.run(["gcc", "-O2", "-o", str(exe), os.path.join(ROOT, "tools", "div_check.c"), "-lm"], check=True)
    out = subprocess.run([str(exe), "300000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert out.stdout.count("bad=0") == out.stdout.count("bad=")
