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


def test_sincos_small_within_one_ulp_of_libm(tmp_path):
    """ch_device.h sincos_small (reduction-free fdlibm kernels, used for the substep's half angle
    0 <= x <= pi/8) and cos_0pi (the flock bump's cos on [0, pi]: Cody-Waite reduction by pi/2, then those
    kernels) stay within 1 ulp of glibc sin/cos, the oracle's libm (tools/sincos_check.c)."""
    exe = tmp_path / "sincos_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(ROOT, "tools", "sincos_check.c"),
                    "-lm"], check=True)
    out = subprocess.run([str(exe), "2000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "cos_0pi:" in out.stdout
