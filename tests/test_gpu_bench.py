"""bench.py's output contract on the GPU (the driver parses this line): one JSON line with the metric, the whole-job
value, the timing fields, the roofline and cpu_baseline objects -- through ch_step_n (the default) and with one launch
per step (--steps-per-launch 1).  Short runs: 20 timed steps after a 50-step burn-in."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _run(args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("spl", [-1, 1])
def test_bench_line_contract(spl):
    d = _run(["--steps", "20", "--warmup", "5", "--burn-in", "50", "--no-cpu-baseline", "--no-extras",
              "--steps-per-launch", str(spl)])
    for k in KEYS:
        assert k in d, k
    assert d["metric"].startswith("env-steps/sec") and d["unit"] == "env-steps/s" and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 5 and d["scaling"] == "weak"
    assert d["dtype"] == "f64" and d["vs_baseline"] is None and d["cpu_baseline"] is None
    # value = envs x steps / wall of the timed region
    assert abs(d["value"] - 4096 * 20 / (d["ms_per_step"] * 20 / 1e3)) < 1e-6 * d["value"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["unit"] == "GB/s" and r["peak"] == 8000.0 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    assert r["algorithmic_bytes_per_launch"] == r["bytes_per_env_step"] * 4096
    assert ("k_step2_multi" in r["kernel"]) == (spl != 1)
    assert d["config"]["envs_per_gpu"] == 4096 and d["config"]["num_drones"] == 4 and d["config"]["num_cattle"] == 16
    assert d["rollout_metrics"]["nan_rewards"] == 0
