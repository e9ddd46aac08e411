"""Counter record of the shipped step kernel, keyed by its code object.

Runs on the GPU box, after the library is built.  For each workload: three rocprofv3 --pmc passes of a short
bench.py run (FETCH_SIZE; WRITE_SIZE; the SQ instruction group -- separate passes, MI355X_MICROARCH.md's TCC
limits), each rocprofv3 a child process of this one (which never touches the GPU itself), then the workgroup
phase trace (tools/wg_trace.py --json: drone chain cycles against workgroup cycles).  The per-launch means of the
dominant kernel go to profiles/counters/<workload>_<dtype>.json together with ``code_object`` =
cattleherd._lib.code_object_hash() of the library measured; bench.py reads the record only when that hash
matches the library it runs (so the line's ``traffic`` / ``valu`` always describe the kernel it timed).

  python tools/counter_record.py --workloads c4 c5 --out profiles/counters --raw gpurun_out/counters
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))

PASSES = {"fetch": "FETCH_SIZE", "write": "WRITE_SIZE",
          "sq": "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY"}


def kernel_means(root, only=None):
    """{kernel name: {counter: (mean per dispatch, dispatches)}} over every counter CSV under root (`only`: kernels whose
    name contains it)."""
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if only is not None and only not in k:
                    continue
                if "k_step2" in k or ("k_env" in k and "Lb1E" not in k):
                    acc[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
    out = defaultdict(dict)
    for (k, c), v in acc.items():
        out[k][c] = (sum(v) / len(v), len(v))
    return out


def record(workload, dtype, raw, steps, timeout, multi=0):
    """multi > 0: ch_step_n's k_step2_multi, dispatches of `multi` steps each (bench.py --counter-probe); the record's
    counters are then per step (per dispatch / multi)."""
    from cattleherd._lib import code_object_hash
    env = dict(os.environ, TMPDIR="/tmp")
    means = defaultdict(dict)
    for tag, ctrs in PASSES.items():
        d = os.path.join(raw, f"{workload}_{dtype}_{tag}" + ("_multi" if multi else ""))
        tail = (["--counter-probe", str(multi)] if multi else
                ["--steps", str(steps), "--warmup", "10", "--no-cpu-baseline", "--no-extras", "--steps-per-launch", "1"])
        cmd = ["timeout", "-s", "KILL", str(timeout), "rocprofv3", "--pmc", *ctrs.split(), "--output-format", "csv",
               "-d", d, "-o", "pmc", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload,
               "--precision", dtype, "--burn-in", "300", *tail]
        print("counter_record:", " ".join(cmd), flush=True)
        r = subprocess.run(cmd, env=env, cwd=ROOT)
        if r.returncode != 0:
            raise SystemExit(f"counter pass {tag} failed with {r.returncode}")
        for k, cs in kernel_means(d, "k_step2_multi" if multi else None).items():
            if not multi and "k_step2_multi" in k:
                continue
            means[k].update(cs)
    # the dominant kernel: the most dispatches with both traffic counters
    best = max((k for k, m in means.items() if "FETCH_SIZE" in m and "WRITE_SIZE" in m),
               key=lambda k: means[k]["FETCH_SIZE"][1])
    m = means[best]
    if multi:   # per step
        m = {c: (v / multi, n) for c, (v, n) in m.items()}
    out = {"code_object": code_object_hash(), "kernel": best, "workload": workload, "dtype": dtype,
           "dispatches": m["FETCH_SIZE"][1], "fetch_kib": m["FETCH_SIZE"][0], "write_kib": m["WRITE_SIZE"][0],
           "traffic_bytes_per_launch": (2.0 * m["FETCH_SIZE"][0] + m["WRITE_SIZE"][0]) * 1024.0,
           "note": "per-launch means over the dispatches of bench.py runs under rocprofv3 --pmc (one pass per counter "
                   "group); traffic = FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE, KiB -> B" +
                   (f"; k_step2_multi dispatches of {multi} steps each (bench.py --counter-probe), every counter divided "
                    f"by {multi}: per step" if multi else "")}
    if multi:
        out["steps_per_dispatch"] = multi
    for c, (v, _n) in m.items():
        if c.startswith("SQ_"):
            out[c.lower()] = v
    # the workgroup timeline of the same library (latency bound: chain cycles against workgroup cycles)
    mode, E, n, mm = {"c4": ("ctde", 4096, 4, 16), "c3": ("ctde", 4096, 2, 8), "c2": ("ctde", 1024, 2, 8),
                      "c5": ("marl", 4096, 4, 32)}[workload]
    tr = subprocess.run(["timeout", "-k", "10", str(timeout), sys.executable, os.path.join(ROOT, "tools", "wg_trace.py"),
                         "--json", mode, str(E), str(n), str(mm)], env=dict(env, CH_TRACE_MULTI="1" if multi else ""),
                        cwd=ROOT, capture_output=True, text=True)
    if tr.returncode == 0:
        lines = [ln for ln in tr.stdout.splitlines() if ln.startswith("{")]
        if lines:
            out["wg_trace"] = json.loads(lines[-1])
    else:
        print(tr.stdout[-2000:], tr.stderr[-2000:], file=sys.stderr)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", nargs="+", default=["c4", "c5"])
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "counters"))
    ap.add_argument("--raw", default=os.path.join(ROOT, "gpurun_out", "counters"))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--timeout", type=int, default=150)
    ap.add_argument("--multi", type=int, default=0, help="steps per ch_step_n dispatch (k_step2_multi); 0 = k_step2")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for w in a.workloads:
        rec = record(w, a.dtype, a.raw, a.steps, a.timeout, a.multi)
        path = os.path.join(a.out, f"{w}_{a.dtype}" + ("_multi" if a.multi else "") + ".json")
        with open(path, "w") as fh:
            json.dump(rec, fh, indent=1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
