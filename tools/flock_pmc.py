"""Flock-only counter record (N1): parse the rocprofv3 --pmc passes of tools/flock_phase.py --state-in runs (every
step-kernel launch of those processes is a flock-only launch, phase mask 13) and the per-launch times of the same
configurations, into HBM bytes per launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md) and
the VALU issue fraction (SQ_INSTS_VALU x 4 cycles per fp64 wave-instruction over the SIMD cycles of the launch).

  python tools/flock_pmc.py ROOT --times times.jsonl --json out.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SIMDS, CLOCK_GHZ, HBM_GBS = 1024, 2.4, 8000.0


def counters(root):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "k_step2" not in row.get("Kernel_Name", ""):
                    continue
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--times", required=True)
    ap.add_argument("--json", required=True)
    ap.add_argument("--drones", type=int, default=4)
    ap.add_argument("--cattle", type=int, default=16)
    a = ap.parse_args()
    times = {}
    with open(a.times) as fh:
        for line in fh:
            line = line.strip()
            if line.startswith("{"):
                d = json.loads(line)
                times[int(d["envs"])] = d["us"]
    out = {"kernel": "ch::k_step2 with phase mask 13 (flock only: staging, cattle integration, alpha / shepherd / "
                     "predator / gamma terms, velocity update)", "records": []}
    for E in sorted(times):
        c = counters(os.path.join(a.root, f"E{E}"))
        if not c:
            continue
        us = times[E]
        fetch = 2.0 * c["FETCH_SIZE"][0] * 1024 if "FETCH_SIZE" in c else None
        write = c["WRITE_SIZE"][0] * 1024 if "WRITE_SIZE" in c else None
        valu = c.get("SQ_INSTS_VALU", (None, 0))[0]
        simd_cycles = SIMDS * us * 1e-6 * CLOCK_GHZ * 1e9
        b_flock = (24 * a.cattle + 8 * a.drones) * E / 2   # SURVEY 8(d) B_flock, half the envs flock per step
        rec = {"envs": E, "us_per_launch": us, "launches_counted": c.get("SQ_INSTS_VALU", (0, 0))[1],
               "fetch_bytes": fetch, "write_bytes": write,
               "traffic_bytes": (fetch or 0) + (write or 0) if fetch is not None and write is not None else None,
               "hbm_gbs_counted": ((fetch or 0) + (write or 0)) / (us * 1e-6) / 1e9 if fetch is not None else None,
               "flock_bytes_survey": b_flock, "hbm_frac_survey_bytes": b_flock / (us * 1e-6) / 1e9 / HBM_GBS,
               "valu_insts": valu, "valu_issue_frac": (valu * 4 / simd_cycles) if valu else None,
               "sq_busy_cycles": c.get("SQ_BUSY_CYCLES", (None, 0))[0], "sq_waves": c.get("SQ_WAVES", (None, 0))[0],
               "sq_active_inst_valu": c.get("SQ_ACTIVE_INST_VALU", (None, 0))[0]}
        if rec["sq_active_inst_valu"]:
            rec["valu_active_frac"] = rec["sq_active_inst_valu"] * 4 / simd_cycles
        out["records"].append(rec)
    out["note"] = ("us_per_launch: HIP events over flock-only launches without counters; valu_issue_frac counts every "
                   "VALU wave-instruction at the fp64 rate (4 cycles per wave64 on a SIMD), an upper bound; "
                   "hbm_frac_survey_bytes = SURVEY 8(d) B_flock / time / 8 TB/s")
    with open(a.json, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
