"""Summarise rocprofv3 --pmc CSVs of the step kernel (tools/gpu_prof.sh) and derive HBM traffic.

Per MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE / WRITE_SIZE are KiB from the L2's memory-side
request counters; on gfx950 FETCH_SIZE reports half of the bytes of a wide coalesced read, so it is
doubled.  `--json OUT` writes {kernel, fetch_kib, write_kib, traffic_bytes_per_launch} for bench.py.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def collect(root):
    acc = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if "k_step2" not in k and "k_env" not in k:
                    continue
                if "Lb1E" in k:          # the RESET_ONLY instantiation of the v1 kernel
                    continue
                acc[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json", default=None)
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--dtype", default="f64")
    a = ap.parse_args()
    acc = collect(a.root)
    means = {}
    for (k, c), v in sorted(acc.items()):
        means.setdefault(k, {})[c] = sum(v) / len(v)
        print(f"{k[:70]:70s} {c:28s} mean={sum(v) / len(v):.6g} n={len(v)}")
    if a.json:
        # the dominant kernel = the one with most dispatches that has both traffic counters
        best = None
        for k, m in means.items():
            if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
                n = len(acc[(k, "FETCH_SIZE")])
                if best is None or n > best[1]:
                    best = (k, n)
        if best:
            m = means[best[0]]
            out = {"kernel": best[0], "workload": a.workload, "dtype": a.dtype, "fetch_kib": m["FETCH_SIZE"],
                   "write_kib": m["WRITE_SIZE"],
                   "traffic_bytes_per_launch": (2.0 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024.0,
                   "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KiB -> bytes, mean over dispatches"}
            # instruction counters of the same kernel (per launch; SQ_ACTIVE_INST_* in quad-cycles)
            for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES"):
                if c in m:
                    out[c.lower()] = m[c]
            with open(a.json, "w") as fh:
                json.dump(out, fh, indent=1)
            print(json.dumps(out))


if __name__ == "__main__":
    main()
