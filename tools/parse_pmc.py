"""Summarise rocprofv3 --pmc CSVs: per-kernel mean of each counter (dispatches of the fused step only)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if "k_env" not in k or "Lb1" in k:
                    continue
                acc[(k[:60], row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{k:60s} {c:28s} mean={sum(v)/len(v):.4g} n={len(v)}")


if __name__ == "__main__":
    main(sys.argv[1])
