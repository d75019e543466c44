#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs: mean of each counter per kernel (largest kernels)."""
import csv
import glob
import sys
from collections import defaultdict


def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for f in glob.glob(p, recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "?")[:60]
                    key = (row.get("Dispatch_Id"), row.get("Counter_Name"))
                    acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, ctrs in acc.items():
        if "gemm" not in name.lower() and "Cijk" not in name:
            continue
        print(name)
        for c, vals in sorted(ctrs.items()):
            print(f"   {c:28s} {sum(vals) / len(vals):16.1f}  (n={len(vals)})")


if __name__ == "__main__":
    main(sys.argv[1:] or ["gpurun_out/pmc/**/*counter_collection.csv"])
