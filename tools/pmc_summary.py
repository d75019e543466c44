#!/usr/bin/env python3
"""Summarise rocprofv3 output: mean of each counter per GEMM kernel, plus (when the run's
kernel_trace.csv is next to it) the mean duration and the effective clock
GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md "DVFS give-back")."""
import csv
import glob
import os
import sys
from collections import defaultdict


_MATCH = os.environ.get("PMC_MATCH")      # regex over kernel names (default: GEMM kernels)


def _is_gemm(name):
    if _MATCH:
        import re

        return re.search(_MATCH, name) is not None
    return "gemm" in name.lower() or "Cijk" in name


def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    seen_dirs = set()
    for p in paths:
        for f in glob.glob(p, recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "?")[:60]
                    acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
            seen_dirs.add(os.path.dirname(f))
    for d in seen_dirs:
        for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "?")[:60]
                    try:
                        durs[name].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
                    except (KeyError, ValueError):
                        pass
    for name, ctrs in acc.items():
        if not _is_gemm(name):
            continue
        print(name)
        means = {c: sum(v) / len(v) for c, v in ctrs.items()}
        for c, v in sorted(ctrs.items()):
            print(f"   {c:28s} {means[c]:16.1f}  (n={len(v)})")
        if "SQ_INSTS_MFMA" in means and means["SQ_INSTS_MFMA"]:
            if "SQ_INSTS_VALU" in means:
                print(f"   {'VALU insts per MFMA':28s} {means['SQ_INSTS_VALU'] / means['SQ_INSTS_MFMA']:16.2f}")
        if means.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in means:
            print(f"   {'bank conflicts per LDS inst':28s} {means['SQ_LDS_BANK_CONFLICT'] / means['SQ_INSTS_LDS']:16.2f}")
        if durs.get(name):
            d = sorted(durs[name])[len(durs[name]) // 2]
            print(f"   {'duration_ns (median)':28s} {d:16.1f}")
            if "GRBM_GUI_ACTIVE" in means:
                print(f"   {'effective clock GHz':28s} {means['GRBM_GUI_ACTIVE'] / 8 / d:16.3f}")


if __name__ == "__main__":
    main(sys.argv[1:] or ["gpurun_out/pmc/**/*counter_collection.csv"])
