#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 counter CSVs from tools/llm_pmc.sh (LLM decode kernels).

No clock column: GRBM_GUI_ACTIVE accumulates over the dispatch window rocprofv3 brackets, which
for these 5-20 us kernels is longer than the kernel's own timestamps, so GRBM / duration read as
3-7 GHz on a <= 2.4 GHz part.  The clock of a long kernel comes from the validator's
GEMM counter pass (operator/validator.py rocprof_counter_summary) or amd-smi telemetry."""
import collections
import csv
import glob
import sys


def main(pattern):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "qgemv" not in name and "attn" not in name and "rope" not in name:
                continue
            short = name.replace("void ", "").replace("(anonymous namespace)::", "")
            key = short.split("(")[0][:40] + \
                f" grid={r.get('Grid_Size', r.get('Grid_Size_X', ''))}"
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            dur[(key, r["Dispatch_Id"])] = d
    bykey = collections.defaultdict(list)
    for (k, _), d in dur.items():
        bykey[k].append(d)
    for k in sorted(acc, key=lambda k: -sum(bykey[k]) / max(1, len(bykey[k]))):
        m = {c: sum(v) / len(v) for c, v in acc[k].items()}
        d = sum(bykey[k]) / len(bykey[k])
        line = f"{k:52s} n={len(bykey[k]):4d} {d / 1e3:8.2f} us"
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            wc = m["SQ_WAVE_CYCLES"]
            line += (f"  wait {m.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} valu "
                     f"{m.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.2f} lds {m.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.2f}")
        if "TCC_EA0_RDREQ_sum" in m:
            line += f"  hbm_rd {m['TCC_EA0_RDREQ_sum'] * 128 / d:6.0f} GB/s(x128B)  l2hit {m.get('TCC_HIT_sum', 0) / max(1, m.get('TCC_HIT_sum', 0) + m.get('TCC_MISS_sum', 0)):4.2f}"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
