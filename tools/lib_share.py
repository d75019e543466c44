#!/usr/bin/env python3
"""Which kernels of a request path are ours and which come from libraries: classify every kernel of
a ``rocprofv3 --kernel-trace --stats`` run (its ``*kernel_stats.csv``) as

  in-tree      a __global__ function of this repository's HIP sources (found by scanning them)
  hipBLASLt    Tensile / hipBLASLt GEMMs (``Cijk_*``)
  MIOpen       MIOpen / composable-kernel convolutions and norms
  AOTriton     Triton-compiled kernels PyTorch dispatches to (SDPA's ``attn_fwd`` ...)
  torch        PyTorch's own ATen kernels (elementwise, reductions, copies, RNG)
  other        anything else

and print each class's share of the GPU time, with its largest kernels.

    python tools/lib_share.py gpurun_out/prof/<host>/<pid>_kernel_stats.csv [--top 5]
    python tools/lib_share.py run_kernel_trace.csv --window-ms 223   # the last 223 ms only

A ``*kernel_trace.csv`` (one row per dispatch) can be cut to a window at the end of the run:
MIOpen's ``find`` benchmarks every candidate solver (naive ones included) on the first call of a
convolution shape, so whole-run stats over-count library time; the steady-state request is the
last ``--window-ms`` of GPU time (``--skip-ms``: leave out that much at the very end).
"""
from __future__ import annotations

import argparse
import csv
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ours() -> set:
    names = set()
    skip = {"__launch_bounds__", "__attribute__", "amdgpu_waves_per_eu", "void",
            "amdgpu_flat_work_group_size", "__align__", "alignas"}
    ident = re.compile(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(")
    for d in ("k8s_nvidia_gpus_amd/ops/csrc", "native/src"):
        base = os.path.join(ROOT, d)
        for f in os.listdir(base):
            if not f.endswith((".hip", ".h", ".inc")):
                continue
            with open(os.path.join(base, f), errors="replace") as fh:
                src = fh.read()
            for m in re.finditer(r"__global__", src):
                for cand in ident.findall(src, m.end(), m.end() + 400):
                    if cand not in skip:
                        names.add(cand)
                        break
    return names


def classify(name: str, mine: set) -> str:
    for m in mine:                  # first: our attn_fwd_kernel is not AOTriton's attn_fwd
        if re.search(rf"\b{re.escape(m)}\b", name):
            return "in-tree"
    if name.startswith("Cijk_") or "Cijk_" in name:
        return "hipBLASLt"
    if re.search(r"\battn_fwd\b|triton", name, re.I):
        return "AOTriton"
    if re.search(r"miopen|MIOpen|naive_conv|igemm|ck::|ck_tile|ck\d+tensor_operation|Im2Col|"
                 r"batchnorm|gridwise|SubTensorOp", name):
        return "MIOpen"
    if "at::" in name or "c10::" in name or name.startswith("void at"):
        return "torch"
    return "other"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--window-ms", type=float, default=0.0,
                    help="kernel-trace input: only dispatches in the last this many ms")
    ap.add_argument("--skip-ms", type=float, default=0.0,
                    help="kernel-trace input: end the window this many ms before the last dispatch")
    a = ap.parse_args(argv)
    mine = ours()
    by = defaultdict(float)
    calls = defaultdict(int)
    top = defaultdict(list)
    with open(a.csv) as f:
        rows = list(csv.DictReader(f))
    if rows and "Start_Timestamp" in rows[0]:            # per-dispatch trace: aggregate here
        ends = [int(r["End_Timestamp"]) for r in rows]
        hi = max(ends) - a.skip_ms * 1e6
        lo = hi - a.window_ms * 1e6 if a.window_ms > 0 else -1
        agg = defaultdict(lambda: [0.0, 0])
        for r in rows:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if st >= lo and en <= hi:
                agg[r["Kernel_Name"]][0] += en - st
                agg[r["Kernel_Name"]][1] += 1
        rows = [{"Name": n, "TotalDurationNs": v[0], "Calls": v[1]} for n, v in agg.items()]
    for row in rows:
        name = row.get("Name") or row.get("KernelName") or ""
        ns = float(row.get("TotalDurationNs") or row.get("TotalDuration") or 0)
        c = int(float(row.get("Calls") or 0))
        k = classify(name, mine)
        by[k] += ns
        calls[k] += c
        top[k].append((ns, c, name))
    total = sum(by.values()) or 1.0
    print(f"# {a.csv}: {total / 1e6:.3f} ms of kernel time")
    for k, ns in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"{k:10s} {ns / 1e6:10.3f} ms  {100 * ns / total:6.2f} %  {calls[k]:7d} calls")
        for tns, c, name in sorted(top[k], reverse=True)[:a.top]:
            print(f"    {tns / 1e6:9.3f} ms {100 * tns / total:6.2f} % {c:6d}x  {name[:150]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
