#!/usr/bin/env python3
"""Per-launch timing of the validator GEMM over a long back-to-back run (DVFS / power transient).

The rocprofv3 kernel trace of bench.py (profiles/r01_session5/) shows the 8192^3 bf16 GEMM at
~680 us for the first two launches, ~900 us at launches 4-6 (power-management reaction to the
load step), then a slow recovery over ~20 launches.  This tool records every launch with HIP
events for --launches back-to-back GEMMs and prints the duration sequence in buckets, so the
steady state and the length of the transient can be read off.

    python tools/gemm_settle_probe.py --launches 3000 --bucket 100
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--launches", type=int, default=3000)
    ap.add_argument("--bucket", type=int, default=100)
    ap.add_argument("--head", type=int, default=40, help="print each of the first N launches")
    ap.add_argument("--variant", default="w4a")
    args = ap.parse_args()
    s = args.size
    dev = torch.device("cuda", 0)
    a = torch.empty((s, s), dtype=torch.bfloat16, device=dev)
    b = torch.empty((s, s), dtype=torch.bfloat16, device=dev)
    c = torch.empty((s, s), dtype=torch.bfloat16, device=dev)
    K.fill_uniform_bf16(a, seed=1000)
    K.fill_uniform_bf16(b, seed=2000)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.launches + 1)]
    ev[0].record()
    for i in range(args.launches):
        K.gemm_bf16_nt(a, b, out=c, variant=args.variant)
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.launches)]
    flop = 2.0 * s ** 3
    print("first launches (us):", " ".join(f"{m * 1e3:.0f}" for m in ms[:args.head]))
    t = 0.0
    for lo in range(0, args.launches, args.bucket):
        chunk = ms[lo:lo + args.bucket]
        t += sum(chunk)
        print(json.dumps({"launches": f"{lo}-{lo + len(chunk) - 1}", "t_end_ms": round(t, 1),
                          "mean_us": round(sum(chunk) / len(chunk) * 1e3, 1),
                          "tflops": round(flop * len(chunk) / (sum(chunk) * 1e-3) / 1e12, 1)}))
    print(json.dumps({"summary": True, "launches": args.launches, "total_ms": round(sum(ms), 1),
                      "tflops_all": round(flop * len(ms) / (sum(ms) * 1e-3) / 1e12, 1),
                      "tflops_best_launch": round(flop / (min(ms) * 1e-3) / 1e12, 1)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
