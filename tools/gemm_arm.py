#!/usr/bin/env python3
"""Run ONE GEMM arm for a fixed number of iterations (for rocprofv3 counter collection)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, ".")
from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--arm", default="w4")
ap.add_argument("--shape", default="8192x8192x8192")
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
if "@" in args.arm:  # VARIANT@ENV=VALUE, as in tools/gemm_sweep.py
    args.arm, kvs = args.arm.split("@", 1)
    os.environ.update(dict(kv.split("=", 1) for kv in kvs.split(",")))
m, n, k = (int(x) for x in args.shape.split("x"))
dev = torch.device("cuda", 0)
a = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
b = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
K.fill_uniform_bf16(a, 11)
K.fill_uniform_bf16(b, 12)
c = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
for _ in range(args.iters):
    if args.arm == "blt":
        torch.matmul(a, b.t(), out=c)
    else:
        K.gemm_bf16_nt(a, b, out=c, variant=args.arm)
torch.cuda.synchronize()
print("done", args.arm, args.shape)
