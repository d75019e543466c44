#!/usr/bin/env python3
"""Fused-epilogue GEMM (gemm_bf16_epi.hip) vs hipBLASLt (torch) on the Wan2.1 DiT projection
shapes: time per call, TFLOPS, and the gated-residual epilogue against GEMM + separate update."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from k8s_nvidia_gpus_amd.ops import gemm_epi as GE  # noqa: E402
from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
ITERS = int(os.environ.get("ITERS", "50"))


def bench(fn, iters=ITERS):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


res = {}
for tokens in [int(t) for t in os.environ.get("TOKENS", "2560,32768").split(",")]:
    M = 2 * tokens
    for name, n, k in [("qkv", 4608, 1536), ("o", 1536, 1536), ("ffn0", 8960, 1536), ("ffn2", 1536, 8960)]:
        x = torch.randn(M, k, device=dev).bfloat16()
        w = (torch.randn(n, k, device=dev) / k ** 0.5).bfloat16()
        b = torch.randn(n, device=dev).bfloat16()
        fl = 2.0 * M * n * k
        row = {}
        if name == "ffn0":
            row["ours_us"] = bench(lambda: GE.linear_gelu(x, w, b))
            row["torch_us"] = bench(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True))
        elif name in ("o", "ffn2"):
            r = torch.randn(2, tokens, n, device=dev)
            g = torch.randn(2, n, device=dev)
            x3 = x.view(2, tokens, k)
            row["ours_us"] = bench(lambda: GE.linear_residual_(r, x3, w, b, g))
            row["torch_us"] = bench(lambda: r.add_(F.linear(x3, w, b) * g[:, None, :]))
            row["ours_store_us"] = bench(lambda: GE.linear(x, w, b))
            row["torch_gemm_us"] = bench(lambda: F.linear(x, w, b))
        else:
            row["ours_us"] = bench(lambda: GE.linear(x, w, b))
            row["torch_us"] = bench(lambda: F.linear(x, w, b))
        if M % 256 == 0 and n % 256 == 0:          # the validator's 256x256 w4a kernel, plain store
            row["w4a_us"] = bench(lambda: K.gemm_bf16_nt(x, w))
        for key in list(row):
            row[key] = round(row[key], 1)
        row["ours_tflops"] = round(fl / row["ours_us"] / 1e6, 1)
        if "w4a_us" in row:
            row["w4a_tflops"] = round(fl / row["w4a_us"] / 1e6, 1)
        row["torch_tflops"] = round(fl / row["torch_us"] / 1e6, 1)
        res[f"{tokens}_{name}"] = row
        print(tokens, name, row, flush=True)
print(json.dumps(res))
