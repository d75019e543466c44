#!/usr/bin/env python3
"""A/B the hand-written gfx950 GEMM against torch.matmul (hipBLASLt) — same random data, one process.

Interleaved rounds (methodology: perf deltas come from interleaved rounds in ONE process), report
median and min ms per call and TFLOPS for each arm.
"""
import argparse
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402


def time_arm(fn, iters):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[8192])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--fp16", action="store_true", help="also A/B the fp16 kernel against hipBLASLt fp16")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    print(f"device {torch.cuda.get_device_name(dev)} torch {torch.__version__}")
    for s in args.sizes:
        a = torch.empty((s, s), dtype=torch.bfloat16, device=dev)
        b = torch.empty((s, s), dtype=torch.bfloat16, device=dev)
        K.fill_uniform_bf16(a, 11)
        K.fill_uniform_bf16(b, 12)
        c = torch.empty((s, s), dtype=torch.bfloat16, device=dev)
        arms = {
            "amdk8s w8": lambda: K.gemm_bf16_nt(a, b, out=c, variant="w8"),
            "amdk8s w4": lambda: K.gemm_bf16_nt(a, b, out=c, variant="w4"),
            "amdk8s w4a": lambda: K.gemm_bf16_nt(a, b, out=c, variant="w4a"),
            "torch.matmul(hipBLASLt)": lambda: torch.matmul(a, b.t(), out=c),
        }
        if args.fp16:
            ah, bh = a.half(), b.half()
            ch = torch.empty((s, s), dtype=torch.float16, device=dev)
            arms["amdk8s w4a fp16"] = lambda: K.gemm_f16_nt(ah, bh, out=ch)
            arms["torch.matmul fp16 (hipBLASLt)"] = lambda: torch.matmul(ah, bh.t(), out=ch)
        for fn in arms.values():
            time_arm(fn, 5)
        res = {k: [] for k in arms}
        for _ in range(args.rounds):
            for k, fn in arms.items():
                res[k].append(time_arm(fn, args.iters))
        flop = 2.0 * s ** 3
        for k, v in res.items():
            med, mn = statistics.median(v), min(v)
            print(f"{s}^3 {k:28s} median {med:.4f} ms ({flop / med / 1e9:.1f} TFLOPS)  "
                  f"min {mn:.4f} ms ({flop / mn / 1e9:.1f} TFLOPS)")
        ref = torch.matmul(a, b.t())
        for v in ("w8", "w4", "w4a"):
            # a fresh NaN-filled output per variant: a kernel that skipped any element of C shows
            # up as NaN instead of inheriting the previous arm's (hipBLASLt's) result
            out = torch.full((s, s), float("nan"), dtype=torch.bfloat16, device=dev)
            K.gemm_bf16_nt(a, b, out=out, variant=v)
            unwritten = int(torch.isnan(out).sum().item())
            err = (out.float() - ref.float()).abs().max().item()
            print(f"{s}^3 max |amdk8s {v} - hipBLASLt| = {err:.4e}  (NaN/unwritten: {unwritten})")
        if args.fp16:
            out = torch.full((s, s), float("nan"), dtype=torch.float16, device=dev)
            K.gemm_f16_nt(ah, bh, out=out)
            ref16 = torch.matmul(ah, bh.t())
            err = (out.float() - ref16.float()).abs().max().item()
            print(f"{s}^3 max |amdk8s fp16 - hipBLASLt fp16| = {err:.4e}  "
                  f"(NaN/unwritten: {int(torch.isnan(out).sum().item())})")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
