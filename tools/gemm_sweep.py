#!/usr/bin/env python3
"""Interleaved A/B of GEMM arms over (M, N, K) shapes in one process (random [-1,1) bf16 data).

usage: gemm_sweep.py --shapes 4096x4096x4096 8192x8192x4096 ... [--arms w8 w4 blt] [--rounds 5]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402


def timed(fn, iters):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["8192x8192x8192"])
    ap.add_argument("--arms", nargs="+", default=["w8", "w4", "blt"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--min-ms", type=float, default=20.0, help="time per round per arm")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for shp in args.shapes:
        m, n, k = (int(x) for x in shp.split("x"))
        a = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
        b = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
        K.fill_uniform_bf16(a, 11)
        K.fill_uniform_bf16(b, 12)
        c = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
        arms = {}
        if any(x in ("f8", "f8h", "blt8") or x.startswith("f8@") for x in args.arms):
            a8 = K.uniform_fp8((m, k), 13, dev)
            b8 = K.uniform_fp8((n, k), 14, dev)
            one = torch.ones((), device=dev)
        for arm in args.arms:
            if arm == "f8":  # hand-written fp8 e4m3 kernel (default: generated-assembly K-loop)
                arms[arm] = lambda: K.gemm_fp8_nt(a8, b8, out=c)
            elif arm.startswith("f8@"):  # f8@ENV=VALUE: the fp8 kernel with a launcher env knob
                k_, v_ = arm[3:].split("=", 1)

                def fn(k_=k_, v_=v_):
                    os.environ[k_] = v_
                    try:
                        K.gemm_fp8_nt(a8, b8, out=c)
                    finally:
                        os.environ.pop(k_, None)
                arms[arm] = fn
            elif arm == "f8h":  # the hipcc-scheduled fp8 kernel
                arms[arm] = lambda: K.gemm_fp8_nt(a8, b8, out=c, variant="hipcc")
            elif arm == "blt8":  # hipBLASLt fp8 through torch._scaled_mm (unit scales)
                arms[arm] = lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one,
                                                     out_dtype=torch.bfloat16)
            elif arm == "blt":
                arms[arm] = lambda: torch.matmul(a, b.t(), out=c)
            elif "@" in arm or arm == "w4x":
                # VARIANT@ENV=VALUE: the variant with a launcher env knob set (A/B of kernel options);
                # w4x = w4 without the super-block tile order
                spec = "w4@AMDK8S_W4_SUPERBLOCK=0" if arm == "w4x" else arm
                var, kvs = spec.split("@", 1)
                env = dict(kv.split("=", 1) for kv in kvs.split(","))  # VARIANT@K1=V1,K2=V2

                def f(var=var, env=env):
                    os.environ.update(env)
                    K.gemm_bf16_nt(a, b, out=c, variant=var)
                    for key in env:
                        os.environ.pop(key, None)
                arms[arm] = f
            else:
                arms[arm] = (lambda v: (lambda: K.gemm_bf16_nt(a, b, out=c, variant=v)))(arm)
        est = {}
        for name, fn in arms.items():
            timed(fn, 3)
            est[name] = max(1, int(args.min_ms / max(timed(fn, 3), 1e-3)))
        res = {name: [] for name in arms}
        for _ in range(args.rounds):
            for name, fn in arms.items():
                res[name].append(timed(fn, est[name]))
        flop = 2.0 * m * n * k
        line = [f"{shp:>18s}"]
        for name, v in res.items():
            med = statistics.median(v)
            line.append(f"{name} {flop / med / 1e9:7.1f}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
