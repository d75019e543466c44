#!/usr/bin/env python3
"""Numerics gate for a w4 K-loop schedule (AMDK8S_W4_SCHEDULE=<x>) before timing it.

Runs the w4 kernel under the schedule on shapes that exercise T = 1, 2, 3 K-tiles, odd tile
counts and multi-round grids, and checks (a) no NaN from the NaN-filled output, (b) the max error
against an fp32 torch reference, (c) bit-equality with the default REGION schedule (same per-lane
MFMA order, so any difference is a schedule bug).

usage: python tools/gemm_schedule_check.py interleaved   (any AMDK8S_W4_SCHEDULE value, or a
       GEMM variant name such as w4a, or w4a:<schedule>)
"""
import os
import sys

import torch

sys.path.insert(0, ".")
from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402

SHAPES = [(4096, 4096, 64), (8192, 8192, 64), (8192, 8192, 128), (8192, 4096, 192),
          (256, 256, 64), (768, 256, 1024), (4096, 8192, 1024), (12288, 12288, 1024),
          (8192, 8192, 8192)]


def main() -> int:
    sched = sys.argv[1]
    dev = torch.device("cuda", 0)
    ok = True
    for (m, n, k) in SHAPES:
        a = torch.empty((m, k), dtype=torch.bfloat16, device=dev)
        b = torch.empty((n, k), dtype=torch.bfloat16, device=dev)
        K.fill_uniform_bf16(a, 1)
        K.fill_uniform_bf16(b, 2)
        c = torch.full((m, n), float("nan"), dtype=torch.bfloat16, device=dev)
        if sched.split(":")[0] in K.GEMM_VARIANTS:  # a variant, optionally variant:schedule
            variant, _, w4a_sched = sched.partition(":")
            if w4a_sched:
                os.environ["AMDK8S_W4A_SCHEDULE"] = w4a_sched
            K.gemm_bf16_nt(a, b, out=c, variant=variant)
            os.environ.pop("AMDK8S_W4A_SCHEDULE", None)
        else:
            os.environ["AMDK8S_W4_SCHEDULE"] = sched
            K.gemm_bf16_nt(a, b, out=c, variant="w4")
        os.environ["AMDK8S_W4_SCHEDULE"] = "region"
        c2 = K.gemm_bf16_nt(a, b, variant="w4")
        ref = a.float() @ b.float().t()
        err = (c.float() - ref).abs().max().item()
        same = torch.equal(c, c2)
        nan = bool(torch.isnan(c.float()).any().item())
        good = (not nan) and same and err < 0.05 * (k ** 0.5) / 8 + 0.05
        ok &= good
        print(f"{m}x{n}x{k}: max_abs_err {err:.4f} equal_to_region {same} nan {nan} "
              f"{'ok' if good else 'FAIL'}", flush=True)
    print("ALL OK" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
