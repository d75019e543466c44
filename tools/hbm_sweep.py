#!/usr/bin/env python3
"""Sweep the HBM streaming kernels (ops/csrc/loadgen.hip) over cache policy, in-flight depth and
grid size, interleaved in ONE process (cdna_hip_programming.md §5.4 rule 24), on 2 GiB buffers.

    python tools/hbm_sweep.py [--gib 2] [--rounds 3] [--modes read,write,copy]

Prints one line per variant: mode, nt_load, nt_store, unroll, blocks/CU, median and min GB/s.
"""
from __future__ import annotations

import argparse
import itertools
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--modes", default="read,write,copy")
    ap.add_argument("--unrolls", default="1,2,4,8")
    ap.add_argument("--bpc", default="4,8,16")
    ap.add_argument("--layouts", default="0,1", help="0 = grid-stride window, 1 = chunk per workgroup")
    ap.add_argument("--nt", default="0,1", help="cache policies to sweep (0 = default, 1 = nt)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    nbytes = int(args.gib * (1 << 30)) // 16 * 16
    src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    dst = torch.empty_like(src)
    K.hbm_stream("write", None, src)  # toggling pattern, never zeros
    K.hbm_stream("write", None, dst)
    variants = []
    for mode in args.modes.split(","):
        nt = [int(x) for x in args.nt.split(",")]
        ntls = nt if mode != "write" else (0,)
        ntss = nt if mode != "read" else (0,)
        for ntl, nts, u, b, c in itertools.product(ntls, ntss, map(int, args.unrolls.split(",")),
                                                   map(int, args.bpc.split(",")),
                                                   map(int, args.layouts.split(","))):
            variants.append((mode, ntl, nts, u, b, c))
    res = {v: [] for v in variants}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.rounds):
        for v in variants:
            mode, ntl, nts, u, b, c = v
            s = src if mode != "write" else None
            d = dst if mode != "read" else None
            for _ in range(3):
                K.hbm_stream(mode, s, d, nbytes, blocks_per_cu=b, variant=(ntl, nts, u, c))
            e0.record()
            moved = 0
            for _ in range(args.iters):
                moved += K.hbm_stream(mode, s, d, nbytes, blocks_per_cu=b, variant=(ntl, nts, u, c))
            e1.record()
            e1.synchronize()
            res[v].append(moved / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    print(f"# {torch.cuda.get_device_name(dev)}; {nbytes / 2**30:.2f} GiB buffers, "
          f"{args.rounds} interleaved rounds x {args.iters} launches")
    print("mode   ntl nts unroll bpc chunk  median_GBps   min_GBps")
    for v in sorted(variants, key=lambda v: (v[0], -statistics.median(res[v]))):
        print(f"{v[0]:6s} {v[1]:3d} {v[2]:3d} {v[3]:6d} {v[4]:3d} {v[5]:5d} "
              f"{statistics.median(res[v]):12.1f} {min(res[v]):10.1f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
