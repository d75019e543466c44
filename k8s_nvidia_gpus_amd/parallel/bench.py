"""Collective bandwidth benchmark, one process per GPU (launch with torchrun in an amd.com/gpu: N pod).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m k8s_nvidia_gpus_amd.parallel.bench --op all_reduce -b 8 -e 4G -f 4

Prints an nccl-tests style table on rank 0 and a final JSON line (used by the gpu-bench Job and by
the validator's exporter integration).  ``--backend gloo`` runs the same code on CPU.
"""
from __future__ import annotations

import argparse
import json
import sys

import torch
import torch.distributed as dist

from .collectives import BUSBW_FACTOR, format_table, init_distributed, results_json, sweep


def parse_size(s: str) -> int:
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    s = s.strip().upper()
    if s and s[-1] in mult:
        return int(float(s[:-1]) * mult[s[-1]])
    return int(s)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--op", default="all_reduce", choices=sorted(BUSBW_FACTOR))
    ap.add_argument("-b", "--minbytes", default="1M")
    ap.add_argument("-e", "--maxbytes", default="1G")
    ap.add_argument("-f", "--stepfactor", type=int, default=4)
    ap.add_argument("-n", "--iters", type=int, default=20)
    ap.add_argument("-w", "--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16", "float16"])
    ap.add_argument("--backend", default=None, choices=[None, "nccl", "gloo"])
    args = ap.parse_args(argv)
    device = init_distributed(args.backend)
    rows = sweep(args.op, parse_size(args.minbytes), parse_size(args.maxbytes), args.stepfactor,
                 dtype=getattr(torch, args.dtype), iters=args.iters, warmup=args.warmup, device=device)
    doc = results_json(rows)
    if dist.get_rank() == 0:
        print(f"# {args.op} over {dist.get_world_size()} rank(s), backend {dist.get_backend()}")
        print(format_table(rows))
        print(json.dumps({k: v for k, v in doc.items() if k != "rows"}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if doc["passed"] else 1


if __name__ == "__main__":
    sys.exit(main())
