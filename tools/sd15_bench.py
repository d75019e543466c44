#!/usr/bin/env python3
"""SD1.5 on one MI355X: UNet-pass latency and end-to-end text-to-image throughput.

The reference's SD15 service returns the per-request latency in ``X-Gen-Time`` but publishes no
value (reference sd15-api/configmap.yaml:113-121).  This measures the in-tree model
family (``k8s_nvidia_gpus_amd/models/sd15``) at the reference's request defaults — 512×512, 30
steps, CFG 7.5, fp16 — with random-init weights of the exact SD1.5 architecture (no network for
checkpoints; the maths per step is identical).

Arms (``--arms``):
  * ``torch-eager``  — PyTorch ops only (SDPA, F.group_norm), launched from Python each step;
  * ``native-eager`` — the HIP kernels (GroupNorm+SiLU, GEGLU, attention), launched from Python;
  * ``native-graph`` — the same, one UNet+CFG pass replayed from a HIP graph (the serving default).
Then the end-to-end pipeline (text encoder → 30 PNDM steps → VAE decode) at ``--batches``.

Prints one JSON object (``--out`` also writes it).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_nvidia_gpus_amd.models.sd15 import StableDiffusion, functional as SF  # noqa: E402
from k8s_nvidia_gpus_amd.models.sd15.config import SD15, tiny  # noqa: E402


def heartbeat(period: float = 30.0) -> None:
    """Print a progress line while long first calls (MIOpen solver search / kernel JIT) run."""
    import threading

    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f"[sd15_bench] still running ({time.time() - t0:.0f} s)", file=sys.stderr,
                  flush=True)

    threading.Thread(target=run, daemon=True).start()


def time_unet(pipe: StableDiffusion, batch: int, graphs: bool, iters: int, warmup: int) -> float:
    dev = pipe.device
    lat = torch.randn(batch, 4, 64, 64, device=dev)
    ctx = pipe.encode_prompt(["a photo"] * batch, [""] * batch)
    pipe.runner.use_graphs = graphs
    pipe.runner.reset()
    for _ in range(warmup):
        pipe.runner(lat, 981, ctx, 7.5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        pipe.runner(lat, 981, ctx, 7.5)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--dtype", default="float16", choices=["float16", "bfloat16"])
    ap.add_argument("--arms", default="torch-eager,native-eager,native-graph")
    ap.add_argument("--unet-batch", type=int, default=1, help="images per UNet pass (CFG doubles it)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batches", default="1,8", help="end-to-end batch sizes ('' = skip)")
    ap.add_argument("--tiny", action="store_true", help="miniature config (plumbing check only)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--miopen-find", action="store_true",
                    help="torch.backends.cudnn.benchmark: MIOpen solver search per conv shape")
    args = ap.parse_args(argv)
    if args.miopen_find:
        torch.backends.cudnn.benchmark = True
    if not torch.cuda.is_available():
        print("sd15_bench needs an MI355X", file=sys.stderr)
        return 2
    heartbeat()
    dtype = getattr(torch, args.dtype)
    cfg = tiny() if args.tiny else SD15
    t0 = time.perf_counter()
    pipe = StableDiffusion(device="cuda", dtype=dtype, cfg=cfg)
    res = {"model": "SD1.5 (random-init weights, exact architecture)" if not args.tiny else "tiny",
           "dtype": args.dtype, "device": torch.cuda.get_device_name(0),
           "load_s": round(time.perf_counter() - t0, 2), "unet_ms": {}, "e2e": []}
    b = args.unet_batch
    flops = None
    for arm in [a for a in args.arms.split(",") if a]:
        SF.set_backend("torch" if arm.startswith("torch") else "native")
        ms = time_unet(pipe, b, arm.endswith("graph"), args.iters, args.warmup)
        res["unet_ms"][arm] = round(ms, 3)
        print(f"unet batch {b} (x2 CFG) {arm}: {ms:.3f} ms", file=sys.stderr, flush=True)
    SF.set_backend("native")
    pipe.runner.use_graphs = True
    for nb in [int(x) for x in args.batches.split(",") if x]:
        gens = [torch.Generator(device="cuda").manual_seed(i) for i in range(nb)]
        pipe(["a cozy cabin in the woods"] * nb, num_inference_steps=2, generator=gens)  # capture
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = pipe(["a cozy cabin in the woods"] * nb, num_inference_steps=args.steps,
                   generator=gens)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        row = {"batch": nb, "steps": args.steps, "size": "512x512", "seconds": round(dt, 4),
               "images_per_s": round(nb / dt, 3),
               "timings": {k: round(v, 4) for k, v in out.timings.items()}}
        res["e2e"].append(row)
        print(f"e2e batch {nb}: {dt:.3f} s ({nb / dt:.2f} img/s) {row['timings']}",
              file=sys.stderr, flush=True)
    res["graph_captures"] = pipe.runner.captures
    res["flops_note"] = flops
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
