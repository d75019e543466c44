#!/usr/bin/env python3
"""Generate Wan2.1 text-to-video (or text-to-image) outputs through the cluster's ComfyUI.

Same CLI as the reference script (reference cluster-config/apps/llm/scripts/generate_wan_t2v.py:
300-322); the logic lives in k8s_nvidia_gpus_amd/models/comfy_client.py.

    ./generate_wan_t2v.py --prompt "a red panda surfing" --count 3 --port-forward
"""
import argparse
import random
import sys
from datetime import datetime
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[4]))
from k8s_nvidia_gpus_amd.models.comfy_client import (ComfyClient, ComfyError, WanJob,  # noqa: E402
                                                     port_forward, run_jobs)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--prompt", required=True)
    ap.add_argument("--negative", default="blurry, low quality, artifacts")
    ap.add_argument("--count", type=int, default=5)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=320)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--cfg", type=float, default=6.0)
    ap.add_argument("--sampler", default="uni_pc")
    ap.add_argument("--scheduler", default="simple")
    ap.add_argument("--denoise", type=float, default=1.0)
    ap.add_argument("--mode", choices=["video", "image"], default="video")
    ap.add_argument("--format", choices=["webm", "webp", "both"], default="webm")
    ap.add_argument("--comfy-url", default="http://127.0.0.1:8181")
    ap.add_argument("--output-dir", default="generated")
    ap.add_argument("--seed", type=int, default=None, help="base seed; outputs use seed, seed+1, ...")
    ap.add_argument("--port-forward", action="store_true", help="start kubectl port-forward if needed")
    ap.add_argument("--namespace", default="comfyui")
    ap.add_argument("--deployment", default="wan-video-gen")
    ap.add_argument("--skip-check", action="store_true", help="skip the model-file preflight")
    ap.add_argument("--timeout", type=float, default=3600)
    args = ap.parse_args(argv)

    rnd = random.SystemRandom()
    seeds = [args.seed + i if args.seed is not None else rnd.randrange(1 << 63) for i in range(args.count)]
    formats = ("webm", "webp") if args.format == "both" else (args.format,)
    prefix = "wan_t2v" if args.mode == "video" else "wan_t2i"
    jobs = [WanJob(prompt=args.prompt, negative=args.negative, seed=s, width=args.width,
                   height=args.height, frames=args.frames, steps=args.steps, cfg=args.cfg,
                   sampler=args.sampler, scheduler=args.scheduler, denoise=args.denoise,
                   mode=args.mode, formats=formats, prefix=f"{prefix}_{i:02d}")
            for i, s in enumerate(seeds, 1)]
    dest = Path(args.output_dir).expanduser().resolve() / datetime.now().strftime("%Y%m%d_%H%M%S")
    client = ComfyClient(args.comfy_url)
    try:
        if client.reachable():
            saved = run_jobs(client, jobs, dest, not args.skip_check, args.timeout)
        elif args.port_forward:
            from urllib.parse import urlparse

            port = urlparse(args.comfy_url).port or 8181
            with port_forward(args.namespace, args.deployment, port):
                if not client.wait_reachable(30):
                    raise ComfyError("port-forward started but ComfyUI is not reachable")
                saved = run_jobs(client, jobs, dest, not args.skip_check, args.timeout)
        else:
            raise ComfyError("ComfyUI is not reachable; use --port-forward or --comfy-url")
    except (ComfyError, TimeoutError, ValueError) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    if saved:
        print(f"\nDone. Open {dest / 'index.html'}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
