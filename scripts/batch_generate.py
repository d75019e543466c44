#!/usr/bin/env python3
"""Generate several images from the SD1.5 API (cluster-config/apps/sd15-api) over HTTP.

Same CLI as the reference client (reference scripts/batch_generate.py:44-58) with its two bugs
fixed — the missing `traceback` import (:32,35) and `--steps` defaulting to 40 while documented as
30 (:50) — plus `--parallel` to send requests concurrently, which the API batches on the GPU.

    scripts/batch_generate.py "a panda riding a motorbike" 8 panda out/ --parallel 8
"""
import argparse
import sys
import time
import traceback
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import requests

DEFAULT_URL = "http://127.0.0.1:30800/generate"


def generate_one(session, url, payload, target: Path, timeout: float) -> str:
    resp = session.post(url, json=payload, timeout=timeout)
    resp.raise_for_status()
    target.write_bytes(resp.content)
    return resp.headers.get("X-Gen-Time", "?")


def generate(prompt: str, steps: int, url: str, out_dir: Path, prefix: str, count: int, delay: float,
             parallel: int = 1, seed=None, timeout: float = 600.0) -> int:
    out_dir.mkdir(parents=True, exist_ok=True)
    session = requests.Session()
    failures = 0

    def task(idx: int):
        name = f"{prefix}_{idx:02d}.png"
        payload = {"prompt": prompt, "steps": steps}
        if seed is not None:
            payload["seed"] = seed + idx - 1
        print(f"[*] generating {name}")
        try:
            t = generate_one(session, url, payload, out_dir / name, timeout)
            print(f"    done {name} in {t}")
            return True
        except requests.exceptions.RequestException as e:
            print(f"    request failed for {name}: {e}")
        except Exception as e:  # noqa: BLE001 - keep going with the remaining images
            print(f"    unexpected error for {name}: {e}")
            traceback.print_exc()
        return False

    if parallel > 1:
        with ThreadPoolExecutor(max_workers=parallel) as ex:
            failures = sum(1 for ok in ex.map(task, range(1, count + 1)) if not ok)
    else:
        for idx in range(1, count + 1):
            failures += 0 if task(idx) else 1
            if delay > 0 and idx != count:
                time.sleep(delay)
    print(f"[*] finished: {count - failures}/{count} images")
    return failures


def main(argv) -> int:
    ap = argparse.ArgumentParser(description="Batch-generate images via the SD1.5 API")
    ap.add_argument("prompt")
    ap.add_argument("count", type=int)
    ap.add_argument("prefix", help="output filename prefix, e.g. piggy")
    ap.add_argument("out_dir", nargs="?", default="outputs")
    ap.add_argument("--steps", type=int, default=30, help="diffusion steps per image (default: 30)")
    ap.add_argument("--url", default=DEFAULT_URL)
    ap.add_argument("--delay", type=float, default=0, help="seconds between sequential requests")
    ap.add_argument("--parallel", type=int, default=1, help="concurrent requests (batched on the GPU)")
    ap.add_argument("--seed", type=int, default=None, help="base seed (image i uses seed+i-1)")
    args = ap.parse_args(argv)
    failures = generate(args.prompt, args.steps, args.url, Path(args.out_dir), args.prefix, args.count,
                        args.delay, args.parallel, args.seed)
    print(f"images under {Path(args.out_dir).resolve()}")
    return 1 if failures else 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1:]))
