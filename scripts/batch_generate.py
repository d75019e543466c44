#!/usr/bin/env python3
"""Batch client for the SD1.5 image API (cluster-config/apps/sd15-api, NodePort 30800).

Command-line compatible with the reference client (reference scripts/batch_generate.py:44-58:
``prompt count prefix [out_dir] --steps --url --delay``).  Its two defects are gone — the
``traceback`` module it calls but never imports (:32,35) and ``--steps`` defaulting to 40 while
the help says 30 (:50).  Additions:

* ``--parallel N`` keeps N requests in flight; the service coalesces concurrent requests into one
  batched denoising loop on the GPU (k8s_nvidia_gpus_amd/models/sd15_api.py), so this is how the
  MI355X is actually kept busy;
* ``--seed S`` makes a run reproducible (image i gets seed S+i-1);
* ``--retries R`` re-sends a request that failed at the connection level (not on HTTP 4xx);
* each PNG is written to a temporary name and renamed, so an interrupted run never leaves a
  truncated image that looks complete;
* the run ends with a latency summary (server-side ``X-Gen-Time`` and client round trip).

    scripts/batch_generate.py "a panda riding a motorbike" 8 panda out/ --parallel 8
"""

import argparse
import os
import statistics
import sys
import time
import traceback
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional

import requests

DEFAULT_URL = "http://127.0.0.1:30800/generate"


@dataclass
class Request:
    index: int
    target: Path
    payload: dict


@dataclass
class Outcome:
    request: Request
    ok: bool
    server_s: Optional[float] = None
    round_trip_s: float = 0.0
    error: str = ""


def plan(prompt: str, count: int, prefix: str, out_dir: Path, steps: int,
         seed: Optional[int]) -> List[Request]:
    """One request per image; file names follow the reference (``<prefix>_NN.png``)."""
    reqs = []
    for i in range(1, count + 1):
        body = {"prompt": prompt, "steps": steps}
        if seed is not None:
            body["seed"] = seed + i - 1
        reqs.append(Request(i, out_dir / f"{prefix}_{i:02d}.png", body))
    return reqs


def _write_atomic(target: Path, data: bytes) -> None:
    tmp = target.with_name(f".{target.name}.part")
    tmp.write_bytes(data)
    os.replace(tmp, target)


def _seconds(header: Optional[str]) -> Optional[float]:
    """``X-Gen-Time`` as seconds; the service sends e.g. ``2.59s``, the reference sent ``2.59``."""
    try:
        return float(header.strip().rstrip("s")) if header else None
    except ValueError:
        return None


def send(session: requests.Session, url: str, req: Request, timeout: float, retries: int) -> Outcome:
    t0 = time.perf_counter()
    last = ""
    for attempt in range(retries + 1):
        try:
            resp = session.post(url, json=req.payload, timeout=timeout)
            if 400 <= resp.status_code < 500:   # the request itself is wrong: do not resend
                return Outcome(req, False, round_trip_s=time.perf_counter() - t0,
                               error=f"HTTP {resp.status_code}: {resp.text[:200]}")
            resp.raise_for_status()
            _write_atomic(req.target, resp.content)
            return Outcome(req, True, _seconds(resp.headers.get("X-Gen-Time")), time.perf_counter() - t0)
        except requests.exceptions.RequestException as e:
            last = f"{type(e).__name__}: {e}"
            if attempt < retries:
                time.sleep(min(2.0 ** attempt, 10.0))
        except Exception as e:  # noqa: BLE001 - report and continue with the other images
            traceback.print_exc()
            return Outcome(req, False, round_trip_s=time.perf_counter() - t0, error=repr(e))
    return Outcome(req, False, round_trip_s=time.perf_counter() - t0, error=last)


def run(reqs: List[Request], url: str, parallel: int = 1, delay: float = 0.0, timeout: float = 600.0,
        retries: int = 0) -> List[Outcome]:
    if reqs:
        reqs[0].target.parent.mkdir(parents=True, exist_ok=True)
    session = requests.Session()

    def one(req: Request) -> Outcome:
        print(f"[*] {req.target.name}: requesting ({req.payload['steps']} steps)", flush=True)
        out = send(session, url, req, timeout, retries)
        if out.ok:
            gen = f"{out.server_s:.2f}s on the GPU, " if out.server_s is not None else ""
            print(f"    {req.target.name}: ok ({gen}{out.round_trip_s:.2f}s round trip)", flush=True)
        else:
            print(f"    {req.target.name}: FAILED {out.error}", flush=True)
        return out

    if parallel > 1:
        with ThreadPoolExecutor(max_workers=parallel) as pool:
            return list(pool.map(one, reqs))
    outcomes = []
    for n, req in enumerate(reqs):
        outcomes.append(one(req))
        if delay > 0 and n + 1 < len(reqs):
            time.sleep(delay)
    return outcomes


def summarize(outcomes: List[Outcome], wall_s: float) -> str:
    ok = [o for o in outcomes if o.ok]
    line = f"[*] {len(ok)}/{len(outcomes)} images in {wall_s:.1f}s"
    gen = [o.server_s for o in ok if o.server_s is not None]
    if gen:
        line += f"; X-Gen-Time median {statistics.median(gen):.2f}s max {max(gen):.2f}s"
    if ok:
        line += f"; {len(ok) / wall_s:.2f} images/s"
    return line


def main(argv) -> int:
    ap = argparse.ArgumentParser(description="Batch-generate images via the SD1.5 API")
    ap.add_argument("prompt", help="prompt sent with every request")
    ap.add_argument("count", type=int, help="number of images")
    ap.add_argument("prefix", help="output filename prefix, e.g. piggy")
    ap.add_argument("out_dir", nargs="?", default="outputs", help="output directory (default: outputs)")
    ap.add_argument("--steps", type=int, default=30, help="diffusion steps per image (default: 30)")
    ap.add_argument("--url", default=DEFAULT_URL, help=f"API endpoint (default: {DEFAULT_URL})")
    ap.add_argument("--delay", type=float, default=0, help="seconds between sequential requests")
    ap.add_argument("--parallel", type=int, default=1, help="requests in flight (batched on the GPU)")
    ap.add_argument("--seed", type=int, default=None, help="base seed (image i uses seed+i-1)")
    ap.add_argument("--retries", type=int, default=0, help="resends after a connection-level failure")
    ap.add_argument("--timeout", type=float, default=600.0, help="per-request timeout in seconds")
    args = ap.parse_args(argv)

    out_dir = Path(args.out_dir)
    reqs = plan(args.prompt, args.count, args.prefix, out_dir, args.steps, args.seed)
    t0 = time.perf_counter()
    outcomes = run(reqs, args.url, args.parallel, args.delay, args.timeout, args.retries)
    print(summarize(outcomes, time.perf_counter() - t0))
    print(f"images under {out_dir.resolve()}")
    return 0 if all(o.ok for o in outcomes) else 1


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1:]))
