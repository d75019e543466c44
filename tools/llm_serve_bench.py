#!/usr/bin/env python3
"""The LLM server measured as a service: HTTP + SSE streaming + continuous batching + chunked
prompt processing, on one MI355X.

The reference's LLM pod is llama-server behind a Service (reference
cluster-config/apps/llm/deployment.yaml:61,76-84); its users see aggregate tokens/s, time to first
token and inter-token latency, not engine step times.  This starts the in-tree server
(``python -m k8s_nvidia_gpus_amd.models.llm.server --synthetic 7b``: the Qwen2.5-7B Q4_K_M layout,
random blocks, synthetic vocabulary — no checkpoint offline) with the Deployment's settings and
drives it with streaming ``/v1/chat/completions`` clients:

* ``concurrency``: for N in --clients, N clients each send one chat request whose rendered prompt
  is --prompt tokens (distinct content per request: no prompt-cache hits) for --gen new tokens
  (``ignore_eos``, greedy).  Reports aggregate tok/s over the whole run and over the window in
  which all N streams decode, TTFT p50/p99 and inter-token-latency p50/p99/max.
* ``admit``: N-1 clients stream (long outputs); once they all decode, one more request with a
  --long-prompt-token prompt arrives.  Reports the worst gap between two chunks of any running
  stream while that prompt is processed, and its TTFT.

One JSON line on stdout (and --out).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def heartbeat(period=20.0):
    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f"[serve_bench] running ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q / 100 * (len(xs) - 1))))]


WORDS = ("cabin forest river mountain kernel matrix wave tile cache stream token slot prompt "
         "model server graph launch memory bandwidth latency throughput quantum ledger harbor "
         "violet copper meadow lantern orbit signal").split()


class Client:
    def __init__(self, base: str):
        import aiohttp

        self.base = base
        self.session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=3600))

    async def close(self):
        await self.session.close()

    async def post(self, path, body):
        async with self.session.post(self.base + path, json=body) as r:
            r.raise_for_status()
            return await r.json()

    async def prompt_messages(self, n_tokens: int, seed: int):
        """Chat messages whose rendered prompt tokenises to ``n_tokens`` (+- a few)."""
        rng = random.Random(seed)
        words = [rng.choice(WORDS) + str(rng.randrange(100)) for _ in range(4 * n_tokens)]

        async def count(k):
            msgs = [{"role": "user", "content": " ".join(words[:k])}]
            p = (await self.post("/apply-template", {"messages": msgs}))["prompt"]
            return len((await self.post("/tokenize", {"content": p}))["tokens"]), msgs

        lo, hi = 1, len(words)
        while lo < hi:                      # smallest word count reaching n_tokens
            mid = (lo + hi) // 2
            if (await count(mid))[0] >= n_tokens:
                hi = mid
            else:
                lo = mid + 1
        n, msgs = await count(lo)
        return msgs, n

    async def stream(self, msgs, max_tokens: int, rec: dict):
        """One streaming chat request; ``rec`` gets send time, chunk times and the usage."""
        body = {"messages": msgs, "max_tokens": max_tokens, "temperature": 0, "stream": True,
                "ignore_eos": True}
        rec["t_send"] = time.perf_counter()
        rec["chunks"] = []
        async with self.session.post(self.base + "/v1/chat/completions", json=body) as r:
            r.raise_for_status()
            async for line in r.content:
                if not line.startswith(b"data: "):
                    continue
                data = line[6:].strip()
                if data == b"[DONE]":
                    break
                obj = json.loads(data)
                ch = obj["choices"][0]
                if ch.get("delta", {}).get("content"):
                    rec["chunks"].append(time.perf_counter())
                if ch.get("finish_reason"):
                    rec["usage"] = obj.get("usage")
                    rec["timings"] = obj.get("timings")
        rec["t_done"] = time.perf_counter()
        return rec


def summarise(recs):
    ttft = [r["chunks"][0] - r["t_send"] for r in recs if r["chunks"]]
    itl = [b - a for r in recs for a, b in zip(r["chunks"], r["chunks"][1:])]
    ntok = sum(r["usage"]["completion_tokens"] for r in recs)
    t0 = min(r["t_send"] for r in recs)
    t1 = max(r["t_done"] for r in recs)
    # the window in which every stream is decoding: tokens counted by their chunk times
    w0 = max(r["chunks"][0] for r in recs)
    w1 = min(r["chunks"][-1] for r in recs)
    inside = sum(1 for r in recs for c in r["chunks"] if w0 < c <= w1)
    return {"requests": len(recs), "completion_tokens": ntok, "wall_s": round(t1 - t0, 3),
            "agg_tok_s": round(ntok / (t1 - t0), 1),
            "steady_tok_s": round(inside / (w1 - w0), 1) if w1 > w0 else None,
            "ttft_ms_p50": round(pct(ttft, 50) * 1e3, 1), "ttft_ms_p99": round(pct(ttft, 99) * 1e3, 1),
            "itl_ms_p50": round(pct(itl, 50) * 1e3, 2), "itl_ms_p99": round(pct(itl, 99) * 1e3, 2),
            "itl_ms_max": round(max(itl) * 1e3, 2) if itl else None,
            "prompt_tokens": recs[0]["usage"]["prompt_tokens"]}


async def run(args, base):
    cl = Client(base)
    out = {"concurrency": [], "admit": None}
    try:
        seed = 0
        # warm-up request: first-touch allocations of the prefill path
        msgs, _ = await cl.prompt_messages(64, seed=10 ** 6)
        await cl.stream(msgs, 8, {})
        for n in [int(x) for x in args.clients.split(",") if x]:
            prompts = []
            for i in range(n):
                seed += 1
                prompts.append((await cl.prompt_messages(args.prompt, seed))[0])
            recs = await asyncio.gather(*(cl.stream(m, args.gen, {}) for m in prompts))
            row = dict(clients=n, **summarise(recs))
            # what the scheduler did until every stream had its first token (TTFT window)
            try:
                async with cl.session.get(cl.base + "/debug/iterations") as r:
                    dbg = await r.json()
                a0 = min(r_["t_send"] for r_ in recs) - 0.05
                a1 = max(r_["chunks"][0] for r_ in recs if r_["chunks"]) + 0.05
                its = [x for x in dbg["iterations"] if a0 <= x["t"] <= a1]
                row["ttft_window"] = {
                    "iterations": len(its),
                    "first_iteration_after_send_ms": round((its[0]["t"] - a0 - 0.05) * 1e3, 1)
                    if its else None,
                    "prefill_ms": round(sum(x["prefill_s"] for x in its) * 1e3, 1),
                    "step_ms": round(sum(x["step_s"] for x in its) * 1e3, 1),
                    "prompt_tokens": sum(x["prompt_tokens"] for x in its),
                    "gc_pauses_ms": [round(g["s"] * 1e3, 1) for g in dbg.get("gc_pauses", [])
                                     if a0 <= g["t"] <= a1]}
            except Exception as e:  # noqa: BLE001 - diagnostics only
                row["ttft_window"] = {"error": repr(e)[:120]}
            out["concurrency"].append(row)
            print(f"concurrency {row}", file=sys.stderr, flush=True)
        if args.admit:
            n = args.admit
            prompts = []
            for i in range(n - 1):
                seed += 1
                prompts.append((await cl.prompt_messages(args.prompt, seed))[0])
            seed += 1
            long_msgs, long_n = await cl.prompt_messages(args.long_prompt, seed)
            recs = [{} for _ in range(n - 1)]
            tasks = [asyncio.create_task(cl.stream(m, args.admit_gen, r))
                     for m, r in zip(prompts, recs)]
            while not all(r.get("chunks") and len(r["chunks"]) >= 16 for r in recs):
                await asyncio.sleep(0.01)
            await asyncio.sleep(0.2)
            lrec = {}
            await cl.stream(long_msgs, 4, lrec)
            t_in, t_first = lrec["t_send"], lrec["chunks"][0] if lrec["chunks"] else lrec["t_done"]
            await asyncio.gather(*tasks)
            gaps, gaps_all = [], []
            for r in recs:
                for a, b in zip(r["chunks"], r["chunks"][1:]):
                    gaps_all.append(b - a)
                    if b > t_in and a < t_first:       # a gap overlapping the admission
                        gaps.append(b - a)
            # what the scheduler did meanwhile (same CLOCK_MONOTONIC as perf_counter here)
            async with cl.session.get(cl.base + "/debug/iterations") as r:
                dbg = await r.json()
            its = [x for x in dbg["iterations"] if t_in - 0.05 <= x["t"] <= t_first + 0.05]
            worst = sorted(its, key=lambda x: -(x["admit_s"] + x["prefill_s"] + x["step_s"]
                                                + x["wake_s"]))[:6]
            gcs = [g for g in dbg["gc_pauses"] if t_in - 0.05 <= g["t"] <= t_first + 0.05]
            out["admit_trace"] = {
                "iterations": len(its),
                "worst": [{k: (round(v * 1e3, 2) if k.endswith("_s") else v) for k, v in x.items()
                           if k != "t"} | {"at_ms": round((x["t"] - t_in) * 1e3, 1)} for x in worst],
                "gc_pauses_ms": [round(g["s"] * 1e3, 2) for g in gcs]}
            out["admit"] = {"running_streams": n - 1, "long_prompt_tokens": long_n,
                            "long_ttft_ms": round((t_first - t_in) * 1e3, 1),
                            "worst_gap_during_admit_ms": round(max(gaps) * 1e3, 2) if gaps else None,
                            "gaps_during_admit": len(gaps),
                            "itl_ms_p50": round(pct(gaps_all, 50) * 1e3, 2),
                            "itl_ms_p99": round(pct(gaps_all, 99) * 1e3, 2),
                            "long_timings": lrec.get("timings")}
            print(f"admit {out['admit']}", file=sys.stderr, flush=True)
            print(f"admit_trace {out['admit_trace']}", file=sys.stderr, flush=True)
        out["metrics"] = await metrics(cl)
    finally:
        await cl.close()
    return out


async def metrics(cl):
    async with cl.session.get(cl.base + "/metrics") as r:
        txt = await r.text()
    m = {}
    for ln in txt.splitlines():
        if ln and not ln.startswith("#"):
            k, v = ln.split()
            m[k.replace("llamacpp_amdk8s_", "")] = float(v)
    return m


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--clients", default="1,4,8")
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--gen", type=int, default=512)
    ap.add_argument("--admit", type=int, default=8, help="streams in the admission test (0: skip)")
    ap.add_argument("--admit-gen", type=int, default=1024)
    ap.add_argument("--long-prompt", type=int, default=3584)
    ap.add_argument("--parallel", type=int, default=8)
    ap.add_argument("--ctx-size", type=int, default=32768)
    ap.add_argument("--ubatch-size", type=int, default=512)
    ap.add_argument("--synthetic", default="7b")
    ap.add_argument("--server-log", default=None)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    heartbeat()
    port = free_port()
    cmd = [sys.executable, "-u", "-m", "k8s_nvidia_gpus_amd.models.llm.server", "--synthetic",
           args.synthetic, "--parallel", str(args.parallel), "--ctx-size", str(args.ctx_size),
           "--ubatch-size", str(args.ubatch_size), "--host", "127.0.0.1", "--port", str(port)]
    log = open(args.server_log or os.devnull, "w")
    t0 = time.time()
    srv = subprocess.Popen(cmd, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT)
    base = f"http://127.0.0.1:{port}"
    try:
        import urllib.request

        while True:                      # /health is 503 until the model and graphs are ready
            if srv.poll() is not None:
                raise SystemExit(f"server exited with {srv.returncode}")
            try:
                with urllib.request.urlopen(base + "/health", timeout=2) as r:
                    if r.status == 200:
                        break
            except Exception:  # noqa: BLE001 - not up yet
                pass
            if time.time() - t0 > 900:
                raise SystemExit("server not ready after 900 s")
            time.sleep(1)
        ready_s = time.time() - t0
        print(f"server ready after {ready_s:.1f} s", file=sys.stderr, flush=True)
        res = asyncio.run(run(args, base))
        res.update(server_ready_s=round(ready_s, 1), parallel=args.parallel,
                   ctx_size=args.ctx_size, ubatch=args.ubatch_size, gen=args.gen,
                   prompt=args.prompt,
                   model="Qwen2.5-7B architecture, Q4_K_M type mix, random blocks, synthetic vocab")
    finally:
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
        log.close()
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
