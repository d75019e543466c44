#!/usr/bin/env python3
"""Qwen2.5-7B (Q4_K_M layout, random-init blocks) on one MI355X: decode tokens/s and prefill.

The reference serves this model with llama.cpp at ``--ctx-size 4096`` and publishes no speed
(reference cluster-config/apps/llm/deployment.yaml:61-84).  This measures the in-tree
engine (``k8s_nvidia_gpus_amd/models/llm``) on the exact architecture and quantisation mix with
random weights (no network for the checkpoint): bytes streamed per token are those of the real file.

Reports, as one JSON line:
  * weight bytes and the HBM-roofline decode time per step (bytes / 6.3 TB/s measured copy peak);
  * decode ms/step and tokens/s for T = 1..4 and 8 concurrent sequences (HIP-graph replay, greedy
    sampling of every step on the GPU, per-step host sync as a server does);
  * prefill tokens/s for a ``--prompt``-token prompt (fp16 dense path);
  * per-GEMV-shape achieved bandwidth (``--gemv``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_nvidia_gpus_amd.models.llm import QWEN25_7B  # noqa: E402
from k8s_nvidia_gpus_amd.models.llm.engine import Engine  # noqa: E402
from k8s_nvidia_gpus_amd.models.llm.weights import ModelWeights  # noqa: E402
from k8s_nvidia_gpus_amd.ops import llm_kernels as LK  # noqa: E402


def heartbeat(period=30.0):
    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f"[llm_bench] running ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


GEMV_CASES = ("qkv", "o_proj", "gate_up", "gate_up_q8", "down_q4k", "down_q6k", "lm_head")
GEMV_CFGS = [(0, 0), (4, 4), (4, 16), (4, 32), (8, 8), (8, 16), (8, 32), (2, 4), (2, 8),
             (1, 2), (1, 4), (8, 7), (4, 7), (8, 14), (4, 37), (8, 37), (8, 74), (4, 74)]
# MFMA GEMV: (K-waves, rows per workgroup = 16 x row groups)
MFMA_CFGS = [(0, 0), (1, 64), (2, 32), (4, 16), (8, 16)]      # the instantiated shapes
# long rows (ffn_down): (K-waves, rows per workgroup, split-K slices over workgroups)
SPLIT_CFGS = [(0, 0, -1), (8, 16, 1), (4, 16, 1), (8, 16, 2), (4, 16, 2), (4, 16, 3), (4, 16, 4),
              (2, 16, 4), (4, 16, 6), (2, 16, 8), (4, 16, 8), (8, 16, 4)]


def bench_gemv(eng: Engine, iters: int = 56, sweep4: bool = False, only=GEMV_CASES,
               cfgs=GEMV_CFGS) -> list:
    """Achieved bandwidth of every decode GEMV shape, default decomposition and a sweep.

    Each timed launch reads ANOTHER layer's copy of the matrix (cycling over every layer that has
    it in the same quantisation type): 28 × 76 MB of gate|up does not fit the 256 MB Infinity
    Cache, so the numbers are the cold-weight rates of a real decode step, not MALL re-reads."""
    LK = eng.LK
    layers = eng.w.layers
    per_case = {
        "qkv": [(x.wqkv[0], None) for x in layers],
        "o_proj": [(x.wo, None) for x in layers],
        "gate_up": [(x.wg, x.wu) for x in layers],
        "gate_up_q8": [(x.wg, x.wu) for x in layers],
        "down_q4k": [(x.wd, None) for x in layers if x.wd.qtype == 0],
        "down_q6k": [(x.wd, None) for x in layers if x.wd.qtype == 1],
        "lm_head": [(eng.w.output, None)],
    }
    modes = {"qkv": "store", "o_proj": "resid", "gate_up": "pair", "gate_up_q8": "pair",
             "down_q4k": "resid", "down_q6k": "resid", "lm_head": "store"}
    rows = []
    for name in [c for c in GEMV_CASES if c in only]:
        mats = per_case[name]
        if not mats:
            continue
        mode = modes[name]
        w = mats[0][0]
        for T in (1, 4):
            x8 = torch.randint(-127, 127, (T, w.k), dtype=torch.int8, device=eng.device)
            dx = torch.full((T, w.k // 32), 0.01, device=eng.device)
            sx = torch.zeros(T, w.k // 16, device=eng.device)
            out = torch.zeros(T, w.n, device=eng.device)
            q8o = None
            if name == "gate_up_q8":
                q8o = (torch.zeros(T, w.n, dtype=torch.int8, device=eng.device),
                       torch.zeros(T, w.n // 32, device=eng.device),
                       torch.zeros(T, w.n // 16, device=eng.device))
            m = {"store": LK.STORE, "resid": LK.RESID, "pair": LK.PAIR}[mode]
            todo = cfgs if (T == 1 or sweep4) else cfgs[:1]
            if name == "gate_up_q8":          # 32 rows per workgroup are fixed there
                todo = [(wv, 0) for wv in (0, 2, 4, 8)]
            todo = [(wv, rp, 1) for wv, rp in todo]
            if LK.gemv_impl() == LK.GEMV_MFMA and w.mfma is not None:
                todo = [(wv, rp, 1) for wv, rp in MFMA_CFGS] if name not in ("gate_up", "gate_up_q8") \
                    else [(0, 0, 1), (1, 32, 1), (2, 32, 1)]
                if name.startswith("down"):
                    todo = SPLIT_CFGS
            for waves, rpw, ks in todo:
                def launch(i):
                    w0, w1 = mats[i % len(mats)]
                    LK.qgemv(w0, x8, dx, sx, out, m, w1=w1, waves=waves, rows_per_wg=rpw,
                             q8_out=q8o, kscratch=eng.kscratch, ksplit=ks)
                try:
                    for i in range(3):
                        launch(i)
                except RuntimeError:          # decomposition not supported for this shape
                    continue
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                e0.record()
                for i in range(iters):
                    launch(i)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / iters * 1e3
                nbytes = w.nbytes() * (2 if mode == "pair" else 1)
                r = {"gemv": name, "T": T, "N": w.n, "K": w.k, "type": ["Q4_K", "Q6_K"][w.qtype],
                     "cfg": [waves, rpw, ks], "copies": len(mats), "us": round(us, 2),
                     "GBps": round(nbytes / us / 1e3, 1)}
                rows.append(r)
                print(r, file=sys.stderr, flush=True)
    return rows


def bench_small_kernels(eng: Engine, iters: int = 100) -> list:
    """Per-launch time of the non-GEMV decode kernels (T = 1), attention at several lengths."""
    import math

    LK, c = eng.LK, eng.cfg
    b = eng._buffers(1)
    qd = eng._q8(b, c.dim)
    L = eng.w.layers[0]
    rows = []

    def timed(name, fn, **extra):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        r = dict(kernel=name, us=round(e0.elapsed_time(e1) / iters * 1e3, 2), **extra)
        rows.append(r)
        print(r, file=sys.stderr, flush=True)

    timed("rmsnorm_q8_dim", lambda: LK.rmsnorm_q8(b.h, L.attn_norm, c.eps, *qd))
    qf = eng._q8(b, c.ffn)
    timed("quant_ffn", lambda: LK.rmsnorm_q8(b.t, None, 0.0, *qf))
    timed("rope_kv", lambda: LK.rope_kv(b.qkv, b.pos, b.slot, eng.cos, eng.sin, c.heads,
                                        c.kv_heads, c.head_dim, eng.max_ctx, b.qrot,
                                        eng.k_cache[0], eng.v_cache[0]))
    for p in (100, 1000, 4000):
        if p >= eng.max_ctx:
            continue
        b.pos.fill_(p)
        span = eng._span(p)
        timed("attn_decode+combine", lambda: LK.attn_decode(
            b.qrot, b.pos, b.slot, eng.k_cache[0], eng.v_cache[0], c.heads, c.kv_heads,
            c.head_dim, eng.max_ctx, 1 / math.sqrt(c.head_dim), b.po, b.pml, *qd, span=span),
            pos=p, span=span)
    timed("embed_dequant", lambda: LK.dequant(eng.w.tok_embd, b.h, rows=b.tok))
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--layers", type=int, default=QWEN25_7B.layers)
    ap.add_argument("--steps", type=int, default=128, help="decode steps per T")
    ap.add_argument("--ctx", type=int, default=0,
                    help="KV-cache context (reference --ctx-size); 0 = max(4096, room for the "
                         "prompt and every timed step)")
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--tokens", default="1,2,3,4,8", help="decode T list ('' = no decode timing)")
    ap.add_argument("--gemv", action="store_true")
    ap.add_argument("--gemv-sweep4", action="store_true", help="also sweep the decomposition at T=4")
    ap.add_argument("--gemv-cases", default=",".join(GEMV_CASES), help="GEMV shapes to time")
    ap.add_argument("--kernels", action="store_true", help="time the non-GEMV decode kernels")
    ap.add_argument("--gemv-impl", choices=["valu", "mfma"],
                    default=os.environ.get("AMDK8S_LLM_GEMV_IMPL", "mfma"),
                    help="Q4_K GEMV kernel (A/B; env AMDK8S_LLM_GEMV_IMPL)")
    ap.add_argument("--norm-prologue-t", type=int,
                    default=int(os.environ.get("AMDK8S_LLM_NORM_PROLOGUE_T", "0")),
                    help="A/B: steps of up to this many tokens normalise in the GEMV prologues "
                         "(0 = the engine default; env AMDK8S_LLM_NORM_PROLOGUE_T)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    LK.gemv_impl(LK.GEMV_MFMA if args.gemv_impl == "mfma" else LK.GEMV_VALU)
    if not torch.cuda.is_available():
        print("llm_bench needs an MI355X", file=sys.stderr)
        return 2
    heartbeat()
    from dataclasses import replace

    cfg = replace(QWEN25_7B, layers=args.layers)
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    w = ModelWeights.random(cfg, device=dev, seed=0)
    torch.cuda.synchronize()
    ctx = args.ctx or max(4096, args.prompt + args.steps + 64)
    eng = Engine(w, max_ctx=ctx, slots=8, dense=True)
    if args.norm_prologue_t:
        eng.norm_prologue_t = args.norm_prologue_t
    eng.dense_weights()
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t0
    wbytes = w.nbytes()
    res = {"model": f"Qwen2.5-7B architecture, Q4_K_M type mix, random blocks ({cfg.layers} layers)",
           "weight_bytes": wbytes, "roofline_ms_at_6.3TBps": round(wbytes / 6.3e12 * 1e3, 4),
           "load_s": round(load_s, 2), "ctx": eng.max_ctx, "decode": [], "device":
           torch.cuda.get_device_name(0)}
    # prefill (dense fp16 path) — also fills the KV caches the decode steps attend over
    prompt = list(range(100, 100 + args.prompt))
    for s in range(4):
        eng.prefill(prompt, slot=s)
    torch.cuda.synchronize()
    t = time.perf_counter()
    eng.prefill(prompt, slot=0)
    torch.cuda.synchronize()
    pf = time.perf_counter() - t
    res["prefill"] = {"tokens": args.prompt, "s": round(pf, 4), "tok_s": round(args.prompt / pf, 1)}
    print(f"prefill {args.prompt} tokens: {pf * 1e3:.1f} ms", file=sys.stderr, flush=True)
    for T in [int(x) for x in args.tokens.split(",") if x]:
        pos = [args.prompt] * T
        toks = [11] * T
        slots = list(range(T))
        eng.decode_greedy(toks, pos, slots)          # capture (the timed loop's graph)
        for i in range(3):
            eng.decode_greedy(toks, [p + 1 + i for p in pos], slots)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(args.steps):
            # greedy on the GPU inside the step's graph, host sync per step like a server
            nxt = eng.decode_greedy(toks, [p + 4 + i for p in pos], slots)
            toks = [int(x) % cfg.vocab for x in nxt]
        dt = time.perf_counter() - t
        row = {"T": T, "ms_per_step": round(dt / args.steps * 1e3, 4),
               "tok_s": round(T * args.steps / dt, 1),
               "eff_GBps": round(wbytes / (dt / args.steps) / 1e9, 1)}
        res["decode"].append(row)
        print(f"decode T={T}: {row}", file=sys.stderr, flush=True)
    if args.gemv:
        res["gemv"] = bench_gemv(eng, sweep4=args.gemv_sweep4, only=args.gemv_cases.split(","))
    if args.kernels:
        res["kernels"] = bench_small_kernels(eng)
    res["graph_captures"] = eng.stats["graph_captures"]
    res["gemv_impl"] = args.gemv_impl
    res["norm_prologue_t"] = eng.norm_prologue_t
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
