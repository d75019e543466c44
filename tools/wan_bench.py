#!/usr/bin/env python3
"""Wan2.1 T2V-1.3B on one MI355X: DiT step latency and end-to-end text-to-video time.

The reference runs Wan2.1 through an external ComfyUI server at 512×320, 16 frames, 25 steps,
CFG 6, uni_pc/simple (reference cluster-config/apps/llm/scripts/generate_wan_t2v.py:305-312) and
publishes no timing.  This measures the in-tree family (``k8s_nvidia_gpus_amd/models/wan``) at
exactly those defaults with random-init weights of the published architectures (no network for
checkpoints; the arithmetic per step is identical): the 1.3B DiT (30 blocks, 1536 wide, 12 heads),
the Wan VAE decoder and, with ``--t5``, the umT5-xxl encoder (5.7 B parameters).

Arms: ``native-graph`` (HIP row kernels + flash attention, the step replayed from a HIP graph —
the serving path), ``native`` (same kernels launched eagerly) and ``torch`` (the same model through
PyTorch ops) for one CFG step (batch 2, 2560 tokens); then the end-to-end job on the serving path.
Prints one JSON object (``--out`` also writes it).
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

from k8s_nvidia_gpus_amd.models.sd15 import functional as SF  # noqa: E402
from k8s_nvidia_gpus_amd.models.wan import functional as WF  # noqa: E402
from k8s_nvidia_gpus_amd.models.wan.config import (UMT5Config, WanDiTConfig,  # noqa: E402
                                                   WanVAEConfig, latent_frames)
from k8s_nvidia_gpus_amd.models.wan.pipeline import WanPipeline  # noqa: E402


def heartbeat(period: float = 30.0) -> None:
    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f"[wan_bench] still running ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def step_ms(pipe: WanPipeline, kv, shape, iters: int, warmup: int, graph: bool = False) -> float:
    x = torch.randn(shape, device=pipe.device)
    model = pipe.runner.model(kv, 6.0, pipe.device) if graph else pipe.denoiser(kv, 6.0)
    for _ in range(warmup):
        model(x, 0.7)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        model(x, 0.7)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


def dit_flops(cfg: WanDiTConfig, tokens: int, text: int, batch: int) -> float:
    d, f = cfg.dim, cfg.ffn_dim
    per_tok = 2 * (3 * d * d + d * d + d * d + d * d + 2 * d * f)           # qkv, o, cross q, o, ffn
    attn = 2 * 2 * tokens * tokens * d + 2 * 2 * tokens * text * d          # self + cross (QK, PV)
    return batch * cfg.layers * (tokens * per_tok + attn)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=320)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--arms", default="native-graph,native,torch")
    ap.add_argument("--t5", action="store_true", help="include the umT5-xxl encoder (11 GB bf16)")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--model", default="1.3b", choices=["1.3b", "14b"])
    ap.add_argument("--out")
    a = ap.parse_args(argv)
    heartbeat()
    dev = torch.device("cuda", 0)
    dcfg = WanDiTConfig.wan21_t2v_14b() if a.model == "14b" else WanDiTConfig.wan21_t2v_1_3b()
    t0 = time.time()
    pipe = WanPipeline.synthetic(dev, dcfg, UMT5Config.umt5_xxl() if a.t5 else None,
                                 WanVAEConfig.wan21())
    init_s = time.time() - t0
    vc = pipe.vae.cfg
    lat = (1, 16, latent_frames(a.frames), a.height // 8, a.width // 8)
    tokens = lat[2] * (lat[3] // 2) * (lat[4] // 2)
    pos, neg = pipe.encode("a panda riding a motorbike through a neon city"), pipe.encode("blurry")
    res = {"model": f"Wan2.1-T2V-{a.model.upper()} (random-init weights of the published architecture)",
           "video": {"width": a.width, "height": a.height, "frames_requested": a.frames,
                     "latent": list(lat), "tokens": tokens},
           "dtype": "bf16", "init_s": round(init_s, 2), "arms": {}}
    flops = dit_flops(dcfg, tokens, dcfg.text_len, 2)
    for arm in [s for s in a.arms.split(",") if s]:
        WF.set_backend("torch" if arm == "torch" else "auto")
        SF.set_backend("torch" if arm == "torch" else "auto")
        kv = pipe.text_kv(pos, neg)
        ms = step_ms(pipe, kv, lat, a.iters, a.warmup, graph=arm == "native-graph")
        res["arms"][arm] = {"cfg_step_ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1)}
        print(f"[wan_bench] {arm}: CFG step {ms:.2f} ms ({flops / ms / 1e9:.0f} TFLOPS)", file=sys.stderr,
              flush=True)
    WF.set_backend("auto")
    SF.set_backend("auto")
    if not a.no_e2e:
        pipe.generate("warm-up", "blurry", a.width, a.height, a.frames, steps=2, cfg=6.0)
        # a prompt not seen before: encode_s is the umT5 cost of a new request (cached afterwards)
        r = pipe.generate("a red fox running through fresh snow at dawn, cinematic", "low quality", a.width,
                          a.height, a.frames, steps=a.steps, cfg=6.0, sampler="uni_pc",
                          scheduler="simple", seed=0)
        res["e2e"] = {k: round(v, 3) for k, v in r.timings.items()}
        res["e2e"].update({"steps": a.steps, "frames_out": int(r.frames.shape[0]),
                           "sampler": "uni_pc", "scheduler": "simple", "cfg": 6.0})
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipe.vae.decode(r.latent.to(dev))
        torch.cuda.synchronize()
        res["vae_decode_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    res["device"] = torch.cuda.get_device_name(dev)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
