#!/usr/bin/env python3
"""Steady-state workload for a rocprofv3 kernel profile: warm up (MIOpen find, graph capture,
lazy kernel loads), sleep 300 ms, then run N iterations — tools/rocpd_summary.py
--after-gap-ms 200 --per N then reports only the steady-state dispatches.

    python tools/steady_prof.py sd15-unet  [--iters 20]   # one SD1.5 UNet CFG pass (512², fp16)
    python tools/steady_prof.py wan-step   [--iters 5]    # one Wan2.1-1.3B CFG DiT step (2560 tokens)
    python tools/steady_prof.py llm-decode [--iters 64]   # one Qwen2.5-7B Q4_K_M decode step, T=1
                                                          #   (position 512, host sync per token)
    python tools/steady_prof.py llm-prefill [--iters 10]  # one 512-token prompt prefill (fp16 path)
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def sd15_unet():
    from k8s_nvidia_gpus_amd.models.sd15 import StableDiffusion

    torch.backends.cudnn.benchmark = True          # the service's MIOpen find mode
    pipe = StableDiffusion(device="cuda", dtype=torch.float16)
    lat = torch.randn(1, 4, 64, 64, device="cuda")
    ctx = torch.randn(2, 77, 768, device="cuda", dtype=torch.float16)
    return lambda: pipe.runner(lat, 500, ctx, 7.5)


def wan_step():
    from k8s_nvidia_gpus_amd.models.wan.config import WanDiTConfig, WanVAEConfig
    from k8s_nvidia_gpus_amd.models.wan.pipeline import WanPipeline

    pipe = WanPipeline.synthetic(torch.device("cuda", 0), WanDiTConfig.wan21_t2v_1_3b(), None,
                                 WanVAEConfig.wan21())
    kv = pipe.text_kv(pipe.encode("a panda"), pipe.encode("blurry"))
    model = pipe.runner.model(kv, 6.0, pipe.device)
    x = torch.randn(1, 16, 4, 40, 64, device="cuda")
    return lambda: model(x, 0.7)


def llm_decode(T: int = 1, P: int = 512):
    from k8s_nvidia_gpus_amd.models.llm.config import QWEN25_7B
    from k8s_nvidia_gpus_amd.models.llm.engine import Engine
    from k8s_nvidia_gpus_amd.models.llm.weights import ModelWeights

    w = ModelWeights.random(QWEN25_7B, device=torch.device("cuda", 0), seed=0)
    ctx = max(4096, P + 512)
    eng = Engine(w, max_ctx=ctx, slots=8, dense=True)
    prompt = list(range(100, 100 + P))
    for s in range(T):
        eng.prefill(prompt, slot=s)
    state = {"pos": len(prompt), "tok": [11] * T}

    def step():
        p = state["pos"]
        nxt = eng.decode_greedy(state["tok"], [p] * T, list(range(T)))
        state["tok"] = [int(x) % QWEN25_7B.vocab for x in nxt]
        state["pos"] = p + 1 if p + 1 < min(P + 488, ctx - 8) else len(prompt)
    return step


def llm_prefill(P: int = 512):
    from k8s_nvidia_gpus_amd.models.llm.config import QWEN25_7B
    from k8s_nvidia_gpus_amd.models.llm.engine import Engine
    from k8s_nvidia_gpus_amd.models.llm.weights import ModelWeights

    w = ModelWeights.random(QWEN25_7B, device=torch.device("cuda", 0), seed=0)
    eng = Engine(w, max_ctx=max(4096, P + 256), slots=1 if P > 4096 else 8, dense=True)
    eng.dense_weights()
    prompt = list(range(100, 100 + P))
    return lambda: eng.prefill(prompt, slot=0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["sd15-unet", "wan-step", "llm-decode", "llm-prefill"])
    ap.add_argument("--tokens", type=int, default=1, help="llm-decode: concurrent sequences")
    ap.add_argument("--prompt", type=int, default=512, help="llm-decode / llm-prefill: prompt tokens (per sequence)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    fn = (llm_decode(a.tokens, a.prompt) if a.what == "llm-decode" else llm_prefill(a.prompt) if a.what == "llm-prefill"
          else {"sd15-unet": sd15_unet, "wan-step": wan_step}[a.what]())
    for _ in range(a.warmup):
        fn()
    torch.cuda.synchronize()
    time.sleep(0.3)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    print(f"{a.what}: {(time.perf_counter() - t0) * 1e3 / a.iters:.3f} ms/iter under the profiler",
          flush=True)


if __name__ == "__main__":
    main()
