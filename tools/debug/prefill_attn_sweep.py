#!/usr/bin/env python3
"""Plan sweep of the hand-written prompt attention (ops/csrc/llm_prefill_attn.hip): waves per
workgroup x key splits, per (P, start), Qwen2.5-7B layout (28 q heads / 4 KV heads, d 128, fp16).
One JSON line per point; the auto plan is marked.  Usage: prefill_attn_sweep.py [P:start ...]"""
from __future__ import annotations

import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main(argv):
    from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

    dev = torch.device("cuda")
    H, Hkv, d = 28, 4, 128
    cases = [tuple(int(x) for x in a.split(":")) for a in argv] or \
        [(512, 0), (512, 3072), (512, 31488), (64, 8192), (2048, 0), (8192, 0)]
    for P, start in cases:
        end = start + P
        if os.environ.get("SWEEP_TOKEN_MAJOR") == "1":     # the engine's [P][H][128] storage
            q = torch.randn(P, H, d, device=dev, dtype=torch.float16).transpose(0, 1)
            out = torch.empty(P, H, d, device=dev, dtype=torch.float16).transpose(0, 1)
        else:
            q = torch.randn(H, P, d, device=dev, dtype=torch.float16)
            out = torch.empty(H, P, d, device=dev, dtype=torch.float16)
        k = torch.randn(Hkv, end, d, device=dev, dtype=torch.float16)
        v = torch.randn(Hkv, end, d, device=dev, dtype=torch.float16)
        auto = LK.prefill_attn_plan(P, start, H, Hkv)
        flop = 4 * H * d * P * (start + (P + 1) / 2)
        us = timed(lambda: LK.prefill_attn(q, k, v, out, start, 1 / math.sqrt(d)),
                   iters=int(os.environ.get("SWEEP_ITERS", "20")))
        print(json.dumps({"P": P, "start": start, "plan": "auto", **auto, "us": round(us, 1),
                          "tflops": round(flop / us / 1e6, 1)}), flush=True)
        ntiles = (end + 63) // 64
        if os.environ.get("SWEEP_AUTO_ONLY") == "1":
            continue
        splits = [int(x) for x in os.environ.get("SWEEP_SPLITS", "1,2,3,4,6,8,12,16,24").split(",")]
        for ks in (1, 2):
            for nw in (4, 8):
                for ns in splits:
                    if ns > ntiles:
                        continue
                    us = timed(lambda: LK.prefill_attn(q, k, v, out, start, 1 / math.sqrt(d),
                                                       nsplit=ns, nw=nw, ks=ks))
                    print(json.dumps({"P": P, "start": start, "waves": nw, "key_slots": ks,
                                      "nsplit": ns, "us": round(us, 1),
                                      "tflops": round(flop / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
