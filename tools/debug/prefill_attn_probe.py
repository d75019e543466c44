#!/usr/bin/env python3
"""Chunked-prefill attention on one MI355X: a 512-query chunk at offset ``start`` attending to
``start + 512`` cached keys (Qwen2.5-7B layout: 28 q heads over 4 kv heads, d = 128, fp16),
formulations timed and checked against the fp32 softmax:

  mask      SDPA with an explicit [P, end] boolean mask (the engine's chunk path before round 5)
  lowright  SDPA with torch.nn.attention.bias.causal_lower_right (bottom-right causal)
  split     prefix part (non-causal over [0, start)) + chunk part (causal over the chunk) from
            _scaled_dot_product_efficient_attention with log-sum-exp, merged on the host side
  hand      the hand-written causal GQA prefill attention kernel (when the library has it)

One JSON line per (variant, start)."""
from __future__ import annotations

import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


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


def main():
    dev = torch.device("cuda")
    H, Hkv, d = 28, 4, 128
    P = int(os.environ.get("PROBE_P", "512"))
    only = os.environ.get("PROBE_VARIANTS")
    g = torch.Generator(device=dev).manual_seed(0)
    starts = [int(v) for v in os.environ.get("PROBE_STARTS", "0,1536,3072,8192,16384,31488").split(",")]
    for start in starts:
        end = start + P
        q = torch.randn(1, H, P, d, device=dev, dtype=torch.float16, generator=g)
        k = torch.randn(1, Hkv, end, d, device=dev, dtype=torch.float16, generator=g)
        v = torch.randn(1, Hkv, end, d, device=dev, dtype=torch.float16, generator=g)
        kk = k.repeat_interleave(H // Hkv, 1)
        vv = v.repeat_interleave(H // Hkv, 1)
        qi = torch.arange(start, end, device=dev)[:, None]
        kj = torch.arange(end, device=dev)[None, :]
        mask = kj <= qi
        # fp32 reference on a few heads
        s = (q[:, :4].float() @ kk[:, :4].float().transpose(-1, -2)) / math.sqrt(d)
        s = s.masked_fill(~mask, float("-inf"))
        ref = torch.softmax(s, -1) @ vv[:, :4].float()
        variants = {}
        variants["mask"] = lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=mask[None, None],
                                                                  enable_gqa=True)
        try:
            from torch.nn.attention.bias import causal_lower_right
            bias = causal_lower_right(P, end)
            variants["lowright"] = lambda: F.scaled_dot_product_attention(q, kk, vv, attn_mask=bias)
            variants["lowright_gqa"] = lambda: F.scaled_dot_product_attention(
                q, k, v, attn_mask=bias, enable_gqa=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"variant": "lowright", "error": repr(e)[:200]}), flush=True)

        def split():
            if start == 0:
                return F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
            o1, l1 = torch.ops.aten._scaled_dot_product_efficient_attention(
                q, kk[:, :, :start], vv[:, :, :start], None, True)[:2]
            o2, l2 = torch.ops.aten._scaled_dot_product_efficient_attention(
                q, kk[:, :, start:], vv[:, :, start:], None, True, is_causal=True)[:2]
            l1, l2 = l1[..., :P, None], l2[..., :P, None]
            m = torch.maximum(l1, l2)
            w1, w2 = torch.exp(l1 - m), torch.exp(l2 - m)
            return ((o1.float() * w1 + o2.float() * w2) / (w1 + w2)).to(q.dtype)
        variants["split"] = split
        try:
            from k8s_nvidia_gpus_amd.ops import llm_kernels as LK
            out = torch.empty(H, P, d, device=dev, dtype=torch.float16)
            variants["hand"] = lambda: LK.prefill_attn(q[0], k[0], v[0], out, start,
                                                       1 / math.sqrt(d)) or out[None]
            plan = LK.prefill_attn_plan(P, start, H, Hkv)
            print(json.dumps({"variant": "hand_plan", "start": start, **plan}), flush=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"variant": "hand", "error": repr(e)[:200]}), flush=True)
        for name, fn in variants.items():
            if only and name not in only.split(","):
                continue
            try:
                o = fn()
                err = (o[:, :4].float() - ref).abs().max().item()
                us = timed(fn)
                flop = 4 * H * d * P * (start + P / 2)
                print(json.dumps({"variant": name, "start": start, "us": round(us, 1),
                                  "tflops": round(flop / us / 1e6, 1), "max_err": round(err, 4)}),
                      flush=True)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"variant": name, "start": start, "error": repr(e)[:300]}), flush=True)


if __name__ == "__main__":
    main()
