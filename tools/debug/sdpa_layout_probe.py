#!/usr/bin/env python3
"""Which kernels does the LLM prefill's attention call launch (engine._forward_dense_native: SDPA
GQA path on the fp16 KV-cache slabs, q in [H][P][128]) and does a q in [P][H][128] layout return
an output whose transpose(0, 1).reshape(P, H * 128) is a free view?  Qwen2.5-7B shapes, P = 512.

    python tools/debug/sdpa_layout_probe.py
"""
import time

import torch
import torch.nn.functional as F
from torch.profiler import ProfilerActivity, profile

H, HKV, D, P, CTX = 28, 4, 128, 512, 4096
dev = torch.device("cuda", 0)
kc = torch.randn(HKV, CTX, D, device=dev, dtype=torch.float16)
vc = torch.randn(HKV, CTX, D, device=dev, dtype=torch.float16)
q_hpd = torch.randn(H, P, D, device=dev, dtype=torch.float16)
q_phd = q_hpd.transpose(0, 1).contiguous().transpose(0, 1)      # same values, [P][H][D] storage


def attn(q):
    o = F.scaled_dot_product_attention(q[None], kc[None, :, :P], vc[None, :, :P], is_causal=True,
                                       enable_gqa=True)
    return o, o[0].transpose(0, 1).reshape(P, H * D)


for name, q in (("q [H][P][D]", q_hpd), ("q [P][H][D]", q_phd)):
    for _ in range(3):
        attn(q)
    torch.cuda.synchronize()
    o, o2 = attn(q)
    print(f"{name}: q strides {tuple(q.stride())}, out strides {tuple(o.stride())}, "
          f"reshape is a view: {o2.data_ptr() == o.data_ptr()}", flush=True)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(10):
            attn(q)
        torch.cuda.synchronize()
    for ev in prof.key_averages():
        if ev.device_type is not None and "cuda" in str(ev.device_type).lower():
            print(f"   {ev.count:4d} x {ev.device_time / 1.0 if hasattr(ev, 'device_time') else 0:8.1f} us  {ev.key[:110]}",
                  flush=True)
    t0 = time.perf_counter()
    for _ in range(50):
        attn(q)
    torch.cuda.synchronize()
    print(f"   {(time.perf_counter() - t0) / 50 * 1e6:.1f} us per call (eager)", flush=True)
ref = attn(q_hpd)[1]
alt = attn(q_phd)[1]
print("max |diff| between layouts:", (ref.float() - alt.float()).abs().max().item(), flush=True)
