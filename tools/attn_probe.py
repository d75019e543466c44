#!/usr/bin/env python3
"""Flash-attention kernel sweep over query tiles per wave (QT) at the Wan2.1 / SD1.5 shapes:
time per call, TFLOPS, and max error against PyTorch SDPA (fp32 math)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from k8s_nvidia_gpus_amd.ops import sd_kernels as SK  # noqa: E402

dev = torch.device("cuda", 0)
ONLY = os.environ.get("ATTN_ONLY")          # e.g. wan_self (PMC passes)
QTS = [int(x) for x in os.environ.get("ATTN_QTS", "").split(",") if x]
VARIANTS = [int(x) for x in os.environ.get("ATTN_VARIANTS", "0,2").split(",") if x]
SHAPES = {  # name: (N, heads, Lq, Lk, d)
    "wan_self": (2, 12, 2560, 2560, 128),
    "wan_cross": (2, 12, 2560, 512, 128),
    "wan_long": (2, 12, 32760, 32760, 128),
    "sd_64x64": (2, 8, 4096, 4096, 40),
    "sd_32x32": (2, 8, 1024, 1024, 80),
    "sd_16x16": (2, 8, 256, 256, 160),
}
res = {}
for name, (n, h, lq, lk, d) in SHAPES.items():
    if ONLY and name != ONLY:
        continue
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(n, lq, h * d, generator=g, device=dev).bfloat16()
    k = torch.randn(n, lk, h * d, generator=g, device=dev).bfloat16()
    v = torch.randn(n, lk, h * d, generator=g, device=dev).bfloat16()
    ref = None
    if lq * lk <= 2560 * 4096:     # the fp32 reference of the 32 760-token case would need ~100 GB
        ref = F.scaled_dot_product_attention(*(t.float().view(n, -1, h, d).transpose(1, 2) for t in (q, k, v)))
        ref = ref.transpose(1, 2).reshape(n, lq, h * d)
    flops = 4.0 * n * h * lq * lk * d
    res[name] = {}
    combos = []
    for vv in VARIANTS:
        if vv == 2:
            combos += [(2, nw) for nw in (4, 8)]
        else:
            combos += [(vv, qq) for qq in (QTS or ((1, 2, 4) if d == 128 else (1, 2)))]
    for var, qt in combos:
        SK.attention_set_variant(var)
        if var == 2:
            SK.attention_d128_set_nw(qt)
        else:
            SK.attention_set_qt(qt)
        o = SK.attention(q, k, v, h, d ** -0.5)
        err = (o.float() - ref).abs().max().item() if ref is not None else float("nan")
        for _ in range(3):
            SK.attention(q, k, v, h, d ** -0.5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        it = 50 if lq < 10000 else 5
        for _ in range(it):
            SK.attention(q, k, v, h, d ** -0.5)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) * 1e6 / it
        key = f"v{var}_qt{qt}"
        res[name][key] = {"us": round(us, 1), "tflops": round(flops / us / 1e6, 1), "max_err": round(err, 4)}
        print(name, key, res[name][key], flush=True)
    SK.attention_set_qt(0)
    SK.attention_set_variant(-1)
    SK.attention_d128_set_nw(0)
    o = SK.attention(q, k, v, h, d ** -0.5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it = 50 if lq < 10000 else 5
    for _ in range(it):
        SK.attention(q, k, v, h, d ** -0.5)
    torch.cuda.synchronize()
    res[name]["heuristic_us"] = round((time.perf_counter() - t0) * 1e6 / it, 1)
print(json.dumps(res))
