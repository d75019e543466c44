#!/usr/bin/env python3
"""The SD1.5 UNet's 3×3 convolutions (CFG batch 2, 64² latents, fp16 channels-last): MIOpen (find
mode) vs the implicit-GEMM kernel (gemm_bf16_epi.hip) under its planner and under every forced
(tile, split) pair — per shape and weighted by calls per UNet pass.

    python tools/conv_probe.py            # prints one line per shape, then the weighted sums
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from k8s_nvidia_gpus_amd.ops import gemm_epi as GE  # noqa: E402

dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
ITERS = int(os.environ.get("ITERS", "30"))
B = 2 * int(os.environ.get("BATCH", "1"))

# (name, cin, cout, H (input), mode, calls per UNet pass)
SHAPES = [
    ("d0_res", 320, 320, 64, "s1", 4), ("d0_down", 320, 320, 64, "s2", 1),
    ("d1_res_in", 320, 640, 32, "s1", 1), ("d1_res", 640, 640, 32, "s1", 3), ("d1_down", 640, 640, 32, "s2", 1),
    ("d2_res_in", 640, 1280, 16, "s1", 1), ("d2_res", 1280, 1280, 16, "s1", 3), ("d2_down", 1280, 1280, 16, "s2", 1),
    ("d3_res", 1280, 1280, 8, "s1", 4), ("mid_res", 1280, 1280, 8, "s1", 4),
    ("u0_res_in", 2560, 1280, 8, "s1", 3), ("u0_res", 1280, 1280, 8, "s1", 3), ("u0_up", 1280, 1280, 8, "up2", 1),
    ("u1_res_in_a", 2560, 1280, 16, "s1", 2), ("u1_res_in_b", 1920, 1280, 16, "s1", 1),
    ("u1_res", 1280, 1280, 16, "s1", 3), ("u1_up", 1280, 1280, 16, "up2", 1),
    ("u2_res_in_a", 1920, 640, 32, "s1", 1), ("u2_res_in_b", 1280, 640, 32, "s1", 1),
    ("u2_res_in_c", 960, 640, 32, "s1", 1), ("u2_res", 640, 640, 32, "s1", 3), ("u2_up", 640, 640, 32, "up2", 1),
    ("u3_res_in_a", 960, 320, 64, "s1", 1), ("u3_res_in_b", 640, 320, 64, "s1", 2), ("u3_res", 320, 320, 64, "s1", 3),
]
MODES = {"s1": GE.CONV_S1, "s2": GE.CONV_S2, "up2": GE.CONV_UP2}


def bench(fn, iters=ITERS):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


rows = {}
tot = {}
for name, cin, cout, h, mode, calls in SHAPES:
    x = torch.randn(B, cin, h, h, device=dev).half().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 3, 3, device=dev) / (3 * cin ** 0.5)).half().contiguous(memory_format=torch.channels_last)
    b = torch.randn(cout, device=dev).half()
    wk = GE.conv_weight(w)
    m = MODES[mode]

    def miopen():
        xi = F.interpolate(x, scale_factor=2.0, mode="nearest") if mode == "up2" else x
        return F.conv2d(xi, w, b, stride=2 if mode == "s2" else 1, padding=1)

    ho = h // 2 if mode == "s2" else (2 * h if mode == "up2" else h)
    M, K = B * ho * ho, 9 * cin
    row = {"M": M, "N": cout, "K": K, "calls": calls, "plan": GE.plan(M, cout, K)}
    row["miopen_us"] = bench(miopen)
    row["auto_us"] = bench(lambda: GE.conv3x3(x, wk, b, m))
    err = (GE.conv3x3(x, wk, b, m).float() - miopen().float()).abs().max().item()
    row["max_abs_diff"] = round(err, 4)
    for t in range(4):
        GE.set_tile(t)
        for sp in (1, 2, 3, 4, 6, 8):
            if sp > 1 and K // 64 // sp < 4:
                continue
            GE.set_splits(sp)
            row[f"t{t}s{sp}_us"] = bench(lambda: GE.conv3x3(x, wk, b, m))
    GE.set_tile(-1)
    GE.set_splits(-1)
    best = min((k for k in row if k.startswith("t") and k.endswith("_us")), key=lambda k: row[k])
    row["best"] = best
    for k in [k for k in row if k.endswith("_us")]:
        row[k] = round(row[k], 1)
        tot[k] = tot.get(k, 0.0) + row[k] * calls
    tot["best_us"] = tot.get("best_us", 0.0) + row[best] * calls
    fl = 2.0 * M * cout * K
    row["auto_tflops"] = round(fl / row["auto_us"] / 1e6, 1)
    row["miopen_tflops"] = round(fl / row["miopen_us"] / 1e6, 1)
    rows[name] = row
    print(name, {k: row[k] for k in ("M", "N", "K", "plan", "miopen_us", "auto_us", "best", "max_abs_diff")},
          row[best], flush=True)
tot = {k: round(v, 1) for k, v in tot.items()}
print("weighted sums (us per UNet pass):", {k: tot[k] for k in ("miopen_us", "auto_us", "best_us")}, flush=True)
print(json.dumps({"rows": rows, "sum": tot}))
