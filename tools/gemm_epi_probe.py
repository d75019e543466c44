#!/usr/bin/env python3
"""Fused-epilogue GEMMs (gemm_bf16_epi.hip wave-grid family, w4a epilogues) vs hipBLASLt (torch).

MODE=wan (default): the Wan2.1 DiT projection shapes — time per call, TFLOPS, and the gated-residual
epilogue against GEMM + separate update.  MODE=sd: the SD1.5 UNet's fp16 projections at a CFG batch
of 64² latents — the auto-picked path, every forced block tile, and torch."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from k8s_nvidia_gpus_amd.ops import gemm_epi as GE  # noqa: E402
from k8s_nvidia_gpus_amd.ops import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
ITERS = int(os.environ.get("ITERS", "50"))


def bench(fn, iters=ITERS):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


res = {}
if os.environ.get("MODE", "wan") == "sd":
    lat = int(os.environ.get("LATENT", "64"))
    rows = {}
    for lvl, c in enumerate((320, 640, 1280, 1280)):
        m = 2 * (lat >> lvl) ** 2
        for name, n, k in [("proj", c, c), ("qkv", 3 * c, c), ("geglu", 8 * c, c), ("ff_out", c, 4 * c)]:
            x = torch.randn(m, k, device=dev).half()
            w = (torch.randn(n, k, device=dev) / k ** 0.5).half()
            b = torch.randn(n, device=dev).half()
            fl = 2.0 * m * n * k
            row = {"m": m, "n": n, "k": k, "auto_plan": GE.plan(m, n, k),
                   "w4a": GE.use_w4a(m, n, k, torch.float16)}
            row["auto_us"] = bench(lambda: GE.linear(x, w, b))
            out = torch.empty(m, n, device=dev).half()
            for t in range(4):
                GE.set_tile(t)
                row[f"tile{t}_us"] = bench(lambda: GE._run(GE.EPI_STORE, x, w, b, out,
                                                           None, None, 0, 0, n, 0))
            GE.set_tile(-1)
            row["torch_us"] = bench(lambda: F.linear(x, w, b))
            for key in [k2 for k2 in row if k2.endswith("_us")]:
                row[key] = round(row[key], 1)
            row["auto_tflops"] = round(fl / row["auto_us"] / 1e6, 1)
            rows[f"L{lvl}_{name}"] = row
            print(f"L{lvl}_{name}", row, flush=True)
    tot = {k2: round(sum(r[k2] for r in rows.values()), 1)
           for k2 in ("auto_us", "torch_us", "tile0_us", "tile1_us", "tile2_us", "tile3_us")}
    tot["best_forced_us"] = round(sum(min(r[f"tile{t}_us"] for t in range(4)) for r in rows.values()), 1)
    print("sum", tot, flush=True)
    print(json.dumps({"rows": rows, "sum": tot}))
    sys.exit(0)
for tokens in [int(t) for t in os.environ.get("TOKENS", "2560,32768").split(",")]:
    M = 2 * tokens
    for name, n, k in [("qkv", 4608, 1536), ("o", 1536, 1536), ("ffn0", 8960, 1536), ("ffn2", 1536, 8960)]:
        x = torch.randn(M, k, device=dev).bfloat16()
        w = (torch.randn(n, k, device=dev) / k ** 0.5).bfloat16()
        b = torch.randn(n, device=dev).bfloat16()
        fl = 2.0 * M * n * k
        row = {}
        if name == "ffn0":
            row["ours_us"] = bench(lambda: GE.linear_gelu(x, w, b))
            row["torch_us"] = bench(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True))
        elif name in ("o", "ffn2"):
            r = torch.randn(2, tokens, n, device=dev)
            g = torch.randn(2, n, device=dev)
            x3 = x.view(2, tokens, k)
            row["ours_us"] = bench(lambda: GE.linear_residual_(r, x3, w, b, g))
            row["torch_us"] = bench(lambda: r.add_(F.linear(x3, w, b) * g[:, None, :]))
            row["ours_store_us"] = bench(lambda: GE.linear(x, w, b))
            row["torch_gemm_us"] = bench(lambda: F.linear(x, w, b))
        else:
            row["ours_us"] = bench(lambda: GE.linear(x, w, b))
            row["torch_us"] = bench(lambda: F.linear(x, w, b))
        if M % 256 == 0 and n % 256 == 0:          # the validator's 256x256 w4a kernel, plain store
            row["w4a_us"] = bench(lambda: K.gemm_bf16_nt(x, w))
        # the wave-grid kernel's 256x128 tile (8 waves of 64x64) on every shape
        out = torch.empty(M, n, device=dev).bfloat16()
        for t in (0,):
            GE.set_tile(t)
            if name in ("o", "ffn2"):
                r2 = torch.randn(2, tokens, n, device=dev)
                g2 = torch.randn(2, n, device=dev)
                row[f"resid_t{t}_us"] = bench(lambda: GE._run(GE.EPI_RESID, x, w, b, None, r2.view(-1, n),
                                                              g2, tokens, n, 0, n))
            else:
                epi = GE.EPI_GELU if name == "ffn0" else GE.EPI_STORE
                row[f"epi_t{t}_us"] = bench(lambda: GE._run(epi, x, w, b, out, None, None, 0, 0, n, 0))
        GE.set_tile(-1)
        for key in list(row):
            row[key] = round(row[key], 1)
        row["ours_tflops"] = round(fl / row["ours_us"] / 1e6, 1)
        if "w4a_us" in row:
            row["w4a_tflops"] = round(fl / row["w4a_us"] / 1e6, 1)
        row["torch_tflops"] = round(fl / row["torch_us"] / 1e6, 1)
        res[f"{tokens}_{name}"] = row
        print(tokens, name, row, flush=True)
print(json.dumps(res))
