#!/usr/bin/env python3
"""The LLM prompt-prefill GEMMs (Qwen2.5-7B layout, fp16, M = prompt tokens): every path of
ops/gemm_epi.py against hipBLASLt (torch) — the planner's pick, the 256x256 w4a kernel, the
wave-grid family with each block tile and split-K factor.

    python tools/llm_prefill_gemm_probe.py [--m 512] [--out probe.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from k8s_nvidia_gpus_amd.ops import gemm_epi as GE  # noqa: E402

SHAPES = (("qkv", 4608, 3584, "store"), ("o", 3584, 3584, "resid"),
          ("gate_up", 37888, 3584, "store"), ("down", 3584, 18944, "resid"))


def bench(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--quick", action="store_true", help="planner / w4a / torch only (no sweep)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="", help="comma-separated GEMM names (qkv,o,gate_up,down)")
    ap.add_argument("--splitk-sweep", action="store_true",
                    help="time the split-K w4a form at every slice count 2..8")
    ap.add_argument("--cold", action="store_true",
                    help="cycle through weight copies totalling > 512 MB, so every call streams its "
                         "weights from HBM as in a prefill (not from the Infinity Cache)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows = []
    for name, n, k, kind in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        m = a.m
        x = torch.randn(m, k, device=dev, dtype=torch.float16)
        copies = max(1, -(-(512 << 20) // (n * k * 2))) if a.cold else 1
        ws = [torch.randn(n, k, device=dev, dtype=torch.float16) / k ** 0.5 for _ in range(copies)]
        w = ws[0]
        res = torch.zeros(m, n, device=dev)
        flop = 2.0 * m * n * k
        it = [0]

        def run():
            wi = ws[it[0] % copies]
            it[0] += 1
            return GE.linear(x, wi) if kind == "store" else GE.linear_residual_(res, x, wi)

        def rec(variant, us):
            r = {"gemm": name, "m": m, "n": n, "k": k, "variant": variant, "us": round(us, 1),
                 "tflops": round(flop / us / 1e6, 1)}
            rows.append(r)
            print(r, flush=True)

        rec(f"auto plan={GE.plan(m, n, k)} w4a={GE.use_w4a(m, n, k, x.dtype)} "
            f"hybrid={GE.hybrid_plan(m, n, k)} splitk={GE.splitk_plan(m, n, k)}"
            f"{' cold' if a.cold else ''}", bench(run))
        if GE.use_w4a(m, n, k, x.dtype):
            GE._HYBRID = False
            rec("w4a plain (no partial-wave split)", bench(run))
            GE._HYBRID = True
        if GE.splitk_plan(m, n, k) > 1 and a.splitk_sweep:
            for ks in (2, 3, 4, 5, 6, 7, 8):
                GE.set_w4a_splitk(ks)
                rec(f"split-K w4a ks={GE.splitk_plan(m, n, k)}", bench(run))
            GE.set_w4a_splitk(0)
        if GE.splitk_plan(m, n, k) > 1:
            GE._W4A_SPLITK = False
            rec(f"wave-grid plan={GE.plan(m, n, k)} (split-K w4a off)", bench(run))
            GE._W4A_SPLITK = True

        def tl():
            wi = ws[it[0] % copies]
            it[0] += 1
            return F.linear(x, wi)
        rec("torch", bench(tl))
        if a.quick:
            continue
        wide = GE._WIDE
        GE._WIDE = "epi"
        for tile in range(len(GE.TILES)):
            for sp in (1, 2, 3, 4, 6, 8):
                GE.set_tile(tile)
                GE.set_splits(sp)
                try:
                    rec(f"epi tile={GE.TILES[tile]} splits={sp}", bench(run))
                except RuntimeError as e:
                    print(f"{name} tile {tile} splits {sp}: {e}", flush=True)
        GE.set_tile(-1)
        GE.set_splits(-1)
        GE._WIDE = wide
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
