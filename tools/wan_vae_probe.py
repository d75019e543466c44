#!/usr/bin/env python3
"""Wan VAE decode latency at the reference job size (13 frames 512x320) per dtype / MIOpen mode."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_nvidia_gpus_amd.models.wan.config import WanVAEConfig  # noqa: E402
from k8s_nvidia_gpus_amd.models.wan.vae import WanVAE  # noqa: E402

dev = torch.device("cuda", 0)
res = {}
z = torch.randn(1, 16, 4, 40, 64, device=dev)
for dt in (torch.bfloat16, torch.float16):
    for det in (False, True):
        if det and dt == torch.bfloat16:
            continue
        torch.manual_seed(0)
        with torch.device(dev):
            v = WanVAE(WanVAEConfig.wan21())
        v = v.to(dev, dt).eval()
        torch.backends.cudnn.deterministic = det
        outs = []
        for i in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            o = v.decode(z)
            torch.cuda.synchronize()
            outs.append(round((time.perf_counter() - t0) * 1e3, 1))
            print(str(dt), det, i, outs[-1], "ms", flush=True)
        res[f"{str(dt).split('.')[-1]}{'_det' if det else ''}"] = {"ms": outs, "finite": bool(torch.isfinite(o).all())}
torch.backends.cudnn.deterministic = False
print(json.dumps(res))
