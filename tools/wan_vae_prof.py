#!/usr/bin/env python3
"""Warm Wan VAE decode (13 frames 512x320) for rocprofv3 --stats: one untimed call (MIOpen kernel
compilation), then 3 decodes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_nvidia_gpus_amd.models.wan.config import WanVAEConfig  # noqa: E402
from k8s_nvidia_gpus_amd.models.wan.vae import WanVAE  # noqa: E402

dev = torch.device("cuda", 0)
if os.environ.get("VAE_BENCHMARK") == "1":
    torch.backends.cudnn.benchmark = True      # MIOpen find (exhaustive solver search) per shape
with torch.device(dev):
    v = WanVAE(WanVAEConfig.wan21())
v = v.to(dev, torch.bfloat16).eval()
z = torch.randn(1, 16, 4, 40, 64, device=dev)
t0 = time.perf_counter()
v.decode(z)
torch.cuda.synchronize()
print(f"first decode (kernel compile / solver search): {time.perf_counter() - t0:.1f} s", flush=True)
for i in range(3):
    t0 = time.perf_counter()
    v.decode(z)
    torch.cuda.synchronize()
    print(f"decode {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
