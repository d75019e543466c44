#!/usr/bin/env python3
"""Run torch.matmul (hipBLASLt) on the validator shapes so rocprofv3 records its kernel names."""
import torch

dev = torch.device("cuda", 0)
for s in (4096, 8192):
    a = (torch.rand((s, s), device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand((s, s), device=dev) * 2 - 1).to(torch.bfloat16)
    for _ in range(5):
        c = torch.matmul(a, b.t())
torch.cuda.synchronize()
print("ok")
