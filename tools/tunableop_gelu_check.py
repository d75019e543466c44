import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from k8s_nvidia_gpus_amd.models.wan import functional as WF
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(5120, 1536, generator=g, device=dev).bfloat16()
w = (torch.randn(8960, 1536, generator=g, device=dev) * 0.03).bfloat16()
b = (torch.randn(8960, generator=g, device=dev) * 0.5).bfloat16()
ref = torch.nn.functional.gelu(x.float() @ w.float().t() + b.float(), approximate="tanh")
for i in range(3):
    y = WF.linear_gelu(x, w, b)
print("tunableop", os.environ.get("PYTORCH_TUNABLEOP_ENABLED"), "max|y-ref|", (y.float() - ref).abs().max().item(),
      "min(y)", y.float().min().item())
