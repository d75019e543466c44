#!/usr/bin/env python3
"""Same-process A/B of two prompt-attention launch plans per case (ops/csrc/llm_prefill_attn.hip),
Qwen2.5-7B layout, alternating 3 times.  Usage: prefill_attn_plan_ab.py P:start:nw:ks:ns ..."""
from __future__ import annotations

import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from tools.debug.prefill_attn_sweep import timed  # noqa: E402


def main(argv):
    from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

    dev = torch.device("cuda")
    H, Hkv, d = 28, 4, 128
    for spec in argv:
        P, start, nw, ks, ns = (int(x) for x in spec.split(":"))
        end = start + P
        q = torch.randn(H, P, d, device=dev, dtype=torch.float16)
        k = torch.randn(Hkv, end, d, device=dev, dtype=torch.float16)
        v = torch.randn(Hkv, end, d, device=dev, dtype=torch.float16)
        out = torch.empty(H, P, d, device=dev, dtype=torch.float16)
        auto = LK.prefill_attn_plan(P, start, H, Hkv)
        res = {"auto": [], "other": []}
        for _ in range(3):
            res["auto"].append(timed(lambda: LK.prefill_attn(q, k, v, out, start, 1 / math.sqrt(d)), 50))
            res["other"].append(timed(lambda: LK.prefill_attn(q, k, v, out, start, 1 / math.sqrt(d),
                                                               nsplit=ns, nw=nw, ks=ks), 50))
        print(json.dumps({"P": P, "start": start, "auto": auto,
                          "auto_us": [round(x, 1) for x in res["auto"]],
                          "other": {"waves": nw, "key_slots": ks, "nsplit": ns},
                          "other_us": [round(x, 1) for x in res["other"]]}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
