#!/usr/bin/env python3
"""Prompt batching on one MI355X (Qwen2.5-7B Q4_K_M layout, random blocks): time
``Engine.prefill_many`` of k prompts of n tokens against k separate ``prefill`` calls and one
monolithic k*n-token prefill.  One JSON line per case."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    from k8s_nvidia_gpus_amd.models.llm import QWEN25_7B
    from k8s_nvidia_gpus_amd.models.llm.engine import Engine
    from k8s_nvidia_gpus_amd.models.llm.weights import ModelWeights

    dev = torch.device("cuda")
    w = ModelWeights.random(QWEN25_7B, device=dev, seed=0)
    eng = Engine(w, max_ctx=8192, slots=8, dense=True)
    eng.warmup(lengths=(512, 2048))
    for k, n in [(2, 512), (4, 512), (8, 256), (4, 128)]:
        ids = [[(7 * s + j) % 1000 + 10 for j in range(n)] for s in range(k)]
        sep = timed(lambda: [eng.prefill(ids[s], s) for s in range(k)])
        many = timed(lambda: eng.prefill_many([(ids[s], s, 0) for s in range(k)]))
        mono = timed(lambda: eng.prefill(sum(ids, []), 0))
        print(json.dumps({"prompts": k, "tokens": n, "separate_ms": round(sep, 2),
                          "prefill_many_ms": round(many, 2), "one_prompt_of_all_ms": round(mono, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
