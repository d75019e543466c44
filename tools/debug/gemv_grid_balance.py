#!/usr/bin/env python3
"""Does the pair GEMV (gate|up, T = 1) lose bandwidth to an uneven grid?  Times the default MFMA
launch for N = 16384 (512 workgroups of 32 rows: 2 per CU), 18944 (592, Qwen2.5-7B) and others,
cycling over 8 random Q4_K pairs so the weights stream from HBM (8 x 2 x N x 3584 x 144/256 B
exceeds the 256 MB Infinity Cache).  One JSON line per N."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def main(argv):
    from k8s_nvidia_gpus_amd.models.llm import gguf
    from k8s_nvidia_gpus_amd.models.llm.weights import QWeight
    from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

    dev = torch.device("cuda")
    K = 3584
    ns = [int(x) for x in argv] or [8192, 16384, 18944, 20480, 24576]
    per, size = gguf.BLOCK[gguf.Q4_K]
    for N in ns:
        mats = []
        for i in range(8):
            pair = []
            for _ in range(2):
                raw = torch.randint(0, 256, (N, K // 256 * size), dtype=torch.uint8, device=dev)
                w = QWeight.from_device_raw(raw, gguf.Q4_K)
                assert w.mfma_pack()
                pair.append(w)
            mats.append(pair)
        x8 = torch.randint(-127, 127, (1, K), dtype=torch.int8, device=dev)
        dx = torch.full((1, K // 32), 0.01, device=dev)
        sx = torch.zeros(1, K // 16, device=dev)
        out = torch.zeros(1, N, device=dev)

        def launch(i):
            g, u = mats[i % len(mats)]
            LK.qgemv(g, x8, dx, sx, out, LK.PAIR, w1=u)

        for i in range(8):
            launch(i)
        torch.cuda.synchronize()
        iters = 80
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for i in range(iters):
            launch(i)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / iters * 1e3
        nbytes = 2 * mats[0][0].nbytes()
        print(json.dumps({"N": N, "workgroups": N // 32, "us": round(us, 2),
                          "GBps": round(nbytes / us / 1e3, 1)}), flush=True)
        del mats
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main(sys.argv[1:])
