"""Compare the decode step's intermediate buffers for T=4 vs T=1 (eager, no graphs)."""
import math
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from k8s_nvidia_gpus_amd.models.llm import tiny
from k8s_nvidia_gpus_amd.models.llm.synthetic import write_synthetic_gguf, load

p = "/tmp/dbg.gguf"
write_synthetic_gguf(p, tiny(layers=4, dim=512, heads=4, kv_heads=2, ffn=1024))
eng, tok = load(p, device="cuda", max_ctx=512, dense=True)
eng.use_graphs = False
LK, c = eng.LK, eng.cfg
prompts = [tok.encode(s) for s in ("hello", "the quick brown fox", "a cozy cabin in", "you")]
for s, pr in enumerate(prompts):
    eng.prefill(pr, slot=s)
toks = [7, 8, 9, 10]
pos = [len(pr) for pr in prompts]

def run(T, idx):
    b = eng._buffers(T)
    host = torch.tensor([[toks[i] for i in idx], [pos[i] for i in idx], list(idx)], dtype=torch.int32)
    b.tok.copy_(host[0]); b.pos.copy_(host[1]); b.slot.copy_(host[2])
    rec = {}
    LK.dequant(eng.w.tok_embd, b.h, rows=b.tok); rec["emb"] = b.h.clone()
    qd = eng._q8(b, c.dim); qf = eng._q8(b, c.ffn)
    L = eng.w.layers[0]
    LK.rmsnorm_q8(b.h, L.attn_norm, c.eps, *qd); rec["x8a"] = qd[0].clone(); rec["dxa"] = qd[1].clone()
    off = 0
    for w in L.wqkv:
        LK.qgemv(w, *qd, b.qkv[:, off:], LK.STORE, bias=L.bqkv[off:], ldo=b.qkv.stride(0)); off += w.n
    rec["qkv"] = b.qkv.clone()
    LK.rope_kv(b.qkv, b.pos, b.slot, eng.cos, eng.sin, c.heads, c.kv_heads, c.head_dim, eng.max_ctx, b.qrot, eng.k_cache[0], eng.v_cache[0])
    rec["qrot"] = b.qrot.clone()
    LK.attn_decode(b.qrot, b.pos, b.slot, eng.k_cache[0], eng.v_cache[0], c.heads, c.kv_heads, c.head_dim, eng.max_ctx, 1/math.sqrt(128), b.po, b.pml, *qd, span=256)
    rec["attn_x8"] = qd[0].clone()
    LK.qgemv(L.wo, *qd, b.h, LK.RESID); rec["h_o"] = b.h.clone()
    LK.rmsnorm_q8(b.h, L.ffn_norm, c.eps, *qd)
    LK.qgemv(L.wg, *qd, b.t, LK.PAIR, w1=L.wu); rec["t"] = b.t.clone()
    LK.rmsnorm_q8(b.t, None, 0.0, *qf); rec["x8f"] = qf[0].clone()
    LK.qgemv(L.wd, *qf, b.h, LK.RESID); rec["h_d"] = b.h.clone()
    torch.cuda.synchronize()
    return rec

r4 = run(4, [0, 1, 2, 3])
for s in range(4):
    r1 = run(1, [s])
    for k in r4:
        a, b_ = r4[k][s].float(), r1[k][0].float()
        d = (a - b_).abs().max().item()
        print(f"slot {s} {k:8s} maxdiff {d:.3g}", flush=True)
