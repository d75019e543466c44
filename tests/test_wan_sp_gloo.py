"""Wan2.1 DiT sequence parallelism (models/wan/parallel.py) across real processes on gloo: the
Ulysses all-to-all forward and a full sampling run equal the single-process results."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    from k8s_nvidia_gpus_amd.models.wan.config import WanDiTConfig
    from k8s_nvidia_gpus_amd.models.wan.dit import WanDiT
    from k8s_nvidia_gpus_amd.models.wan.parallel import SequenceParallel
    from k8s_nvidia_gpus_amd.models.wan.pipeline import ksample

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.manual_seed(0)
        cfg = WanDiTConfig(dim=256 * world // 2 if world > 2 else 256, ffn_dim=512, freq_dim=32,
                           heads=world * 2 if world > 2 else 2, layers=2, text_dim=64, text_len=32)
        m = WanDiT(cfg)
        with torch.no_grad():
            for p in m.parameters():
                p.add_(torch.randn(p.shape, generator=torch.Generator().manual_seed(1)) * 0.02)
        sp = SequenceParallel.from_env()
        x = torch.randn(2, 16, 2, 8, 12, generator=torch.Generator().manual_seed(2))
        t = torch.tensor([600.0, 600.0])
        ctx = torch.randn(2, 9, cfg.text_dim, generator=torch.Generator().manual_seed(3))
        kv = m.text_kv(m.embed_text(ctx))
        ref = m(x, t, kv)
        par = m(x, t, kv, sp=sp)
        fwd_err = (par - ref).abs().max().item()
        lat = torch.zeros(1, 16, 2, 8, 12)
        a = ksample(m, ctx[:1], ctx[1:], lat, seed=5, steps=3, cfg=4.0)
        b = ksample(m, ctx[:1], ctx[1:], lat, seed=5, steps=3, cfg=4.0, sp=sp)
        q.put((rank, fwd_err, (a - b).abs().max().item(), ref.abs().max().item()))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None, None))


@pytest.mark.parametrize("world", [2, 4])
def test_sequence_parallel_dit_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(60)
    for rank, fwd_err, samp_err, scale in res:
        assert not isinstance(fwd_err, str), fwd_err
        assert fwd_err < 1e-4 * max(1.0, scale), (rank, fwd_err)
        assert samp_err < 1e-4, (rank, samp_err)
