"""RCCL-over-xGMI collectives for the multi-GPU validator / benchmark pods (BASELINE config 4).

The reference has no collective call sites at all; its only multi-GPU artefacts
are two independent single-GPU pods (reference README.md:301-349) and a "one pod, two GPUs — TBD"
(README.md:389-391).  This module is the MI355X answer: one process per GPU, ``torch.distributed``
with backend ``nccl`` (= RCCL on ROCm) over the node's xGMI mesh, measuring the collectives a
data/tensor/expert-parallel job would run, nccl-tests style:

    op              algbw = bytes / t      busbw factor (what a ring moves per rank per link)
    all_reduce      S / t                  2(n−1)/n
    all_gather      S·n / t (S per rank)   (n−1)/n
    reduce_scatter  S / t  (S in total)    (n−1)/n
    all_to_all      S / t                  (n−1)/n

Every measurement is preceded by an exact correctness pass (rank r contributes r+1, or a rank/index
pattern for gather/scatter/all-to-all), and the reported time is the MAX over ranks (the slowest
rank bounds the collective).  On CPU the same code runs on ``gloo`` (tests use world_size 2).

xGMI budget: each MI355X has 7 links to its 7 peers (full mesh, ≈76 GB/s per direction per link
from the KFD io_links); a single ring uses one outgoing link per GPU, so busbw beyond one link's
rate means RCCL is spreading channels over several rings — report what is measured.
"""
from __future__ import annotations

import os
import time
from dataclasses import asdict, dataclass
from typing import Dict, Iterable, List, Optional

import torch
import torch.distributed as dist

BUSBW_FACTOR = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_to_all": lambda n: (n - 1) / n,
    "broadcast": lambda n: 1.0,
}


@dataclass
class CollectiveResult:
    op: str
    bytes: int
    dtype: str
    world: int
    time_us: float
    algbw_gbps: float
    busbw_gbps: float
    wrong: int

    def as_dict(self) -> dict:
        return asdict(self)


def env_rank() -> tuple:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0) -> torch.device:
    """Initialise the default process group from torchrun env vars; return this rank's device.

    backend None → ``nccl`` (RCCL) when a GPU is visible, else ``gloo``.  The device is bound to the
    process group (``device_id``) so RCCL creates its communicator eagerly on the right GPU.
    """
    import datetime

    rank, world, local = env_rank()
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    backend = backend or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if not dist.is_initialized():
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device
        if "MASTER_ADDR" not in os.environ:
            os.environ["MASTER_ADDR"] = "127.0.0.1"
            os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group(rank=rank, world_size=world, **kw)
    return device


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def _max_over_ranks(x: float, device: torch.device, group=None) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def _check_and_prepare(op: str, nbytes: int, dtype: torch.dtype, device, rank: int, world: int,
                       group=None):
    """Build input/output buffers, run the op once, count wrong elements exactly."""
    esize = torch.tensor([], dtype=dtype).element_size()
    count = max(world, nbytes // esize)
    count -= count % world  # scatter-type ops need divisibility
    if op == "all_reduce":
        x = torch.full((count,), float(rank + 1), dtype=dtype, device=device)
        dist.all_reduce(x, group=group)
        expect = world * (world + 1) / 2
        wrong = int((x != expect).sum().item())
        return (lambda: dist.all_reduce(x, group=group)), wrong, count * esize
    if op == "all_gather":
        per = count // world
        x = torch.full((per,), float(rank + 1), dtype=dtype, device=device)
        out = torch.empty((per * world,), dtype=dtype, device=device)
        dist.all_gather_into_tensor(out, x, group=group)
        expect = torch.arange(1, world + 1, dtype=dtype, device=device).repeat_interleave(per)
        wrong = int((out != expect).sum().item())
        return (lambda: dist.all_gather_into_tensor(out, x, group=group)), wrong, per * world * esize
    if op == "reduce_scatter":
        per = count // world
        x = torch.full((per * world,), float(rank + 1), dtype=dtype, device=device)
        out = torch.empty((per,), dtype=dtype, device=device)
        dist.reduce_scatter_tensor(out, x, group=group)
        wrong = int((out != world * (world + 1) / 2).sum().item())
        return (lambda: dist.reduce_scatter_tensor(out, x, group=group)), wrong, per * world * esize
    if op == "all_to_all":
        per = count // world
        # chunk j of rank r carries the value r*world + j; after the exchange chunk j of rank r
        # must carry j*world + r
        x = (torch.arange(world, device=device, dtype=torch.float32) + rank * world).to(dtype)
        x = x.repeat_interleave(per)
        out = torch.empty_like(x)
        dist.all_to_all_single(out, x, group=group)
        expect = (torch.arange(world, device=device, dtype=torch.float32) * world + rank).to(dtype)
        wrong = int((out != expect.repeat_interleave(per)).sum().item())
        return (lambda: dist.all_to_all_single(out, x, group=group)), wrong, per * world * esize
    if op == "broadcast":
        x = torch.full((count,), float(rank + 1), dtype=dtype, device=device)
        dist.broadcast(x, src=0, group=group)
        wrong = int((x != 1).sum().item())
        return (lambda: dist.broadcast(x, src=0, group=group)), wrong, count * esize
    raise ValueError(f"unknown collective {op!r}")


def measure(op: str, nbytes: int, dtype: torch.dtype = torch.float32, iters: int = 20,
            warmup: int = 5, device: Optional[torch.device] = None, group=None) -> CollectiveResult:
    """One collective's time (MAX over ranks) and correctness; ``group``: the process group to
    run it on (default: the default group)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    device = device or (torch.device("cuda", torch.cuda.current_device())
                        if torch.cuda.is_available() and dist.get_backend(group) == "nccl"
                        else torch.device("cpu"))
    fn, wrong, size = _check_and_prepare(op, nbytes, dtype, device, rank, world, group)
    wrong = int(_max_over_ranks(float(wrong), device, group))
    for _ in range(warmup):
        fn()
    _sync(device)
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync(device)
    dt = (time.perf_counter() - t0) / iters
    dt = _max_over_ranks(dt, device, group)
    algbw = size / dt / 1e9
    return CollectiveResult(op, size, str(dtype).replace("torch.", ""), world, dt * 1e6, algbw,
                            algbw * BUSBW_FACTOR[op](world) if world > 1 else algbw, wrong)


def sweep(op: str, min_bytes: int, max_bytes: int, factor: int = 4, **kw) -> List[CollectiveResult]:
    out = []
    b = min_bytes
    while b <= max_bytes:
        out.append(measure(op, b, **kw))
        b *= factor
    return out


def format_table(rows: Iterable[CollectiveResult]) -> str:
    lines = [f"# {'op':>14s} {'size(B)':>12s} {'dtype':>8s} {'time(us)':>10s} {'algbw(GB/s)':>12s} "
             f"{'busbw(GB/s)':>12s} {'#wrong':>7s}"]
    for r in rows:
        lines.append(f"  {r.op:>14s} {r.bytes:12d} {r.dtype:>8s} {r.time_us:10.1f} {r.algbw_gbps:12.2f} "
                     f"{r.busbw_gbps:12.2f} {r.wrong:7d}")
    return "\n".join(lines)


class GradientBucketer:
    """Flatten many tensors into ~``bucket_bytes`` buckets and all-reduce them asynchronously.

    The DP-communication pattern (bucketed all-reduce overlapped with compute) at the granularity
    xGMI likes: RCCL reaches its bus bandwidth only for messages of tens of MiB (per-link bound
    rings), so gradients are packed into 64 MiB buckets by default rather than reduced one tensor at
    a time.  ``start()`` launches every bucket with ``async_op=True`` and returns immediately;
    ``wait()`` completes them and scatters the averaged values back into the original tensors.
    """

    def __init__(self, tensors: List[torch.Tensor], bucket_bytes: int = 64 << 20, average: bool = True):
        self.tensors = tensors
        self.average = average
        self.buckets: List[List[int]] = []
        cur, cur_bytes = [], 0
        for i, t in enumerate(tensors):
            nb = t.numel() * t.element_size()
            if cur and (cur_bytes + nb > bucket_bytes or t.dtype != tensors[cur[0]].dtype):
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(i)
            cur_bytes += nb
        if cur:
            self.buckets.append(cur)
        self._flat: List[torch.Tensor] = []
        self._work = []

    def start(self) -> None:
        self._flat, self._work = [], []
        for b in self.buckets:
            flat = torch.cat([self.tensors[i].reshape(-1) for i in b])
            self._flat.append(flat)
            self._work.append(dist.all_reduce(flat, async_op=True))

    def wait(self) -> None:
        world = dist.get_world_size()
        for b, flat, w in zip(self.buckets, self._flat, self._work):
            w.wait()
            if self.average:
                flat /= world
            off = 0
            for i in b:
                t = self.tensors[i]
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n
        self._flat, self._work = [], []


def results_json(rows: List[CollectiveResult]) -> Dict:
    best = max(rows, key=lambda r: r.busbw_gbps) if rows else None
    return {"check": f"torch_{rows[0].op}" if rows else "torch_collective",
            "world": rows[0].world if rows else 0,
            "peak_busbw_gbps": round(best.busbw_gbps, 2) if best else None,
            "peak_bytes": best.bytes if best else None,
            "wrong": sum(r.wrong for r in rows),
            "passed": bool(rows) and all(r.wrong == 0 for r in rows),
            "rows": [r.as_dict() for r in rows]}
