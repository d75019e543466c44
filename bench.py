#!/usr/bin/env python3
"""Headline benchmark: validator-pod bf16 GEMM TFLOPS on 1/2/4/8 MI355X (+ time-to-first-GPU-result).

BASELINE.json names the metric "validator-pod bf16 GEMM TFLOPS/GPU + time-to-first-GPU-pod,
1/2/4/8 MI355X".  One *step* is what the operator's validator pod runs on each GPU it was
allocated: one 8192×8192×8192 bf16 GEMM (C = A·Bᵀ, fp32 accumulate, bf16 out) through the
hand-written gfx950 MFMA kernels (k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950*.hip; default
w4a, whose K-loop is generated assembly), on random [-1,1) operands (synthetic data).  Work per GPU is fixed as
N grows → weak scaling.

Launch contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 under
``torch.distributed.run`` with one rank per GPU (RCCL backend).  A plain ``python bench.py --gpus N``
(N > 1, no WORLD_SIZE) starts that torchrun itself as a child process after counting GPU agents in
the KFD sysfs topology (fewer than N → exit 2), so it can never report a 1-GPU number for N; under
torchrun, WORLD_SIZE != --gpus is an error, and the JSON carries every rank's PCI BDF (checked
distinct) and the process group's own world size.  The ranks synchronise the timed windows over a
host (gloo) group and create the RCCL group after them, for the all-reduce sweep: an initialised
RCCL communicator slowed the GEMM 3-5 % (see main()).  W untimed steps, then exactly K
timed steps bracketed by barrier + synchronize on both sides; the MAX elapsed over ranks is used;
rank 0 prints ONE JSON line.  Before the W warmup steps each rank runs the GEMM back-to-back for
``--settle-ms`` (default 250 ms, untimed) so that the timed window measures sustained throughput
rather than the chip's power-management transient after a load step (see :func:`settle`).
``value`` is the whole-job aggregate TFLOPS over all N GPUs.

Outside the timed region it also reports:
* ``time_to_first_gpu_result_s`` — process start → first verified GPU result (HIP vectorAdd,
  reference protocol), the in-process part of the "time-to-first-GPU-pod" metric (mostly
  ``import torch``); ``time_to_first_gpu_result_native_s`` — the same check as the validator pod
  runs it (native ``amd-vectoradd``, a child process started before torch loads, this rank's GPU);
* ``numerics_max_rel_err`` — sampled error of the timed kernel against an fp32 on-device reference;
* ``allreduce_busbw_gbps`` — peak RCCL all-reduce bus bandwidth over xGMI across the N ranks, from
  ``allreduce_sweep`` (1 MiB … 1 GiB, ×4; N > 1);
* ``telemetry_per_rank`` — each rank's gfx clock (mean / min), socket power and hotspot temperature
  sampled through amd-smi during the timed window, so a flat weak-scaling curve can be told apart
  into a power-capped clock vs a slow rank from one run (parallel/telemetry.py);
* ``fp8_tflops`` — the validator's second precision: the same GEMM shape in OCP fp8 e4m3 through
  the hand-written ``v_mfma_scale_f32_16x16x128_f8f6f4`` kernel, whole-job aggregate, timed the
  same way (extra field; the headline ``value`` stays bf16).

``--cpu-smoke`` exercises the same launch/timing/JSON path on CPU (fp32 torch.matmul, gloo) for
tests; its numbers are not measurements and are labelled as such.
"""
from __future__ import annotations

import time

_T_PROCESS_START = time.time()

import argparse  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402


def native_first_gpu_result():
    """The validator pod's own first GPU result: seconds for ``native/bin/amd-vectoradd`` (reference
    protocol, 50 000 fp32) to print ``Test PASSED`` on this rank's GPU, as a child process started
    before this process imports torch or touches a GPU. None when the binary is not built."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "bin", "amd-vectoradd")
    if "--cpu-smoke" in sys.argv or not os.access(exe, os.X_OK):
        return None
    local = int(os.environ.get("LOCAL_RANK", "0"))
    visible = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    ids = [d for d in visible.split(",") if d.strip()] if visible else []
    env = dict(os.environ, HIP_VISIBLE_DEVICES=ids[local] if local < len(ids) else str(local))
    env.pop("CUDA_VISIBLE_DEVICES", None)
    t0 = time.time()
    try:
        out = subprocess.run([exe], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                             text=True, timeout=120).stdout
    except (OSError, subprocess.TimeoutExpired):
        return None
    return round(time.time() - t0, 3) if "Test PASSED" in out else None


def _peek_args(argv):
    """(--gpus, --launcher, --cpu-smoke) from argv without argparse's exit-on-error (the full
    parser runs later, in the ranks)."""
    gpus, launcher = 1, "auto"
    for i, a in enumerate(argv):
        for flag in ("--gpus", "--launcher"):
            val = None
            if a == flag and i + 1 < len(argv):
                val = argv[i + 1]
            elif a.startswith(flag + "="):
                val = a.split("=", 1)[1]
            if val is None:
                continue
            if flag == "--gpus":
                try:
                    gpus = int(val)
                except ValueError:
                    pass
            else:
                launcher = val
    return gpus, launcher, "--cpu-smoke" in argv


def visible_gpu_agents(root=None):
    """GPU agents this process could open, from the KFD sysfs topology (never a HIP call: the
    launcher parent must not initialise the GPU before it starts the ranks).  A
    HIP/ROCR/CUDA_VISIBLE_DEVICES list narrows the count.  Returns (count, detail)."""
    from k8s_nvidia_gpus_amd.utils.topology import read_topology

    root = root or os.environ.get("AMDK8S_SYSFS_ROOT", "/")
    topo = read_topology(root)
    n = len(topo.gpus)
    detail = f"{n} GPU agent(s) in {os.path.join(root, 'sys/class/kfd/kfd/topology')}"
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:       # unset or empty: no narrowing (an empty list would fail loudly in the ranks)
            ids = [d for d in v.split(",") if d.strip()]
            if len(ids) < n:
                n = len(ids)
                detail += f", {var}={v!r} leaves {n}"
    return n, detail


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(argv, nproc: int, smoke: bool) -> int:
    """``python bench.py --gpus N`` (N > 1, no WORLD_SIZE): start one rank per GPU under
    ``torch.distributed.run`` as a CHILD process (never an exec: see the launch rules) and relay its
    stdout — rank 0's one JSON line — and its exit code.  Refuses (exit 2) when fewer than N GPU
    agents are visible instead of silently measuring fewer GPUs.  This process imports neither
    torch nor HIP."""
    if not smoke or os.environ.get("AMDK8S_SYSFS_ROOT"):
        try:
            have, detail = visible_gpu_agents()
        except (OSError, FileNotFoundError) as e:
            print(f"bench.py: --gpus {nproc}: cannot count GPU agents ({e})", file=sys.stderr)
            return 2
        if have < nproc:
            print(f"bench.py: --gpus {nproc} but only {detail}; refusing to measure fewer GPUs",
                  file=sys.stderr)
            return 2
    rest = []
    skip = False
    for i, a in enumerate(argv):       # the ranks must not try to launch again
        if skip:
            skip = False
            continue
        if a == "--launcher":
            skip = True
            continue
        if a.startswith("--launcher="):
            continue
        rest.append(a)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + rest
    env = dict(os.environ, AMDK8S_BENCH_LAUNCHER="torchrun (spawned by bench.py)")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"bench.py: launching {nproc} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in proc.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return proc.wait()


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ:
    _gpus, _launcher, _smoke = _peek_args(sys.argv[1:])
    if _launcher not in ("auto", "torchrun", "none"):
        print(f"bench.py: --launcher must be auto|torchrun|none, not {_launcher!r}", file=sys.stderr)
        sys.exit(2)
    if _gpus > 1 and _launcher == "none":
        print(f"bench.py: --gpus {_gpus} needs one rank per GPU; run it under torch.distributed.run "
              "or drop --launcher none", file=sys.stderr)
        sys.exit(2)
    if _gpus > 1 or _launcher == "torchrun":
        sys.exit(self_launch(sys.argv[1:], _gpus, _smoke))

_NATIVE_TTFR = native_first_gpu_result()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "validator-pod bf16 GEMM TFLOPS/GPU + time-to-first-GPU-pod, 1/2/4/8 MI355X"
BASELINE_VALUE = None  # BASELINE.json "published": {} — the reference publishes no numbers


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="untimed back-to-back GEMMs before the warmup steps, until the chip's clock "
                         "has left its load-step transient (see settle())")
    ap.add_argument("--size", type=int, default=8192, help="M = N = K of the validator GEMM")
    ap.add_argument("--variant", default=None, help="GEMM variant (auto | w8 | w4)")
    ap.add_argument("--allreduce-mib", type=int, default=1024,
                    help="largest message of the post-run RCCL all-reduce sweep (1 MiB .. this, x4; N > 1)")
    ap.add_argument("--no-telemetry", action="store_true", help="no amd-smi sampling")
    ap.add_argument("--no-allreduce", action="store_true")
    ap.add_argument("--no-fp8", action="store_true", help="skip the fp8 GEMM extra measurement")
    ap.add_argument("--launcher", choices=("auto", "torchrun", "none"), default="auto",
                    help="auto: a plain run with --gpus N > 1 starts N ranks under "
                         "torch.distributed.run itself; torchrun: do so even for N = 1")
    ap.add_argument("--cpu-smoke", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def settle(step, sync, settle_ms: float, chunk: int = 8, max_launches: int = 4000) -> int:
    """Run ``step`` back-to-back (untimed) for at least ``settle_ms`` of GPU time; return launches.

    MI355X answers a load step with a power-management transient: in back-to-back 8192³ bf16
    GEMMs the first 2 launches run at ~680 us, launches 4-6 at ~900 us, and the chip takes ~40
    launches (~30 ms) to come back to its sustained ~663 us (1655 TFLOPS, flat over 2.6 s / 4000
    launches; profiles/r01_session5/gemm_settle_probe_4000.txt).  A short timed window that starts
    inside the transient measures the DVFS controller, not the kernel: K=20/W=5 read 1463 TFLOPS,
    K=50/W=10 1595, K=200/W=50 1669 on the same box (bench_kw_sweep_before_settle.txt).  The
    validator's number is *sustained* throughput, so every timed window starts after this phase.
    Nothing is skipped inside the timed region: it still holds exactly K full GEMMs.
    """
    if settle_ms <= 0:
        return 0
    n = 0
    t0 = time.perf_counter()
    while n < max_launches:
        for _ in range(chunk):
            step()
        n += chunk
        sync()
        if (time.perf_counter() - t0) * 1e3 >= settle_ms:
            break
    return n


def timed_window(step, sync, barrier, steps: int, warmup: int, settle_ms: float, sampler=None,
                 stats=None):
    """settle → warmup → [sync, barrier, sync] → t0 → K steps → sync → t1 → [barrier, sync].

    Returns ``(elapsed_s, settle_launches)``: this rank's t1 − t0, the caller takes the MAX over
    ranks.  The closing barrier aligns the ranks but is not inside the elapsed time: a 1-rank RCCL
    barrier cost a self-launched ``--gpus 1`` run 3.8 % of a 100-step window (1626.8 vs 1691.1 /
    1692.4 TFLOPS plain, r06), which at the driver's 20 steps would understate every N > 1 point;
    ``stats["end_barrier_ms"]`` records what it took.  The sampler (already constructed: ``amdsmi_init``
    and the handle scan are the slow part) starts its thread *before* the settle phase; inside the
    bracket it is only told the clock (``mark_start``/``mark_end``) and is held quiet while the K
    steps are launched (``hold`` … ``mark_launched``: no GIL contention with the launches).
    Nothing but synchronisation
    may sit between the last warmup step and ``t0``: any idle gap — r03's amd-smi init there cost
    the driver's K=20/W=5 run 14 % — puts the chip back into the load-step DVFS transient that the
    settle phase exists to skip (tests/test_parallel_gloo.py::test_bench_timed_window_order).
    """
    if sampler is not None:
        sampler.__enter__()
    try:
        launches = settle(step, sync, settle_ms)
        for _ in range(warmup):
            step()
        if sampler is not None:
            sampler.hold()      # quiet from here to the last timed launch (waits under warmup work)
        sync()
        barrier()
        sync()
        if sampler is not None:
            sampler.mark_start()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        if sampler is not None:
            sampler.mark_launched()     # sample while the enqueued steps run, not between launches
        sync()
        t1 = time.perf_counter()
        if sampler is not None:
            sampler.mark_end()
        barrier()
        sync()
        if stats is not None:
            stats["end_barrier_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
        elapsed = t1 - t0
    finally:
        if sampler is not None:
            sampler.__exit__(None, None, None)
    return elapsed, launches


def first_gpu_result(K, device: torch.device) -> float:
    """Reference-protocol vectorAdd (50 000 fp32, 196×256) — returns seconds since process start."""
    n = 50000
    g = torch.Generator().manual_seed(1234)
    ha, hb = torch.rand(n, generator=g), torch.rand(n, generator=g)
    c = K.vector_add(ha.to(device), hb.to(device))
    if not torch.allclose(c.cpu(), ha + hb, atol=1e-5, rtol=0):
        raise RuntimeError("vectorAdd verification failed")
    return time.time() - _T_PROCESS_START


def check_numerics(K, a, b, c, samples: int = 1024) -> float:
    m, n = c.shape
    g = torch.Generator().manual_seed(7)
    coords = torch.stack([torch.randint(0, m, (samples,), generator=g),
                          torch.randint(0, n, (samples,), generator=g)], dim=1).to(torch.int32)
    ref = K.gemm_sample_check(a, b, coords)
    got = c[coords[:, 0].long().to(c.device), coords[:, 1].long().to(c.device)].float()
    err = (got - ref).abs()
    tol = 0.01 * ref.abs() + 0.02 * (a.shape[1] ** 0.5) / 16
    bad = int((err > tol).sum().item())
    if bad:
        raise RuntimeError(f"GEMM numerics check failed: {bad}/{samples} samples out of tolerance, "
                           f"max err {err.max().item():.3e}")
    return float((err / (ref.abs() + 1.0)).max().item())


def rank_identity(device: torch.device) -> dict:
    """Which GPU this rank measured: PCI BDF (distinct across ranks, checked), device index, host."""
    import socket

    from k8s_nvidia_gpus_amd.parallel.telemetry import device_bdf

    return {"rank": int(os.environ.get("RANK", "0")),
            "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "device": str(device),
            "bdf": device_bdf(device.index or 0) if device.type == "cuda" else None,
            "host": socket.gethostname()}


def main(argv=None) -> int:
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        # a mismatched launch would report a different N than the one asked for
        if rank == 0:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    # torchrun with one rank still takes the RCCL path (a 1-GPU rehearsal of the N>1 code)
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    smoke = args.cpu_smoke
    if not smoke and not torch.cuda.is_available():
        print("bench.py needs an MI355X (no GPU visible)", file=sys.stderr)
        return 2
    from k8s_nvidia_gpus_amd.parallel.collectives import init_distributed, sweep

    # Process groups (N > 1, or torchrun with one rank): the default group is gloo, on the host —
    # the timing barriers and the gathering of per-rank results; the RCCL group (xGMI) is created
    # after the timed windows, for the all-reduce bus-bandwidth sweep.  An initialised RCCL
    # communicator cost the GEMM itself 3-5 % (one rank under torchrun: 1588 / 1615 / 1618 TFLOPS
    # with the RCCL group vs 1663 with gloo and 1672 plain, profiles/r06/bench_pg_probe.log), which
    # would read as a scaling loss at every N > 1.  AMDK8S_BENCH_PG=nccl: RCCL from the start
    # (barriers included), for A/B runs.
    rccl_first = os.environ.get("AMDK8S_BENCH_PG", "gloo") == "nccl"
    rccl = None
    if distributed:
        if smoke:
            device = init_distributed("gloo")
        else:
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            init_distributed("gloo")
            device = torch.device("cuda", local)
            if rccl_first:
                rccl = dist.new_group(backend="nccl", device_id=device)
    elif smoke:
        device = torch.device("cpu")
    else:
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(device)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    s = args.size
    max_rel_err = None
    ttfr = None
    variant = None
    if smoke:
        a = torch.rand((s, s)) * 2 - 1
        b = torch.rand((s, s)) * 2 - 1
        c = torch.empty((s, s))

        def step():
            torch.matmul(a, b.t(), out=c)
    else:
        from k8s_nvidia_gpus_amd.ops import kernels as K

        ttfr = first_gpu_result(K, device)
        if not K.gemm_shape_supported(s, s, s):
            raise SystemExit(f"--size {s} must be a multiple of 256")
        a = torch.empty((s, s), dtype=torch.bfloat16, device=device)
        b = torch.empty((s, s), dtype=torch.bfloat16, device=device)
        c = torch.empty((s, s), dtype=torch.bfloat16, device=device)
        K.fill_uniform_bf16(a, seed=1000 + rank)
        K.fill_uniform_bf16(b, seed=2000 + rank)
        variant = args.variant or K.DEFAULT_GEMM_VARIANT
        if variant == "auto":
            variant = K.pick_gemm_variant(s, s, s)
        K.gemm_bf16_nt(a, b, out=c, variant=variant)
        max_rel_err = check_numerics(K, a, b, c)

        def step():
            K.gemm_bf16_nt(a, b, out=c, variant=variant)

    from k8s_nvidia_gpus_amd.parallel import telemetry

    def barrier():
        if distributed:
            dist.barrier(group=rccl)            # gloo (host) unless AMDK8S_BENCH_PG=nccl

    # amd-smi init + handle scan happen here, before the settle phase (see timed_window)
    sampler = (telemetry.timed(period=0.005,
                               device_index=device.index if device.index is not None else 0)
               if not smoke and not args.no_telemetry else None)
    wstats: dict = {}
    elapsed, settle_launches = timed_window(step, sync, barrier, args.steps, args.warmup,
                                            0.0 if smoke else args.settle_ms, sampler, wstats)
    tel = sampler.summary() if sampler is not None else None

    flop_per_gpu = 2.0 * s * s * s * args.steps
    per_rank = [round(flop_per_gpu / elapsed / 1e12, 2)]
    if distributed:
        t = torch.tensor([elapsed, ttfr or 0.0], dtype=torch.float64)      # host tensors: gloo
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        ttfr = float(t[1].item()) if ttfr is not None else None
        mine = torch.tensor([per_rank[0]], dtype=torch.float64)
        gathered = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(gathered, mine)
        per_rank = [round(float(x.item()), 2) for x in gathered]
        tels = [None] * world
        dist.all_gather_object(tels, tel)
        pg_world = dist.get_world_size()
        ranks = [None] * world
        dist.all_gather_object(ranks, rank_identity(device))
    else:
        tels = [tel]
        pg_world = None
        ranks = [rank_identity(device)]
    if not smoke:
        bdfs = [r["bdf"] for r in ranks]
        if None in bdfs or len(set(bdfs)) != len(bdfs):
            raise RuntimeError(f"ranks did not each get their own GPU: {bdfs}")
    if distributed and pg_world != args.gpus:
        raise RuntimeError(f"process group has {pg_world} ranks, --gpus {args.gpus}")
    fp8_tflops = None
    if not smoke and not args.no_fp8 and K.gemm_fp8_shape_supported(s, s, s):
        del a, b
        a8 = K.uniform_fp8((s, s), seed=3000 + rank, device=device)
        b8 = K.uniform_fp8((s, s), seed=4000 + rank, device=device)

        def step8():
            K.gemm_fp8_nt(a8, b8, out=c)

        e8, _ = timed_window(step8, sync, barrier, args.steps, args.warmup, args.settle_ms)
        if distributed:
            t = torch.tensor([e8], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e8 = float(t[0].item())
        fp8_tflops = flop_per_gpu * world / e8 / 1e12
        del a8, b8

    busbw = None
    ar_sweep = None
    if distributed and not args.no_allreduce:
        if rccl is None and not smoke:          # now that the GEMM windows are done
            rccl = dist.new_group(backend="nccl", device_id=device)
        top = (4 if smoke else args.allreduce_mib) << 20
        rows = sweep("all_reduce", 1 << 20, top, factor=4, iters=3 if smoke else 10,
                     warmup=1 if smoke else 3, device=device, group=rccl)
        bad = sum(r.wrong for r in rows)
        if bad:
            raise RuntimeError(f"all-reduce returned {bad} wrong elements")
        ar_sweep = [{"bytes": r.bytes, "time_us": round(r.time_us, 1),
                     "algbw_gbps": round(r.algbw_gbps, 2), "busbw_gbps": round(r.busbw_gbps, 2)}
                    for r in rows]
        busbw = max(r.busbw_gbps for r in rows)

    value = flop_per_gpu * world / elapsed / 1e12
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "TFLOPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / BASELINE_VALUE, 3) if BASELINE_VALUE else None),
            "dtype": "fp32 (cpu smoke test, not a measurement)" if smoke else "bf16",
            "data": "synthetic (uniform [-1,1) operands generated on device)",
            "config": {
                "model": f"validator bf16 MFMA GEMM {s}x{s}x{s} (C=A*B^T, hand-written gfx950 kernel)",
                "global_batch": world,
                "seq_len": s,
                "parallelism": f"dp{world}" if world > 1 else "single",
                "m": s, "n": s, "k": s,
                "kernel": {"w8": "amdk8s_gemm_bf16_nt_256x256", "w4": "amdk8s_gemm_bf16_nt_256x256_w4",
                           "w4a": "amdk8s_gemm_bf16_nt_256x256_w4a"}
                .get(variant, "torch.matmul (cpu smoke)"),
            },
            "world_size": world,
            "process_group_world_size": pg_world,
            "process_group_backend": (dist.get_backend() if distributed else None),
            "allreduce_backend": (dist.get_backend(rccl) if rccl is not None else
                                  ("gloo" if distributed and smoke and not args.no_allreduce
                                   else None)),
            "launcher": os.environ.get("AMDK8S_BENCH_LAUNCHER",
                                       "torchrun" if distributed else "single process"),
            "ranks": ranks,
            "tflops_per_gpu": round(value / world, 2),
            "tflops_per_rank": per_rank,
            "settle": {"ms": 0.0 if smoke else args.settle_ms, "launches": settle_launches},
            "end_barrier_ms": wstats.get("end_barrier_ms"),
            "time_to_first_gpu_result_s": round(ttfr, 3) if ttfr is not None else None,
            "time_to_first_gpu_result_native_s": _NATIVE_TTFR,
            "numerics_max_rel_err": max_rel_err,
            "allreduce_busbw_gbps": (round(busbw, 2) if busbw is not None else None),
            "allreduce_sweep": ar_sweep,
            "telemetry_per_rank": tels,
            "fp8_tflops": (round(fp8_tflops, 2) if fp8_tflops is not None else None),
            "device": torch.cuda.get_device_name(device) if device.type == "cuda" else "cpu",
        }
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
