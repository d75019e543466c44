"""Collectives + gradient bucketing across real processes on the gloo backend (CPU, world 2 and 4)."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch.multiprocessing as mp

REPO = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    from k8s_nvidia_gpus_amd.parallel import collectives as C

    try:
        C.init_distributed("gloo")
        out = {}
        for op in ("all_reduce", "all_gather", "reduce_scatter", "all_to_all", "broadcast"):
            r = C.measure(op, 1 << 16, iters=3, warmup=1)
            out[op] = (r.wrong, r.world, r.bytes, r.busbw_gbps > 0)
        rows = C.sweep("all_reduce", 1 << 10, 1 << 14, factor=4, iters=2, warmup=1)
        out["sweep"] = [r.bytes for r in rows]
        # bucketed gradient all-reduce: rank r holds r+1 → average (world+1)/2 everywhere
        tensors = [torch.full((n,), float(rank + 1)) for n in (1000, 3, 70000, 12)]
        tensors.append(torch.full((5,), float(rank + 1), dtype=torch.float64))
        b = C.GradientBucketer(tensors, bucket_bytes=64 * 1024)
        b.start()
        b.wait()
        out["buckets"] = len(b.buckets)
        out["avg_ok"] = all(bool((t == (world + 1) / 2).all()) for t in tensors)
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced in the parent
        q.put((rank, {"error": repr(e)}))


@pytest.mark.parametrize("world", [2, 4])
def test_collectives_correct_on_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, out in res.items():
        assert "error" not in out, out
        for op in ("all_reduce", "all_gather", "reduce_scatter", "all_to_all", "broadcast"):
            wrong, w, nbytes, positive = out[op]
            assert wrong == 0 and w == world and positive, (op, out[op])
        assert out["sweep"] == [1024, 4096, 16384]
        assert out["avg_ok"] and out["buckets"] >= 3  # fp64 tensor forces its own bucket


def test_busbw_factors():
    from k8s_nvidia_gpus_amd.parallel.collectives import BUSBW_FACTOR

    assert BUSBW_FACTOR["all_reduce"](8) == pytest.approx(1.75)
    assert BUSBW_FACTOR["all_gather"](8) == pytest.approx(0.875)


def _torchrun(args, nproc, timeout=300):
    env = dict(os.environ, PYTHONPATH=str(REPO), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    return subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=str(REPO), timeout=timeout)


def test_parallel_bench_cli_under_torchrun_gloo():
    p = _torchrun(["-m", "k8s_nvidia_gpus_amd.parallel.bench", "--backend", "gloo", "--op",
                   "all_reduce", "-b", "4K", "-e", "64K", "-n", "2", "-w", "1"], 2)
    assert p.returncode == 0, p.stderr[-2000:]
    doc = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert doc["passed"] and doc["world"] == 2 and doc["wrong"] == 0


@pytest.mark.parametrize("world", [2, 8])
def test_bench_py_distributed_contract_on_cpu(world):
    """bench.py --cpu-smoke under torchrun (gloo): one JSON line, MAX over ranks, N-rank aggregate.
    world 8 rehearses the driver's 8-GPU launch shape (8 ranks, one per GPU)."""
    p = _torchrun(["bench.py", "--gpus", str(world), "--steps", "2", "--warmup", "1", "--cpu-smoke",
                   "--size", "256"], world)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    doc = json.loads(lines[0])
    assert doc["n_gpus"] == world and doc["steps"] == 2 and doc["warmup"] == 1
    assert doc["higher_is_better"] is True and doc["scaling"] == "weak"
    assert doc["config"]["parallelism"] == f"dp{world}" and doc["config"]["global_batch"] == world
    assert len(doc["tflops_per_rank"]) == world
    assert doc["allreduce_busbw_gbps"] is not None
    sw = doc["allreduce_sweep"]
    assert [r["bytes"] for r in sw] == [1 << 20, 4 << 20]            # 1 MiB .. top, x4
    assert doc["allreduce_busbw_gbps"] == pytest.approx(max(r["busbw_gbps"] for r in sw), abs=0.01)
    assert len(doc["telemetry_per_rank"]) == world                    # None on CPU (no GPU)
    # world x flop / MAX elapsed <= sum of per-rank rates (equal only when every rank is as slow as
    # the slowest; CPU ranks under a loaded test runner are not)
    assert 0 < doc["value"] <= sum(doc["tflops_per_rank"]) * 1.01 + 0.01 * world


def _plain_bench(args, env_extra=None, timeout=300):
    env = dict(os.environ, PYTHONPATH=str(REPO), OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py"] + args, capture_output=True, text=True,
                          env=env, cwd=str(REPO), timeout=timeout)


def test_bench_py_plain_gpus_n_self_launches_n_ranks():
    """``python bench.py --gpus 2`` without a launcher starts 2 ranks itself (VERDICT r05 weak 1:
    it used to print n_gpus 1 with rc 0) and relays rank 0's single JSON line."""
    p = _plain_bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--cpu-smoke", "--size", "256",
                      "--no-allreduce"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    doc = json.loads(lines[0])
    assert doc["n_gpus"] == 2 and doc["world_size"] == 2
    assert doc["process_group_world_size"] == 2 and doc["process_group_backend"] == "gloo"
    assert len(doc["tflops_per_rank"]) == 2
    assert [r["rank"] for r in doc["ranks"]] == [0, 1]
    assert doc["launcher"].startswith("torchrun (spawned")


def test_bench_py_refuses_more_gpus_than_visible_agents(tmp_path):
    """--gpus 3 on a node with 2 visible GPU agents exits non-zero before starting any rank."""
    from tests.fakes.sysfs import build_node

    root = build_node(tmp_path, n_gpus=2)
    p = _plain_bench(["--gpus", "3", "--steps", "1", "--warmup", "0", "--cpu-smoke", "--size", "256"],
                     {"AMDK8S_SYSFS_ROOT": str(root)})
    assert p.returncode == 2, (p.stdout, p.stderr)
    assert "only 2 GPU agent" in p.stderr and not p.stdout.strip()
    # the same node with 2 GPUs asked for runs
    p = _plain_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--cpu-smoke", "--size", "128",
                      "--no-allreduce"], {"AMDK8S_SYSFS_ROOT": str(root)})
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 2
    # HIP_VISIBLE_DEVICES narrows what is visible
    p = _plain_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--cpu-smoke", "--size", "128"],
                     {"AMDK8S_SYSFS_ROOT": str(root), "HIP_VISIBLE_DEVICES": "1"})
    assert p.returncode == 2 and "HIP_VISIBLE_DEVICES" in p.stderr


def test_bench_py_world_size_mismatch_is_an_error():
    """Under torchrun, WORLD_SIZE != --gpus fails instead of reporting the other N."""
    p = _torchrun(["bench.py", "--gpus", "3", "--steps", "1", "--warmup", "0", "--cpu-smoke",
                   "--size", "128"], 2)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "WORLD_SIZE=2" in p.stderr


def test_bench_py_single_gpu_path_unchanged():
    """N = 1 without a launcher stays one process (BENCH comparability across rounds)."""
    p = _plain_bench(["--steps", "1", "--warmup", "0", "--cpu-smoke", "--size", "128"])
    assert p.returncode == 0, p.stderr[-2000:]
    doc = json.loads(p.stdout.strip().splitlines()[-1])
    assert doc["n_gpus"] == 1 and doc["launcher"] == "single process"
    assert doc["process_group_world_size"] is None and "launching" not in p.stderr


def test_bench_settle_phase_bounds():
    """bench.settle(): untimed launches until settle_ms of synchronized time, capped, off at 0."""
    import importlib.util
    import time

    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    calls, syncs = [], []

    def step():
        calls.append(1)
        time.sleep(0.001)

    assert bench.settle(step, lambda: syncs.append(1), 0.0) == 0 and not calls
    t0 = time.perf_counter()
    n = bench.settle(step, lambda: syncs.append(1), 20.0, chunk=4)
    assert (time.perf_counter() - t0) * 1e3 >= 20.0
    assert n == len(calls) and n % 4 == 0 and len(syncs) == n // 4
    calls.clear()
    assert bench.settle(step, lambda: None, 1e6, chunk=4, max_launches=12) == 12 == len(calls)


def test_bench_timed_window_order():
    """Sampler init → thread start → settle → warmup → t0 → K steps: between the last warmup step
    and the first timed step only sync/barrier and the sampler's clock marks may run (r03's
    amd-smi init in that gap cost the driver's K=20/W=5 headline 14 %)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    log = []

    class FakeSampler:
        def __init__(self):
            log.append("init")                       # amdsmi_init + handle scan

        def __enter__(self):
            log.append("thread")
            return self

        def hold(self):
            log.append("hold")

        def mark_start(self):
            log.append("mark_start")

        def mark_launched(self):
            log.append("mark_launched")

        def mark_end(self):
            log.append("mark_end")

        def __exit__(self, *exc):
            log.append("exit")

    sampler = FakeSampler()
    elapsed, launches = bench.timed_window(lambda: log.append("step"), lambda: log.append("sync"),
                                           lambda: log.append("barrier"), steps=20, warmup=5,
                                           settle_ms=0.5, sampler=sampler)
    assert elapsed > 0 and launches >= 8
    assert log[:2] == ["init", "thread"]
    i_start = log.index("mark_start")
    # exactly K steps inside the marks, and they are the last K steps issued
    inside = log[i_start:log.index("mark_end")]
    assert inside.count("step") == 20
    assert log.count("step") == launches + 5 + 20
    # the gap between the last untimed step and the first timed one holds no real work
    last_warm = max(i for i, e in enumerate(log[:i_start]) if e == "step")
    assert set(log[last_warm + 1:i_start + 1]) <= {"sync", "barrier", "hold", "mark_start"}
    assert log[last_warm + 1] == "hold"             # quiet before the GPU drains the warmup
    assert log[i_start + 1] == "step" and log[-1] == "exit"
    # the window closes at this rank's own sync: the aligning barrier comes after mark_end
    i_end = log.index("mark_end")
    assert log[i_end - 1] == "sync" and "barrier" not in log[i_start:i_end]
    assert "barrier" in log[i_end:]
    # held quiet while the K steps are launched, sampling again while they execute
    i_launched = log.index("mark_launched")
    assert log.index("hold") < i_start and log[i_start:i_launched].count("step") == 20 and "sync" not in log[i_start:i_launched]
    # the real Sampler does its amd-smi setup in the constructor, not in __enter__/mark_start
    from k8s_nvidia_gpus_amd.parallel.telemetry import Sampler

    calls = []

    class FakeSmi:
        def amdsmi_init(self):
            calls.append("init")

        def amdsmi_get_processor_handles(self):
            calls.append("handles")
            return ["h0"]

        def amdsmi_get_gpu_device_bdf(self, h):
            return "0000:05:00.0"

        def amdsmi_get_gpu_metrics_info(self, h):
            return {"current_gfxclk": 2100, "current_socket_power": 900, "temperature_hotspot": 70}

        def amdsmi_shut_down(self):
            calls.append("shutdown")

    s = Sampler("0000:05:00.0", period=0.001, amdsmi_module=FakeSmi())
    assert calls == ["init", "handles"]
    before = len(calls)
    with s:
        import time as _t

        _t.sleep(0.01)
        s.hold()
        s.mark_start()
        n_held = len(s.rows)
        _t.sleep(0.01)
        assert len(s.rows) == n_held          # quiet while launching
        s.mark_launched()
        _t.sleep(0.01)
        s.mark_end()
        assert len(calls) == before
    summ = s.summary()
    assert summ["gfxclk_mhz_mean"] == 2100 and 1 <= summ["samples"] < len(s.rows)
    assert summ["coverage"] in ("window", "tail-only") and summ["window_ms"] >= 20
    assert summ["coverage"] == ("window" if summ["samples"] >= 3 else "tail-only")
    assert summ["pre_window"]["samples"] >= 1 and summ["pre_window"]["gfxclk_mhz_mean"] == 2100
    assert calls[-1] == "shutdown"


def test_rccl_bench_multiprocess_plan_under_torchrun():
    """rccl-allreduce-bench --mp takes its rank/world/device from torchrun (--no-python) — the
    launch the gpu-bench Job uses; --plan stops before any HIP call so this runs on CPU."""
    import json
    import socket
    import subprocess
    import sys
    from pathlib import Path

    import yaml

    repo = Path(__file__).resolve().parent.parent
    exe = repo / "native/bin/rccl-allreduce-bench"
    if not exe.exists():
        from k8s_nvidia_gpus_amd.ops import build as B

        B.build_native(only=["rccl-allreduce-bench"])
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=3", "--master-addr=127.0.0.1", f"--master-port={port}",
                        "--no-python", str(exe), "--mp", "--plan"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    plans = sorted((json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")),
                   key=lambda d: d["rank"])
    assert [(d["rank"], d["world"], d["device"]) for d in plans] == [(0, 3, 0), (1, 3, 1), (2, 3, 2)]
    assert len({d["id_file"] for d in plans}) == 1 and str(port) in plans[0]["id_file"]
    # a second launch on the SAME port gets a different id file (launcher pid in
    # the key) ...
    p2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                         "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={port}",
                         "--no-python", str(exe), "--mp", "--plan"],
                        capture_output=True, text=True, timeout=120)
    assert p2.returncode == 0, p2.stderr[-2000:]
    second = [json.loads(ln) for ln in p2.stdout.splitlines() if ln.startswith("{")]
    assert second[0]["id_file"] != plans[0]["id_file"] and str(port) in second[0]["id_file"]
    # ... and a stale file at the launch's path (crashed earlier run, reused /tmp) is not accepted
    import os
    import tempfile
    import time

    stale = Path(tempfile.mkdtemp()) / "rccl.id"
    stale.write_bytes(b"\0" * 128)
    old = time.time() - 3600
    os.utime(stale, (old, old))
    p3 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                         "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={port}",
                         "--no-python", str(exe), "--mp", "--plan", "--id-file", str(stale)],
                        capture_output=True, text=True, timeout=120)
    third = [json.loads(ln) for ln in p3.stdout.splitlines() if ln.startswith("{")]
    assert third and all(d["existing_id_file_fresh"] is False for d in third)
    assert all(d["launcher_start"] > old for d in third)
    job = yaml.safe_load((repo / "cluster-config/apps/gpu-bench/job-rccl-allreduce.yaml").read_text())
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert c["command"][-1] == "torch.distributed.run" and "--no-python" in c["args"] and "--mp" in c["args"]
    nproc = next(a for a in c["args"] if a.startswith("--nproc-per-node=")).split("=")[1]
    assert int(nproc) == int(c["resources"]["limits"]["amd.com/gpu"])
    # the rendezvous id is the pod UID (downward API), unique per Job pod
    assert "--rdzv-id=$(POD_UID)" in c["args"]
    env = {e["name"]: e for e in c["env"]}
    assert env["POD_UID"]["valueFrom"]["fieldRef"]["fieldPath"] == "metadata.uid"


def test_telemetry_sampler_matches_gpu_by_pci_address():
    """The sampler picks the amd-smi handle of THIS rank's GPU by BDF, summarises clock / power /
    hotspot, and degrades to an error record without amd-smi."""
    import time

    from fakes.amdsmi import FakeAmdSmi
    from k8s_nvidia_gpus_amd.parallel.telemetry import Sampler

    fake = FakeAmdSmi()
    bdf = fake.amdsmi_get_gpu_device_bdf(fake.amdsmi_get_processor_handles()[5])
    with Sampler(bdf, period=0.005, amdsmi_module=fake) as s:
        time.sleep(0.05)
    summ = s.summary()
    assert s.handle is not None and int(s.handle) == 5
    assert summ["samples"] >= 2 and summ["bdf"] == bdf.lower()
    assert summ["gfxclk_mhz_mean"] and summ["power_w_mean"] and summ["temp_hotspot_c_max"]
    missing = Sampler("0000:ff:00.0", amdsmi_module=FakeAmdSmi())
    with missing:
        pass
    assert missing.summary() == {"error": "no amd-smi handle for 0000:ff:00.0"}
