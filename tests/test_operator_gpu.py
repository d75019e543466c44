"""Operator components on a real MI355X node (run on the GPU box: pytest -m gpu).

The CPU suite drives these components against fakes; here the same code runs against the real
KFD sysfs, the real amd-smi library and the real native validator binaries.
"""
import json
import os

import pytest

from k8s_nvidia_gpus_amd.operator import deviceplugin_api as api
from k8s_nvidia_gpus_amd.operator.config import load_config
from k8s_nvidia_gpus_amd.operator.validator import Validator
from k8s_nvidia_gpus_amd.ops import build as B
from k8s_nvidia_gpus_amd.utils.topology import read_topology

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    B.build_native()
    return B.NATIVE_BIN


def test_real_topology_has_visible_gfx950(tmp_path):
    t = read_topology("/", 90500)
    assert t.gpus, "no gfx950 agent visible in /sys/class/kfd"
    g = t.gpus[0]
    assert g.gfx_name == "gfx950" and g.cu_count in (256, 128, 64, 32)
    assert g.vram_bytes > 30 * (1 << 30)
    assert os.path.exists(g.render_path)


def test_device_plugin_enumerates_real_node(tmp_path):
    from k8s_nvidia_gpus_amd.operator.device_plugin import AmdGpuDevicePlugin

    cfg = load_config(text="expectedGpusPerNode: 1\n")
    p = AmdGpuDevicePlugin(cfg, root="/", kubelet_dir=str(tmp_path), pause_marker=str(tmp_path / "p"))
    devs = p.list_response().devices
    assert len(devs) >= 1 and all(d.health == api.HEALTHY for d in devs)
    req = api.AllocateRequest()
    req.container_requests.add(devices_ids=[devs[0].ID])
    (c,) = p.Allocate(req, None).container_responses
    assert c.devices[0].host_path == "/dev/kfd" and os.path.exists(c.devices[1].host_path)


def test_exporter_on_real_amdsmi():
    from prometheus_client import generate_latest

    from k8s_nvidia_gpus_amd.operator import exporter as ex

    col = ex.GpuCollector(ex.AmdSmiBackend(), "box", "/nonexistent")
    text = generate_latest(ex.make_registry(col)).decode()
    assert "amd_gpu_exporter_up 1.0" in text
    assert "amd_gpu_info{" in text and 'gfx="gfx950"' in text
    assert "amd_gpu_vram_total_bytes{" in text
    assert "amd_gpu_pcie_link_width{" in text and "amd_gpu_power_limit_watts{" in text
    out = os.environ.get("AMDK8S_EVIDENCE_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "exporter_metrics.txt"), "w") as f:
            f.write(text)


def test_validator_chain_with_native_binaries(tmp_path, native):
    cfg = load_config(text="expectedGpusPerNode: 1\nvalidator: {podResourcesRequired: false, gemmSize: 4096, gemmMinTflops: 600, "
                           "rccl: false, pluginTest: false, rocprofCounters: true}\n")
    v = Validator(cfg, str(tmp_path), bin_dir=str(native))
    for step in ("driver", "vectoradd", "gemm", "bandwidth", "profile"):
        r = v.run_step(step)
        assert r.passed, (step, r.reason)
    (tmp_path / "runtime-ready").write_text("1")  # no runtime installer on the box
    assert v.run_step("report").passed
    gemm = json.loads((tmp_path / "gemm.json").read_text())
    assert all(d["tflops"] > 600 for d in gemm["devices"])
    pmc = json.loads((tmp_path / "profile.json").read_text())["rocprof_counters"]
    assert pmc.get("flop_matches_shape") is True, pmc  # MFMA FLOPs counted == 2·4096³
    assert 50 < pmc["mfma_util_pct"] <= 100 and 1.0 < pmc["clock_ghz"] < 2.5
    out = os.environ.get("AMDK8S_EVIDENCE_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        for f in ("driver.json", "vectoradd.json", "gemm.json", "bandwidth.json", "profile.json",
                  "report.json"):
            with open(tmp_path / f) as src, open(os.path.join(out, "validator_" + f), "w") as dst:
                dst.write(src.read())


def test_rccl_bench_single_gpu_passes(native):
    import subprocess

    p = subprocess.run([str(native / "rccl-allreduce-bench"), "-b", "1M", "-e", "16M", "-n", "5",
                        "--json"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "Test PASSED" in p.stdout


def test_rccl_bench_multiprocess_mode_one_rank(native):
    """The one-process-per-GPU launch of the gpu-bench Job (torchrun --no-python ... --mp): the
    ncclUniqueId file exchange, ncclCommInitRank and the MAX-over-ranks timing on the real GPU."""
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=1", "--master-addr=127.0.0.1", f"--master-port={port}",
                        "--no-python", str(native / "rccl-allreduce-bench"), "--mp", "-b", "1M",
                        "-e", "16M", "-n", "5", "--json"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    doc = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert doc["mode"] == "mp" and doc["ngpus"] == 1 and doc["passed"] and doc["wrong"] == 0
    assert "Test PASSED" in p.stdout


def test_bench_py_rccl_path_under_torchrun_one_rank():
    """bench.py under torchrun with one rank takes the N>1 code path (RCCL process group, MAX over
    ranks, all_gather of per-rank TFLOPS, post-run all-reduce probe) on the real GPU."""
    import socket
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "1",
           "--steps", "5", "--warmup", "2", "--settle-ms", "20", "--size", "2048",
           "--allreduce-mib", "16", "--no-fp8"]
    p = subprocess.run(cmd, capture_output=True, text=True, cwd=str(repo), timeout=240,
                       env=dict(os.environ, PYTHONPATH=str(repo)))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    doc = json.loads(lines[0])
    assert doc["n_gpus"] == 1 and doc["steps"] == 5 and doc["value"] > 0
    assert doc["allreduce_busbw_gbps"] is not None and len(doc["tflops_per_rank"]) == 1
    assert doc["settle"]["launches"] > 0
    assert len(doc["allreduce_sweep"]) == 3          # 1, 4, 16 MiB
    tel = doc["telemetry_per_rank"][0]
    assert tel is None or "error" in tel or tel["samples"] >= 1


def test_bench_py_self_launched_torchrun_matches_plain_run():
    """``bench.py --gpus 1 --launcher torchrun`` (the self-launch path a plain
    ``--gpus N`` takes) measures the same GEMM as the plain single-process run, within 2 %, and
    reports the rank's own PCI BDF and the process group's world size."""
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    common = ["--gpus", "1", "--steps", "100", "--warmup", "10", "--no-fp8", "--no-allreduce",
              "--no-telemetry"]
    env = dict(os.environ, PYTHONPATH=str(repo))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    docs = []
    # plain, self-launched, plain: the launched run is compared with the plain runs on both sides
    # of it, so a drift of the chip's sustained clock between back-to-back runs is not read as a
    # launcher cost
    for extra in ([], ["--launcher", "torchrun"], []):
        p = subprocess.run([sys.executable, "bench.py"] + common + extra, capture_output=True,
                           text=True, cwd=str(repo), timeout=300, env=env)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, p.stdout
        docs.append(json.loads(lines[0]))
    plain, launched, plain2 = docs
    assert plain["launcher"] == "single process" and launched["launcher"].startswith("torchrun")
    assert launched["process_group_world_size"] == 1 and launched["n_gpus"] == 1
    assert plain["ranks"][0]["bdf"] and plain["ranks"][0]["bdf"] == launched["ranks"][0]["bdf"]
    lo = min(plain["value"], plain2["value"]) * 0.98
    hi = max(plain["value"], plain2["value"]) * 1.02
    assert lo <= launched["value"] <= hi, (plain["value"], launched["value"], plain2["value"])


@pytest.mark.parametrize("gated", [True, False])
def test_node_bringup_rehearsal_on_real_hardware(tmp_path, native, gated):
    """Node-local time-to-first-GPU-pod: real kfd-probe, runtime shim + CDI, device plugin over gRPC
    (kubelet stand-in), Allocate, OCI spec edit, vectorAdd on the allocated GPU, validator chain.
    Gated (shipped): the plugin advertises the GPU only after the validator's vectorAdd + GEMMs
    passed on it, and the first pod is allocated then (<= 5 s)."""
    import torch

    from k8s_nvidia_gpus_amd.operator import bringup

    n = torch.cuda.device_count()
    cfg = load_config(text=f"expectedGpusPerNode: {n}\n")
    rep = bringup.rehearse(cfg, str(native), workdir=str(tmp_path / "work"), gated=gated)
    assert rep["passed"], json.dumps(rep["stages"][-1])
    st = {s["name"]: s for s in rep["stages"]}
    assert st["plugin"]["detail"]["healthy"] == (0 if gated else n)
    if gated:
        assert st["allocatable"]["detail"]["healthy"] == n
        assert rep["time_to_first_gpu_pod_s"] <= 5.0, rep["time_to_first_gpu_pod_s"]
    assert st["create"]["detail"]["device_nodes"][-1] == "/dev/kfd"
    assert rep["time_to_first_gpu_pod_s"] < 30 and rep["time_to_validated_s"] < 120
    out = os.environ.get("AMDK8S_EVIDENCE_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"bringup_{'gated' if gated else 'ungated'}.json"), "w") as f:
            json.dump(rep, f, indent=1)


def test_validator_stress_step_on_real_hardware(tmp_path, native):
    """5 s of sustained MFMA load with real amd-smi telemetry: steady rate, no ECC, sane temperatures."""
    cfg = load_config(text="expectedGpusPerNode: 1\nvalidator: {podResourcesRequired: false, stress: true, stressSeconds: 5}\n")
    v = Validator(cfg, str(tmp_path), bin_dir=str(native))
    r = v.run_step("stress")
    assert r.passed, r.reason
    g = r.detail["gpus"]["0"]
    assert g["tflops"] > 1000 and g["tflops_min_window"] >= 0.85 * g["tflops"]
    assert r.detail["telemetry_samples"] >= 3 and g.get("ecc_uncorrectable_delta", 0) == 0
    out = os.environ.get("AMDK8S_EVIDENCE_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(tmp_path / "stress.json") as src, open(os.path.join(out, "validator_stress.json"), "w") as dst:
            dst.write(src.read())
