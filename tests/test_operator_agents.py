"""Node agents of the AMD GPU operator against fakes: sysfs tree, Kubernetes API, amd-smi (CPU-only)."""
import json
import os
import subprocess
import sys
import threading
import urllib.request
from pathlib import Path

import pytest

from fakes import sysfs as fake_sysfs
from fakes.amdsmi import FakeAmdSmi
from fakes.kubeapi import FakeKubeAPI
from k8s_nvidia_gpus_amd.operator import exporter as ex
from k8s_nvidia_gpus_amd.operator import labeller as lb
from k8s_nvidia_gpus_amd.operator import partition as pm
from k8s_nvidia_gpus_amd.operator.labeller import compute_labels
from k8s_nvidia_gpus_amd.operator import runtime as rt
from k8s_nvidia_gpus_amd.operator.config import ConfigError, load_config
from k8s_nvidia_gpus_amd.utils.kube import KubeClient, pod_gpu_request
from k8s_nvidia_gpus_amd.utils.topology import read_topology

REPO = Path(__file__).resolve().parent.parent


@pytest.fixture
def api():
    a = FakeKubeAPI().start()
    a.add_node("gpu-node-1", {"kubernetes.io/os": "linux"})
    yield a
    a.stop()


@pytest.fixture
def client(api):
    return KubeClient(base_url=api.url)


# ----------------------------------------------------------------------------- config
def test_config_defaults_and_validation():
    cfg = load_config()
    assert cfg.resource_name == "amd.com/gpu" and cfg.min_gfx == 90500
    with pytest.raises(ConfigError):
        load_config(text="resourceName: amd.com/gpu\nbogus: 1\n")
    with pytest.raises(ConfigError):
        load_config(text="partition: {compute: MIG}\n")
    with pytest.raises(ConfigError):
        load_config(text="validator: {gemmSize: 1000}\n")


def test_shipped_operator_config_parses():
    import yaml

    cm = yaml.safe_load((REPO / "cluster-config/apps/amd-gpu-operator/config.yaml").read_text())
    cfg = load_config(text=cm["data"]["operator.yaml"])
    assert cfg["expectedGpusPerNode"] == 8
    assert cfg.section("allocation")["mode"] == "deviceSpecs"


# ----------------------------------------------------------------------------- labeller
def test_labeller_labels_mi355x_node(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    (root / "sys/module/amdgpu").mkdir(parents=True)
    (root / "sys/module/amdgpu/version").write_text("6.16.6\n")
    patch = lb.NodeLabeller(client, "gpu-node-1", str(root)).reconcile()
    labels = api.nodes["gpu-node-1"]["metadata"]["labels"]
    assert labels["amd.com/gpu.present"] == "true"
    assert labels["amd.com/gpu.product"] == "MI355X"
    assert labels["amd.com/gpu.family"] == "gfx950"
    assert labels["amd.com/gpu.count"] == "8"
    assert labels["amd.com/gpu.cu-count"] == "256"
    assert labels["amd.com/gpu.vram"] == "288G"
    assert labels["amd.com/gpu.compute-partition"] == "SPX"
    assert labels["amd.com/gpu.xgmi-links"] == "7"
    assert labels["amd.com/gpu.numa-nodes"] == "2"
    assert labels["amd.com/gpu.driver-version"] == "6.16.6"
    assert labels["kubernetes.io/os"] == "linux"  # untouched
    assert patch
    # idempotent: second pass patches nothing
    assert lb.NodeLabeller(client, "gpu-node-1", str(root)).reconcile() == {}


def test_labeller_cpx_and_removal(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r", compute_partition="CPX")
    lab = lb.NodeLabeller(client, "gpu-node-1", str(root))
    lab.reconcile()
    labels = api.nodes["gpu-node-1"]["metadata"]["labels"]
    assert labels["amd.com/gpu.count"] == "64" and labels["amd.com/gpu.cu-count"] == "32"
    assert labels["amd.com/gpu.compute-partition"] == "CPX"
    api.nodes["gpu-node-1"]["metadata"]["labels"]["amd.com/gpu.validated"] = "true"
    # GPUs gone (driver unloaded): owned labels removed, foreign ones kept
    lb.NodeLabeller(client, "gpu-node-1", str(tmp_path / "empty")).reconcile()
    labels = api.nodes["gpu-node-1"]["metadata"]["labels"]
    assert not any(k in labels for k in ("amd.com/gpu.present", "amd.com/gpu.count"))
    assert labels["amd.com/gpu.validated"] == "true"


def test_label_value_sanitizer():
    assert lb.sanitize("Linuxversion 6.18 (gcc)") == "Linuxversion_6.18_gcc"
    assert len(lb.sanitize("x" * 100)) == 63


# ----------------------------------------------------------------------------- exporter
def _scrape(collector):
    from prometheus_client import generate_latest

    return generate_latest(ex.make_registry(collector)).decode()


def _samples(text):
    """{(metric, frozenset(labels)): value} from Prometheus text."""
    from prometheus_client.parser import text_string_to_metric_families

    out = {}
    for fam in text_string_to_metric_families(text):
        for s in fam.samples:
            out[(s.name, frozenset(s.labels.items()))] = s.value
    return out


def _find(samples, name, **labels):
    return [v for (n, ls), v in samples.items()
            if n == name and all((k, str(val)) in ls for k, val in labels.items())]


def test_exporter_amdsmi_backend_metrics(tmp_path):
    marker = tmp_path / "v"
    marker.mkdir()
    (marker / "gemm.json").write_text(json.dumps({"passed": True, "devices": [
        {"device": 0, "tflops": 1389.4}, {"device": 1, "tflops": 1380.0}],
        "fp8": {"devices": [{"device": 0, "tflops": 2858.1}]}, "duration_s": 2.25}))
    (marker / "rccl.json").write_text(json.dumps({"passed": True, "ngpus": 8, "peak_busbw_gbps": 310.5}))
    (marker / "report.json").write_text(json.dumps({"passed": True, "chain_seconds": 7.5,
                                                    "duration_s": 0.01}))
    fake = FakeAmdSmi()
    col = ex.GpuCollector(ex.AmdSmiBackend(fake), "gpu-node-1", str(marker))
    text = _scrape(col)
    sm = _samples(text)
    assert _find(sm, "amd_gpu_exporter_up") == [1.0]
    info = _find(sm, "amd_gpu_info")
    assert len(info) == 8
    assert _find(sm, "amd_gpu_info", product="AMD Instinct MI355 OAM", gfx="gfx950", gpu=0)
    assert _find(sm, "amd_gpu_power_watts", gpu=0) == [249.0]
    assert _find(sm, "amd_gpu_temperature_celsius", gpu=0, sensor="hotspot") == [45.0]
    assert _find(sm, "amd_gpu_utilization_percent", gpu=3) == [30.0]
    assert _find(sm, "amd_gpu_vram_total_bytes", gpu=0) == [294896 * 1024 * 1024]
    links = _find(sm, "amd_gpu_xgmi_data_bytes_total", gpu=0, direction="read")
    assert len(links) == 8 and max(links) > 1e10
    assert _find(sm, "amd_gpu_ecc_errors_total", gpu=0, type="uncorrectable") == [0.0]
    assert _find(sm, "amd_gpu_validator_gemm_tflops", gpu=0, node="gpu-node-1") == [1389.4]
    assert _find(sm, "amd_gpu_validator_gemm_fp8_tflops", gpu=0) == [2858.1]
    assert _find(sm, "amd_gpu_validator_allreduce_busbw_gbps", ngpus=8) == [310.5]
    assert _find(sm, "amd_gpu_validation_passed", step="gemm") == [1.0]
    assert _find(sm, "amd_gpu_validator_step_seconds", step="gemm") == [2.25]
    assert _find(sm, "amd_gpu_validator_step_seconds", step="report") == [7.5]
    # PCIe / xGMI link state and the power cap, from the recorded MI355X amd-smi output
    assert _find(sm, "amd_gpu_pcie_link_speed_gts", gpu=0) == [32.0]
    assert _find(sm, "amd_gpu_pcie_link_width", gpu=0) == [16.0]
    assert _find(sm, "amd_gpu_pcie_events_total", gpu=0, event="replay") == [0.0]
    assert _find(sm, "amd_gpu_pcie_events_total", gpu=0, event="nak_received") == [0.0]
    assert _find(sm, "amd_gpu_power_limit_watts", gpu=0) == [1400.0]
    assert _find(sm, "amd_gpu_xgmi_link_width", gpu=0) == [16.0]
    # N/A fields (edge temperature) are omitted, not exported as 0
    assert not _find(sm, "amd_gpu_temperature_celsius", sensor="edge")


def test_exporter_omits_incomplete_validation_chain_time(tmp_path):
    marker = tmp_path / "v"
    marker.mkdir()
    (marker / "report.json").write_text(json.dumps({"passed": True, "chain_seconds": 1.2,
                                                    "chain_complete": False,
                                                    "step_seconds_missing": ["runtime"]}))
    col = ex.GpuCollector(ex.AmdSmiBackend(FakeAmdSmi()), "n", str(marker))
    sm = _samples(_scrape(col))
    assert not _find(sm, "amd_gpu_validator_step_seconds", step="report")
    assert _find(sm, "amd_gpu_validation_passed", step="report") == [1.0]


def test_exporter_survives_unsupported_calls():
    fake = FakeAmdSmi(n_gpus=2, fail={"amdsmi_get_gpu_metrics_info", "amdsmi_get_gpu_total_ecc_count"})
    text = _scrape(ex.GpuCollector(ex.AmdSmiBackend(fake), "n", "/nonexistent"))
    assert text.count("amd_gpu_info{") == 2
    assert "amd_gpu_power_watts{" not in text
    assert "amd_gpu_vram_used_bytes{" in text


def test_exporter_sysfs_fallback(tmp_path):
    root = fake_sysfs.build_node(tmp_path / "r")
    text = _scrape(ex.GpuCollector(ex.SysfsBackend(str(root)), "n", "/nonexistent"))
    assert text.count("amd_gpu_info{") == 8
    assert 'amd_gpu_vram_total_bytes{gpu="0"' in text


def test_exporter_http_server(tmp_path):
    srv = ex.ExporterServer(ex.GpuCollector(ex.AmdSmiBackend(FakeAmdSmi(2)), "n", str(tmp_path)),
                            port=0, host="127.0.0.1")
    srv.serve_background()
    try:
        base = f"http://127.0.0.1:{srv.port}"
        assert urllib.request.urlopen(base + "/healthz", timeout=5).read() == b"ok\n"
        body = urllib.request.urlopen(base + "/metrics", timeout=5).read().decode()
        assert "amd_gpu_info{" in body
    finally:
        srv.shutdown()


# ----------------------------------------------------------------------------- partition manager
class FakeSysfsPartitionBackend:
    """Applies a mode by re-enumerating the fake sysfs tree, as the driver would."""

    def __init__(self, root, n_gpus=8):
        self.root, self.n = root, n_gpus
        self.applied = []

    def set_memory(self, dev, mode):
        self.applied.append(("memory", dev.pci_bdf, mode))

    def set_compute(self, dev, mode):
        self.applied.append(("compute", dev.pci_bdf, mode))
        if len([a for a in self.applied if a[0] == "compute"]) == self.n:
            mem = next((a[2] for a in self.applied if a[0] == "memory"), "NPS1")
            fake_sysfs.set_partition(self.root, self.n, mode, mem)


def test_partition_manager_spx_to_cpx(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    api.nodes["gpu-node-1"]["metadata"]["labels"][pm.LABEL_DESIRED] = "CPX"
    backend = FakeSysfsPartitionBackend(root)
    marker = tmp_path / "run/partition-in-progress"
    mgr = pm.PartitionManager(client, "gpu-node-1", backend, str(root), poll=0.01,
                              pause_marker=str(marker), sleep=lambda s: None, ack_components=())
    assert mgr.reconcile() == "applied"
    assert len(read_topology(str(root), 90500).gpus) == 64
    assert not marker.exists()
    node = api.nodes["gpu-node-1"]
    assert node["metadata"]["annotations"][pm.ANNOT_STATE].startswith("idle")
    assert not [t for t in node["spec"].get("taints", []) if t["key"] == pm.TAINT_KEY]
    assert node["metadata"]["labels"]["amd.com/gpu.compute-partition"] == "CPX"
    assert len([a for a in backend.applied if a[0] == "compute"]) == 8
    # steady state
    assert mgr.reconcile() == "idle"


def test_partition_manager_waits_for_gpu_pods_then_times_out(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    api.nodes["gpu-node-1"]["metadata"]["labels"][pm.LABEL_DESIRED] = "CPX"
    api.add_pod("default", "busy", "gpu-node-1", gpus=1)
    api.add_pod("default", "cpu-only", "gpu-node-1", gpus=0)
    seen = {}

    def sleep(_s):
        node = api.nodes["gpu-node-1"]
        seen["taint"] = [t for t in node["spec"].get("taints", []) if t["key"] == pm.TAINT_KEY]
        seen["marker"] = os.path.exists(str(tmp_path / "pause"))

    mgr = pm.PartitionManager(client, "gpu-node-1", FakeSysfsPartitionBackend(root), str(root),
                              drain_timeout=0.05, poll=0.01, pause_marker=str(tmp_path / "pause"),
                              sleep=sleep, drain_policy="wait", ack_components=())
    assert mgr.reconcile() == "failed"
    assert seen["taint"] and seen["marker"]  # drained with taint + device-plugin pause
    node = api.nodes["gpu-node-1"]
    assert "drain timeout" in node["metadata"]["annotations"][pm.ANNOT_STATE]
    assert not [t for t in node["spec"].get("taints", []) if t["key"] == pm.TAINT_KEY]
    assert not os.path.exists(str(tmp_path / "pause"))
    assert len(read_topology(str(root), 90500).gpus) == 8  # untouched


def test_partition_manager_rejects_unavailable_mode(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    api.nodes["gpu-node-1"]["metadata"]["labels"][pm.LABEL_DESIRED] = "XPX"
    mgr = pm.PartitionManager(client, "gpu-node-1", FakeSysfsPartitionBackend(root), str(root),
                              pause_marker=str(tmp_path / "p"), sleep=lambda s: None, ack_components=())
    assert mgr.reconcile() == "failed"


def test_amdsmi_partition_backend_maps_bdf(tmp_path):
    from fakes.amdsmi_partition import FakeAmdSmiPartitionable
    from k8s_nvidia_gpus_amd.operator.partition_amdsmi import AmdSmiPartitionBackend

    fake = FakeAmdSmiPartitionable()
    root = fake_sysfs.build_node(tmp_path / "r")
    dev = read_topology(str(root), 90500).gpus[5]
    AmdSmiPartitionBackend(fake).set_compute(dev, "CPX")
    h = [fake.amdsmi_get_gpu_device_bdf(i) for i in range(8)].index(dev.pci_bdf)
    assert fake.calls == [("compute", h, "CPX")]


def test_pod_gpu_request():
    assert pod_gpu_request({"spec": {"containers": [
        {"resources": {"limits": {"amd.com/gpu": "2"}}}, {"resources": {"requests": {"amd.com/gpu": 1}}}]}}) == 3


# ----------------------------------------------------------------------------- runtime / CDI
def test_cdi_spec_and_runtime_install(tmp_path):
    root = fake_sysfs.build_node(tmp_path / "r", compute_partition="CPX")
    src = tmp_path / "amd-container-runtime"
    src.write_bytes(b"#!/bin/sh\nexit 0\n")
    dst = tmp_path / "host/usr/local/bin/amd-container-runtime"
    info = rt.install_runtime(str(src), str(dst), str(tmp_path / "cdi"), str(tmp_path / "m"), str(root))
    assert os.access(dst, os.X_OK) and info["updated"]
    spec = json.loads((tmp_path / "cdi" / rt.CDI_FILE).read_text())
    assert spec["kind"] == "amd.com/gpu" and spec["cdiVersion"] == "0.6.0"
    assert len(spec["devices"]) == 65  # 64 CPX partitions + "all"
    assert spec["containerEdits"]["deviceNodes"] == [{"path": "/dev/kfd", "permissions": "rw"}]
    names = {d["name"] for d in spec["devices"]}
    assert "all" in names and all(n == "all" or "-p" in n for n in names)
    assert (tmp_path / "m" / "runtime-ready").exists()
    assert rt.install_runtime(str(src), str(dst), str(tmp_path / "cdi"), str(tmp_path / "m"), str(root))["updated"] is False


def test_wait_markers(tmp_path):
    m = tmp_path / "x-ready"
    assert rt.wait_markers([str(m)], timeout=0.05, poll=0.01) is False
    threading.Timer(0.05, lambda: m.write_text("1")).start()
    assert rt.wait_markers([str(m)], timeout=5, poll=0.01) is True


def test_cli_topology_and_cdi(tmp_path):
    root = fake_sysfs.build_node(tmp_path / "r")
    env = dict(os.environ, PYTHONPATH=str(REPO))
    out = subprocess.run([sys.executable, "-m", "k8s_nvidia_gpus_amd.operator", "topology",
                          "--root", str(root), "--config", "/nonexistent"], capture_output=True,
                         text=True, env=env, check=True).stdout
    doc = json.loads(out)
    assert len(doc["gpus"]) == 8 and doc["cpu_nodes"] == 2
    out = subprocess.run([sys.executable, "-m", "k8s_nvidia_gpus_amd.operator", "cdi",
                          "--root", str(root), "--config", "/nonexistent"], capture_output=True,
                         text=True, env=env, check=True).stdout
    assert json.loads(out)["kind"] == "amd.com/gpu"


def test_driver_module_loading(tmp_path):
    calls = []
    dev = tmp_path / "dev"
    dev.mkdir()
    host = tmp_path / "host"
    host.mkdir()
    runner = lambda argv: (calls.append(argv) or (0, ""))  # noqa: E731
    assert rt.ensure_module(str(dev), str(host), runner) is True
    assert calls == [["chroot", str(host), "modprobe", "amdgpu"]]
    (dev / "kfd").write_text("")
    assert rt.ensure_module(str(dev), str(host), runner) is None  # driver already up
    os.unlink(dev / "kfd")
    assert rt.ensure_module(str(dev), str(host), lambda a: (1, "FATAL: Module amdgpu not found")) is False


def test_validator_gemm_step_under_rocprof(tmp_path):
    from k8s_nvidia_gpus_amd.operator.validator import Validator

    prof = Path(__file__).resolve().parent.parent / "profiles"
    logs = {"bf16": (prof / "r01_gemm_validator.log").read_text(),
            "fp8": (prof / "r01_gemm_validator_fp8.log").read_text()}
    kernels = {"bf16": "amdk8s_gemm_bf16_nt_256x256", "fp8": "amdk8s_gemm_fp8_nt_256x256"}
    seen = []

    def runner(argv, timeout):
        seen.append(argv)
        dtype = argv[argv.index("--dtype") + 1] if "--dtype" in argv else "bf16"
        d = Path(argv[argv.index("-d") + 1]) / "run"
        d.mkdir(parents=True)
        (d / "gemm_kernel_stats.csv").write_text(
            '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
            f'"{kernels[dtype]}",60,47700000,795000.0,98.9,782807,1030849,66849.2\n')
        return 0, logs[dtype]

    cfg = load_config(text="validator: {rocprof: true, podResourcesRequired: false}\n")
    # the profiled GEMMs are the profile step's (after the gate); the gate step runs them plain
    r = Validator(cfg, str(tmp_path), bin_dir="/b", runner=runner).run_step("profile")
    assert r.passed and seen[0][:3] == ["rocprofv3", "--kernel-trace", "--stats"]
    assert r.detail["rocprof_kernels"][0]["name"] == "amdk8s_gemm_bf16_nt_256x256"
    assert r.detail["fp8"]["rocprof_kernels"][0]["name"] == "amdk8s_gemm_fp8_nt_256x256"


class PerAsicPartitionBackend:
    """Switches ONE ASIC per call (what the driver does per PCI device); can fail on one ASIC."""

    def __init__(self, root, n_gpus=8, fail_on=None):
        self.root, self.n, self.fail_on = root, n_gpus, fail_on
        self.applied = []
        self.bdfs = [g["bdf"] for g in fake_sysfs.LAYOUT["gpus"][:n_gpus]]
        self.fail_bdf = sorted(self.bdfs)[fail_on] if fail_on is not None else None
        topo = read_topology(str(root), 90500)
        by_bdf = {m[0].pci_bdf: m[0] for m in topo.asics().values()}
        self.modes = [by_bdf[b].compute_partition for b in self.bdfs]
        self.mems = [by_bdf[b].memory_partition for b in self.bdfs]

    def set_memory(self, dev, mode):
        self.mems[self.bdfs.index(dev.pci_bdf)] = mode
        self.applied.append(("memory", dev.pci_bdf, mode))

    def set_compute(self, dev, mode):
        a = self.bdfs.index(dev.pci_bdf)
        if dev.pci_bdf == self.fail_bdf:    # "ASIC 3" = 4th by PCI bus
            raise OSError(f"amdsmi: device {dev.pci_bdf} busy")
        self.modes[a] = mode
        self.applied.append(("compute", dev.pci_bdf, mode))
        fake_sysfs.set_partition(self.root, self.n, list(self.modes), list(self.mems))


def test_partition_failure_mid_node_is_mixed_and_reconverges_per_asic(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    api.nodes["gpu-node-1"]["metadata"]["labels"][pm.LABEL_DESIRED] = "CPX"
    kw = dict(poll=0.01, pause_marker=str(tmp_path / "p"), sleep=lambda s: None, reenum_timeout=0.2,
              ack_components=())
    bad = PerAsicPartitionBackend(root, fail_on=3)
    assert pm.PartitionManager(client, "gpu-node-1", bad, str(root), **kw).reconcile() == "failed"
    state = api.nodes["gpu-node-1"]["metadata"]["annotations"][pm.ANNOT_STATE]
    assert "after 3 of 8 ASIC(s) switched" in state
    # the node is half CPX, half SPX: reported as mixed, not as the head GPU's CPX
    mgr = pm.PartitionManager(client, "gpu-node-1", PerAsicPartitionBackend(root), str(root), **kw)
    c, m, topo = mgr.current()
    assert (c, m) == ("mixed", "NPS1") and len(topo.gpus) == 3 * 8 + 5
    assert compute_labels(str(root))["amd.com/gpu.compute-partition"] == "mixed"
    # the next reconcile switches only the 5 ASICs still in SPX
    assert mgr.reconcile() == "applied"
    assert len([a for a in mgr.backend.applied if a[0] == "compute"]) == 5
    assert len(read_topology(str(root), 90500).gpus) == 64
    assert compute_labels(str(root))["amd.com/gpu.compute-partition"] == "CPX"
    assert mgr.reconcile() == "idle"


def test_labeller_pci_present_without_driver_and_not_on_cpu_nodes(tmp_path):
    import shutil

    root = fake_sysfs.build_node(tmp_path / "gpu")
    shutil.rmtree(root / "sys/class/kfd")          # amdgpu not loaded yet: no KFD topology
    labels = compute_labels(str(root))
    assert labels["amd.com/gpu.pci-present"] == "true" and labels["amd.com/gpu.present"] is None
    cpu = tmp_path / "cpu"
    fake_sysfs.add_cpu_only_pci(cpu)                # BMC VGA (ASPEED), no AMD device
    assert all(v is None for v in compute_labels(str(cpu)).values())
    # a CPU worker with an AMD Radeon (display class) must not get the driver DaemonSet
    radeon = tmp_path / "radeon"
    fake_sysfs.add_cpu_only_pci(radeon, bdf="0000:03:00.0", vendor="0x1002", cls="0x030000",
                                device="0x744c")   # Radeon RX 7900 XTX
    assert compute_labels(str(radeon))["amd.com/gpu.pci-present"] is None
    # an older Instinct (MI300X, gfx942: class 0x12) is below minGfxTargetVersion gfx950
    mi300 = tmp_path / "mi300"
    fake_sysfs.add_cpu_only_pci(mi300, bdf="0000:05:00.0", vendor="0x1002", cls="0x120000",
                                device="0x74a1")
    assert compute_labels(str(mi300))["amd.com/gpu.pci-present"] is None
    assert compute_labels(str(mi300), min_gfx=90402)["amd.com/gpu.pci-present"] == "true"
    # an MI355X (0x75a3) on the bus, driver not loaded yet
    mi355 = tmp_path / "mi355"
    fake_sysfs.add_cpu_only_pci(mi355, bdf="0000:05:00.0", vendor="0x1002", cls="0x120000",
                                device="0x75a3")
    assert compute_labels(str(mi355))["amd.com/gpu.pci-present"] == "true"
