"""Validator chain: gating logic on the REAL outputs the native tools produced on an MI355X.

tests/fixtures/native_logs/ (copies of profiles/r01_vectoradd.log, r01_gemm_validator*.log and
profiles/r02_session1/proftester_all.log) are the stdout of native/bin/
amd-vectoradd and amd-gemm-validator from the first gpurun session; the driver step runs the real
kfd-probe binary (host C++, built here) against a fabricated MI355X sysfs tree.
"""
import json
import os
import subprocess
from pathlib import Path

import pytest

from fakes import sysfs as fake_sysfs
from fakes.kubeapi import FakeKubeAPI
from k8s_nvidia_gpus_amd.ops import build as B
from k8s_nvidia_gpus_amd.operator.config import load_config
from k8s_nvidia_gpus_amd.operator.validator import (Validator, json_lines, protocol_passed)
from k8s_nvidia_gpus_amd.utils.kube import KubeClient

REPO = Path(__file__).resolve().parent.parent
VECTORADD_LOG = (REPO / "tests/fixtures/native_logs/r01_vectoradd.log").read_text()
GEMM_LOG = (REPO / "tests/fixtures/native_logs/r01_gemm_validator.log").read_text()
GEMM_FP8_LOG = (REPO / "tests/fixtures/native_logs/r01_gemm_validator_fp8.log").read_text()
# stdout of native/bin/amd-proftester --json on one MI355X (round 2, session 1)
PROFTESTER_LOG = (REPO / "tests/fixtures/native_logs/proftester_all.log").read_text()


def _pt_line(test, device, value, peer=-1, engine="", passed=True, skipped=False):
    return json.dumps({"check": "proftester", "test": test, "device": device, "peer": peer,
                       "engine": engine, "value": value, "min": value, "max": value, "unit": "GB/s",
                       "seconds": 0.01, "skipped": skipped, "passed": passed, "note": ""})
RCCL_8GPU = """# rccl-allreduce-bench: 8 GPU(s), RCCL 22703, in-place float sum, 20 iters
{"check": "rccl_allreduce", "ngpus": 8, "peak_busbw_gbps": 301.20, "peak_algbw_gbps": 172.11, "peak_bytes": 1073741824, "wrong": 0, "passed": true}
Test PASSED
Done
"""


class Runner:
    def __init__(self, outputs):
        self.outputs = outputs
        self.calls = []

    def __call__(self, argv, timeout):
        self.calls.append(list(argv))
        if argv and argv[0] == "env":   # ROCR_VISIBLE_DEVICES=... narrowing (GPU scope)
            argv = argv[1:]
            while argv and "=" in argv[0]:
                argv = argv[1:]
        name = os.path.basename(argv[0])
        if "--dtype" in argv:  # e.g. "amd-gemm-validator:fp8"
            name += ":" + argv[argv.index("--dtype") + 1]
        rc, out = self.outputs[name]
        return rc, out


@pytest.fixture
def cfg():
    return load_config(text="expectedGpusPerNode: 1\nvalidator: {podResourcesRequired: false, gemmMinTflops: 900, rcclMinBusbwGBps: 100}\n")


def test_protocol_parser():
    assert protocol_passed(VECTORADD_LOG)
    assert not protocol_passed("Test FAILED\nDone\n")
    assert not protocol_passed("Test PASSED\n")  # no Done
    assert len(json_lines(GEMM_LOG)) == 1


def test_vectoradd_and_gemm_steps_on_real_outputs(tmp_path, cfg):
    r = Runner({"amd-vectoradd": (0, VECTORADD_LOG), "amd-gemm-validator": (0, GEMM_LOG),
                "amd-gemm-validator:fp8": (0, GEMM_FP8_LOG)})
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=r)
    va = v.run_step("vectoradd")
    assert va.passed and va.detail["devices"][0]["elements"] == 50000
    g = v.run_step("gemm")
    assert g.passed
    assert g.detail["devices"][0]["tflops"] > 1300
    assert (tmp_path / "gemm-ready").exists()
    assert json.loads((tmp_path / "gemm.json").read_text())["aggregate_tflops"] > 1300
    assert r.calls[1][:3] == ["/x/amd-gemm-validator", "--size", "8192"]


def test_report_carries_per_step_durations(tmp_path):
    """Every step records its wall time; the report sums the required ones (time-to-validated)."""
    cfg = load_config(text="expectedGpusPerNode: 1\nvalidator: {podResourcesRequired: false, gemmMinTflops: 900, rccl: false, "
                           "pluginTest: false}\n")
    r = Runner({"amd-vectoradd": (0, VECTORADD_LOG), "amd-gemm-validator": (0, GEMM_LOG),
                "amd-gemm-validator:fp8": (0, GEMM_FP8_LOG), "amd-proftester": (0, PROFTESTER_LOG)})
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=r)
    for st in ("driver", "runtime"):  # markers as the driver/runtime agents publish them
        (tmp_path / f"{st}.json").write_text(json.dumps({"step": st, "passed": True, "duration_s": 1.5}))
        (tmp_path / f"{st}-ready").write_text("0\n")
    assert v.run_step("vectoradd").detail["duration_s"] >= 0
    assert v.run_step("gemm").passed
    assert v.run_step("bandwidth").passed
    rep = v.run_step("report")
    assert rep.passed
    steps = rep.detail["step_seconds"]
    assert set(steps) >= {"driver", "runtime", "vectoradd", "gemm", "bandwidth"}
    assert rep.detail["chain_seconds"] == pytest.approx(sum(steps.values()), abs=1e-3)
    assert json.loads((tmp_path / "report.json").read_text())["chain_seconds"] >= 3.0


def test_gemm_step_enforces_tflops_floor(tmp_path):
    cfg = load_config(text="validator: {podResourcesRequired: false, gemmMinTflops: 2000}\n")
    v = Validator(cfg, str(tmp_path), bin_dir="/x",
                  runner=Runner({"amd-gemm-validator": (0, GEMM_LOG),
                                 "amd-gemm-validator:fp8": (0, GEMM_FP8_LOG)}))
    g = v.run_step("gemm")
    assert not g.passed and "below 2000" in g.reason
    assert not (tmp_path / "gemm-ready").exists()


def test_gemm_step_fails_on_numerics(tmp_path, cfg):
    bad = GEMM_LOG.replace('"passed": true', '"passed": false').replace("Test PASSED", "Test FAILED")
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=Runner({
        "amd-gemm-validator": (1, bad), "amd-gemm-validator:fp8": (0, GEMM_FP8_LOG)}))
    assert not v.run_step("gemm").passed


def test_rccl_step(tmp_path, cfg):
    v = Validator(cfg, str(tmp_path), bin_dir="/x",
                  runner=Runner({"rccl-allreduce-bench": (0, RCCL_8GPU)}))
    r = v.step_rccl(8)
    assert r.passed and r.detail["peak_busbw_gbps"] == pytest.approx(301.2)
    assert v.step_rccl(1).passed  # single GPU: skipped
    wrong = RCCL_8GPU.replace('"wrong": 0, "passed": true', '"wrong": 12, "passed": false')
    v2 = Validator(cfg, str(tmp_path), bin_dir="/x",
                   runner=Runner({"rccl-allreduce-bench": (1, wrong)}))
    assert not v2.step_rccl(8).passed


@pytest.mark.skipif(not B.toolchain_available(), reason="needs the native build")
def test_driver_step_runs_real_kfd_probe(tmp_path):
    B.build_native(only=["kfd-probe"])
    root = fake_sysfs.build_node(tmp_path / "r")
    cfg = load_config(text="expectedGpusPerNode: 8\n")
    v = Validator(cfg, str(tmp_path / "m"), bin_dir=str(B.NATIVE_BIN), root=str(root))
    r = v.run_step("driver")
    assert r.passed, r.reason
    assert r.detail["gpus"] == 8 and len(r.detail["agents"]) == 8
    assert {a["render_minor"] for a in r.detail["agents"]} == set(range(128, 192, 8))
    # one GPU falls off the bus → driver step fails, marker withdrawn
    fake_sysfs.remove_gpu(root, 2)
    cfg9 = load_config(text="expectedGpusPerNode: 8\n")
    v9 = Validator(cfg9, str(tmp_path / "m"), bin_dir=str(B.NATIVE_BIN), root=str(root))
    v9.run_cmd = lambda argv, t: _no_wait(argv, t)
    r2 = v9.run_step("driver")
    assert not r2.passed and "expected 8" in r2.reason
    assert not (tmp_path / "m" / "driver-ready").exists()


def _no_wait(argv, timeout):
    argv = [a for a in argv]
    i = argv.index("--wait")
    argv[i + 1] = "0"
    p = subprocess.run(argv, capture_output=True, text=True)
    return p.returncode, p.stdout + p.stderr


@pytest.mark.skipif(not B.toolchain_available(), reason="needs the native build")
def test_kfd_probe_cpx_counts_partitions(tmp_path):
    B.build_native(only=["kfd-probe"])
    root = fake_sysfs.build_node(tmp_path / "r", compute_partition="CPX")
    p = subprocess.run([str(B.NATIVE_BIN / "kfd-probe"), "--sysfs-root",
                        str(root / "sys/class/kfd/kfd/topology"), "--dev-root", str(root / "dev"),
                        "--no-open", "--expect-gpus", "64"], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    doc = json.loads(p.stdout)
    assert doc["gpus"] == 64 and {a["cu"] for a in doc["agents"]} == {32}
    assert {a["num_xcc"] for a in doc["agents"]} == {1}


def test_plugin_step_schedules_a_gpu_pod(tmp_path, cfg, monkeypatch):
    api = FakeKubeAPI().start()
    api.add_node("gpu-node-1")
    api.pods[("amd-gpu-operator", "validator-xyz")] = {
        "metadata": {"name": "validator-xyz", "namespace": "amd-gpu-operator"},
        "spec": {"nodeName": "gpu-node-1", "initContainers": [
            {"name": "driver-validation", "image": "ghcr.io/example-org/amd-gpu-operator:9.9.9"}],
            "containers": []},
        "status": {"phase": "Running"}}
    created = []

    def kubelet(a, pod):  # play kubelet: the pod ran and printed the reference protocol
        created.append(pod)
        pod["status"]["phase"] = "Succeeded"
        a.logs[("amd-gpu-operator", pod["metadata"]["name"])] = VECTORADD_LOG

    api.on_pod_created = kubelet
    monkeypatch.setenv("POD_NAME", "validator-xyz")
    monkeypatch.setenv("POD_NAMESPACE", "amd-gpu-operator")
    try:
        v = Validator(cfg, str(tmp_path), kube=KubeClient(base_url=api.url), node_name="gpu-node-1")
        r = v.run_step("plugin")
        assert r.passed, r.reason
        (pod,) = created
        c = pod["spec"]["containers"][0]
        assert c["resources"]["limits"] == {"amd.com/gpu": "1"}
        assert c["image"] == "ghcr.io/example-org/amd-gpu-operator:9.9.9"
        assert pod["spec"]["runtimeClassName"] == "amd" and pod["spec"]["nodeName"] == "gpu-node-1"
        assert ("amd-gpu-operator", pod["metadata"]["name"]) not in api.pods  # cleaned up
        # report: label the node
        for s in ("driver", "runtime", "vectoradd", "gemm", "bandwidth", "rccl"):
            (tmp_path / f"{s}-ready").write_text("1")
        rep = v.run_step("report")
        assert rep.passed and api.nodes["gpu-node-1"]["metadata"]["labels"]["amd.com/gpu.validated"] == "true"
        assert (tmp_path / "validator-ready").exists()
        os.unlink(tmp_path / "gemm-ready")
        rep2 = v.run_step("report")
        assert not rep2.passed and "gemm" in rep2.reason
        assert api.nodes["gpu-node-1"]["metadata"]["labels"]["amd.com/gpu.validated"] == "false"
    finally:
        api.stop()


def test_gemm_step_runs_fp8_on_real_output(tmp_path, cfg):
    """The fp8 half of the GEMM step: parsed from the native validator's real MI355X output,
    reported next to bf16, and held to its own floor."""
    r = Runner({"amd-gemm-validator": (0, GEMM_LOG), "amd-gemm-validator:fp8": (0, GEMM_FP8_LOG)})
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=r)
    g = v.run_step("gemm")
    assert g.passed, g.reason
    assert r.calls[-1][-2:] == ["--dtype", "fp8"]
    d = json.loads((tmp_path / "gemm.json").read_text())
    assert d["fp8"]["aggregate_tflops"] > 2 * 1300
    assert d["fp8"]["devices"][0]["check"] == "gemm_fp8"

    strict = load_config(text="validator: {podResourcesRequired: false, gemmFp8MinTflops: 10000}\n")
    v2 = Validator(strict, str(tmp_path / "s"), bin_dir="/x", runner=r)
    g2 = v2.run_step("gemm")
    assert not g2.passed and "fp8" in g2.reason


def test_gemm_step_fp8_can_be_disabled(tmp_path):
    cfg = load_config(text="validator: {podResourcesRequired: false, gemmFp8: false}\n")
    r = Runner({"amd-gemm-validator": (0, GEMM_LOG)})  # no fp8 output available: must not be run
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=r)
    assert v.run_step("gemm").passed
    assert len(r.calls) == 1 and "fp8" not in json.loads((tmp_path / "gemm.json").read_text())


class _PendingKube:
    """A kube client whose validation pod never leaves Pending (0 devices advertised)."""

    def __init__(self):
        self.deleted = []

    def get_pod(self, ns, name):
        return {"spec": {"containers": [{"image": "img:1"}]}}

    def delete_pod(self, ns, name):
        self.deleted.append(name)

    def create_pod(self, ns, pod):
        pass

    def wait_pod_phase(self, ns, name, timeout=600.0, **kw):
        raise TimeoutError(f"pod {ns}/{name} not in ('Succeeded', 'Failed') (phase Pending)")

    def pod_logs(self, ns, name):
        return ""

    def set_node_labels(self, node, labels):
        self.labels = labels


def test_step_that_raises_is_recorded_as_failed_and_withdraws_markers(tmp_path, cfg):
    """a plugin pod stuck in Pending used to escape run_step, leaving the previous
    plugin.json / plugin-ready (hostPath, survives restarts) and the node label untouched."""
    kube = _PendingKube()
    v = Validator(cfg, str(tmp_path), kube=kube, node_name="gpu-node-1")
    (tmp_path / "plugin-ready").write_text("stale\n")
    (tmp_path / "plugin.json").write_text(json.dumps({"step": "plugin", "passed": True}))
    r = v.run_step("plugin")
    assert not r.passed and "TimeoutError" in r.reason
    assert not (tmp_path / "plugin-ready").exists()
    rec = json.loads((tmp_path / "plugin.json").read_text())
    assert rec["passed"] is False and rec["exception"] == "TimeoutError" and "duration_s" in rec
    assert kube.deleted  # the pod was still cleaned up
    # the report then fails the node instead of keeping the old pass
    for s in ("driver", "runtime", "vectoradd", "gemm", "bandwidth", "rccl"):
        (tmp_path / f"{s}-ready").write_text("1")
    rep = v.run_step("report")
    assert not rep.passed and "plugin" in rep.detail["missing"]
    assert kube.labels == {"amd.com/gpu.validated": "false"}


def test_unknown_step_still_raises(tmp_path, cfg):
    with pytest.raises(ValueError):
        Validator(cfg, str(tmp_path)).run_step("nope")


def test_report_lists_required_steps_without_duration(tmp_path):
    """chain_seconds must not silently treat an untimed required step as 0 s."""
    cfg = load_config(text="expectedGpusPerNode: 1\nvalidator: {podResourcesRequired: false, rccl: false, pluginTest: false, "
                           "gemm: false, vectorAdd: false, bandwidth: false}\n")
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=Runner({}))
    (tmp_path / "driver.json").write_text(json.dumps({"step": "driver", "passed": True, "duration_s": 2.0}))
    for st in ("driver", "runtime"):
        (tmp_path / f"{st}-ready").write_text("0\n")   # runtime marker without runtime.json timing
    rep = v.run_step("report")
    assert rep.passed
    assert rep.detail["step_seconds"] == {"driver": 2.0}
    assert rep.detail["step_seconds_missing"] == ["runtime"]
    assert rep.detail["chain_complete"] is False


# ----------------------------------------------------------------------------- bandwidth step
def test_bandwidth_step_on_real_mi355x_output(tmp_path, cfg):
    r = Runner({"amd-proftester": (0, PROFTESTER_LOG)})
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=r)
    b = v.run_step("bandwidth")
    assert b.passed, b.reason
    argv = r.calls[0]
    assert argv[0] == "/x/amd-proftester" and argv[-1] == "--json"
    assert set(argv[argv.index("-t") + 1].split(",")) == {"hbm-copy", "pcie-h2d", "pcie-d2h", "xgmi"}
    summary = b.detail["min_by_test_gbps"]
    assert summary["hbm-copy"] > 4000 and summary["pcie-h2d"] > 20
    assert "xgmi-sdma" not in summary  # one GPU: the xGMI test is skipped, not failed
    assert (tmp_path / "bandwidth-ready").exists()


def test_bandwidth_step_enforces_floors(tmp_path):
    cfg = load_config(text="validator: {podResourcesRequired: false, hbmMinGBps: 9000}\n")
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=Runner({"amd-proftester": (0, PROFTESTER_LOG)}))
    b = v.run_step("bandwidth")
    assert not b.passed and "hbm-copy dev 0" in b.reason and "< 9000" in b.reason
    assert not (tmp_path / "bandwidth-ready").exists()


def test_bandwidth_step_gates_every_sdma_xgmi_pair(tmp_path, cfg):
    """Synthetic 2-GPU output (no 2-GPU box in this pool): one slow SDMA pair fails the node; the
    copy-kernel pulls and the all-peer aggregate are reported but not gated."""
    lines = [_pt_line("hbm-copy", d, 5200.0) for d in (0, 1)]
    lines += [_pt_line(t, d, 56.0, engine="sdma") for t in ("pcie-h2d", "pcie-d2h") for d in (0, 1)]
    lines += [_pt_line("xgmi", 1, 48.0, peer=0, engine="sdma"), _pt_line("xgmi", 0, 12.0, peer=1, engine="sdma"),
              _pt_line("xgmi", 1, 5.0, peer=0, engine="kernel"), _pt_line("xgmi", 0, 90.0, engine="kernel-all-peers")]
    out = "\n".join(lines) + "\nTest PASSED\nDone\n"
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=Runner({"amd-proftester": (0, out)}))
    b = v.run_step("bandwidth")
    assert not b.passed and "xgmi dev 0<-1 12.0 < 30" in b.reason
    assert "dev 1<-0" not in b.reason  # the slow copy-kernel pull is not gated
    assert b.detail["min_by_test_gbps"]["xgmi-sdma"] == 12.0


def test_bandwidth_step_fails_on_failed_copy_and_missing_tests(tmp_path, cfg):
    out = _pt_line("hbm-copy", 0, 5200.0, passed=False) + "\nTest FAILED\n"
    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=Runner({"amd-proftester": (1, out)}))
    b = v.run_step("bandwidth")
    assert not b.passed and "1 check(s) failed" in b.reason and "pcie-h2d" in b.reason


def test_exporter_publishes_bandwidth_results(tmp_path, cfg):
    from prometheus_client import generate_latest

    from k8s_nvidia_gpus_amd.operator import exporter as ex

    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=Runner({"amd-proftester": (0, PROFTESTER_LOG)}))
    assert v.run_step("bandwidth").passed
    col = ex.GpuCollector(ex.SysfsBackend(str(tmp_path / "nosys")), "node-a", str(tmp_path))  # no GPUs
    text = generate_latest(ex.make_registry(col)).decode()
    assert 'amd_gpu_validator_bandwidth_gbps{engine="",gpu="0",node="node-a",peer="",test="hbm-copy"}' in text
    assert 'test="pcie-h2d"' in text and 'amd_gpu_validation_passed{node="node-a",step="bandwidth"} 1.0' in text


# ----------------------------------------------------------------------------- rocprof counters
PMC_DIR = REPO / "tests/fixtures/pmc_validator"   # copy of profiles/r02_session2/pmc_validator


def test_rocprof_counter_summary_on_real_mi355x_csv():
    from k8s_nvidia_gpus_amd.operator.validator import rocprof_counter_summary

    s = rocprof_counter_summary(str(PMC_DIR), cus=256)
    assert s["dispatches"] >= 80  # settle + warmup + timed launches of the 8192³ GEMM
    assert s["mfma_flop"] == 2.0 * 8192 ** 3  # the hardware counted exactly the requested GEMM
    assert 1.5 < s["clock_ghz"] < 2.4 and 70 < s["mfma_util_pct"] < 100 and 60 < s["l2_hit_pct"] < 100
    assert 1300 < s["tflops_profiled"] < 2000


def test_profile_step_runs_a_counter_pass(tmp_path):
    import shutil

    cfg = load_config(text="validator: {podResourcesRequired: false, gemmMinTflops: 900, rocprofCounters: true, gemmFp8: false}\n")
    gemm_log = GEMM_LOG.replace('"arch": "gfx950:sramecc+:xnack-", ', '"arch": "gfx950:sramecc+:xnack-", "cus": 256, ')
    calls = []

    def runner(argv, timeout):
        calls.append(list(argv))
        if argv[0] == "rocprofv3":
            assert "--pmc" in argv and "--sys-trace" not in argv  # counters never share a traced run
            d = argv[argv.index("-d") + 1]
            shutil.copytree(PMC_DIR, d)
            return 0, (PMC_DIR / "pmc.log").read_text()
        return 0, gemm_log

    v = Validator(cfg, str(tmp_path), bin_dir="/x", runner=runner)
    g = v.run_step("gemm")
    assert g.passed, g.reason and "rocprof_counters" not in g.detail    # the gate step runs plain
    assert all(c[0] != "rocprofv3" for c in calls)
    g = v.run_step("profile")
    assert g.passed, g.reason
    rc = g.detail["rocprof_counters"]
    assert rc["flop_matches_shape"] is True and rc["mfma_util_pct"] > 70
    pmc = calls[-1]
    assert pmc[pmc.index("--pmc") + 1:pmc.index("-d")] == ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES",
                                                           "SQ_INSTS_VALU_MFMA_MOPS_BF16", "GRBM_GUI_ACTIVE",
                                                           "TCC_HIT_sum", "TCC_MISS_sum"]

    from prometheus_client import generate_latest

    from k8s_nvidia_gpus_amd.operator import exporter as ex

    col = ex.GpuCollector(ex.SysfsBackend(str(tmp_path / "nosys")), "n1", str(tmp_path))
    text = generate_latest(ex.make_registry(col)).decode()
    assert 'amd_gpu_validator_gemm_profile{node="n1",quantity="mfma_util_pct"}' in text


# ----------------------------------------------------------------------------- stress step
def _stress_out(rows):
    lines = [json.dumps({"check": "proftester", "test": "tensor", "device": d, "peer": -1, "engine": "",
                         "value": mean, "min": lo, "max": hi, "unit": "TFLOPS", "seconds": 30.1,
                         "skipped": False, "passed": True, "note": ""}) for d, mean, lo, hi in rows]
    return "[amd-proftester: sustained load]\n" + "\n".join(lines) + "\nTest PASSED\nDone\n"


class Telemetry:
    """Synthetic amd-smi samples (exporter GpuSample keys); ``ecc_step`` adds uncorrectable errors."""

    def __init__(self, n=2, hotspot=78.0, ecc_step=0):
        self.n, self.hot, self.ecc_step, self.calls = n, hotspot, ecc_step, 0

    def __call__(self):
        self.calls += 1
        return [{"index": i, "temp_hotspot": self.hot + i, "power_w": 1390.0, "gfxclk_mhz": 1900.0,
                 "ecc_uncorrectable": float(self.ecc_step * self.calls if i == 1 else 0),
                 "ecc_correctable": 3.0} for i in range(self.n)]


def _stress_validator(tmp_path, out, tel, rc=0):
    cfg = load_config(text="validator: {podResourcesRequired: false, stress: true, stressSeconds: 0.3}\n")

    def runner(argv, timeout):
        import time as _t

        assert argv[1:5] == ["-t", "tensor", "--duration", "0.3"]
        _t.sleep(0.3)  # the load runs while telemetry is sampled
        return rc, out

    return Validator(cfg, str(tmp_path), bin_dir="/x", runner=runner, telemetry=tel)


def test_stress_step_passes_under_steady_load(tmp_path):
    tel = Telemetry()
    v = _stress_validator(tmp_path, _stress_out([(0, 1650.0, 1601.0, 1702.0), (1, 1640.0, 1590.0, 1690.0)]), tel)
    r = v.run_step("stress")
    assert r.passed, r.reason
    g = r.detail["gpus"]
    assert g["0"]["tflops_min_window"] == 1601.0 and g["1"]["hotspot_max_c"] == 79.0
    assert g["0"]["ecc_uncorrectable_delta"] == 0 and g["0"]["power_mean_w"] == 1390.0
    assert r.detail["telemetry_samples"] >= 1 and (tmp_path / "stress-ready").exists()


@pytest.mark.parametrize("case,needle", [
    ("cliff", "GPU 1: 100 ms window 900 < 0.85"),
    ("ecc", "GPU 1: "),
    ("hot", "hotspot 111 C > 105 C"),
])
def test_stress_step_fails_on_throttle_ecc_or_heat(tmp_path, case, needle):
    rows = [(0, 1650.0, 1601.0, 1702.0), (1, 1640.0, 900.0 if case == "cliff" else 1590.0, 1690.0)]
    tel = Telemetry(hotspot=110.0 if case == "hot" else 78.0, ecc_step=1 if case == "ecc" else 0)
    r = _stress_validator(tmp_path, _stress_out(rows), tel).run_step("stress")
    assert not r.passed and needle in r.reason, r.reason
    if case == "ecc":
        assert "uncorrectable ECC error(s) under load" in r.reason
