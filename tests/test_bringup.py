"""Node bring-up rehearsal (operator/bringup.py) on CPU: the real kfd-probe and runtime shim against
a fabricated 8 × MI355X sysfs/dev tree, the real device plugin over unix-socket gRPC, and recorded
MI355X outputs for the GPU tools. The same code runs on the GPU box (test_operator_gpu.py)."""
import json
import os
import sys
from pathlib import Path

import pytest

from fakes import sysfs as fake_sysfs
from k8s_nvidia_gpus_amd.ops import build as B
from k8s_nvidia_gpus_amd.operator import bringup
from k8s_nvidia_gpus_amd.operator.config import load_config
from k8s_nvidia_gpus_amd.operator.validator import default_runner

REPO = Path(__file__).resolve().parent.parent
LOGS = {
    "amd-vectoradd": (REPO / "tests/fixtures/native_logs/r01_vectoradd.log").read_text(),
    "amd-gemm-validator": (REPO / "tests/fixtures/native_logs/r01_gemm_validator.log").read_text(),
    "amd-gemm-validator:fp8": (REPO / "tests/fixtures/native_logs/r01_gemm_validator_fp8.log").read_text(),
    "amd-proftester": (REPO / "tests/fixtures/native_logs/proftester_all.log").read_text(),
    "rccl-allreduce-bench": '{"check": "rccl_allreduce", "ngpus": 8, "peak_busbw_gbps": 301.2, '
                            '"wrong": 0, "passed": true}\nTest PASSED\nDone\n',
}
CONTAINER_OK = [sys.executable, "-c", "print('Test PASSED'); print('Done')"]


@pytest.fixture(scope="module")
def bins():
    B.build_native(only=["kfd-probe", "amd-container-runtime"])
    return str(B.NATIVE_BIN)


def runner(argv, timeout):
    name = os.path.basename(argv[0])
    if name == "kfd-probe":
        return default_runner(argv, timeout)  # the real probe against the fake tree
    if "--dtype" in argv:
        name += ":" + argv[argv.index("--dtype") + 1]
    return 0, LOGS[name]


@pytest.mark.parametrize("gated", [True, False])
def test_rehearsal_reaches_first_pod_and_validated(tmp_path, bins, gated):
    """Gated (the shipped order): the plugin advertises nothing Healthy until the validator's
    vectorAdd and GEMM passed, the pod comes after them, the node-wide steps after the pod.
    Ungated: plugin → pod → the whole chain."""
    root = fake_sysfs.build_node(tmp_path / "node")
    cfg = load_config(text="expectedGpusPerNode: 8\nvalidator: {gateGraceSeconds: 0}\n")
    rep = bringup.rehearse(cfg, bins, workdir=str(tmp_path / "work"), root=str(root), runner=runner,
                           container_cmd=CONTAINER_OK, timeout=30, gated=gated)
    names = [s["name"] for s in rep["stages"]]
    pod = ["allocate", "create", "container", "validate"]
    if gated:
        assert names == ["driver", "runtime", "plugin", "vectoradd", "gemm", "allocatable"] + pod, rep
    else:
        assert names == ["driver", "runtime", "plugin"] + pod, rep
    assert rep["passed"] and rep["order"] == ("gated" if gated else "ungated"), rep
    st = {s["name"]: s for s in rep["stages"]}
    assert st["plugin"]["detail"]["advertised"] == 8 and st["plugin"]["detail"]["resource"] == "amd.com/gpu"
    assert st["plugin"]["detail"]["healthy"] == (0 if gated else 8)
    if gated:
        assert st["allocatable"]["detail"]["healthy"] == 8 and st["gemm"]["detail"]["validated_devices"] == 8
        assert "gemm" not in st["validate"]["detail"] and "bandwidth" in st["validate"]["detail"]
    nodes = st["create"]["detail"]["device_nodes"]
    assert nodes[0] == "/dev/dri/renderD" + st["allocate"]["detail"]["annotations"]["amd.com/gpu.render-minors"]
    assert nodes[1] == "/dev/kfd" and len(nodes) == 2  # exactly one GPU injected
    assert 0 < rep["time_to_first_gpu_pod_s"] <= rep["time_to_validated_s"]
    assert st["validate"]["detail"]["report"]["passed"]
    assert st["validate"]["detail"]["rccl"]["passed"]  # 8 GPUs: the node-local RCCL step ran
    # stages are contiguous and ordered
    for a, b in zip(rep["stages"], rep["stages"][1:]):
        assert a["end_s"] <= b["start_s"] + 1e-3
    json.dumps(rep)


def test_rehearsal_stops_at_the_failing_stage(tmp_path, bins):
    root = fake_sysfs.build_node(tmp_path / "node", n_gpus=4)
    cfg = load_config(text="expectedGpusPerNode: 8\n")  # the probe must see 8 → driver fails
    rep = bringup.rehearse(cfg, bins, workdir=str(tmp_path / "work"), root=str(root), runner=runner,
                           container_cmd=CONTAINER_OK, timeout=30, driver_wait=1)
    assert not rep["passed"] and [s["name"] for s in rep["stages"]] == ["driver"]
    assert rep["time_to_first_gpu_pod_s"] is None


def test_rehearsal_fails_when_the_pod_process_fails(tmp_path, bins):
    root = fake_sysfs.build_node(tmp_path / "node")
    cfg = load_config(text="expectedGpusPerNode: 8\n")
    bad = [sys.executable, "-c", "print('Test FAILED')"]
    rep = bringup.rehearse(cfg, bins, workdir=str(tmp_path / "work"), root=str(root), runner=runner,
                           container_cmd=bad, timeout=30, validate=False)
    assert not rep["passed"] and rep["stages"][-1]["name"] == "container"
    assert rep["stages"][-1]["detail"]["log_tail"] == ["Test FAILED"]
