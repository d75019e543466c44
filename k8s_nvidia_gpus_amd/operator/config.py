"""Operator configuration: one YAML document shared by every component.

The reference configures its GPU stack through Helm values of an external chart (reference
cluster-config/apps/gpu-operator/helmrelease.yaml:17-29) plus per-pod env.  Here the whole operator
reads one in-repo file (ConfigMap ``amd-gpu-operator-config`` → ``/etc/amd-gpu-operator/operator.yaml``,
cluster-config/apps/amd-gpu-operator/config.yaml); unknown keys are rejected so a typo cannot
silently fall back to a default.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import yaml

DEFAULTS: Dict[str, Any] = {
    "resourceName": "amd.com/gpu",
    "runtimeClass": "amd",
    "minGfxTargetVersion": 90500,
    "expectedGpusPerNode": 8,
    "deviceIdStrategy": "uuid",
    "allocation": {
        "mode": "deviceSpecs",       # deviceSpecs | cdi
        "cardNodes": False,          # also expose /dev/dri/card<N> (not needed by ROCm compute)
        "preferXgmiLocality": True,
    },
    "driver": {
        "loadModule": True,          # modprobe amdgpu (chroot into hostRoot) if /dev/kfd is missing
        "hostRoot": "/host",
    },
    "health": {
        "intervalSeconds": 10,
        "eccUncorrectableThreshold": 1,
    },
    "partition": {
        "compute": "SPX",
        "memory": "NPS1",
        "drainTimeoutSeconds": 600,
        # evict: GPU pods are evicted through the Eviction API (PodDisruptionBudgets honoured);
        # wait: only wait for them to finish
        "drainPolicy": "evict",
        # how long to wait for the exporter / driver probe / device plugin to release the GPUs
        "pauseAckSeconds": 60,
        # sysfs / amd-smi writes that find the device busy (EBUSY): retries, 1 s doubling backoff
        "applyRetries": 5,
    },
    "exporter": {
        "port": 9400,
        "intervalSeconds": 5,
    },
    "validator": {
        "vectorAdd": True,
        "gemm": True,
        "gemmSize": 8192,
        "gemmMinTflops": 900,
        "gemmFp8": True,             # also run the fp8 (OCP e4m3) MFMA GEMM
        "gemmFp8MinTflops": 1800,
        # profile step (after the gate): the GEMMs under rocprofv3 --kernel-trace --stats, and one
        # rocprofv3 --pmc pass (MFMA util, clock, L2 hit rate)
        "rocprof": False,
        "rocprofCounters": False,
        "bandwidth": True,           # amd-proftester: HBM copy, PCIe H2D/D2H, xGMI peer copies
        "hbmMinGBps": 4000,          # HBM3E copy (read + write bytes), per GPU
        "pcieMinGBps": 20,           # pinned host <-> device, each direction, per GPU
        "xgmiMinGBps": 30,           # each ordered GPU pair, SDMA peer copy (>= 2 GPUs)
        "stress": False,             # sustained MFMA load + amd-smi telemetry (DCGM diag level 3)
        "stressSeconds": 30,
        "stressMinFraction": 0.85,   # every 100 ms window >= this x the mean rate (no throttle cliffs)
        "stressMaxHotspotC": 105,
        "rccl": True,
        "rcclMinBusbwGBps": 100,
        "pluginTest": True,
        # GPUs kubelet has allocated to pods are never loaded: gemm / bandwidth / stress / rccl run
        # on the free ones only (kubelet PodResources API), and are deferred when none is free
        "podResourcesSocket": "/var/lib/kubelet/pod-resources/kubelet.sock",
        # an absent socket fails the load steps (a node cannot prove a GPU is free); false only for
        # runs outside Kubernetes (bring-up rehearsal on a bare box), where every agent is free
        "podResourcesRequired": True,
        # device plugin advertises a GPU Healthy only once the gate steps have passed on it this
        # boot (validated-devices.json), so pods cannot take GPUs before the first validation
        "gateOnValidation": True,
        # the per-device steps that open the gate (vectorAdd runs before them in the chain); the
        # node-wide steps (bandwidth pairs, stress, rccl) only decide the node label and run after
        # the gate opened — list them here too for the strict all-steps gate
        "gateSteps": ["gemm"],
        # node-wide steps start this long after the gate first opened this boot, so pods already
        # pending for the node get their GPUs before the steps reserve the free ones
        "gateGraceSeconds": 5,
        # the device plugin's registration socket: a load step whose reservation is not acked while
        # this socket accepts connections is deferred (never loads GPUs a live plugin may hand out)
        "pluginSocket": "/var/lib/kubelet/device-plugins/amd-gpu.sock",
        # load steps reserve their GPUs (in-test.json → the plugin reports them Unhealthy) and wait
        # this long for the plugin's ack before re-reading PodResources
        "reserveAckSeconds": 15,
        # the report container re-runs the chain when a deferred/partial node gets a free,
        # not-yet-validated GPU; PodResources is polled at this period
        "retryDeferredSeconds": 300,
        # a validator restart with the node's fingerprint (boot id, amdgpu version, operator image)
        # unchanged since the last full pass re-uses that pass instead of re-running the load steps
        "skipUnchangedNode": True,
        # compute-partitioned GPUs (DPX/QPX/CPX): per-partition GEMM size; the TFLOPS / HBM floors
        # are scaled by the partition's share of the ASIC (CUs / memory)
        "gemmSizePartitioned": 4096,
    },
}

COMPUTE_PARTITIONS = ("SPX", "DPX", "QPX", "CPX")
MEMORY_PARTITIONS = ("NPS1", "NPS2", "NPS4")


class ConfigError(ValueError):
    pass


def _merge(base: Dict[str, Any], over: Dict[str, Any], path: str = "") -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        where = f"{path}.{k}" if path else k
        if k not in base:
            raise ConfigError(f"unknown operator config key '{where}'")
        if isinstance(base[k], dict):
            if not isinstance(v, dict):
                raise ConfigError(f"'{where}' must be a mapping")
            out[k] = _merge(base[k], v, where)
        else:
            out[k] = v
    return out


@dataclass
class OperatorConfig:
    raw: Dict[str, Any] = field(default_factory=lambda: copy.deepcopy(DEFAULTS))

    def __getitem__(self, key: str) -> Any:
        return self.raw[key]

    @property
    def resource_name(self) -> str:
        return self.raw["resourceName"]

    @property
    def min_gfx(self) -> int:
        return int(self.raw["minGfxTargetVersion"])

    def section(self, name: str) -> Dict[str, Any]:
        return self.raw[name]

    def validate(self) -> "OperatorConfig":
        r = self.raw
        if "/" not in r["resourceName"]:
            raise ConfigError("resourceName must be vendor-qualified, e.g. amd.com/gpu")
        if r["deviceIdStrategy"] not in ("uuid", "index"):
            raise ConfigError("deviceIdStrategy must be 'uuid' or 'index'")
        if r["allocation"]["mode"] not in ("deviceSpecs", "cdi"):
            raise ConfigError("allocation.mode must be 'deviceSpecs' or 'cdi'")
        if r["partition"]["compute"] not in COMPUTE_PARTITIONS:
            raise ConfigError(f"partition.compute must be one of {COMPUTE_PARTITIONS}")
        if r["partition"]["memory"] not in MEMORY_PARTITIONS:
            raise ConfigError(f"partition.memory must be one of {MEMORY_PARTITIONS}")
        if r["partition"]["drainPolicy"] not in ("evict", "wait"):
            raise ConfigError("partition.drainPolicy must be 'evict' or 'wait'")
        if not 1 <= int(r["exporter"]["port"]) <= 65535:
            raise ConfigError("exporter.port out of range")
        if float(r["validator"]["reserveAckSeconds"]) < 0 or float(r["validator"]["retryDeferredSeconds"]) <= 0:
            raise ConfigError("validator.reserveAckSeconds must be >= 0, retryDeferredSeconds > 0")
        gs = r["validator"]["gateSteps"]
        if not isinstance(gs, list) or any(x not in ("gemm", "bandwidth", "stress", "rccl") for x in gs):
            raise ConfigError("validator.gateSteps must list load steps (gemm, bandwidth, stress, rccl)")
        if float(r["validator"]["gateGraceSeconds"]) < 0:
            raise ConfigError("validator.gateGraceSeconds must be >= 0")
        if int(r["validator"]["gemmSize"]) % 256:
            raise ConfigError("validator.gemmSize must be a multiple of 256 (MFMA block tile)")
        return self


def load_config(path: Optional[str] = None, text: Optional[str] = None) -> OperatorConfig:
    if text is None and path:
        with open(path) as f:
            text = f.read()
    data = yaml.safe_load(text) if text else {}
    if data is None:
        data = {}
    if not isinstance(data, dict):
        raise ConfigError("operator config must be a YAML mapping")
    return OperatorConfig(_merge(DEFAULTS, data)).validate()
