"""Operator validator — the gate between "driver loaded" and "node usable".

The reference reproduces NVIDIA's validator by hand: a ``cuda-sample:vectoradd`` Job whose log must
end in ``Test PASSED`` / ``Done`` (reference README.md:264-299), plus a two-pod isolation check
(README.md:301-387); multi-GPU-in-one-pod is "TBD" (README.md:389-391).  Here the chain runs
automatically on every GPU node as init containers of the validator DaemonSet, each step gated on
the previous one's marker under ``/run/amd/validations``:

  driver    kfd-probe: ≥ expectedGpusPerNode gfx950 agents, /dev/kfd + render nodes usable
  runtime   the runtime installer published runtime-ready (amd-container-runtime + CDI spec)
  vectoradd hand-written HIP vectorAdd on every GPU, reference stdout protocol
  gemm      hand-written gfx950 bf16 (and fp8 e4m3) MFMA GEMMs on every GPU: numerics vs fp32 +
            TFLOPS ≥ floor per precision
  bandwidth amd-proftester (the dcgmproftester counterpart): HBM3E copy, PCIe H2D / D2H and, with
            ≥ 2 GPUs, every xGMI peer pair — verified copies, GB/s ≥ floor per link type
  stress    (optional, DCGM diag level 3's targeted stress) every GPU under a sustained MFMA load
            for stressSeconds while amd-smi telemetry is sampled: no uncorrectable ECC error, no
            100 ms window below stressMinFraction of the mean rate, hotspot ≤ stressMaxHotspotC
  rccl      RCCL all-reduce over xGMI across all GPUs of the node: exact sums + bus bandwidth floor
  profile   (optional, BASELINE config 3) the validator GEMMs again under rocprofv3: kernel trace +
            stats, and one --pmc pass (MFMA utilisation, clock, L2 hit rate, FLOP check)
  plugin    a pod requesting amd.com/gpu: 1 is scheduled THROUGH the device plugin and passes
  report    node label amd.com/gpu.validated=true|partial|deferred|false, validator-ready marker

The load steps (gemm, bandwidth, stress, rccl, profile) never touch a GPU that kubelet has allocated to a
pod: the kubelet PodResources API (``podresources_api.py``) lists the device IDs pods hold, and the
native tools run with ``ROCR_VISIBLE_DEVICES`` narrowed to the free agents.  Closing the window
between that answer and the launch: the step first *reserves* its agents (``in-test.json``; the
device plugin reports them Unhealthy and acks with ``in-test.ack``), then re-reads PodResources
and drops any agent a pod took in between — that agent is never loaded.  When no agent is free
the step is *deferred*: no ``-ready`` marker, the init chain continues, and the node label says
``deferred`` (never ``true``) until a full pass exists.  A kubelet that cannot be asked (socket
absent or List failing) or an allocated ID that cannot be mapped *fails* the step: "nothing was
validated" is never reported as validated.  Every agent a load step passed on is recorded per
fingerprint (``device-passes.json``); the agents on which every enabled load step passed this
boot are published in ``validated-devices.json``, which the device plugin gates on
(``gateOnValidation``).  The gate is per device: it opens on the ``gateSteps`` (default: the GEMM,
after vectorAdd earlier in the chain), so a GPU becomes allocatable seconds after the driver is up.
The node-wide steps after it (bandwidth pairs, stress, RCCL, profiling) decide only the node label;
they start ``gateGraceSeconds`` after the gate first opened, so pods already pending for the node get
their GPUs first, and then reserve whatever is still free.  A reservation that a live device plugin
(its registration socket accepts connections) does not ack defers the step: GPUs a serving plugin
may still hand out are never loaded.

A validator restart whose node fingerprint (boot id, amdgpu version, operator image, validator
config, partition modes, agent set) equals the one of the last full pass re-uses that pass instead
of loading the GPUs again.  On compute-partitioned
GPUs (DPX/QPX/CPX) the TFLOPS and HBM floors scale with the partition's share of the ASIC, the
GEMM runs at ``gemmSizePartitioned``, xGMI pair copies are skipped and RCCL runs over one agent
per ASIC.

Each step writes ``<step>.json`` (the metrics exporter publishes TFLOPS / busbw / pass flags from
them) and ``<step>-ready`` on success.  Command execution is injectable so the parsing and gating
logic is tested on CPU against the real outputs the native tools produced on an MI355X
(profiles/r01_*.log).
"""
from __future__ import annotations

import json
import logging
import os
import re
import subprocess
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from . import podresources_api
from .config import OperatorConfig

log = logging.getLogger("amd-gpu-validator")

STEPS = ("driver", "runtime", "vectoradd", "gemm", "bandwidth", "stress", "rccl", "profile", "plugin",
         "report")
LOAD_STEPS = ("gemm", "bandwidth", "stress", "rccl", "profile")
LABEL_VALIDATED = "amd.com/gpu.validated"
FINGERPRINT = "fingerprint.json"
IN_TEST = "in-test.json"                  # {nonce, step, device_uids, expires}: plugin → Unhealthy
IN_TEST_ACK = "in-test.ack"               # the plugin's ack: the nonce it has published
DEVICE_PASSES = "device-passes.json"      # {fingerprint, steps: {step: [device_uid]}}
VALIDATED_DEVICES = "validated-devices.json"  # {boot_id, device_uids}: the plugin's gate
LABEL_TRUE, LABEL_PARTIAL, LABEL_DEFERRED, LABEL_FALSE = "true", "partial", "deferred", "false"
# upper bound of a load step's run time, for the reservation's expiry (a crashed validator must not
# leave GPUs reported Unhealthy forever)
STEP_TIMEOUT = {"gemm": 2400.0, "bandwidth": 900.0, "rccl": 900.0, "profile": 1200.0}
# kubelet device ID -> device_uid, written by the device plugin (needed for deviceIdStrategy: index)
DEVICE_ID_MAP = "/run/amd/device-plugin/ids.json"

Runner = Callable[[Sequence[str], float], Tuple[int, str]]


def default_runner(argv: Sequence[str], timeout: float) -> Tuple[int, str]:
    try:
        p = subprocess.run(list(argv), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=timeout)
        return p.returncode, p.stdout
    except subprocess.TimeoutExpired as e:
        out = e.stdout.decode() if isinstance(e.stdout, bytes) else (e.stdout or "")
        return 124, out + f"\n[validator] timed out after {timeout}s"
    except FileNotFoundError as e:
        return 127, str(e)


def find_bin_dir() -> str:
    env = os.environ.get("AMDK8S_BIN_DIR")
    if env:
        return env
    here = os.path.dirname(os.path.abspath(__file__))
    for cand in ("/opt/amd-gpu-operator/bin",
                 os.path.normpath(os.path.join(here, "..", "..", "native", "bin"))):
        if os.path.isdir(cand):
            return cand
    return "/opt/amd-gpu-operator/bin"


def json_lines(text: str) -> List[dict]:
    out = []
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{") and line.endswith("}"):
            try:
                out.append(json.loads(line))
            except ValueError:
                continue
    return out


def protocol_passed(text: str) -> bool:
    """Reference protocol: 'Test PASSED' then 'Done', no 'Test FAILED'."""
    lines = [ln.strip() for ln in text.splitlines() if ln.strip()]
    return ("Test PASSED" in lines and "Done" in lines and "Test FAILED" not in lines
            and lines.index("Done") > lines.index("Test PASSED"))


def rocprof_kernel_stats(prof_dir: str) -> List[dict]:
    """Rows of rocprofv3's *_kernel_stats.csv (name, calls, average ns) under ``prof_dir``."""
    import csv
    import glob

    rows = []
    for f in glob.glob(os.path.join(prof_dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append({"name": r.get("Name", "")[:120], "calls": int(r.get("Calls", 0) or 0),
                             "avg_ns": float(r.get("AverageNs", 0) or 0),
                             "percent": float(r.get("Percentage", 0) or 0)})
    return sorted(rows, key=lambda r: -r["percent"])


# One rocprofv3 --pmc pass over the validator GEMM (BASELINE.json config 3: "with rocprof counters").
# Within gfx950's per-pass limits (≤ 8 SQ, ≤ 4 TCC, ≤ 2 GRBM counters; MI355X_MICROARCH.md).
GEMM_COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16",
                 "GRBM_GUI_ACTIVE", "TCC_HIT_sum", "TCC_MISS_sum")


def rocprof_counter_summary(prof_dir: str, cus: int, kernel_filter: str = "gemm") -> Dict:
    """Median over the profiled GEMM dispatches of rocprofv3's counter_collection.csv, turned into
    the numbers the validator reports: MFMA utilisation (busy MFMA cycles per SIMD-cycle), the
    effective clock (GRBM_GUI_ACTIVE is summed over the XCDs: cycles = GRBM / XCDs), the L2 hit rate,
    and the MFMA FLOPs the hardware counted (SQ_INSTS_VALU_MFMA_MOPS_* × 512), which must equal
    2·M·N·K — a check that the counters measure the kernel that ran."""
    import csv
    import glob
    import statistics

    per: Dict[str, Dict[str, float]] = {}
    for f in glob.glob(os.path.join(prof_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                if kernel_filter not in name or "sample" in name:
                    continue
                d = per.setdefault(r["Dispatch_Id"], {})
                d[r["Counter_Name"]] = float(r["Counter_Value"])
                try:
                    d["duration_ns"] = float(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                except (KeyError, ValueError):
                    pass
    if not per:
        return {}
    keys = set().union(*per.values())
    med = {k: statistics.median(d[k] for d in per.values() if k in d) for k in keys}
    xcds = max(1, (cus + 16) // 32)
    out: Dict = {"dispatches": len(per), "counters": {k: med[k] for k in sorted(keys)}}
    cycles = med.get("GRBM_GUI_ACTIVE", 0) / xcds
    if cycles and med.get("duration_ns"):
        out["clock_ghz"] = round(cycles / med["duration_ns"], 3)
    if cycles and "SQ_VALU_MFMA_BUSY_CYCLES" in med:
        out["mfma_util_pct"] = round(100 * med["SQ_VALU_MFMA_BUSY_CYCLES"] / (cus * 4 * cycles), 2)
    hit, miss = med.get("TCC_HIT_sum"), med.get("TCC_MISS_sum")
    if hit is not None and miss is not None and hit + miss > 0:
        out["l2_hit_pct"] = round(100 * hit / (hit + miss), 2)
    if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in med:
        out["mfma_flop"] = med["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512
        if med.get("duration_ns"):
            out["tflops_profiled"] = round(out["mfma_flop"] / med["duration_ns"] / 1e3, 1)
    return out


@dataclass
class GpuScope:
    """Which GPU agents the load steps may use.  ``devices`` are in ROCr enumeration order (KFD
    node id), so a position in it is a ``ROCR_VISIBLE_DEVICES`` index."""
    devices: List = field(default_factory=list)
    free: List[int] = field(default_factory=list)
    allocated: Dict[str, str] = field(default_factory=dict)   # device_uid -> namespace/pod
    note: str = ""
    split: int = 1                                            # partitions per ASIC (CPX: 8)
    error: str = ""                                           # kubelet could not be asked
    from_kubelet: bool = False                                # free set came from PodResources

    @property
    def full(self) -> bool:
        return len(self.free) == len(self.devices)

    @property
    def free_uids(self) -> List[str]:
        return [self.devices[i].device_uid for i in self.free]

    @property
    def known(self) -> bool:
        """False when the KFD topology is unreadable here (the tools then run unrestricted and
        fail on their own if there really is no GPU)."""
        return bool(self.devices)

    def env_prefix(self, indices: Optional[Sequence[int]] = None) -> List[str]:
        if not self.known:
            return []
        idx = list(self.free if indices is None else indices)
        if indices is None and self.full:
            return []
        return ["env", "ROCR_VISIBLE_DEVICES=" + ",".join(str(i) for i in idx)]

    def to_dict(self) -> Dict:
        return {"full": self.full, "agents": len(self.devices), "split": self.split,
                "validated": self.free_uids if self.devices else [],
                "allocated": dict(self.allocated), "note": self.note}


@dataclass
class StepResult:
    """``passed`` → ``<step>-ready``.  ``deferred`` steps did not run (no free GPU): not a pass
    (no marker, the report never says ``true`` for them) but not a failure either (the init chain
    continues)."""
    step: str
    passed: bool
    detail: Dict = field(default_factory=dict)
    reason: str = ""
    deferred: bool = False

    @property
    def proceed(self) -> bool:
        return self.passed or self.deferred

    def to_json(self) -> dict:
        d = {"step": self.step, "passed": self.passed, "reason": self.reason, "time": time.time()}
        if self.deferred:
            d["deferred_step"] = True
        d.update(self.detail)
        return d


class Validator:
    def __init__(self, config: OperatorConfig, marker_dir: str = "/run/amd/validations",
                 bin_dir: Optional[str] = None, runner: Runner = default_runner, root: str = "/",
                 kube=None, node_name: Optional[str] = None, driver_wait: float = 120,
                 telemetry: Optional[Callable[[], List[Dict]]] = None,
                 device_id_map: str = DEVICE_ID_MAP, pause_marker: Optional[str] = None,
                 sleep: Callable[[float], None] = time.sleep):
        from .pause import PAUSE_MARKER

        self.cfg = config
        self.sleep = sleep
        self.device_id_map = device_id_map
        # no load step starts while the partition manager switches modes
        self.pause_marker = pause_marker if pause_marker is not None else (
            PAUSE_MARKER if root == "/" else os.path.join(root, PAUSE_MARKER.lstrip("/")))
        self._scope: Optional[GpuScope] = None
        self._fp: Optional[Dict[str, str]] = None
        self.telemetry = telemetry  # per-GPU samples for the stress step (default: amd-smi)
        self.driver_wait = driver_wait  # kfd-probe --wait: how long the driver may take to appear
        self.vcfg = config.section("validator")
        self.marker_dir = marker_dir
        self.bin_dir = bin_dir or find_bin_dir()
        self.run_cmd = runner
        self.root = root
        self.kube = kube
        self.node = node_name or os.environ.get("NODE_NAME", "")

    # ---------------------------------------------------------------- markers
    def _path(self, name: str) -> str:
        return os.path.join(self.marker_dir, name)

    def write_result(self, r: StepResult) -> None:
        os.makedirs(self.marker_dir, exist_ok=True)
        tmp = self._path(f".{r.step}.json.tmp")
        with open(tmp, "w") as f:
            json.dump(r.to_json(), f, indent=1)
        os.replace(tmp, self._path(f"{r.step}.json"))
        ready = self._path(f"{r.step}-ready")
        if r.passed:
            with open(ready, "w") as f:
                f.write(f"{time.time()}\n")
        elif os.path.exists(ready):
            os.unlink(ready)

    def ready(self, step: str) -> bool:
        return os.path.exists(self._path(f"{step}-ready"))

    def wait_for(self, marker: str, timeout: float, poll: float = 2.0) -> bool:
        deadline = time.monotonic() + timeout
        while not os.path.exists(self._path(marker)):
            if time.monotonic() >= deadline:
                return False
            time.sleep(poll)
        return True

    def _bin(self, name: str) -> str:
        return os.path.join(self.bin_dir, name)

    # ---------------------------------------------------------------- GPU scope / fingerprint
    def _kubelet_id_map(self, devs) -> Dict[str, str]:
        if self.cfg["deviceIdStrategy"] != "index":
            return {g.device_uid: g.device_uid for g in devs}
        try:
            with open(self.device_id_map) as f:
                return {str(k): str(v) for k, v in json.load(f).items()}
        except (OSError, ValueError):
            return {}

    def _devices(self) -> List:
        from ..utils import topology as topo_mod

        try:
            topo = topo_mod.read_topology(self.root, self.cfg.min_gfx)
            return sorted(topo.gpus, key=lambda g: g.node_id)
        except FileNotFoundError:
            return []

    def _allocated(self, devs) -> Tuple[Optional[Dict[str, str]], str]:
        """({device_uid: "ns/pod"} held by pods, error).  ``None`` with no error: no kubelet here
        and ``podResourcesRequired: false``."""
        sock = str(self.vcfg["podResourcesSocket"])
        try:
            alloc = podresources_api.allocated(self.cfg.resource_name, sock)
        except Exception as e:  # noqa: BLE001 - kubelet unreachable: cannot prove a GPU is free
            return None, f"kubelet PodResources List failed: {e}"[:300]
        if alloc is None:
            if self.vcfg.get("podResourcesRequired", True):
                return None, f"kubelet PodResources socket {sock} absent: cannot prove any GPU is free"
            return None, ""
        idmap = self._kubelet_id_map(devs)
        busy: Dict[str, str] = {}
        unknown = []
        for kid, pod in sorted(alloc.items()):
            uid = idmap.get(kid)
            if uid is None:
                unknown.append(kid)
            else:
                busy[uid] = pod
        if unknown:
            return busy, "cannot map allocated device id(s) " + ",".join(unknown) + \
                " to GPUs (device plugin id map missing or stale)"
        return busy, ""

    def gpu_scope(self) -> GpuScope:
        """The free GPU agents: every agent minus what kubelet's PodResources API says pods hold.
        Fails closed — an unreadable kubelet answer or an ID that cannot be mapped to a GPU sets
        ``error`` and leaves no GPU free (the load step then fails, never runs on a tenant's GPU)."""
        devs = self._devices()
        split = max((g.partitions_on_asic for g in devs), default=1)
        busy, err = self._allocated(devs)
        if err:
            return GpuScope(devs, [], busy or {}, "", split, error=err)
        if busy is None:
            return GpuScope(devs, list(range(len(devs))), {},
                            "no kubelet PodResources socket (podResourcesRequired: false): all agents",
                            split)
        free = [i for i, g in enumerate(devs) if g.device_uid not in busy]
        return GpuScope(devs, free, busy, "", split, from_kubelet=True)

    def scope(self) -> GpuScope:
        if self._scope is None:
            self._scope = self.gpu_scope()
        return self._scope

    # ---------------------------------------------------------------- reservation (TOCTOU)
    def _write_json(self, name: str, doc) -> None:
        os.makedirs(self.marker_dir, exist_ok=True)
        tmp = self._path(f".{name}.tmp")
        with open(tmp, "w") as f:
            json.dump(doc, f)
        os.replace(tmp, self._path(name))

    def _read_json(self, name: str):
        try:
            with open(self._path(name)) as f:
                return json.load(f)
        except (OSError, ValueError):
            return None

    def reserve(self, step: str, sc: GpuScope) -> Tuple[GpuScope, Dict]:
        """Reserve ``sc``'s free agents for ``step`` and re-check them against kubelet.

        1. ``in-test.json`` names the agents; the device plugin reports them Unhealthy (kubelet
           stops handing them out) and writes the nonce to ``in-test.ack``.
        2. After the ack (or ``reserveAckSeconds`` without one: no plugin is serving, so nothing
           can be allocated through it) PodResources is read again; an agent a pod took since the
           first answer is dropped from the scope and never loaded.
        Returns the narrowed scope (``error`` set when the second answer cannot be had) and a
        detail dict."""
        secs = float(self.vcfg.get("reserveAckSeconds", 15))
        nonce = f"{step}-{os.getpid()}-{time.time_ns()}"
        timeout = STEP_TIMEOUT.get(step, float(self.vcfg.get("stressSeconds", 30)) + 300.0)
        self._write_json(IN_TEST, {"nonce": nonce, "step": step, "device_uids": sc.free_uids,
                                   "expires": time.time() + timeout})
        deadline = time.monotonic() + secs
        acked = False
        while True:
            try:
                with open(self._path(IN_TEST_ACK)) as f:
                    acked = f.read().strip() == nonce
            except OSError:
                acked = False
            if acked or time.monotonic() >= deadline:
                break
            time.sleep(0.05)
        info: Dict = {"nonce": nonce, "acked": acked}
        if not acked and self._plugin_serving():
            # a serving plugin that has not published the reservation may still hand these GPUs
            # to pods: load nothing (the caller defers the step)
            info["unacked_live_plugin"] = True
            return GpuScope(sc.devices, [], sc.allocated, sc.note, sc.split, from_kubelet=True), info
        busy, err = self._allocated(sc.devices)
        if err:
            return GpuScope(sc.devices, [], busy or {}, "", sc.split, error=err), info
        busy = busy or {}
        taken = {u: busy[u] for u in sc.free_uids if u in busy}
        if taken:
            info["taken_while_reserving"] = taken
            log.warning("%s: %d GPU(s) allocated to pods while being reserved, left untouched: %s",
                        step, len(taken), taken)
        free = [i for i in sc.free if sc.devices[i].device_uid not in busy]
        narrowed = GpuScope(sc.devices, free, busy, sc.note, sc.split, from_kubelet=True)
        if taken:   # keep only the agents actually under test reported Unhealthy
            self._write_json(IN_TEST, {"nonce": nonce, "step": step, "device_uids": narrowed.free_uids,
                                       "expires": time.time() + timeout})
        return narrowed, info

    def _plugin_serving(self) -> bool:
        """The device plugin's registration socket accepts a connection (a plugin is serving)."""
        import socket

        path = str(self.vcfg.get("pluginSocket") or "")
        if not path:
            return False
        if not os.path.exists(path) and self.root != "/":
            path = os.path.join(self.root, path.lstrip("/"))
        if not os.path.exists(path):
            return False
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(0.5)
        try:
            s.connect(path)
            return True
        except OSError:
            return False
        finally:
            s.close()

    def release(self) -> None:
        for name in (IN_TEST,):
            try:
                os.unlink(self._path(name))
            except FileNotFoundError:
                pass

    # ---------------------------------------------------------------- per-device passes (gate)
    def _gating_steps(self) -> List[str]:
        """The per-device steps whose passes open the plugin's gate (``gateSteps``, enabled ones);
        the driver check alone when none is enabled."""
        gs = list(self.vcfg.get("gateSteps") or ["gemm"])
        return [s for s in LOAD_STEPS if s in gs and self._enabled(s)] or ["driver"]

    def _wait_gate_grace(self, step: str) -> float:
        """Node-wide steps start ``gateGraceSeconds`` after the gate first opened this boot, so a
        pod pending for the node is allocated before they reserve the free GPUs.  Returns the
        seconds waited."""
        if not self.vcfg.get("gateOnValidation") or step in self._gating_steps():
            return 0.0
        doc = self._read_json(VALIDATED_DEVICES) or {}
        if doc.get("boot_id") != self.fingerprint().get("boot_id") or not doc.get("opened"):
            return 0.0
        wait = float(doc["opened"]) + float(self.vcfg.get("gateGraceSeconds", 0)) - time.time()
        if wait > 0:
            self.sleep(wait)
            return round(wait, 3)
        return 0.0

    def record_pass(self, step: str, uids: Sequence[str]) -> List[str]:
        """Add ``uids`` to ``step``'s passes for the current fingerprint; republish the agents on
        which every gating step has passed (``validated-devices.json``).  Returns that list."""
        fp = self.fingerprint()
        doc = self._read_json(DEVICE_PASSES) or {}
        if doc.get("fingerprint") != fp:
            doc = {"fingerprint": fp, "steps": {}}
        doc["steps"][step] = sorted(set(doc["steps"].get(step, [])) | set(uids))
        self._write_json(DEVICE_PASSES, doc)
        sets = [set(doc["steps"].get(s, [])) for s in self._gating_steps()]
        validated = sorted(set.intersection(*sets)) if sets else []
        prev = self._read_json(VALIDATED_DEVICES) or {}
        opened = prev.get("opened") if (prev.get("boot_id") == fp.get("boot_id", "")
                                        and prev.get("device_uids")) else None
        if validated and opened is None:
            opened = time.time()             # the gate opens now (first GPU allocatable)
        self._write_json(VALIDATED_DEVICES, {"boot_id": fp.get("boot_id", ""), "device_uids": validated,
                                             "time": time.time(), "opened": opened})
        return validated

    def validated_devices(self) -> List[str]:
        doc = self._read_json(VALIDATED_DEVICES) or {}
        if doc.get("boot_id") != self.fingerprint().get("boot_id"):
            return []
        return list(doc.get("device_uids") or [])

    def _cmd(self, argv: List[str], indices: Optional[Sequence[int]] = None) -> List[str]:
        """argv narrowed to the free agents (or to ``indices``) with ROCR_VISIBLE_DEVICES."""
        if self._scope is None:
            return list(argv)
        return self._scope.env_prefix(indices) + list(argv)

    def fingerprint(self) -> Dict[str, str]:
        """What a full pass is valid for.  Besides boot / driver / image / config it covers the GPU
        topology: a compute/memory partition switch re-enumerates the agents without a reboot, so
        the partition modes, the agent count and the sorted device UIDs are part of it (an SPX pass
        must not stand in for the CPX agents after a switch)."""
        if self._fp is None:
            self._fp = self._fingerprint()
        return self._fp

    def _fingerprint(self) -> Dict[str, str]:
        from .labeller import driver_version

        fp: Dict[str, str] = {}
        try:
            with open(os.path.join(self.root, "proc/sys/kernel/random/boot_id")) as f:
                fp["boot_id"] = f.read().strip()
        except OSError:
            fp["boot_id"] = ""
        fp["amdgpu"] = driver_version(self.root) or ""
        fp["image"] = os.environ.get("VALIDATOR_IMAGE_ID") or self._own_image_id()
        fp["config"] = json.dumps(self.vcfg, sort_keys=True, default=str)
        devs = self._devices()
        fp["partition"] = ",".join(sorted({f"{g.compute_partition}/{g.memory_partition}" for g in devs}))
        fp["agents"] = str(len(devs))
        fp["device_uids"] = ",".join(sorted(g.device_uid for g in devs))
        return fp

    def _own_image_id(self) -> str:
        pod_name = os.environ.get("POD_NAME")
        if not pod_name or self.kube is None:
            return ""
        try:
            pod = self.kube.get_pod(os.environ.get("POD_NAMESPACE", "amd-gpu-operator"), pod_name)
        except Exception as e:  # noqa: BLE001
            log.warning("cannot read own pod: %s", e)
            return ""
        st = pod.get("status", {})
        for c in st.get("initContainerStatuses", []) + st.get("containerStatuses", []):
            if c.get("imageID"):
                return c["imageID"]
        return ""

    def _unchanged_pass(self, step: str) -> Optional[Dict]:
        """The previous result of ``step`` when the node has not changed since a FULL pass."""
        if not self.vcfg.get("skipUnchangedNode") or not self.ready(step):
            return None
        try:
            with open(self._path(FINGERPRINT)) as f:
                saved = json.load(f)
            with open(self._path(f"{step}.json")) as f:
                prev = json.load(f)
        except (OSError, ValueError):
            return None
        if not saved.get("full") or saved.get("fingerprint") != self.fingerprint() or not prev.get("passed"):
            return None
        keep = {k: prev[k] for k in ("aggregate_tflops", "min_by_test_gbps", "peak_busbw_gbps", "time",
                                     "reused") if k in prev}
        return {"since": saved.get("time"), **keep}

    # ---------------------------------------------------------------- steps
    def step_driver(self) -> StepResult:
        n = int(self.cfg["expectedGpusPerNode"])
        argv = [self._bin("kfd-probe"), "--expect-gpus", str(n), "--min-gfx", str(self.cfg.min_gfx),
                "--wait", str(int(self.driver_wait))]
        if self.root != "/":
            argv += ["--sysfs-root", os.path.join(self.root, "sys/class/kfd/kfd/topology"),
                     "--dev-root", os.path.join(self.root, "dev"), "--no-open"]
        rc, out = self.run_cmd(argv, self.driver_wait + 60)
        docs = json_lines(out)
        detail = docs[-1] if docs else {}
        ok = rc == 0 and bool(detail.get("ready"))
        return StepResult("driver", ok, {"gpus": detail.get("gpus"), "agents": detail.get("agents", [])},
                          "" if ok else (detail.get("reason") or out.strip()[-300:]))

    def step_runtime(self, timeout: float = 600) -> StepResult:
        ok = self.wait_for("runtime-ready", timeout)
        return StepResult("runtime", ok, {}, "" if ok else "runtime-ready marker not published")

    def step_vectoradd(self) -> StepResult:
        rc, out = self.run_cmd([self._bin("amd-vectoradd"), "--json"], 300)
        devs = [d for d in json_lines(out) if d.get("check") == "vectoradd"]
        ok = rc == 0 and protocol_passed(out) and devs and all(d.get("passed") for d in devs)
        return StepResult("vectoradd", bool(ok), {"devices": devs},
                          "" if ok else f"rc={rc}: " + out.strip()[-300:])

    def _gemm_run(self, dtype: str, size: int, floor: float, rocprof: bool) -> Tuple[bool, Dict, str]:
        argv = [self._bin("amd-gemm-validator"), "--size", str(size), "--iters", "50", "--json"]
        if dtype != "bf16":
            argv += ["--dtype", dtype]
        prof_dir = None
        if rocprof:
            # BASELINE config 3: the validator GEMM "shown in rocprof" — kernel trace + stats of the
            # validator run itself, kept next to the step result (and exported as an artefact)
            prof_dir = self._path("gemm-rocprof" if dtype == "bf16" else f"gemm-{dtype}-rocprof")
            argv = ["rocprofv3", "--kernel-trace", "--stats", "-d", prof_dir, "-o", "gemm",
                    "--output-format", "csv", "--"] + argv
        rc, out = self.run_cmd(self._cmd(argv), 900)
        devs = [d for d in json_lines(out) if d.get("check") == f"gemm_{dtype}"]
        slow = [d for d in devs if float(d.get("tflops", 0)) < floor]
        bad = [d for d in devs if not d.get("passed")]
        ok = rc == 0 and protocol_passed(out) and bool(devs) and not slow and not bad
        reason = ""
        if not ok:
            reason = (f"{len(bad)} GPU(s) failed {dtype} numerics; " if bad else "") + \
                     (f"{len(slow)} GPU(s) below {floor} {dtype} TFLOPS; " if slow else "") + \
                     (f"{dtype} rc={rc}" if rc else "") + ("" if devs else f" no {dtype} result")
        total = sum(float(d.get("tflops", 0)) for d in devs)
        detail = {"devices": devs, "size": size, "floor_tflops": floor,
                  "aggregate_tflops": round(total, 1)}
        if prof_dir:
            detail["rocprof_kernels"] = rocprof_kernel_stats(prof_dir)
        return ok, detail, reason.strip()

    def _gemm_counters(self, size: int, cus: int) -> Dict:
        """A separate short rocprofv3 --pmc pass (counters never share a run with tracing domains)."""
        prof_dir = self._path("gemm-rocprof-counters")
        argv = ["rocprofv3", "--kernel-trace", "--pmc", *GEMM_COUNTERS, "-d", prof_dir, "-o", "pmc",
                "--output-format", "csv", "--", self._bin("amd-gemm-validator"), "--size", str(size),
                "--iters", "10", "--settle-ms", "50", "--json"]
        rc, out = self.run_cmd(self._cmd(argv), 300)
        summary = rocprof_counter_summary(prof_dir, cus) if rc == 0 else {}
        if rc != 0:
            summary["error"] = f"rocprofv3 --pmc rc={rc}: {out.strip()[-200:]}"
        elif summary.get("mfma_flop") is not None:
            # the hardware's MFMA FLOP count must match the GEMM that was asked for
            summary["flop_matches_shape"] = summary["mfma_flop"] == 2.0 * size ** 3
        return summary

    def _gemm_size(self) -> Tuple[int, int]:
        split = self._scope.split if self._scope else 1
        # a compute partition owns 1/split of the ASIC's CUs: per-partition floor and a GEMM sized
        # for 32 CUs (CPX) rather than the whole chip
        return int(self.vcfg["gemmSize"] if split == 1 else self.vcfg["gemmSizePartitioned"]), split

    def step_gemm(self, rocprof: bool = False) -> StepResult:
        """bf16 (+ fp8) GEMMs: numerics vs fp32 and the TFLOPS floor on every free GPU.  A gate
        step, so it runs plain; the profiled runs are the ``profile`` step's."""
        size, split = self._gemm_size()
        ok, detail, reason = self._gemm_run("bf16", size, float(self.vcfg["gemmMinTflops"]) / split,
                                            rocprof)
        detail["partition_split"] = split
        if self.vcfg.get("gemmFp8"):
            ok8, detail8, reason8 = self._gemm_run("fp8", size,
                                                   float(self.vcfg["gemmFp8MinTflops"]) / split, rocprof)
            detail["fp8"] = detail8
            ok = ok and ok8
            reason = "; ".join(r for r in (reason, reason8) if r)
        return StepResult("gemm", bool(ok), detail, reason)

    def step_profile(self) -> StepResult:
        """BASELINE config 3, "the validator GEMM shown in rocprof": the GEMM runs again under
        ``rocprofv3 --kernel-trace --stats`` (``rocprof``), then one separate ``--pmc`` pass
        (``rocprofCounters``: MFMA utilisation, clock, L2 hit rate, the MFMA FLOPs the hardware
        counted vs 2·n³).  After the gate: profiling is evidence, not admission."""
        size, split = self._gemm_size()
        detail: Dict = {"size": size, "partition_split": split}
        ok, reason = True, ""
        if self.vcfg.get("rocprof"):
            r = self.step_gemm(rocprof=True)
            ok, reason = r.passed, r.reason
            detail["rocprof_kernels"] = r.detail.get("rocprof_kernels", [])
            detail["devices"] = r.detail.get("devices", [])
            if "fp8" in r.detail:
                detail["fp8"] = {"rocprof_kernels": r.detail["fp8"].get("rocprof_kernels", []),
                                 "devices": r.detail["fp8"].get("devices", [])}
        if self.vcfg.get("rocprofCounters") and ok:
            devs = detail.get("devices") or []
            cus = min((int(d.get("cus", 256)) for d in devs), default=256 // split)
            pmc = self._gemm_counters(size, cus)
            detail["rocprof_counters"] = pmc
            if pmc.get("error"):
                ok, reason = False, pmc["error"]
        return StepResult("profile", bool(ok), detail, reason)

    def step_bandwidth(self) -> StepResult:
        split = self._scope.split if self._scope else 1
        floors = {"hbm-copy": float(self.vcfg["hbmMinGBps"]) / split,
                  "pcie-h2d": float(self.vcfg["pcieMinGBps"]),
                  "pcie-d2h": float(self.vcfg["pcieMinGBps"]), "xgmi": float(self.vcfg["xgmiMinGBps"])}
        extra: Dict[str, str] = {}
        if split > 1:
            # partitions of one ASIC share its HBM and talk over the on-package fabric, not xGMI; the
            # ASIC-to-ASIC links are exercised by the RCCL step (one agent per ASIC)
            del floors["xgmi"]
            extra["xgmi_skipped"] = f"compute-partitioned ({split} agents per ASIC)"
        rc, out = self.run_cmd(self._cmd([self._bin("amd-proftester"), "-t", ",".join(floors), "--json"]),
                               900)
        docs = [d for d in json_lines(out) if d.get("check") == "proftester" and d.get("test") in floors]
        # pairs: SDMA copies are gated; the copy-kernel pulls and the all-peer aggregate are reported
        gated = [d for d in docs if not d.get("skipped")
                 and (d.get("test") != "xgmi" or d.get("engine") == "sdma")]
        slow = [d for d in gated if float(d.get("value", 0)) < floors[d["test"]]]
        bad = [d for d in docs if not d.get("passed")]
        seen = {d.get("test") for d in docs}
        missing = [t for t in ("hbm-copy", "pcie-h2d", "pcie-d2h") if t not in seen]
        ok = rc == 0 and protocol_passed(out) and not slow and not bad and not missing
        summary: Dict[str, float] = {}
        for d in docs:
            if d.get("skipped"):
                continue
            key = d["test"] if d["test"] != "xgmi" else f"xgmi-{d.get('engine')}"
            summary[key] = round(min(summary.get(key, float("inf")), float(d.get("value", 0))), 1)
        reason = ""
        if not ok:
            reason = "; ".join(filter(None, [
                f"{len(bad)} check(s) failed" if bad else "",
                ", ".join(f"{d['test']} dev {d['device']}"
                          + (f"<-{d['peer']}" if d.get("peer", -1) >= 0 else "")
                          + f" {d['value']:.1f} < {floors[d['test']]}" for d in slow),
                f"no result for {','.join(missing)}" if missing else "",
                f"rc={rc}" if rc else ""]))
        return StepResult("bandwidth", bool(ok), {"results": docs, "min_by_test_gbps": summary,
                                                  "floors_gbps": floors, **extra}, reason)

    def _telemetry_fn(self) -> Optional[Callable[[], List[Dict]]]:
        if self.telemetry is not None:
            return self.telemetry
        try:
            from .exporter import AmdSmiBackend

            return AmdSmiBackend().samples
        except Exception as e:  # noqa: BLE001 - no amd-smi: the load still runs, unmonitored
            log.warning("no amd-smi telemetry for the stress step: %s", e)
            return None

    def step_stress(self) -> StepResult:
        import threading

        secs = float(self.vcfg["stressSeconds"])
        frac = float(self.vcfg["stressMinFraction"])
        tmax = float(self.vcfg["stressMaxHotspotC"])
        sample = self._telemetry_fn()
        samples: List[List[Dict]] = []
        stop = threading.Event()

        def poll():
            while not stop.is_set():
                try:
                    samples.append(sample())
                except Exception as e:  # noqa: BLE001
                    log.debug("telemetry sample failed: %s", e)
                stop.wait(1.0)

        th = threading.Thread(target=poll, daemon=True) if sample else None
        if th:
            th.start()
        try:
            rc, out = self.run_cmd(self._cmd([self._bin("amd-proftester"), "-t", "tensor", "--duration",
                                              str(secs), "--json"]), secs + 300)
        finally:
            stop.set()
            if th:
                th.join(5)
        if sample:  # one more snapshot after the load: ECC counters raised at its very end count too
            try:
                samples.append(sample())
            except Exception as e:  # noqa: BLE001
                log.debug("telemetry sample failed: %s", e)
        docs = [d for d in json_lines(out) if d.get("check") == "proftester" and d.get("test") == "tensor"]
        problems = []
        per_gpu: Dict[str, Dict] = {}
        for d in docs:
            g = per_gpu.setdefault(str(d["device"]), {})
            g.update(tflops=d["value"], tflops_min_window=d["min"], seconds=d["seconds"])
            if d["value"] <= 0 or d["min"] < frac * d["value"]:
                problems.append(f"GPU {d['device']}: 100 ms window {d['min']:.0f} < {frac:.2f} x "
                                f"mean {d['value']:.0f} TFLOPS")
        if len(samples) >= 1:
            first = {str(x.get("index")): x for x in samples[0]}
            last = {str(x.get("index")): x for x in samples[-1]}
            for idx, x in last.items():
                g = per_gpu.setdefault(idx, {})
                temps = [s_.get("temp_hotspot") for snap in samples for s_ in snap
                         if str(s_.get("index")) == idx and s_.get("temp_hotspot") is not None]
                power = [s_.get("power_w") for snap in samples for s_ in snap
                         if str(s_.get("index")) == idx and s_.get("power_w") is not None]
                clocks = [s_.get("gfxclk_mhz") for snap in samples for s_ in snap
                          if str(s_.get("index")) == idx and s_.get("gfxclk_mhz") is not None]
                if temps:
                    g["hotspot_max_c"] = max(temps)
                    if max(temps) > tmax:
                        problems.append(f"GPU {idx}: hotspot {max(temps):.0f} C > {tmax:.0f} C")
                if power:
                    g["power_mean_w"] = round(sum(power) / len(power), 1)
                if clocks:
                    g["gfxclk_min_mhz"], g["gfxclk_mean_mhz"] = min(clocks), round(sum(clocks) / len(clocks))
                u0, u1 = (first.get(idx) or {}).get("ecc_uncorrectable"), x.get("ecc_uncorrectable")
                if u0 is not None and u1 is not None:
                    g["ecc_uncorrectable_delta"] = u1 - u0
                    if u1 > u0:
                        problems.append(f"GPU {idx}: {u1 - u0:.0f} uncorrectable ECC error(s) under load")
                c0, c1 = (first.get(idx) or {}).get("ecc_correctable"), x.get("ecc_correctable")
                if c0 is not None and c1 is not None:
                    g["ecc_correctable_delta"] = c1 - c0
        ok = rc == 0 and protocol_passed(out) and bool(docs) and not problems
        if rc != 0 or not docs:
            problems.append(f"rc={rc}" + ("" if docs else ", no load result"))
        return StepResult("stress", ok, {"seconds": secs, "gpus": per_gpu, "telemetry_samples": len(samples),
                                         "min_fraction": frac, "max_hotspot_c": tmax}, "; ".join(problems))

    def step_rccl(self, ngpus: Optional[int] = None) -> StepResult:
        if ngpus is not None and ngpus < 2:
            return StepResult("rccl", True, {"ngpus": ngpus, "skipped": "single GPU"})
        floor = float(self.vcfg["rcclMinBusbwGBps"])
        indices = None
        sc = self._scope
        if sc is not None and sc.devices and (sc.split > 1 or not sc.full):
            # one agent per ASIC (partition 0): RCCL measures the xGMI links between ASICs, not 64
            # partitions contending for eight sets of links
            indices = [i for i in sc.free if sc.devices[i].partition_index == 0] if sc.split > 1 else sc.free
            if len(indices) < 2:
                return StepResult("rccl", True, {"ngpus": len(indices),
                                                 "skipped": "fewer than 2 free ASICs"})
        rc, out = self.run_cmd(self._cmd([self._bin("rccl-allreduce-bench"), "-b", "1M", "-e", "1G",
                                          "-f", "4", "-n", "20", "--json"], indices), 900)
        docs = [d for d in json_lines(out) if d.get("check") == "rccl_allreduce"]
        d = docs[-1] if docs else {}
        n = d.get("ngpus", ngpus)
        if n is not None and n < 2:
            return StepResult("rccl", rc == 0, {"ngpus": n, "skipped": "single GPU"})
        ok = rc == 0 and bool(d.get("passed")) and float(d.get("peak_busbw_gbps", 0)) >= floor
        return StepResult("rccl", ok, d, "" if ok else
                          f"rc={rc} wrong={d.get('wrong')} busbw={d.get('peak_busbw_gbps')} < {floor}?")

    def step_plugin(self, timeout: float = 600) -> StepResult:
        if self.kube is None or not self.node:
            return StepResult("plugin", False, {}, "no Kubernetes API access / NODE_NAME")
        ns = os.environ.get("POD_NAMESPACE", "amd-gpu-operator")
        image = self._own_image(ns)
        name = f"amd-gpu-plugin-validation-{self.node}"[:63].rstrip("-.")
        pod = {
            "apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": ns,
                         "labels": {"app": "amd-gpu-plugin-validation"}},
            "spec": {
                "restartPolicy": "Never",
                "nodeName": self.node,
                "runtimeClassName": self.cfg["runtimeClass"],
                "tolerations": [{"operator": "Exists"}],
                "containers": [{
                    "name": "vectoradd", "image": image,
                    "command": [os.path.join("/opt/amd-gpu-operator/bin", "amd-vectoradd")],
                    "resources": {"limits": {self.cfg.resource_name: "1"}},
                }],
            },
        }
        self.kube.delete_pod(ns, name)
        self.kube.create_pod(ns, pod)
        try:
            done = self.kube.wait_pod_phase(ns, name, timeout=timeout)
            logs = self.kube.pod_logs(ns, name)
        finally:
            self.kube.delete_pod(ns, name)
        phase = done.get("status", {}).get("phase")
        ok = phase == "Succeeded" and protocol_passed(logs)
        return StepResult("plugin", ok, {"pod": name, "phase": phase},
                          "" if ok else f"phase={phase}: {logs.strip()[-300:]}")

    def _own_image(self, ns: str) -> str:
        pod_name = os.environ.get("POD_NAME")
        if pod_name and self.kube is not None:
            try:
                pod = self.kube.get_pod(ns, pod_name)
                for c in pod.get("spec", {}).get("initContainers", []) + pod.get("spec", {}).get("containers", []):
                    if c.get("image"):
                        return c["image"]
            except Exception as e:  # noqa: BLE001
                log.warning("cannot read own pod image: %s", e)
        return os.environ.get("VALIDATOR_IMAGE", "ghcr.io/example-org/amd-gpu-operator:0.1.0")

    def required_steps(self) -> List[str]:
        required = ["driver", "runtime"]
        if self.vcfg["vectorAdd"]:
            required.append("vectoradd")
        if self.vcfg["gemm"]:
            required.append("gemm")
        if self.vcfg["bandwidth"]:
            required.append("bandwidth")
        if self.vcfg["stress"]:
            required.append("stress")
        if self.vcfg["rccl"]:
            required.append("rccl")
        if self._enabled("profile"):
            required.append("profile")
        if self.vcfg["pluginTest"]:
            required.append("plugin")
        return required

    def _has_full_pass(self) -> bool:
        saved = self._read_json(FINGERPRINT) or {}
        return bool(saved.get("full")) and saved.get("fingerprint") == self.fingerprint()

    def node_label(self) -> Tuple[str, Dict]:
        """(label value, detail) from the recorded step results.

        ``false``    a required step failed or never recorded a result
        ``deferred`` a load step could not run (every GPU allocated) and no full pass exists for
                     the current fingerprint
        ``partial``  every step passed, but a load step ran on a subset of the GPUs, and no full
                     pass exists for the current fingerprint
        ``true``     every step passed on every GPU — now, or in a full pass for this fingerprint
        """
        required = self.required_steps()
        failed, deferred, subset, docs = [], [], [], {}
        for st in required:
            d = self._read_json(f"{st}.json")
            docs[st] = d
            if d is None:
                if not self.ready(st):      # a marker another agent published counts as a pass
                    failed.append(st)
            elif d.get("deferred_step"):
                deferred.append(st)
            elif not d.get("passed") or not self.ready(st):
                failed.append(st)
            elif st in LOAD_STEPS and "previous" not in d and not d.get("skipped") \
                    and not (d.get("gpu_scope") or {}).get("full", True):
                subset.append(st)
        full = not failed and not deferred and not subset
        prior = self._has_full_pass()
        if failed:
            label = LABEL_FALSE
        elif full or prior:
            label = LABEL_TRUE
        else:
            label = LABEL_DEFERRED if deferred else LABEL_PARTIAL
        return label, {"required": required, "failed": failed, "deferred": deferred,
                       "subset": subset, "full_validation": full, "prior_full_pass": prior,
                       "docs": docs}

    def step_report(self) -> StepResult:
        label, info = self.node_label()
        docs = info.pop("docs")
        ok = label == LABEL_TRUE
        if self.kube is not None and self.node:
            try:
                self.kube.set_node_labels(self.node, {LABEL_VALIDATED: label})
            except Exception as e:  # noqa: BLE001
                log.warning("cannot label node: %s", e)
        durations = {}
        no_duration = []
        for st in info["required"]:
            d = (docs.get(st) or {}).get("duration_s")
            if d is not None:
                durations[st] = d
            else:
                no_duration.append(st)
        # chain_seconds is only a complete time-to-validated when every required step is timed;
        # the untimed ones are listed instead of being silently counted as zero
        missing = info["failed"] + info["deferred"]
        reason = ""
        if info["failed"]:
            reason = "failed/missing: " + ",".join(info["failed"])
        elif not ok:
            reason = (f"deferred: {','.join(info['deferred'])}" if info["deferred"] else
                      f"ran on a subset of the GPUs: {','.join(info['subset'])}") + \
                " (no full pass for this boot/topology yet)"
        r = StepResult("report", ok, {**info, "label": label, "missing": missing,
                                      "validated_devices": self.validated_devices(),
                                      "step_seconds": durations,
                                      "step_seconds_missing": no_duration,
                                      "chain_seconds": round(sum(durations.values()), 3),
                                      "chain_complete": not no_duration},
                       reason, deferred=label in (LABEL_DEFERRED, LABEL_PARTIAL))
        if info["full_validation"]:
            self._write_json(FINGERPRINT, {"full": True, "time": time.time(),
                                           "fingerprint": self.fingerprint()})
        if ok:
            with open(self._path("validator-ready"), "w") as f:
                f.write(f"{time.time()}\n")
        elif os.path.exists(self._path("validator-ready")):
            os.unlink(self._path("validator-ready"))
        return r

    def pending_devices(self) -> List[str]:
        """Free agents (per kubelet, now) not yet validated this boot — what a re-run of the chain
        would validate.  Empty when kubelet cannot be asked."""
        sc = self.gpu_scope()
        if sc.error:
            return []
        done = set(self.validated_devices())
        return [u for u in sc.free_uids if u not in done]

    # ---------------------------------------------------------------- driver
    def run_step(self, step: str) -> StepResult:
        """Run one step and ALWAYS record its outcome.  A step that raises (a validation pod that
        never leaves Pending, an API error, a missing binary) is a failed step: its ``-ready``
        marker is withdrawn and ``<step>.json`` says why, so neither a stale pass nor a stale
        node label can survive on the hostPath marker dir."""
        if step not in STEPS:
            raise ValueError(f"unknown step {step!r}; steps: {STEPS}")
        t0 = time.monotonic()
        try:
            r = self._run_step(step)
        except Exception as e:  # noqa: BLE001 - any escape would leave the old markers in place
            log.exception("step %s raised", step)
            r = StepResult(step, False, {"exception": type(e).__name__}, repr(e)[:500])
        # per-step wall time: the report sums them into the node's time-to-validated breakdown
        r.detail.setdefault("duration_s", round(time.monotonic() - t0, 3))
        self.write_result(r)
        log.info("step %s: %s %s", step,
                 "PASSED" if r.passed else "DEFERRED" if r.deferred else "FAILED", r.reason)
        return r

    def _run_step(self, step: str) -> StepResult:
        if step in LOAD_STEPS and self._enabled(step):
            prev = self._unchanged_pass(step)
            if prev is not None:
                return StepResult(step, True, {"reused": "node fingerprint unchanged since the last "
                                                         "full validation", "previous": prev})
            waited = self._wait_gate_grace(step)
            # a fresh kubelet answer per load step (steps run minutes apart)
            sc = self._scope = self.gpu_scope()
            if os.path.exists(self.pause_marker):
                return self._deferred(step, sc, "partition change in progress")
            if sc.error:
                return StepResult(step, False, {"gpu_scope": sc.to_dict()}, sc.error)
            if sc.known and not sc.free:
                return self._deferred(step, sc, f"all {len(sc.devices)} GPU agent(s) allocated to pods")
            reservation = None
            try:
                if sc.known and sc.from_kubelet:
                    sc, reservation = self.reserve(step, sc)
                    self._scope = sc
                    if waited:
                        reservation["gate_grace_waited_s"] = waited
                    if reservation.get("unacked_live_plugin"):
                        return self._deferred(step, sc, "the device plugin is serving but did not "
                                                        "ack the reservation: no GPU loaded",
                                              reservation)
                    if os.path.exists(self.pause_marker):
                        # the partition manager started after the first check
                        return self._deferred(step, sc, "partition change started while "
                                                        "reserving", reservation)
                    if sc.error:
                        return StepResult(step, False, {"gpu_scope": sc.to_dict(),
                                                        "reservation": reservation}, sc.error)
                    if not sc.free:
                        return self._deferred(step, sc, "every free GPU was allocated to a pod "
                                                        "while being reserved", reservation)
                r = self._run_load_step(step)
                if reservation is not None:
                    # the residual window (docs/runbook.md): a pod admitted after the re-read but
                    # before kubelet applied the Unhealthy update shows up here, after the fact
                    after, err2 = self._allocated(sc.devices)
                    late = {u: after[u] for u in sc.free_uids if after and u in after}
                    if late:
                        r.detail["allocated_during_step"] = late
                        log.warning("%s: GPU(s) allocated to pods while under test: %s", step, late)
            finally:
                if reservation is not None:
                    self.release()
            r.detail["gpu_scope"] = sc.to_dict()
            if reservation is not None:
                r.detail["reservation"] = reservation
            if r.passed and sc.known:
                r.detail["validated_devices"] = self.record_pass(step, sc.free_uids)
            return r
        r = self._run_load_step(step)
        if r.passed and step == "driver" and self._gating_steps() == ["driver"]:
            # no load step enabled: the gate opens on the driver check alone
            devs = self._devices()
            if devs:
                r.detail["validated_devices"] = self.record_pass("driver", [g.device_uid for g in devs])
        return r

    def _deferred(self, step: str, sc: GpuScope, why: str, reservation=None) -> StepResult:
        detail = {"deferred": why, "gpu_scope": sc.to_dict()}
        if reservation is not None:
            detail["reservation"] = reservation
        return StepResult(step, False, detail, f"deferred: {why}", deferred=True)

    def _enabled(self, step: str) -> bool:
        if step == "profile":
            return bool(self.vcfg.get("rocprof") or self.vcfg.get("rocprofCounters"))
        return bool(self.vcfg[{"gemm": "gemm", "bandwidth": "bandwidth", "stress": "stress",
                               "rccl": "rccl"}[step]])

    def _run_load_step(self, step: str) -> StepResult:
        if step == "driver":
            r = self.step_driver()
        elif step == "runtime":
            r = self.step_runtime()
        elif step == "vectoradd":
            if not self.vcfg["vectorAdd"]:
                r = StepResult("vectoradd", True, {"skipped": True})
            elif os.path.exists(self.pause_marker):       # no GPU work mid-switch
                r = StepResult("vectoradd", False, {"deferred": "partition change in progress"},
                               "deferred: partition change in progress", deferred=True)
            else:
                r = self.step_vectoradd()
        elif step == "gemm":
            r = self.step_gemm() if self.vcfg["gemm"] else StepResult("gemm", True, {"skipped": True})
        elif step == "bandwidth":
            r = self.step_bandwidth() if self.vcfg["bandwidth"] else StepResult("bandwidth", True, {"skipped": True})
        elif step == "stress":
            r = self.step_stress() if self.vcfg["stress"] else StepResult("stress", True, {"skipped": True})
        elif step == "rccl":
            if not self.vcfg["rccl"]:
                r = StepResult("rccl", True, {"skipped": True})
            else:
                gpus = None
                try:
                    with open(self._path("driver.json")) as f:
                        gpus = json.load(f).get("gpus")
                except (OSError, ValueError):
                    pass
                r = self.step_rccl(gpus)
        elif step == "profile":
            r = self.step_profile() if self._enabled("profile") else StepResult("profile", True, {"skipped": True})
        elif step == "plugin":
            r = self.step_plugin() if self.vcfg["pluginTest"] else StepResult("plugin", True, {"skipped": True})
        elif step == "report":
            r = self.step_report()
        else:
            raise ValueError(f"unknown step {step!r}; steps: {STEPS}")
        return r


def hold_loop(v: "Validator", marker_dir: str, interval: float = 30.0,
              stop: Optional[Callable[[], bool]] = None, sleep: Callable[[float], None] = time.sleep) -> int:
    """The report container's life after the chain: restart the chain when it has to run again.

    * the driver marker is withdrawn (driver restart / GPU reset),
    * the GPU topology changed under it (a partition switch re-enumerated the agents), or
    * the node is ``deferred`` / ``partial`` and kubelet now shows a free GPU that has not been
      validated this boot (polled every ``retryDeferredSeconds``).
    The topology is compared every iteration: after a partition switch the agents
    have new UIDs, the gate is closed for all of them, and waiting out the retry period would
    leave the node with zero allocatable GPUs for minutes.
    A container restart would not re-run init containers, so the chain is restarted by deleting
    this pod (the DaemonSet recreates it); without API access the container exits (code 3).
    Returns the exit code."""
    retry = float(v.vcfg.get("retryDeferredSeconds", 300))
    last_check = time.monotonic()
    why = ""
    while not (stop and stop()):
        if not os.path.exists(os.path.join(marker_dir, "driver-ready")):
            why = "driver-ready withdrawn"
            break
        now = v._fingerprint()
        if any(now.get(k) != v.fingerprint().get(k) for k in ("partition", "agents", "device_uids")):
            why = "GPU topology changed (partition switch / GPU lost): re-validate"
            break
        if time.monotonic() - last_check >= retry:
            last_check = time.monotonic()
            label, _ = v.node_label()
            if label in (LABEL_DEFERRED, LABEL_PARTIAL):
                pending = v.pending_devices()
                if pending:
                    why = f"node {label}: {len(pending)} free GPU(s) not yet validated this boot"
                    break
        sleep(interval)
    else:
        return 0
    log.info("re-running the validation chain: %s", why)
    return 3 if not restart_own_pod(v) else 0


def restart_own_pod(v: "Validator") -> bool:
    pod, ns = os.environ.get("POD_NAME"), os.environ.get("POD_NAMESPACE", "amd-gpu-operator")
    if v.kube is None or not pod:
        return False
    try:
        v.kube.delete_pod(ns, pod)
        return True
    except Exception as e:  # noqa: BLE001 - fall back to exiting
        log.warning("cannot delete own pod %s/%s: %s", ns, pod, e)
        return False
