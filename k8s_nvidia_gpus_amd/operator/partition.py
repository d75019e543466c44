"""Compute / memory partition manager (SURVEY.md §2.2 X7 — the MIG-manager role; BASELINE config 5).

An MI355X can run as one GPU (SPX: 8 XCDs, 256 CUs, 288 GB) or be split into 2/4/8 compute
partitions (DPX/QPX/CPX; CPX = 8 GPUs of 1 XCD / 32 CUs each), with the HBM as one NUMA domain
(NPS1) or two (NPS2).  Changing mode needs the GPU idle, and the driver then re-enumerates: new
KFD agents, new render minors, different device IDs.  The manager drives that safely:

    IDLE ─desired≠current─▶ DRAINING ─no GPU pods─▶ QUIESCING ─acks─▶ APPLYING ─▶ REENUMERATING ─▶ IDLE
                              │ taint NoSchedule +        │ operator GPU      │ amd-smi /   │ KFD shows
                              │ pause marker; evict GPU   │ clients release   │ sysfs per   │ N × split
                              │ pods (Eviction API, PDBs) │ their handles     │ ASIC, EBUSY │ agents
                              └─timeout / PDB-blocked─▶ FAILED (taint + marker removed, reason annotated)

Draining (``partition.drainPolicy``): ``evict`` (default) evicts every pod on the node that holds
``amd.com/gpu`` through the Eviction API, so PodDisruptionBudgets are honoured — a refused (429)
eviction is retried until the drain timeout and then fails the change with the PDB's message; the
reference's GPU workloads are long-lived Deployments (reference llm/deployment.yaml:8-12,
sd15-api/deployment.yaml:8-9) whose pods a NoSchedule taint alone never removes.  ``wait`` only
waits for them to finish.  A validator load step in flight (its ``in-test.json`` reservation)
also holds the drain.

Quiescing (:mod:`.pause`): the operator's own GPU clients — exporter, driver-readiness probe, device
plugin — see the pause marker's nonce, close their amd-smi sessions / stop opening ``/dev/kfd`` and
ack; the mode is applied after every ack (or ``pauseAckSeconds``).  A write that still finds the
device busy (EBUSY) is retried with exponential backoff (``applyRetries``) before the change fails.

The desired mode comes from the node label ``amd.com/gpu.compute-partition.desired`` (and
``…memory-partition.desired``), else from operator.yaml.  The state is published as the node
annotation ``amd.com/gpu.partition-state`` so it survives agent restarts and is visible with kubectl.

Convergence is per ASIC: every ASIC's current mode is read (a node whose change stopped half-way —
``set_compute`` raising on ASIC 3 after ASICs 0-2 switched — reads as ``mixed``, never as the head
GPU's mode), and a reconcile re-applies the desired mode only to the ASICs that are off target.

How the driver applies the two modes (and what the manager does about it):

* **Memory partition (NPS) is hive-wide and needs a driver reload.**  It is applied ONCE per node,
  before any compute change.  amd-smi's set call performs the reload itself (every KFD agent is
  withdrawn and re-created, every processor handle becomes invalid); the manager then waits for
  every ASIC to re-appear in the new mode.  A sysfs write only *requests* the mode for the next
  reload: with ``partition.driverReloadCommand`` set the manager runs it (the GPUs are already
  drained and quiesced), otherwise the change stops in state ``pending-reload`` (taint and pause
  lifted, the GPUs keep serving in the old mode) instead of waiting out a re-enumeration that
  cannot happen; later reconciles report the same state without draining again.
* **Compute partition is per ASIC and re-enumerates that ASIC's agents** (SPX → CPX turns one
  agent into eight, new render nodes and device IDs).  Handles are looked up fresh for every
  write after a change (the amd-smi backend re-initialises its session), never reused.

Between draining and the first write the manager checks again that no validator load step holds
a reservation (``in-test.json``): one that started in that window is waited for.
"""
from __future__ import annotations

import errno
import json
import logging
import os
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from ..utils import kube as kube_mod
from ..utils import topology as topo_mod
from . import pause as pause_mod

log = logging.getLogger("amd-partition-manager")

LABEL_DESIRED = "amd.com/gpu.compute-partition.desired"
LABEL_MEM_DESIRED = "amd.com/gpu.memory-partition.desired"
ANNOT_STATE = "amd.com/gpu.partition-state"
TAINT_KEY = "amd.com/gpu-partitioning"
PAUSE_MARKER = pause_mod.PAUSE_MARKER
DRAIN_POLICIES = ("evict", "wait")


def is_busy(e: BaseException) -> bool:
    """The device refused the mode change because it is in use (retryable)."""
    if isinstance(e, OSError) and e.errno == errno.EBUSY:
        return True
    text = str(e).lower()
    return "ebusy" in text or "device or resource busy" in text or "amdsmi_status_busy" in text


MIXED = "mixed"


class PartitionError(RuntimeError):
    pass


def asic_modes(topo: topo_mod.NodeTopology) -> Dict[int, Tuple[str, str]]:
    """{ASIC unique id: (compute mode, memory mode)} from each ASIC's own PCI attributes."""
    return {uid: (members[0].compute_partition, members[0].memory_partition)
            for uid, members in topo.asics().items()}


def node_mode(modes: Dict[int, Tuple[str, str]]) -> Tuple[str, str]:
    """The node's (compute, memory) mode, ``mixed`` where its ASICs disagree."""
    cs = {c for c, _ in modes.values()}
    ms = {m for _, m in modes.values()}
    return (cs.pop() if len(cs) == 1 else MIXED), (ms.pop() if len(ms) == 1 else MIXED)


class SysfsPartitionBackend:
    """Writes ``current_{compute,memory}_partition`` of each ASIC's PCI device (needs root).

    A compute write re-partitions that ASIC at once; a memory write only requests the NPS mode,
    which the driver applies at its next reload (``memory_reloads_driver`` False)."""

    memory_reloads_driver = False

    def __init__(self, root: str = "/"):
        self.root = root

    def _write(self, dev: topo_mod.GpuDevice, attr: str, value: str) -> None:
        path = os.path.join(self.root, topo_mod.DRM_CLASS, f"card{dev.card_minor}", "device", attr)
        with open(path, "w") as f:
            f.write(value + "\n")

    def set_compute(self, dev: topo_mod.GpuDevice, mode: str) -> None:
        self._write(dev, "current_compute_partition", mode)

    def set_memory(self, dev: topo_mod.GpuDevice, mode: str) -> None:
        self._write(dev, "current_memory_partition", mode)


class PartitionManager:
    def __init__(self, client: kube_mod.KubeClient, node_name: str, backend, root: str = "/",
                 default_compute: str = "SPX", default_memory: str = "NPS1",
                 drain_timeout: float = 600.0, reenum_timeout: float = 300.0, poll: float = 2.0,
                 pause_marker: str = PAUSE_MARKER, min_gfx: int = topo_mod.GFX950,
                 resource: str = "amd.com/gpu", sleep: Callable[[float], None] = time.sleep,
                 drain_policy: str = "evict", pause_ack_timeout: float = 60.0,
                 apply_retries: int = 5, retry_backoff: float = 1.0,
                 ack_dir: str = pause_mod.ACK_DIR,
                 ack_components: Sequence[str] = pause_mod.COMPONENTS,
                 reservation: Optional[str] = "/run/amd/validations/in-test.json",
                 reload_cmd: Sequence[str] = (), run_cmd: Optional[Callable] = None):
        if drain_policy not in DRAIN_POLICIES:
            raise ValueError(f"drainPolicy must be one of {DRAIN_POLICIES}")
        self.client = client
        self.node = node_name
        self.backend = backend
        self.root = root
        self.default_compute = default_compute
        self.default_memory = default_memory
        self.drain_timeout = drain_timeout
        self.reenum_timeout = reenum_timeout
        self.poll = poll
        self.pause_marker = pause_marker
        self.min_gfx = min_gfx
        self.resource = resource
        self.sleep = sleep
        self.drain_policy = drain_policy
        self.pause_ack_timeout = pause_ack_timeout
        self.apply_retries = apply_retries
        self.retry_backoff = retry_backoff
        self.ack_dir = ack_dir
        self.ack_components = tuple(ack_components)
        self.reservation = reservation
        # argv that reloads amdgpu (e.g. a host script: modprobe -r amdgpu && modprobe amdgpu) for
        # a sysfs-requested NPS change; empty: report pending-reload instead
        self.reload_cmd = list(reload_cmd)
        self.run_cmd = run_cmd or (lambda argv: __import__("subprocess").run(
            list(argv), capture_output=True, text=True, timeout=600).returncode)

    # ---------------------------------------------------------------- helpers
    def _state(self, state: str, reason: str = "") -> None:
        self.client.set_node_annotations(self.node, {ANNOT_STATE: f"{state}{': ' + reason if reason else ''}"})
        log.info("partition state %s %s", state, reason)

    def _pause(self, on: bool) -> Optional[str]:
        if on:
            return pause_mod.start_pause(self.pause_marker, self.ack_dir)
        pause_mod.end_pause(self.pause_marker)
        return None

    def desired(self) -> tuple:
        labels = self.client.get_node(self.node).get("metadata", {}).get("labels", {}) or {}
        return (labels.get(LABEL_DESIRED, self.default_compute).upper(),
                labels.get(LABEL_MEM_DESIRED, self.default_memory).upper())

    def current(self) -> tuple:
        """(compute, memory, topology) of the node; a mode is ``mixed`` when the ASICs disagree."""
        topo = topo_mod.read_topology(self.root, self.min_gfx)
        if not topo.gpus:
            raise PartitionError("no GPUs in the KFD topology")
        c, m = node_mode(asic_modes(topo))
        return c, m, topo

    def gpu_pods(self) -> list:
        pods = self.client.list_pods(field_selector=f"spec.nodeName={self.node}")
        return [p for p in pods
                if p.get("status", {}).get("phase") in ("Pending", "Running", "Unknown")
                and kube_mod.pod_gpu_request(p, self.resource) > 0]

    # ---------------------------------------------------------------- reconcile
    def reconcile(self) -> str:
        want_c, want_m = self.desired()
        if want_c not in topo_mod.PARTITION_SPLIT:
            self._state("failed", f"unknown compute partition {want_c}")
            return "failed"
        cur_c, cur_m, topo = self.current()
        modes = asic_modes(topo)
        asics = topo.asics()
        # PCI order (ASIC 0 = lowest bus), so a partial failure is reported and resumed predictably
        off = sorted((uid for uid, cm in modes.items() if cm != (want_c, want_m)),
                     key=lambda u: asics[u][0].pci_bdf)
        if not off:
            self._pause(False)
            self.client.set_taint(self.node, TAINT_KEY, "", present=False)
            self._state("idle")
            return "idle"
        mem_off = any(m != want_m for _, m in modes.values())
        reloads = getattr(self.backend, "memory_reloads_driver", False)
        if mem_off and not reloads and not self.reload_cmd:
            annot = (self.client.get_node(self.node).get("metadata", {}).get("annotations") or {})
            if str(annot.get(ANNOT_STATE, "")).startswith(f"pending-reload: {want_m}"):
                return "pending-reload"      # requested before; only a driver reload applies it
        avail = topo_mod.available_partitions(self.root, asics[off[0]][0])
        if want_c not in avail:
            self._state("failed", f"{want_c} not in available {','.join(avail)}")
            return "failed"
        log.info("node %s: %s/%s -> %s/%s on %d of %d ASIC(s)", self.node, cur_c, cur_m, want_c,
                 want_m, len(off), len(asics))
        # 1. stop new GPU work landing here; hide devices from kubelet; pause the operator's own
        #    GPU clients; move the GPU pods off (Eviction API, PDBs honoured)
        self.client.set_taint(self.node, TAINT_KEY, want_c, present=True)
        nonce = self._pause(True)
        self._state("draining", f"{cur_c}->{want_c} (drainPolicy {self.drain_policy})")
        deadline = time.monotonic() + self.drain_timeout
        err = self.drain(deadline)
        if err:
            self._abort(err)
            return "failed"
        # 2. the operator's GPU clients have closed their handles
        self._state("quiescing", "waiting for exporter / driver probe / device plugin to release the GPUs")
        missing = self.wait_acks(nonce)
        if missing:
            log.warning("no pause ack from %s after %.0f s; applying anyway (EBUSY is retried)",
                        ",".join(missing), self.pause_ack_timeout)
        err = self._wait_validator_idle(deadline)
        if err:
            self._abort(err)
            return "failed"
        # 3. memory partition: hive-wide, once per node, before any compute change
        if mem_off:
            head = asics[off[0]][0]
            self._state("applying", f"memory partition {want_m} (hive-wide, driver reload)")
            try:
                self._apply(self.backend.set_memory, head, want_m)
            except Exception as e:  # noqa: BLE001
                self._abort(f"memory partition {want_m} failed on {head.pci_bdf}: {e}")
                return "failed"
            if not reloads:
                if not self.reload_cmd:
                    self._pause(False)
                    self.client.set_taint(self.node, TAINT_KEY, "", present=False)
                    self._state("pending-reload",
                                f"{want_m} requested through sysfs; the amdgpu driver applies it "
                                f"at its next reload (set partition.driverReloadCommand, or "
                                f"reboot); compute {want_c} follows after that")
                    return "pending-reload"
                self._state("applying", f"reloading amdgpu for {want_m}: {' '.join(self.reload_cmd)}")
                rc = self.run_cmd(self.reload_cmd)
                if rc != 0:
                    self._abort(f"driver reload command failed (rc={rc})")
                    return "failed"
            self._state("reenumerating", f"memory partition {want_m}")
            # the reload keeps every ASIC's compute mode, so a CPX ASIC comes back as 8 agents
            agents = sum(topo_mod.PARTITION_SPLIT.get(c, 1) for c, _ in modes.values())
            got = self._wait_modes(lambda ms: all(m == want_m for _, m in ms.values()),
                                   agents, f"every ASIC in {want_m}")
            if isinstance(got, str):
                self._abort(got)
                return "failed"
            topo = got
            modes = asic_modes(topo)
            asics = topo.asics()
        # 4. compute partition per ASIC, each handle looked up fresh (the backend re-opens its
        #    amd-smi session after every change)
        c_off = sorted((uid for uid, (c, _) in modes.items() if c != want_c),
                       key=lambda u: asics[u][0].pci_bdf)
        self._state("applying", f"{want_c} on {len(c_off)} ASIC(s)")
        done: List[str] = []
        for uid in c_off:
            head = asics[uid][0]
            err = self._wait_validator_idle(deadline)
            if err:
                self._abort(err)
                return "failed"
            try:
                self._apply(self.backend.set_compute, head, want_c)
            except Exception as e:  # noqa: BLE001
                self._abort(f"apply failed on {head.pci_bdf} after {len(done)} of {len(c_off)} "
                            f"ASIC(s) switched: {e}")
                return "failed"
            done.append(head.pci_bdf)
        # 5. wait for the driver to re-enumerate every ASIC in the new mode
        self._state("reenumerating")
        got = self._wait_modes(lambda ms: all(cm == (want_c, want_m) for cm in ms.values()),
                               len(asics) * topo_mod.PARTITION_SPLIT[want_c],
                               f"{want_c}/{want_m}")
        if isinstance(got, str):
            self._abort(got)
            return "failed"
        # 6. resume (the paused clients re-open re-enumerated handles)
        self._pause(False)
        self.client.set_taint(self.node, TAINT_KEY, "", present=False)
        self.client.set_node_labels(self.node, {"amd.com/gpu.compute-partition": want_c,
                                                "amd.com/gpu.memory-partition": want_m})
        # the new agents have new device IDs: with the validator's gate on they are allocatable
        # once the validator (its hold loop sees the topology change) has re-run the GEMM on them
        self._state("idle", f"applied {want_c}/{want_m} ({len(done)} compute, "
                            f"{1 if mem_off else 0} memory change); new agents are allocatable "
                            f"after the validator's GEMM pass on them")
        return "applied"

    def _wait_modes(self, ok, agents: int, what: str):
        """Poll the KFD topology until ``ok(asic modes)`` holds with ``agents`` agents; returns
        the topology, or the failure reason past ``reenum_timeout``."""
        deadline = time.monotonic() + self.reenum_timeout
        while True:
            try:
                t = topo_mod.read_topology(self.root, self.min_gfx)
                if t.gpus and ok(asic_modes(t)) and len(t.gpus) == agents:
                    return t
            except (PartitionError, FileNotFoundError):
                pass
            if time.monotonic() >= deadline:
                return f"re-enumeration timeout (expected {agents} agents, {what})"
            self.sleep(self.poll)

    def _wait_validator_idle(self, deadline: float) -> Optional[str]:
        """A validator load step that reserved GPUs after the drain finished is waited for."""
        while self._validator_busy():
            if time.monotonic() >= deadline:
                return "drain timeout: a validator load step is still running"
            self.sleep(self.poll)
        return None

    def _validator_busy(self) -> bool:
        """A validator load step holds a live reservation (it is loading the GPUs right now)."""
        if not self.reservation:
            return False
        try:
            with open(self.reservation) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            return False
        return float(doc.get("expires", 0)) > time.time()

    def drain(self, deadline: float) -> Optional[str]:
        """Empty the node of GPU pods; returns None when drained, else the failure reason."""
        blocked: Dict[str, str] = {}
        while True:
            busy = self.gpu_pods()
            validating = self._validator_busy()
            if not busy and not validating:
                return None
            if self.drain_policy == "evict":
                for p in busy:
                    md = p.get("metadata", {})
                    if md.get("deletionTimestamp"):
                        continue          # already terminating
                    key = f"{md.get('namespace')}/{md.get('name')}"
                    try:
                        self.client.evict_pod(md.get("namespace"), md.get("name"))
                        blocked.pop(key, None)
                        log.info("evicted GPU pod %s", key)
                    except kube_mod.KubeError as e:
                        # 429: the eviction would violate a PodDisruptionBudget — retry later
                        blocked[key] = (e.message if e.status == 429
                                        else f"HTTP {e.status}: {e.message}")[:200]
            if time.monotonic() >= deadline:
                names = ",".join(p["metadata"]["name"] for p in busy[:5])
                if blocked:
                    return "drain timeout: eviction refused for " + "; ".join(
                        f"{k} ({v})" for k, v in sorted(blocked.items())[:5])
                if not busy:
                    return "drain timeout: a validator load step is still running"
                return f"drain timeout: GPU pods still running ({names})" + \
                    (" [drainPolicy wait]" if self.drain_policy == "wait" else "")
            self.sleep(self.poll)

    def wait_acks(self, nonce: Optional[str]) -> List[str]:
        """Wait for every paused component's ack; returns those that never acked."""
        if not nonce or not self.ack_components:
            return []
        deadline = time.monotonic() + self.pause_ack_timeout
        while True:
            got = pause_mod.acks(nonce, self.ack_dir, self.ack_components)
            missing = [c for c, ok in got.items() if not ok]
            if not missing or time.monotonic() >= deadline:
                return missing
            self.sleep(min(self.poll, 1.0))

    def _apply(self, fn, head: topo_mod.GpuDevice, mode: str) -> None:
        """One sysfs / amd-smi write, retried with exponential backoff while the device is busy."""
        for attempt in range(self.apply_retries + 1):
            try:
                fn(head, mode)
                return
            except Exception as e:  # noqa: BLE001
                if not is_busy(e) or attempt == self.apply_retries:
                    raise
                delay = self.retry_backoff * (2 ** attempt)
                log.warning("%s busy (%s); retry %d/%d in %.1f s", head.pci_bdf, e, attempt + 1,
                            self.apply_retries, delay)
                self.sleep(delay)

    def _abort(self, reason: str) -> None:
        self._pause(False)
        self.client.set_taint(self.node, TAINT_KEY, "", present=False)
        self._state("failed", reason)

    def run(self, interval: float = 30.0, stop_event=None) -> None:
        import threading

        stop_event = stop_event or threading.Event()
        while not stop_event.is_set():
            try:
                self.reconcile()
            except Exception as e:  # noqa: BLE001
                log.warning("reconcile failed: %s", e)
            stop_event.wait(interval)
