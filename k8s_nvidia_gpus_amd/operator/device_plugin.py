"""``amd.com/gpu`` kubelet device plugin for MI355X nodes.

Replaces the NVIDIA k8s-device-plugin the reference gets from its GPU Operator chart (the
``nvidia.com/gpu`` requests in reference README.md:286,348, llm/deployment.yaml:90,
sd15-api/deployment.yaml:66; "Device Plugin shows 0 GPUs" troubleshooting in README.md:529-532).

Design (MI355X-first):

* **Enumeration from KFD sysfs** (:mod:`k8s_nvidia_gpus_amd.utils.topology`): one device per GPU in
  SPX mode, one per compute partition in DPX/QPX/CPX mode (8 per MI355X in CPX), each with its own
  ``/dev/dri/renderD*``.  Device IDs are the stable ASIC unique id (+ ``-p<i>`` per partition), so a
  device keeps its ID across reboots and PCI renumbering.
* **Isolation by device cgroup, never by env.**  ``Allocate`` returns ``DeviceSpec`` s for the shared
  ``/dev/kfd`` plus exactly the allocated render nodes (or, in ``cdi`` mode, CDI names resolved from
  /etc/cdi/amd.com-gpu.json).  No ``*_VISIBLE_DEVICES`` variable is involved, so a pod cannot widen
  its access by setting one (the reference's ``NVIDIA_VISIBLE_DEVICES=all`` hazard).
  Container annotations carry the allocated render minors for ``amd-container-runtime``.
* **Topology-aware preferred allocation.**  Every MI355X of a node is one hop from every other over
  xGMI (full mesh, 7 links), so for whole GPUs the useful locality is the host NUMA node (CPU-side
  staging, RCCL proxy threads) — a 2- or 4-GPU request is packed into one socket, best-fit so large
  free blocks survive.  Partitions of one ASIC share its HBM stacks and Infinity Cache, so
  multi-partition requests are packed onto as few ASICs as possible.
* **Health**: devices that vanish from the KFD topology or /dev, or exceed the uncorrectable-ECC
  threshold (amd-smi), are reported ``Unhealthy`` through ``ListAndWatch``.
* **Kubelet restarts**: kubelet deletes every plugin socket when it restarts; the plugin watches
  ``kubelet.sock`` and its own socket and re-serves + re-registers.
* **Partition changes**: while ``/run/amd/partition-in-progress`` exists (the partition manager's
  drain marker) the plugin advertises no devices, releases its amd-smi (ECC) session and acks the
  pause (:mod:`.pause`), then re-enumerates and re-opens when the marker goes away.
* **Validation gate** (:class:`ValidationGate`): with ``validator.gateOnValidation`` a device is
  Healthy only after the validator's load steps passed on it this boot, and the devices a load
  step is about to load are reported Unhealthy for its duration (the validator's TOCTOU guard).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from concurrent import futures
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

from ..utils import topology as topo_mod
from . import deviceplugin_api as api
from .config import OperatorConfig

log = logging.getLogger("amd-device-plugin")

PAUSE_MARKER = "/run/amd/partition-in-progress"
ANNOT_RENDER_MINORS = "amd.com/gpu.render-minors"
ANNOT_DEVICE_IDS = "amd.com/gpu.device-ids"
CDI_KIND = "amd.com/gpu"

HealthFn = Callable[[List[topo_mod.GpuDevice]], Dict[str, str]]


class PresenceHealth:
    """Device is healthy while its KFD agent and its render node exist.

    Optional ``ecc_fn(device) -> uncorrectable count`` adds the ECC criterion (amd-smi backed in
    production, a fake in tests)."""

    def __init__(self, root: str = "/", ecc_fn: Optional[Callable] = None, ecc_threshold: int = 1):
        self.root = root
        self.ecc_fn = ecc_fn
        self.ecc_threshold = ecc_threshold

    def __call__(self, devices: List[topo_mod.GpuDevice]) -> Dict[str, str]:
        out = {}
        for d in devices:
            ok = os.path.exists(os.path.join(self.root, d.render_path.lstrip("/")))
            if ok and self.ecc_fn is not None and self.ecc_threshold > 0:
                try:
                    ok = int(self.ecc_fn(d)) < self.ecc_threshold
                except Exception as e:  # noqa: BLE001 - an unreadable counter is not a failure
                    log.debug("ECC read failed for %s: %s", d.device_uid, e)
            out[d.device_uid] = api.HEALTHY if ok else api.UNHEALTHY
        return out


class AmdSmiEccReader:
    """``ecc_fn`` for :class:`PresenceHealth`: the uncorrectable-ECC count of a device's ASIC, read
    through amd-smi (``amdsmi_get_gpu_total_ecc_count``, the same call the exporter samples).

    Devices are matched to amd-smi processor handles by PCI BDF.  A compute partition that amd-smi
    does not list under its own BDF falls back to the ASIC's other functions (same
    domain:bus:device): ECC is an HBM property, shared by every partition of one MI355X, so the
    highest count among them is the ASIC's.  The BDF → handle map is rebuilt on a miss, because a
    partition change re-enumerates the handles."""

    def __init__(self, amdsmi_module=None):
        if amdsmi_module is None:
            import amdsmi as amdsmi_module  # noqa: N813 - optional dependency
        self.S = amdsmi_module
        self.S.amdsmi_init()
        self.active = True
        self._by_bdf: Dict[str, object] = {}

    def suspend(self) -> None:
        """Release the amd-smi session for a partition change (pause.py); handles go stale."""
        if self.active:
            self.close()
            self.active = False
            self._by_bdf = {}

    def resume(self) -> None:
        if not self.active:
            self.S.amdsmi_init()
            self.active = True

    def _rebuild(self) -> None:
        self._by_bdf = {}
        for h in self.S.amdsmi_get_processor_handles() or []:
            try:
                self._by_bdf[str(self.S.amdsmi_get_gpu_device_bdf(h)).lower()] = h
            except Exception as e:  # noqa: BLE001 - a handle without a BDF cannot be matched
                log.debug("amd-smi BDF read failed: %s", e)

    def _handles(self, bdf: str) -> List[object]:
        for attempt in (0, 1):
            if bdf in self._by_bdf:
                return [self._by_bdf[bdf]]
            asic = bdf.rsplit(".", 1)[0]
            same = [h for b, h in self._by_bdf.items() if b.rsplit(".", 1)[0] == asic]
            if same:
                return same
            if attempt == 0:
                self._rebuild()
        raise LookupError(f"no amd-smi handle for {bdf}")

    def __call__(self, d: topo_mod.GpuDevice) -> int:
        if not self.active:
            raise LookupError("amd-smi session released (partition change in progress)")
        counts = []
        for h in self._handles(d.pci_bdf.lower()):
            ecc = self.S.amdsmi_get_gpu_total_ecc_count(h) or {}
            counts.append(int(ecc.get("uncorrectable_count") or 0))
        return max(counts)

    def close(self) -> None:
        try:
            self.S.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass


def default_ecc_fn(threshold: int) -> Optional[Callable]:
    """The production ECC criterion: amd-smi backed when the threshold is enabled, else None.

    Without amd-smi (no library, no device access) the plugin still runs on presence alone and
    says so, instead of silently ignoring ``health.eccUncorrectableThreshold``."""
    if threshold <= 0:
        return None
    try:
        return AmdSmiEccReader()
    except Exception as e:  # noqa: BLE001 - no amd-smi in this image / no device access
        log.warning("amd-smi unavailable (%s): the uncorrectable-ECC health check "
                    "(threshold %d) is disabled, presence checks only", e, threshold)
        return None


class ValidationGate:
    """The validator's say in what the plugin advertises (files in ``/run/amd/validations``).

    * ``validated-devices.json`` ``{boot_id, device_uids}`` — with ``gate`` on, a device is reported
      Healthy only once every enabled validator load step has passed on it this boot: on first boot
      no pod can be handed a GPU before the validator has loaded it (else a fully allocated node
      would be labelled validated with zero GEMMs run).
    * ``in-test.json`` ``{nonce, device_uids, expires}`` — the agents a load step is about to load;
      reported Unhealthy (kubelet stops allocating them) until the file is removed or expires.
      After publishing that state the plugin writes the nonce to ``in-test.ack``; the validator
      then re-reads PodResources and drops any agent a pod took in between.
    """

    def __init__(self, marker_dir: str, root: str = "/", gate: bool = True,
                 clock: Callable[[], float] = time.time):
        self.marker_dir = marker_dir
        self.root = root
        self.gate = gate
        self.clock = clock

    def _json(self, name: str):
        try:
            with open(os.path.join(self.marker_dir, name)) as f:
                return json.load(f)
        except (OSError, ValueError):
            return None

    def boot_id(self) -> str:
        try:
            with open(os.path.join(self.root, "proc/sys/kernel/random/boot_id")) as f:
                return f.read().strip()
        except OSError:
            return ""

    def stamp(self) -> Tuple:
        """Changes whenever either file does (cheap: polled every plugin loop iteration)."""
        out = []
        for name in ("validated-devices.json", "in-test.json"):
            try:
                st = os.stat(os.path.join(self.marker_dir, name))
                out.append((st.st_mtime_ns, st.st_ino, st.st_size))
            except OSError:
                out.append(None)
        return tuple(out)

    def state(self) -> Tuple[Optional[set], set, Optional[str]]:
        """(validated uids or None when not gating, reserved uids, reservation nonce)."""
        validated = None
        if self.gate:
            doc = self._json("validated-devices.json") or {}
            validated = set(doc.get("device_uids") or []) if doc.get("boot_id") == self.boot_id() else set()
        res = self._json("in-test.json") or {}
        if res and float(res.get("expires", 0)) > self.clock():
            return validated, set(res.get("device_uids") or []), str(res.get("nonce", ""))
        return validated, set(), None

    def ack(self, nonce: str) -> None:
        path = os.path.join(self.marker_dir, "in-test.ack")
        try:
            with open(path + ".tmp", "w") as f:
                f.write(nonce + "\n")
            os.replace(path + ".tmp", path)
        except OSError as e:
            log.warning("cannot ack reservation %s: %s", nonce, e)


def preferred_allocation(available: Sequence[topo_mod.GpuDevice],
                         must_include: Sequence[topo_mod.GpuDevice], size: int) -> List[topo_mod.GpuDevice]:
    """Pick ``size`` devices: must_include first, then pack by ASIC, then NUMA node (best fit)."""
    chosen = list(must_include)
    pool = [d for d in available if d.device_uid not in {c.device_uid for c in chosen}]
    index = {d.device_uid: i for i, d in enumerate(available)}

    def free_by(key_fn, devs):
        out: Dict[object, int] = {}
        for d in devs:
            out[key_fn(d)] = out.get(key_fn(d), 0) + 1
        return out

    while len(chosen) < size and pool:
        need = size - len(chosen)
        asics_used = {d.unique_id for d in chosen}
        numas_used = {d.numa_node for d in chosen}
        free_asic = free_by(lambda d: d.unique_id, pool)
        free_numa = free_by(lambda d: d.numa_node, pool)

        def fit(free: int) -> Tuple[int, int]:
            # best fit: a group that can take the whole remainder with the least left over,
            # otherwise the largest group (fewest groups overall)
            return (0, free - need) if free >= need else (1, -free)

        def score(d: topo_mod.GpuDevice):
            return (
                0 if d.unique_id in asics_used else 1,
                0 if (not numas_used or d.numa_node in numas_used) else 1,
                fit(free_asic[d.unique_id]) if d.partitions_on_asic > 1 else (0, 0),
                fit(free_numa[d.numa_node]),
                index[d.device_uid],
            )

        best = min(pool, key=score)
        chosen.append(best)
        pool.remove(best)
    return chosen[:size] if size > 0 else chosen


class AmdGpuDevicePlugin:
    """The gRPC DevicePlugin service + registration/health/re-registration loops."""

    def __init__(self, config: OperatorConfig, root: str = "/",
                 kubelet_dir: str = api.DEVICE_PLUGIN_PATH, socket_name: str = "amd-gpu.sock",
                 topology_fn: Optional[Callable[[], topo_mod.NodeTopology]] = None,
                 health_fn: Optional[HealthFn] = None, pause_marker: Optional[str] = PAUSE_MARKER,
                 dev_prefix: str = "/dev", ecc_fn: Optional[Callable] = None,
                 id_map_path: Optional[str] = None, gate: Optional[ValidationGate] = None,
                 pause_guard=None):
        self.config = config
        self.gate = gate
        self._gate_stamp = None
        # pause.PauseGuard("device-plugin"): release the ECC reader's amd-smi session while the
        # partition manager switches modes (the pause marker is the same file as pause_marker)
        self.pause_guard = pause_guard
        self._ecc = None
        # {kubelet device ID: device_uid} for the validator, which maps kubelet's PodResources
        # answer to GPUs with it (needed with deviceIdStrategy: index)
        self.id_map_path = id_map_path
        self.root = root
        self.kubelet_dir = kubelet_dir
        self.socket_path = os.path.join(kubelet_dir, socket_name)
        self.kubelet_socket = os.path.join(kubelet_dir, api.KUBELET_SOCKET)
        self.topology_fn = topology_fn or (lambda: topo_mod.read_topology(root, config.min_gfx))
        if health_fn is None:
            threshold = int(config.section("health")["eccUncorrectableThreshold"])
            self._ecc = ecc_fn or default_ecc_fn(threshold)
            health_fn = PresenceHealth(root, ecc_fn=self._ecc, ecc_threshold=threshold)
        self.health_fn = health_fn
        self.pause_marker = pause_marker
        self.dev_prefix = dev_prefix
        self._cond = threading.Condition()
        self._version = 0
        self._devices: List[topo_mod.GpuDevice] = []
        self._health: Dict[str, str] = {}
        self._index: Dict[str, int] = {}   # device_uid -> stable index (deviceIdStrategy: index)
        self._paused = False
        self._server = None
        self._stop = threading.Event()
        self.registrations = 0
        self.refresh()

    # ------------------------------------------------------------------ state
    def _id(self, d: topo_mod.GpuDevice) -> str:
        """Kubelet-facing ID.  With ``deviceIdStrategy: index`` a device keeps the index it got when
        first seen, for the plugin's lifetime: kubelet checkpoints allocated IDs, so an index must
        never move to another physical GPU when an earlier one disappears."""
        if self.config["deviceIdStrategy"] != "index":
            return d.device_uid
        idx = self._index.get(d.device_uid)
        if idx is None:
            idx = self._index[d.device_uid] = len(self._index)
        return str(idx)

    def _id_map(self) -> Dict[str, topo_mod.GpuDevice]:
        return {self._id(d): d for d in self._devices}

    def refresh(self) -> bool:
        """Re-enumerate + re-check health; returns True (and wakes ListAndWatch) on any change."""
        paused = bool(self.pause_marker and os.path.exists(self.pause_marker))
        if not paused and self._ecc is not None and not getattr(self._ecc, "active", True):
            try:
                self._ecc.resume()          # partition change over: re-open on the new handles
            except Exception as e:  # noqa: BLE001 - ECC criterion off until the next refresh
                log.warning("cannot re-open amd-smi after the partition change: %s", e)
        try:
            devices = [] if paused else list(self.topology_fn().gpus)
        except FileNotFoundError as e:
            log.warning("topology unavailable: %s", e)
            devices = []
        # devices that were advertised and disappeared stay listed as Unhealthy
        known = {d.device_uid: d for d in devices}
        if not paused:
            for d in self._devices:
                if d.device_uid not in known:
                    known[d.device_uid] = d
        merged = list(known.values()) if not paused else []
        health = self.health_fn(merged) if merged else {}
        present = {d.device_uid for d in devices}
        for uid in list(health):
            if uid not in present:
                health[uid] = api.UNHEALTHY
        nonce = None
        if self.gate is not None:
            self._gate_stamp = self.gate.stamp()
            validated, reserved, nonce = self.gate.state()
            for uid in health:
                if (validated is not None and uid not in validated) or uid in reserved:
                    health[uid] = api.UNHEALTHY
        with self._cond:
            changed = (paused != self._paused or health != self._health
                       or [d.device_uid for d in merged] != [d.device_uid for d in self._devices])
            if changed:
                self._devices, self._health, self._paused = merged, health, paused
                for d in merged:   # assign indices in enumeration order, once
                    self._id(d)
                self._version += 1
                self._cond.notify_all()
        if changed:
            self._write_id_map()
            log.info("advertising %d device(s) (%d healthy)%s", len(merged),
                     sum(1 for v in health.values() if v == api.HEALTHY), " [paused]" if paused else "")
        if nonce:
            # the reserved devices' Unhealthy state is published (ListAndWatch woken above)
            self.gate.ack(nonce)
        if paused and self.pause_guard is not None:
            # zero devices are published; drop the amd-smi session, then tell the manager
            if self._ecc is not None and hasattr(self._ecc, "suspend"):
                self._ecc.suspend()
            self.pause_guard.ack()
        elif self.pause_guard is not None:
            self.pause_guard.clear()
        return changed

    def _write_id_map(self) -> None:
        if not self.id_map_path:
            return
        with self._cond:
            m = {self._id(d): d.device_uid for d in self._devices}
        try:
            os.makedirs(os.path.dirname(self.id_map_path), exist_ok=True)
            tmp = self.id_map_path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(m, f)
            os.replace(tmp, self.id_map_path)
        except OSError as e:
            log.warning("cannot write %s: %s", self.id_map_path, e)

    def list_response(self):
        resp = api.ListAndWatchResponse()
        with self._cond:
            for d in self._devices:
                dev = resp.devices.add(ID=self._id(d), health=self._health.get(d.device_uid, api.UNHEALTHY))
                if d.numa_node >= 0:
                    dev.topology.nodes.add(ID=d.numa_node)
        return resp

    # ------------------------------------------------------------------ RPCs
    def GetDevicePluginOptions(self, request, context):
        return api.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):
        seen = -1
        while not self._stop.is_set():
            with self._cond:
                if self._version == seen:
                    self._cond.wait(timeout=1.0)
                if self._version == seen:
                    if context is not None and hasattr(context, "is_active") and not context.is_active():
                        return
                    continue
                seen = self._version
            yield self.list_response()

    def GetPreferredAllocation(self, request, context):
        resp = api.PreferredAllocationResponse()
        ids = self._id_map()
        rev = {d.device_uid: k for k, d in ids.items()}
        for creq in request.container_requests:
            avail = [ids[i] for i in creq.available_deviceIDs if i in ids]
            must = [ids[i] for i in creq.must_include_deviceIDs if i in ids]
            if self.config.section("allocation")["preferXgmiLocality"]:
                picked = preferred_allocation(avail, must, int(creq.allocation_size))
            else:
                picked = (must + [d for d in avail if d not in must])[: int(creq.allocation_size)]
            resp.container_responses.add(deviceIDs=[rev[d.device_uid] for d in picked])
        return resp

    def container_response(self, device_ids: Iterable[str]):
        ids = self._id_map()
        devs = []
        for i in device_ids:
            if i not in ids:
                raise KeyError(f"unknown device id {i!r}")
            devs.append(ids[i])
        alloc = self.config.section("allocation")
        r = api.ContainerAllocateResponse()
        if alloc["mode"] == "cdi":
            for i in device_ids:
                r.cdi_devices.add(name=f"{CDI_KIND}={ids[i].device_uid}")
        else:
            kfd = os.path.join(self.dev_prefix, "kfd")
            r.devices.add(container_path="/dev/kfd", host_path=kfd, permissions="rw")
            for d in devs:
                host = os.path.join(self.dev_prefix, "dri", f"renderD{d.render_minor}")
                r.devices.add(container_path=d.render_path, host_path=host, permissions="rw")
                if alloc["cardNodes"] and d.card_minor is not None:
                    r.devices.add(container_path=d.card_path,
                                  host_path=os.path.join(self.dev_prefix, "dri", f"card{d.card_minor}"),
                                  permissions="rw")
        r.annotations[ANNOT_RENDER_MINORS] = ",".join(str(d.render_minor) for d in devs)
        r.annotations[ANNOT_DEVICE_IDS] = ",".join(d.device_uid for d in devs)
        # informational only: isolation never depends on it (see module docstring)
        r.envs["AMD_GPU_DEVICE_IDS"] = ",".join(d.device_uid for d in devs)
        return r

    def Allocate(self, request, context):
        resp = api.AllocateResponse()
        for creq in request.container_requests:
            try:
                resp.container_responses.append(self.container_response(list(creq.devices_ids)))
            except KeyError as e:
                if context is not None:
                    import grpc

                    context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
                raise
        return resp

    def PreStartContainer(self, request, context):
        return api.PreStartContainerResponse()

    # ------------------------------------------------------------------ serving
    def serve(self) -> None:
        import grpc

        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
        self._stop.clear()
        server = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        server.add_generic_rpc_handlers([api.generic_handler("DevicePlugin", {
            "GetDevicePluginOptions": self.GetDevicePluginOptions,
            "ListAndWatch": self.ListAndWatch,
            "GetPreferredAllocation": self.GetPreferredAllocation,
            "Allocate": self.Allocate,
            "PreStartContainer": self.PreStartContainer,
        })])
        server.add_insecure_port(api.unix_target(self.socket_path))
        server.start()
        self._server = server
        log.info("serving DevicePlugin on %s", self.socket_path)

    def register(self, timeout: float = 10.0) -> None:
        import grpc

        with grpc.insecure_channel(api.unix_target(self.kubelet_socket)) as ch:
            grpc.channel_ready_future(ch).result(timeout=timeout)
            api.Stub(ch, "Registration").Register(api.RegisterRequest(
                version=api.VERSION, endpoint=os.path.basename(self.socket_path),
                resource_name=self.config.resource_name,
                options=api.DevicePluginOptions(get_preferred_allocation_available=True)),
                timeout=timeout)
        self.registrations += 1
        log.info("registered %s with kubelet (%d)", self.config.resource_name, self.registrations)

    def stop(self) -> None:
        self._stop.set()
        with self._cond:
            self._cond.notify_all()
        if self._server is not None:
            self._server.stop(grace=0.5).wait()
            self._server = None

    def _inode(self, path: str) -> Optional[int]:
        try:
            return os.stat(path).st_ino
        except OSError:
            return None

    def run(self, health_interval: Optional[float] = None, poll: float = 1.0,
            stop_event: Optional[threading.Event] = None) -> None:
        """Serve, register, then loop: health refresh + re-register on kubelet restart."""
        stop_event = stop_event or threading.Event()
        health_interval = health_interval or float(self.config.section("health")["intervalSeconds"])
        registered_ino = None
        last_health = 0.0
        while not stop_event.is_set():
            kubelet_ino = self._inode(self.kubelet_socket)
            own_missing = self._server is None or not os.path.exists(self.socket_path)
            if kubelet_ino is not None and (own_missing or kubelet_ino != registered_ino):
                try:
                    self.stop()
                    self.serve()
                    self.register()
                    registered_ino = kubelet_ino
                except Exception as e:  # noqa: BLE001 - kubelet may be mid-restart; retry
                    log.warning("registration failed (%s); retrying", e)
                    registered_ino = None
            now = time.monotonic()
            if now - last_health >= health_interval:
                self.refresh()
                last_health = now
            elif self.gate is not None and self.gate.stamp() != self._gate_stamp:
                self.refresh()      # a reservation / validation result: apply it within one poll
            elif self.pause_marker and os.path.exists(self.pause_marker) != self._paused:
                self.refresh()      # a partition change starts / ends: follow it within one poll
            stop_event.wait(poll)
        self.stop()


def main(args) -> int:  # pragma: no cover - container entry point (exercised via run() in tests)
    from .config import load_config

    cfg = load_config(args.config) if args.config and os.path.exists(args.config) else load_config()
    plugin = AmdGpuDevicePlugin(cfg, root=args.root, kubelet_dir=args.kubelet_dir)
    plugin.run()
    return 0
