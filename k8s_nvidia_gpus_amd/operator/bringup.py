"""Node bring-up rehearsal: the node-local half of time-to-first-GPU-pod, measured on real hardware.

BASELINE.json's headline metric pairs the validator GEMM with *time-to-first-GPU-pod*.  On a
cluster that is ``tools/time_to_first_gpu_pod.py`` (``kubectl apply`` → validated node → first
``amd.com/gpu: 1`` pod passing vectorAdd).  The GPU pool this repository is measured on has
MI355X boxes but no Kubernetes, so this module runs every node-local step of that path with the
operator's REAL components against the real KFD sysfs, /dev nodes, amd-smi and GPU, and stands in
only for the parts that are not on the node (API server, scheduler, image pull) and for kubelet's
socket side (:class:`.kubelet_stub.KubeletStub`, the same stand-in the CPU tests use):

  driver      kfd-probe sees the expected gfx950 agents and opens /dev/kfd + render nodes
  runtime     amd-container-runtime + CDI spec installed (into the work dir's host prefix)
  plugin      device plugin serves, registers with kubelet, first ListAndWatch
  vectoradd   (gated order) the validator's vectorAdd on every GPU
  gemm        (gated order) the validator's bf16 + fp8 GEMMs: the per-device gate step
  allocatable (gated order) ListAndWatch turns a GPU Healthy (validated-devices.json)
  allocate    kubelet's GetPreferredAllocation + Allocate for ``amd.com/gpu: 1``
  create      the runtime shim edits the pod's OCI spec from the Allocate annotations: /dev/kfd +
              exactly the allocated render node, with device-cgroup rules
  container   the pod's process (amd-vectoradd, reference protocol) on the allocated GPU
              → time_to_first_gpu_pod_s
  validate    (optional) the rest of the validator chain (ungated order: all of it) → report
              → time_to_validated_s

Two orders.  **Gated** (``gated=True``, the shipped configuration: ``validator.gateOnValidation``)
builds the plugin with the :class:`ValidationGate`, so no GPU is advertised Healthy before the
validator's per-device gate steps (vectorAdd, then the GEMMs of ``gateSteps``) passed on it; the
first pod is allocated only after that, and the node-wide steps (bandwidth, stress, RCCL,
profiling) run after the pod.  **Ungated** is the order without the gate (plugin → pod → chain).
``main`` runs both and reports the two times to first GPU pod side by side.

The reference has no such measurement; it budgets 90 minutes for its in-cluster driver build alone
(reference cluster-config/apps/gpu-operator/helmrelease.yaml:7).  What this does NOT include: API
server / scheduler latency, image pull, and runc's namespace/cgroup setup (no runc on the box; the
container's view is approximated by HIP_VISIBLE_DEVICES on the allocated GPU).

    python -m k8s_nvidia_gpus_amd.operator bringup [--no-validate] [--workdir DIR]
"""
from __future__ import annotations

import copy
import json
import os
import shutil
import subprocess
import tempfile
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

from . import deviceplugin_api as api
from .config import OperatorConfig
from .validator import Validator, default_runner, json_lines, protocol_passed

ContainerRunner = Callable[[Sequence[str], Dict[str, str], float], subprocess.CompletedProcess]


def _run_container(argv: Sequence[str], env: Dict[str, str], timeout: float) -> subprocess.CompletedProcess:
    return subprocess.run(list(argv), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                          text=True, timeout=timeout)


@dataclass
class Stage:
    name: str
    start_s: float
    end_s: float
    ok: bool
    detail: Dict = field(default_factory=dict)


class BringupError(RuntimeError):
    pass


def _pod_spec(bundle_dir: str, annotations: Dict[str, str], command: Sequence[str]) -> Dict:
    """The OCI spec containerd would hand the runtime for the validator's vectorAdd pod."""
    return {
        "ociVersion": "1.2.0",
        "process": {"args": list(command), "env": ["PATH=/usr/local/bin:/usr/bin:/bin"],
                    "capabilities": {"bounding": ["CAP_CHOWN", "CAP_KILL"]}},
        "root": {"path": os.path.join(bundle_dir, "rootfs")},
        "annotations": dict(annotations, **{"io.kubernetes.cri.container-type": "container"}),
        "linux": {"resources": {"devices": [{"allow": False, "access": "rwm"}]}, "devices": []},
    }


def rehearse(cfg: OperatorConfig, bin_dir: str, workdir: Optional[str] = None, root: str = "/",
             validate: bool = True, runner=default_runner,
             container_runner: ContainerRunner = _run_container,
             container_cmd: Optional[Sequence[str]] = None, timeout: float = 120.0,
             driver_wait: float = 120.0, gated: Optional[bool] = None) -> Dict:
    """Run the node-local bring-up once; returns a JSON-able report (raises nothing: a failed stage
    ends the run and is reported).  ``gated``: the validation-gated order (default: the config's
    ``validator.gateOnValidation``)."""
    from .device_plugin import AmdGpuDevicePlugin, ValidationGate
    from .kubelet_stub import KubeletStub
    from .runtime import install_runtime

    if gated is None:
        gated = bool(cfg.section("validator").get("gateOnValidation", True))

    own_tmp = workdir is None
    # absolute: gRPC unix-socket addresses (the kubelet stand-in, the plugin) must not be relative
    workdir = os.path.abspath(workdir or tempfile.mkdtemp(prefix="amdk8s-bringup-"))
    markers = os.path.join(workdir, "run-amd-validations")
    host = os.path.join(workdir, "host")
    os.makedirs(markers, exist_ok=True)
    t0 = time.monotonic()
    wall0 = time.time()
    stages: List[Stage] = []
    report: Dict = {"check": "bringup", "root": root, "workdir": workdir, "start_time": wall0,
                    "order": "gated" if gated else "ungated"}
    dev_root = "" if root == "/" else root.rstrip("/")
    plugin = kubelet = None
    stop = threading.Event()

    def stage(name: str, fn: Callable[[], Dict]) -> Dict:
        s = time.monotonic() - t0
        try:
            detail = fn() or {}
            ok = bool(detail.pop("_ok", True))
        except Exception as e:  # noqa: BLE001 - every failure is a reported stage result
            detail, ok = {"error": f"{type(e).__name__}: {e}"[:500]}, False
        stages.append(Stage(name, round(s, 4), round(time.monotonic() - t0, 4), ok, detail))
        if not ok:
            raise BringupError(name)
        return detail

    # the plugin-pod step needs an API server; everything else in the chain is node-local
    vraw = copy.deepcopy(cfg.raw)
    vraw["validator"]["pluginTest"] = False
    # a bare box has no kubelet: every agent is free (in a cluster an absent socket fails the step)
    vraw["validator"]["podResourcesRequired"] = False
    kdir = os.path.join(workdir, "kubelet-device-plugins")
    if len(kdir) > 80:  # unix socket paths are limited to 107 bytes
        kdir = tempfile.mkdtemp(prefix="amdk8s-kubelet-")
    vraw["validator"]["pluginSocket"] = os.path.join(kdir, "amd-gpu.sock")
    v = Validator(OperatorConfig(vraw), markers, bin_dir=bin_dir, runner=runner, root=root,
                  driver_wait=driver_wait)
    state: Dict = {}
    try:
        def driver():
            r = v.run_step("driver")
            return {"_ok": r.passed, "gpus": r.detail.get("gpus"), "reason": r.reason}

        def runtime():
            info = install_runtime(os.path.join(bin_dir, "amd-container-runtime"),
                                   os.path.join(host, "usr/local/bin/amd-container-runtime"),
                                   os.path.join(host, "etc/cdi"), markers, root=root,
                                   min_gfx=cfg.min_gfx)
            return {"cdi_devices": info["cdi_devices"]}

        def plugin_up():
            nonlocal plugin, kubelet
            if not kdir.startswith(workdir):
                state["kdir_tmp"] = kdir
            kubelet = KubeletStub(kdir).start()
            gate = ValidationGate(markers, root=root, gate=True) if gated else None
            plugin = AmdGpuDevicePlugin(cfg, root=root, kubelet_dir=kdir, pause_marker=None,
                                        dev_prefix=os.path.join(dev_root or "/", "dev"), gate=gate)
            threading.Thread(target=plugin.run, kwargs={"poll": 0.02, "stop_event": stop},
                             daemon=True).start()
            if not kubelet.registered.wait(timeout):
                raise BringupError("device plugin never registered with kubelet")
            reg = kubelet.registrations[-1]
            ch, stub = kubelet.plugin_stub()
            watch = stub.ListAndWatch(api.Empty(), timeout=timeout + 3600)
            first = next(watch)
            healthy = [d.ID for d in first.devices if d.health == api.HEALTHY]
            state.update(channel=ch, stub=stub, healthy=healthy, watch=watch)
            # gated: nothing is Healthy before the validator's gate steps passed this boot
            return {"_ok": bool(first.devices) and (gated or bool(healthy)),
                    "resource": reg.resource_name, "endpoint": reg.endpoint,
                    "advertised": len(first.devices), "healthy": len(healthy), "gated": gated}

        def gate_step(name):
            def run():
                r = v.run_step(name)
                out = {"_ok": r.passed, "duration_s": r.detail.get("duration_s"), "reason": r.reason}
                if name == "gemm":
                    out["tflops"] = [d.get("tflops") for d in r.detail.get("devices", [])]
                    out["validated_devices"] = len(r.detail.get("validated_devices") or [])
                return out
            return run

        def allocatable():
            """The next ListAndWatch answers until a GPU turns Healthy (kubelet can allocate)."""
            healthy: List[str] = []
            n = 0
            for resp in state["watch"]:
                n += 1
                healthy = [d.ID for d in resp.devices if d.health == api.HEALTHY]
                if healthy:
                    break
            state["healthy"] = healthy
            return {"_ok": bool(healthy), "healthy": len(healthy), "updates": n}

        def allocate():
            stub = state["stub"]
            pref = stub.GetPreferredAllocation(api.PreferredAllocationRequest(container_requests=[
                api.ContainerPreferredAllocationRequest(available_deviceIDs=state["healthy"],
                                                        allocation_size=1)]), timeout=timeout)
            ids = list(pref.container_responses[0].deviceIDs)
            req = api.AllocateRequest()
            req.container_requests.add(devices_ids=ids)
            (c,) = stub.Allocate(req, timeout=timeout).container_responses
            state.update(ids=ids, alloc=c)
            return {"device_ids": ids, "device_nodes": [d.host_path for d in c.devices],
                    "annotations": dict(c.annotations)}

        def create():
            c = state["alloc"]
            bundle = os.path.join(workdir, "bundle")
            os.makedirs(os.path.join(bundle, "rootfs"), exist_ok=True)
            cmd = list(container_cmd or [os.path.join(bin_dir, "amd-vectoradd")])
            with open(os.path.join(bundle, "config.json"), "w") as f:
                json.dump(_pod_spec(bundle, dict(c.annotations), cmd), f)
            env = dict(os.environ)
            if dev_root:
                env["AMD_CONTAINER_RUNTIME_DEV_ROOT"] = dev_root
            p = subprocess.run([os.path.join(host, "usr/local/bin/amd-container-runtime"),
                                "--amd-edit-bundle", bundle], capture_output=True, text=True,
                               env=env, timeout=timeout)
            if p.returncode != 0:
                raise BringupError(f"runtime shim rejected the spec: {p.stderr.strip()[-300:]}")
            spec = json.loads(p.stdout)
            nodes = sorted(d["path"] for d in spec["linux"]["devices"])
            want = sorted(["/dev/kfd"] + [f"/dev/dri/renderD{m}" for m in
                                          c.annotations["amd.com/gpu.render-minors"].split(",")])
            rules = [r for r in spec["linux"]["resources"]["devices"] if r.get("allow")]
            state["cmd"] = cmd
            return {"_ok": nodes == want and len(rules) >= len(want), "device_nodes": nodes,
                    "cgroup_allow_rules": len(rules)}

        def container():
            # the container sees only its render node; without runc on the box the same view is
            # HIP_VISIBLE_DEVICES = the allocated GPU's HIP index (HIP enumerates in KFD order)
            from ..utils.topology import read_topology

            uid = state["ids"][0]
            gpus = read_topology(root, cfg.min_gfx).gpus
            order = [g.device_uid for g in gpus] + [str(i) for i in range(len(gpus))]
            idx = order.index(uid) % max(1, len(gpus)) if uid in order else 0
            env = dict(os.environ, HIP_VISIBLE_DEVICES=str(idx))
            env.pop("CUDA_VISIBLE_DEVICES", None)
            p = container_runner(state["cmd"], env, timeout)
            out = p.stdout or ""
            return {"_ok": p.returncode == 0 and protocol_passed(out), "hip_index": idx,
                    "rc": p.returncode, "log_tail": out.strip().splitlines()[-2:]}

        stage("driver", driver)
        stage("runtime", runtime)
        stage("plugin", plugin_up)
        gate_steps = ["vectoradd"] + [s for s in v._gating_steps() if s != "driver"]
        if gated:
            for name in gate_steps:
                stage(name, gate_step(name))
            stage("allocatable", allocatable)
        stage("allocate", allocate)
        stage("create", create)
        stage("container", container)
        report["time_to_first_gpu_pod_s"] = stages[-1].end_s
        if validate:
            def validator_chain():
                out = {}
                for s in ("vectoradd", "gemm", "bandwidth", "stress", "rccl", "profile"):
                    if gated and s in gate_steps:
                        continue                 # ran before the pod
                    r = v.run_step(s)
                    out[s] = {"passed": r.passed, "duration_s": r.detail.get("duration_s"),
                              "reason": r.reason}
                    if s == "gemm":
                        out[s]["tflops"] = [d.get("tflops") for d in r.detail.get("devices", [])]
                rep = v.run_step("report")
                out["report"] = {"passed": rep.passed, "chain_seconds": rep.detail.get("chain_seconds"),
                                 "missing": rep.detail.get("missing")}
                out["_ok"] = rep.passed
                return out

            stage("validate", validator_chain)
            report["time_to_validated_s"] = stages[-1].end_s
    except BringupError:
        pass
    finally:
        stop.set()
        if plugin is not None:
            plugin.stop()
        if kubelet is not None:
            kubelet.stop()
        if "channel" in state:
            state["channel"].close()
        if "kdir_tmp" in state:
            shutil.rmtree(state["kdir_tmp"], ignore_errors=True)
        if own_tmp:
            shutil.rmtree(workdir, ignore_errors=True)
    report["stages"] = [asdict(s) for s in stages]
    report["passed"] = bool(stages) and all(s.ok for s in stages)
    report.setdefault("time_to_first_gpu_pod_s", None)
    report.setdefault("time_to_validated_s", None)
    return report


def main(args, cfg: OperatorConfig, bin_dir: str) -> int:
    """The shipped (gated) order with the validator chain, then the ungated order up to the
    first pod; one JSON document with both times to first GPU pod."""
    reps = {}
    for order in ("gated", "ungated"):
        wd = os.path.join(args.workdir, order) if args.workdir else None
        reps[order] = rehearse(cfg, bin_dir, workdir=wd, root=args.root,
                               validate=(order == "gated") and not args.no_validate,
                               gated=(order == "gated"))
        for s in reps[order]["stages"]:
            print(f"{order:8s} {s['name']:11s} {'ok  ' if s['ok'] else 'FAIL'} "
                  f"{s['start_s']:8.3f} -> {s['end_s']:8.3f} s"
                  + ("" if s["ok"] else f"  {s['detail'].get('error') or s['detail']}"))
    doc = {"check": "bringup", "time_to_first_gpu_pod_s": {
        o: r["time_to_first_gpu_pod_s"] for o, r in reps.items()},
        "time_to_validated_s": reps["gated"]["time_to_validated_s"],
        "passed": all(r["passed"] for r in reps.values()), **reps}
    print(json.dumps(doc))
    return 0 if doc["passed"] else 1


__all__ = ["rehearse", "main", "json_lines"]
