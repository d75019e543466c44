"""``python -m k8s_nvidia_gpus_amd.operator <component>`` — one entry point per DaemonSet container.

Components (cluster-config/apps/amd-gpu-operator/*.yaml):
  driver            keep /run/amd/validations/driver-ready in sync with kfd-probe
  runtime-install   install amd-container-runtime + CDI spec on the host, publish runtime-ready
  device-plugin     amd.com/gpu kubelet device plugin
  labeller          node labels from the KFD topology
  exporter          Prometheus metrics on :9400
  partition-manager SPX/DPX/QPX/CPX + NPS1/NPS2 reconciler
  validator         one validation step (--step), or all of them (--step all)
  wait-marker       block until marker file(s) exist (init containers)
  cdi               print the CDI spec for this node
  topology          print the node's GPU topology as JSON
  bringup           node bring-up rehearsal: driver → runtime → plugin → allocate → container →
                    validator on this node, timed (node-local time-to-first-GPU-pod)
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys

from .config import load_config


def _cfg(path):
    return load_config(path) if path and os.path.exists(path) else load_config()


def _kube(optional: bool = True):
    from ..utils.kube import KubeClient, KubeError

    url = os.environ.get("AMDK8S_KUBE_URL")
    try:
        return KubeClient(base_url=url) if url else KubeClient()
    except KubeError:
        if optional:
            return None
        raise


def _bin_dir():
    from .validator import find_bin_dir

    return find_bin_dir()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m k8s_nvidia_gpus_amd.operator")
    ap.add_argument("component")
    ap.add_argument("--config", default="/etc/amd-gpu-operator/operator.yaml")
    ap.add_argument("--root", default=os.environ.get("AMDK8S_ROOT", "/"),
                    help="filesystem prefix for /sys and /dev (tests)")
    ap.add_argument("--marker-dir", default="/run/amd/validations")
    ap.add_argument("--marker", action="append", default=[])
    ap.add_argument("--timeout", type=float, default=0)
    ap.add_argument("--interval", type=float, default=None)
    ap.add_argument("--kubelet-dir", default="/var/lib/kubelet/device-plugins")
    ap.add_argument("--binary-src", default="/opt/amd-gpu-operator/bin/amd-container-runtime")
    ap.add_argument("--binary-dst", default="/host/usr/local/bin/amd-container-runtime")
    ap.add_argument("--cdi-dir", default="/host/etc/cdi")
    ap.add_argument("--step", default="all")
    ap.add_argument("--hold", action="store_true", help="validator: stay running after the step")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--log-level", default=os.environ.get("LOG_LEVEL", "INFO"))
    ap.add_argument("--workdir", default=None, help="bringup: keep markers/bundle here")
    ap.add_argument("--no-validate", action="store_true", help="bringup: stop after the first pod")
    args = ap.parse_args(argv)
    logging.basicConfig(level=args.log_level.upper(),
                        format='{"ts":"%(asctime)s","level":"%(levelname)s","logger":"%(name)s","msg":"%(message)s"}')
    cfg = _cfg(args.config)
    node = os.environ.get("NODE_NAME", "")
    c = args.component

    if c == "wait-marker":
        from .runtime import wait_markers

        return 0 if wait_markers(args.marker, args.timeout) else 1

    if c == "topology":
        from ..utils.topology import read_topology

        t = read_topology(args.root, cfg.min_gfx)
        print(json.dumps({"gpus": [g.to_dict() for g in t.gpus], "cpu_nodes": t.cpu_nodes}, indent=1))
        return 0

    if c == "cdi":
        from ..utils.topology import read_topology
        from .runtime import cdi_spec

        print(json.dumps(cdi_spec(read_topology(args.root, cfg.min_gfx)), indent=1))
        return 0

    if c == "driver":
        from .runtime import driver_ready_loop

        extra = []
        if args.root != "/":
            extra = ["--sysfs-root", os.path.join(args.root, "sys/class/kfd/kfd/topology"),
                     "--dev-root", os.path.join(args.root, "dev"), "--no-open"]
        drv = cfg.section("driver")
        from .pause import PauseGuard

        driver_ready_loop(os.path.join(_bin_dir(), "kfd-probe"), int(cfg["expectedGpusPerNode"]),
                          cfg.min_gfx, args.marker_dir, args.interval or 30.0, extra=extra,
                          load_module=bool(drv["loadModule"]),
                          dev_root=os.path.join(args.root, "dev"), host_root=drv["hostRoot"],
                          guard=PauseGuard("driver"))
        return 0

    if c == "runtime-install":
        import time

        from .runtime import install_runtime

        info = install_runtime(args.binary_src, args.binary_dst, args.cdi_dir, args.marker_dir,
                               args.root, cfg.min_gfx)
        logging.getLogger("amd-gpu-runtime").info("installed: %s", info)
        if not args.hold:
            return 0
        while True:  # DaemonSet container: stay up; re-install if the host copy or topology changes
            time.sleep(args.interval or 300)
            install_runtime(args.binary_src, args.binary_dst, args.cdi_dir, args.marker_dir,
                            args.root, cfg.min_gfx)

    if c == "device-plugin":
        from .device_plugin import AmdGpuDevicePlugin, ValidationGate
        from .validator import DEVICE_ID_MAP

        from .pause import PauseGuard

        gate = ValidationGate(args.marker_dir, root=args.root,
                              gate=bool(cfg.section("validator")["gateOnValidation"]))
        AmdGpuDevicePlugin(cfg, root=args.root, kubelet_dir=args.kubelet_dir,
                           id_map_path=DEVICE_ID_MAP, gate=gate,
                           pause_guard=PauseGuard("device-plugin")).run()
        return 0

    if c == "labeller":
        from .labeller import NodeLabeller

        NodeLabeller(_kube(optional=False), node, args.root, cfg.min_gfx).run(args.interval or 60)
        return 0

    if c == "exporter":
        from .exporter import ExporterServer, GpuCollector, make_backend
        from .pause import PauseGuard

        srv = ExporterServer(GpuCollector(make_backend(args.root), node, args.marker_dir,
                                          guard=PauseGuard("exporter")),
                             port=args.port or int(cfg.section("exporter")["port"]))
        logging.getLogger("amd-gpu-exporter").info("listening on :%d", srv.port)
        srv.serve_background()
        srv.watch_pause()
        return 0

    if c == "partition-manager":
        from .partition import PartitionManager, SysfsPartitionBackend

        try:
            from .partition_amdsmi import AmdSmiPartitionBackend

            backend = AmdSmiPartitionBackend()
        except Exception:  # noqa: BLE001
            backend = SysfsPartitionBackend(args.root)
        p = cfg.section("partition")
        PartitionManager(_kube(optional=False), node, backend, args.root, p["compute"], p["memory"],
                         float(p["drainTimeoutSeconds"]), drain_policy=p["drainPolicy"],
                         pause_ack_timeout=float(p["pauseAckSeconds"]),
                         apply_retries=int(p["applyRetries"]),
                         reservation=os.path.join(args.marker_dir, "in-test.json"),
                         resource=cfg.resource_name).run(args.interval or 30)
        return 0

    if c == "bringup":
        from . import bringup

        return bringup.main(args, cfg, _bin_dir())

    if c == "validator":
        from .validator import STEPS, Validator

        v = Validator(cfg, args.marker_dir, root=args.root, kube=_kube(), node_name=node)
        steps = STEPS if args.step == "all" else [args.step]
        ok = True
        for s in steps:
            r = v.run_step(s)
            print(json.dumps(r.to_json()), flush=True)
            # a deferred step (no free GPU) is not a pass, but the chain goes on: the report
            # labels the node "deferred" and the hold loop below re-runs the chain later
            ok = ok and r.proceed
            if not r.proceed:
                break
        if args.hold:
            from .validator import hold_loop

            return hold_loop(v, args.marker_dir, interval=args.interval or 30)
        return 0 if ok else 1

    ap.error(f"unknown component {c!r}")
    return 2


if __name__ == "__main__":
    sys.exit(main())
