"""Container-runtime integration, driver readiness and marker helpers.

* :func:`cdi_spec` — the Container Device Interface spec for ``amd.com/gpu`` (containerd 2.x reads
  /etc/cdi): one CDI device per schedulable GPU/partition (its render node) plus ``all``; /dev/kfd
  is a spec-level edit shared by every device.  Used when the device plugin runs in ``cdi`` mode.
* :func:`install_runtime` — what the runtime-installer DaemonSet does: atomically install the native
  ``amd-container-runtime`` on the host, write the CDI spec, publish ``runtime-ready``.  (The
  reference configures NVIDIA's toolkit to rewrite containerd's config.toml directly —
  reference gpu-operator/helmrelease.yaml:22-29 — which RKE2 regenerates on restart; the
  containerd handler is registered via RKE2's config template by amd-host-prep instead.)
* :func:`driver_ready_loop` — the driver DaemonSet: run the native kfd-probe periodically and keep
  ``driver-ready`` in sync with reality (withdrawn when the driver disappears).
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import subprocess
import time
from typing import Dict, List, Optional

from ..utils import topology as topo_mod

log = logging.getLogger("amd-gpu-runtime")

CDI_VERSION = "0.6.0"
CDI_KIND = "amd.com/gpu"
CDI_FILE = "amd.com-gpu.json"


def cdi_spec(topo: topo_mod.NodeTopology) -> Dict:
    devices: List[Dict] = []
    for g in topo.gpus:
        devices.append({
            "name": g.device_uid,
            "annotations": {"amd.com/gpu.pci": g.pci_bdf,
                            "amd.com/gpu.partition": f"{g.compute_partition}:{g.partition_index}"},
            "containerEdits": {"deviceNodes": [{"path": g.render_path, "permissions": "rw"}]},
        })
    if topo.gpus:
        devices.append({"name": "all", "containerEdits": {"deviceNodes": [
            {"path": g.render_path, "permissions": "rw"} for g in topo.gpus]}})
    return {
        "cdiVersion": CDI_VERSION,
        "kind": CDI_KIND,
        "devices": devices,
        "containerEdits": {"deviceNodes": [{"path": "/dev/kfd", "permissions": "rw"}]},
    }


def atomic_write(path: str, data: bytes, mode: int = 0o644) -> None:
    d = os.path.dirname(path) or "."
    os.makedirs(d, exist_ok=True)
    tmp = os.path.join(d, f".{os.path.basename(path)}.tmp.{os.getpid()}")
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.chmod(tmp, mode)
    os.replace(tmp, path)


def write_marker(marker_dir: str, name: str, payload: Optional[dict] = None) -> str:
    path = os.path.join(marker_dir, name)
    atomic_write(path, (json.dumps(payload or {"time": time.time()}) + "\n").encode())
    return path


def clear_marker(marker_dir: str, name: str) -> None:
    try:
        os.unlink(os.path.join(marker_dir, name))
    except FileNotFoundError:
        pass


def wait_markers(paths: List[str], timeout: float = 0, poll: float = 2.0) -> bool:
    """Block until every marker exists; timeout 0 = forever."""
    deadline = time.monotonic() + timeout if timeout > 0 else None
    while True:
        missing = [p for p in paths if not os.path.exists(p)]
        if not missing:
            return True
        if deadline is not None and time.monotonic() >= deadline:
            log.error("markers still missing after %ss: %s", timeout, missing)
            return False
        time.sleep(poll)


def install_runtime(binary_src: str, binary_dst: str, cdi_dir: str, marker_dir: str,
                    root: str = "/", min_gfx: int = topo_mod.GFX950) -> Dict:
    """Install amd-container-runtime + CDI spec; publish runtime-ready. Idempotent."""
    if not os.path.isfile(binary_src):
        raise FileNotFoundError(f"runtime binary {binary_src} missing from the operator image")
    with open(binary_src, "rb") as f:
        blob = f.read()
    changed = True
    if os.path.exists(binary_dst):
        with open(binary_dst, "rb") as f:
            changed = f.read() != blob
    if changed:
        atomic_write(binary_dst, blob, 0o755)  # never a half-written binary on the host
    topo = topo_mod.read_topology(root, min_gfx)
    spec = cdi_spec(topo)
    atomic_write(os.path.join(cdi_dir, CDI_FILE), (json.dumps(spec, indent=1) + "\n").encode())
    info = {"binary": binary_dst, "updated": changed, "cdi_devices": len(spec["devices"]),
            "time": time.time()}
    write_marker(marker_dir, "runtime-ready", info)
    return info


def run_kfd_probe(bin_path: str, expect: int, min_gfx: int, marker: str,
                  extra: Optional[List[str]] = None) -> subprocess.CompletedProcess:
    argv = [bin_path, "--expect-gpus", str(expect), "--min-gfx", str(min_gfx), "--marker", marker,
            "-q"] + (extra or [])
    return subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def ensure_module(dev_root: str = "/dev", host_root: str = "/host", runner=None) -> Optional[bool]:
    """If /dev/kfd is missing, try ``chroot <host_root> modprobe amdgpu`` once.

    The reference's driver container compiles and loads the NVIDIA module inside the cluster
    (README.md:514-517); amdgpu ships inbox / as DKMS on the host (amd-host-prep), so loading the
    host's own module is all that can be needed here.  Returns None when nothing was attempted,
    else whether modprobe succeeded."""
    if os.path.exists(os.path.join(dev_root, "kfd")):
        return None
    if not os.path.isdir(host_root):
        log.warning("/dev/kfd missing and no host root at %s to modprobe from", host_root)
        return False
    argv = ["chroot", host_root, "modprobe", "amdgpu"]
    if runner is None:
        p = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        rc, out = p.returncode, p.stdout
    else:
        rc, out = runner(argv)
    if rc != 0:
        log.error("modprobe amdgpu failed (%d): %s", rc, out.strip())
    else:
        log.info("loaded amdgpu from the host's module tree")
    return rc == 0


def driver_ready_loop(bin_path: str, expect: int, min_gfx: int, marker_dir: str,
                      interval: float = 30.0, stop_event=None, extra: Optional[List[str]] = None,
                      load_module: bool = False, dev_root: str = "/dev",
                      host_root: str = "/host", guard=None, pause_poll: float = 1.0) -> None:
    """Re-probe every ``interval``.  While a partition change is in progress (``guard``, see
    pause.py) the probe — which opens /dev/kfd and every render node — is not run, the marker is
    left as it is, and the pause is acked; probing resumes when the pause ends."""
    import threading

    stop_event = stop_event or threading.Event()
    marker = os.path.join(marker_dir, "driver-ready")
    os.makedirs(marker_dir, exist_ok=True)
    was_ready = None
    tried_modprobe = False
    while not stop_event.is_set():
        if guard is not None and guard.paused():
            guard.ack()
            stop_event.wait(pause_poll)
            continue
        if guard is not None:
            guard.clear()
        if load_module and not tried_modprobe:
            tried_modprobe = ensure_module(dev_root, host_root) is not None
        p = run_kfd_probe(bin_path, expect, min_gfx, marker, extra)
        ready = p.returncode == 0
        if ready != was_ready:
            log.info("driver %s%s", "READY" if ready else "NOT READY",
                     "" if ready else f": {p.stderr.strip()}")
            was_ready = ready
        # wake early for a pause: sleep in short slices while no pause is pending
        waited = 0.0
        while waited < interval and not stop_event.is_set():
            if guard is not None and guard.paused():
                break
            step = min(pause_poll, interval - waited)
            stop_event.wait(step)
            waited += step


def host_binary_present(path: str) -> bool:
    return os.path.isfile(path) and os.access(path, os.X_OK)


def copy_tree_binaries(src_dir: str, dst_dir: str, names: List[str]) -> None:
    os.makedirs(dst_dir, exist_ok=True)
    for n in names:
        shutil.copy2(os.path.join(src_dir, n), os.path.join(dst_dir, n))
