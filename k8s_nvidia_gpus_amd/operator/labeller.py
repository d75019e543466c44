"""Node labeller (SURVEY.md §2.2 X4 — the GPU-Feature-Discovery / NFD role).

The reference relies on the GPU operator's implicit GFD/NFD labels; its heterogeneous GTX 1060 +
1070 node is why its SD15 Deployment carries an (optional) GPU-model nodeSelector (reference
sd15-api/deployment.yaml:17-18).  Here every MI355X node gets labels derived from the KFD / DRM
sysfs topology, so workloads select on product, architecture, partition mode or memory:

    amd.com/gpu.present=true           amd.com/gpu.product=MI355X       amd.com/gpu.family=gfx950
    amd.com/gpu.count=8                amd.com/gpu.asic-count=8         amd.com/gpu.cu-count=256
    amd.com/gpu.vram=288G              amd.com/gpu.compute-partition=SPX
    amd.com/gpu.memory-partition=NPS1  amd.com/gpu.xgmi-links=7         amd.com/gpu.device-id=75a3
    amd.com/gpu.driver-version=...     amd.com/gpu.numa-nodes=2

``amd.com/gpu.present`` is what schedules the rest of the operator's DaemonSets onto the node.
``amd.com/gpu.pci-present=true`` comes from the PCI bus alone, so it is set before amdgpu is
loaded: vendor 0x1002, class 0x12 (processing accelerator) and a device ID of an Instinct part the
operator's ``minGfxTargetVersion`` accepts (:data:`INSTINCT_PCI_IDS`).  It schedules the driver
DaemonSet, whose ``kfd-probe --min-gfx`` can only turn ready on such a part; a CPU worker with an
AMD Radeon (display class 0x03) or an older Instinct never gets it, so no never-ready driver pod
blocks the operator Kustomization's ``wait: true``.  The partition labels read every ASIC and
say ``mixed`` when they disagree (a partition change that stopped half-way), never the head GPU's.
Labels this component owns are removed again when the GPUs go away; labels owned by other
components (``amd.com/gpu.validated``, ``amd.com/gpu.compute-partition.desired``) are left alone.
"""
from __future__ import annotations

import logging
import os
import re
from typing import Dict, Optional

from ..utils import topology as topo_mod

log = logging.getLogger("amd-node-labeller")

PREFIX = "amd.com/gpu"
OWNED = ("present", "pci-present", "count", "asic-count", "product", "family", "device-id", "cu-count", "vram",
         "compute-partition", "memory-partition", "xgmi-links", "driver-version", "numa-nodes")
_LABEL_VALUE = re.compile(r"^(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?$")


def sanitize(value: str) -> str:
    v = re.sub(r"[^A-Za-z0-9_.-]+", "_", value.strip())[:63]
    v = v.strip("-_.")
    return v if _LABEL_VALUE.match(v) else ""


def driver_version(root: str = "/") -> Optional[str]:
    for p in ("sys/module/amdgpu/version", "sys/module/amdgpu/srcversion"):
        try:
            with open(os.path.join(root, p)) as f:
                v = f.read().strip()
                if v:
                    return v
        except OSError:
            continue
    return None


AMD_VENDOR = "0x1002"
PCI_CLASS_ACCELERATOR = 0x12
# Instinct PCI device IDs (PF and SR-IOV VF) → gfx target version; only parts >= minGfxTargetVersion
# count.  MI300A/X/MI308X/MI325X are gfx942; MI350X/MI355X are gfx950 (the target of this operator).
INSTINCT_PCI_IDS = {
    0x74a0: 90402, 0x74a1: 90402, 0x74a2: 90402, 0x74a5: 90402, 0x74a9: 90402,   # MI300 series
    0x74b5: 90402, 0x74b9: 90402, 0x74bd: 90402,                                 # MI300 VFs
    0x75a0: 90500, 0x75a3: 90500,                                                # MI350X, MI355X
    0x75b0: 90500, 0x75b3: 90500,                                                # MI350X/MI355X VFs
}


def amd_accelerators_on_pci(root: str = "/", min_gfx: int = topo_mod.GFX950) -> int:
    """Instinct accelerators on the PCI bus that this operator can drive (needs no driver)."""
    base = os.path.join(root, "sys/bus/pci/devices")
    try:
        names = os.listdir(base)
    except OSError:
        return 0
    n = 0
    for name in names:
        try:
            with open(os.path.join(base, name, "vendor")) as f:
                vendor = f.read().strip().lower()
            with open(os.path.join(base, name, "class")) as f:
                cls = int(f.read().strip(), 16)
            with open(os.path.join(base, name, "device")) as f:
                device = int(f.read().strip(), 16)
        except (OSError, ValueError):
            continue
        if (vendor == AMD_VENDOR and (cls >> 16) == PCI_CLASS_ACCELERATOR
                and INSTINCT_PCI_IDS.get(device, 0) >= min_gfx):
            n += 1
    return n


def compute_labels(root: str = "/", min_gfx: int = topo_mod.GFX950) -> Dict[str, Optional[str]]:
    """Desired values for every owned label (None = remove)."""
    labels: Dict[str, Optional[str]] = {f"{PREFIX}.{k}": None for k in OWNED}
    if amd_accelerators_on_pci(root, min_gfx):
        labels[f"{PREFIX}.pci-present"] = "true"
    try:
        topo = topo_mod.read_topology(root, min_gfx)
    except FileNotFoundError:
        return labels
    gpus = topo.gpus
    if not gpus:
        return labels
    asics = topo.asics()
    head = gpus[0]
    from .partition import asic_modes, node_mode

    compute_mode, memory_mode = node_mode(asic_modes(topo))
    vram_gib = round(sum(g.vram_bytes for g in asics[head.unique_id]) / (1 << 30))
    labels.update({
        f"{PREFIX}.present": "true",
        f"{PREFIX}.count": str(len(gpus)),
        f"{PREFIX}.asic-count": str(len(asics)),
        f"{PREFIX}.product": sanitize(head.product),
        f"{PREFIX}.family": head.gfx_name,
        f"{PREFIX}.device-id": "%04x" % head.device_id,
        f"{PREFIX}.cu-count": str(head.cu_count),
        f"{PREFIX}.vram": f"{vram_gib}G",
        f"{PREFIX}.compute-partition": compute_mode,
        f"{PREFIX}.memory-partition": memory_mode,
        f"{PREFIX}.xgmi-links": str(len({p for p in head.xgmi_peers
                                         if p not in {g.node_id for g in asics[head.unique_id]}})
                                    if head.partitions_on_asic == 1 else
                                    len(asics) - 1),
        f"{PREFIX}.numa-nodes": str(len({g.numa_node for g in gpus if g.numa_node >= 0}) or 1),
    })
    dv = driver_version(root)
    if dv:
        labels[f"{PREFIX}.driver-version"] = sanitize(dv) or None
    return labels


def diff_labels(current: Dict[str, str], desired: Dict[str, Optional[str]]) -> Dict[str, Optional[str]]:
    patch = {}
    for k, v in desired.items():
        if v is None:
            if k in current:
                patch[k] = None
        elif current.get(k) != v:
            patch[k] = v
    return patch


class NodeLabeller:
    def __init__(self, client, node_name: str, root: str = "/", min_gfx: int = topo_mod.GFX950):
        self.client = client
        self.node = node_name
        self.root = root
        self.min_gfx = min_gfx

    def reconcile(self) -> Dict[str, Optional[str]]:
        desired = compute_labels(self.root, self.min_gfx)
        node = self.client.get_node(self.node)
        current = node.get("metadata", {}).get("labels", {}) or {}
        patch = diff_labels(current, desired)
        if patch:
            self.client.set_node_labels(self.node, patch)
            log.info("node %s: %s", self.node, patch)
        return patch

    def run(self, interval: float = 60.0, stop_event=None) -> None:
        import threading

        stop_event = stop_event or threading.Event()
        while not stop_event.is_set():
            try:
                self.reconcile()
            except Exception as e:  # noqa: BLE001 - API server hiccups must not kill the agent
                log.warning("reconcile failed: %s", e)
            stop_event.wait(interval)
