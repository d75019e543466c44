"""KFD / DRM sysfs topology of an AMD GPU node — what every operator component enumerates from.

The amdgpu driver publishes one HSA agent per GPU (or per compute partition) under
``/sys/class/kfd/kfd/topology/nodes/<n>/`` (``properties`` = "key value" lines, ``gpu_id``,
``name``, ``mem_banks/*/properties``, ``io_links/*/properties``).  This is the AMD counterpart of the
NVML enumeration NVIDIA's device plugin / GFD do inside the reference's operator (SURVEY.md §2.2
X3/X4).  The same reader exists in C++ for the native tools (native/src/kfd_topology.cpp).

Facts this code relies on were captured from a live 8× MI355X node (tests/fixtures/):

* gfx950 agents report ``gfx_target_version 90500``, ``simd_count 1024`` (256 CUs × 4 SIMDs),
  ``num_xcc 8`` in SPX mode, one 288 GiB (309 220 868 096 B) ``heap_type 1`` memory bank;
* xGMI is a full mesh: 7 ``io_links`` of ``type 11`` per GPU, ``max_bandwidth 76000`` (MB/s);
* every MI355X owns 8 DRM card/render minors (``card8k`` + ``renderD(128+8k)`` for the PCI device,
  the next 7 for its ``amdgpu_xcp_*`` partition nodes), so in CPX mode each partition agent has its
  own render node while sharing the ASIC's ``unique_id`` / ``location_id``;
* inside a container, agents whose device nodes are not allocated may show no ``properties`` —
  readers must skip such nodes, not fail.

``root`` is a filesystem prefix (default ``/``) so tests run every component against a fabricated
tree (tests/fakes/sysfs.py).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

KFD_TOPOLOGY = "sys/class/kfd/kfd/topology"
DRM_CLASS = "sys/class/drm"
IOLINK_TYPE_XGMI = 11
IOLINK_TYPE_PCIE = 2
HEAP_TYPE_FB_PUBLIC = 1
HEAP_TYPE_FB_PRIVATE = 2
GFX950 = 90500
AMD_VENDOR_ID = 0x1002

# PCI device ids → marketing names for the products this stack targets.
PRODUCT_NAMES = {
    0x75A3: "MI355X",
    0x75A0: "MI350X",
}
PARTITION_SPLIT = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}


def _read(path: str) -> Optional[str]:
    try:
        with open(path, "r", errors="replace") as f:
            return f.read()
    except OSError:
        return None


def parse_properties(text: str) -> Dict[str, int]:
    """Parse a KFD ``properties`` file ("key value" per line, integer values)."""
    out: Dict[str, int] = {}
    for line in text.splitlines():
        parts = line.split()
        if len(parts) != 2:
            continue
        try:
            out[parts[0]] = int(parts[1])
        except ValueError:
            continue
    return out


def _numeric_dirs(path: str) -> List[str]:
    try:
        names = os.listdir(path)
    except OSError:
        return []
    return sorted((n for n in names if n.isdigit()), key=int)


@dataclass
class GpuDevice:
    """One schedulable GPU: a whole MI355X (SPX) or one compute partition of it."""

    node_id: int
    gpu_id: int
    render_minor: int
    gfx_target_version: int
    simd_count: int
    num_xcc: int
    unique_id: int
    location_id: int
    domain: int
    vendor_id: int
    device_id: int
    vram_bytes: int
    hive_id: int = 0
    xgmi_peers: List[int] = field(default_factory=list)   # KFD node ids reachable over xGMI
    xgmi_link_mbps: int = 0                                # per-link max bandwidth (MB/s)
    card_minor: Optional[int] = None
    numa_node: int = -1
    max_engine_clk_mhz: int = 0
    lds_kb: int = 0
    wave_size: int = 64
    partition_index: int = 0        # index of this agent among the ASIC's partitions
    partitions_on_asic: int = 1
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"

    @property
    def cu_count(self) -> int:
        return self.simd_count // 4  # CDNA: 4 SIMDs per CU

    @property
    def pci_bdf(self) -> str:
        loc = self.location_id
        return "%04x:%02x:%02x.%x" % (self.domain, (loc >> 8) & 0xFF, (loc >> 3) & 0x1F, loc & 0x7)

    @property
    def gfx_name(self) -> str:
        v = self.gfx_target_version
        major, minor, step = v // 10000, (v // 100) % 100, v % 100
        return "gfx%d%d%x" % (major, minor, step)

    @property
    def product(self) -> str:
        return PRODUCT_NAMES.get(self.device_id, "0x%04x" % self.device_id)

    @property
    def uuid(self) -> str:
        """Stable per-ASIC identifier (partitions of one ASIC share it)."""
        return "GPU-%016x" % self.unique_id

    @property
    def device_uid(self) -> str:
        """Stable per-schedulable-device identifier (kubelet device ID)."""
        if self.partitions_on_asic > 1:
            return "%s-p%d" % (self.uuid, self.partition_index)
        return self.uuid

    @property
    def render_path(self) -> str:
        return "/dev/dri/renderD%d" % self.render_minor

    @property
    def card_path(self) -> Optional[str]:
        return None if self.card_minor is None else "/dev/dri/card%d" % self.card_minor

    def to_dict(self) -> dict:
        return {
            "node_id": self.node_id, "gpu_id": self.gpu_id, "render_minor": self.render_minor,
            "card_minor": self.card_minor, "gfx": self.gfx_name, "product": self.product,
            "cu": self.cu_count, "num_xcc": self.num_xcc, "vram_bytes": self.vram_bytes,
            "pci": self.pci_bdf, "numa_node": self.numa_node, "uuid": self.uuid,
            "device_uid": self.device_uid, "xgmi_peers": list(self.xgmi_peers),
            "compute_partition": self.compute_partition, "memory_partition": self.memory_partition,
            "partition_index": self.partition_index,
        }


@dataclass
class NodeTopology:
    gpus: List[GpuDevice]
    cpu_nodes: int = 0
    generation_id: int = 0

    def by_uid(self) -> Dict[str, GpuDevice]:
        return {g.device_uid: g for g in self.gpus}

    def asics(self) -> Dict[int, List[GpuDevice]]:
        out: Dict[int, List[GpuDevice]] = {}
        for g in self.gpus:
            out.setdefault(g.unique_id, []).append(g)
        return out


def _drm_attr(root: str, card: Optional[int], render: int, name: str) -> Optional[str]:
    for node in ([f"card{card}"] if card is not None else []) + [f"renderD{render}"]:
        v = _read(os.path.join(root, DRM_CLASS, node, "device", name))
        if v is not None:
            return v.strip()
    return None


def _card_for_render(root: str, render_minor: int) -> Optional[int]:
    """DRM pairs card<N> with renderD<128+N> for the same device; verify via the device link."""
    drm = os.path.join(root, DRM_CLASS)
    guess = render_minor - 128
    rlink = os.path.join(drm, f"renderD{render_minor}", "device")
    clink = os.path.join(drm, f"card{guess}", "device")
    if os.path.lexists(rlink) and os.path.lexists(clink):
        try:
            if os.path.realpath(rlink) == os.path.realpath(clink):
                return guess
        except OSError:
            pass
        # links differ: search every card for the render node's device
        target = os.path.realpath(rlink)
        try:
            for name in os.listdir(drm):
                if name.startswith("card") and name[4:].isdigit():
                    if os.path.realpath(os.path.join(drm, name, "device")) == target:
                        return int(name[4:])
        except OSError:
            return None
        return None
    return guess if guess >= 0 else None


def read_topology(root: str = "/", min_gfx: int = 0) -> NodeTopology:
    """Enumerate GPU agents; agents below ``min_gfx`` (gfx_target_version) are ignored."""
    base = os.path.join(root, KFD_TOPOLOGY)
    nodes_dir = os.path.join(base, "nodes")
    if not os.path.isdir(nodes_dir):
        raise FileNotFoundError(f"no KFD topology at {nodes_dir} (amdgpu driver not loaded?)")
    gen = _read(os.path.join(base, "generation_id"))
    raw: List[GpuDevice] = []
    cpu_nodes = 0
    for nid in _numeric_dirs(nodes_dir):
        nd = os.path.join(nodes_dir, nid)
        text = _read(os.path.join(nd, "properties"))
        if not text or not text.strip():
            continue  # hidden agent (e.g. not allocated to this container)
        p = parse_properties(text)
        gpu_id_txt = (_read(os.path.join(nd, "gpu_id")) or "0").strip() or "0"
        gpu_id = int(gpu_id_txt) if gpu_id_txt.isdigit() else 0
        if p.get("simd_count", 0) == 0 or gpu_id == 0:
            if p.get("cpu_cores_count", 0) > 0:
                cpu_nodes += 1
            continue
        if p.get("gfx_target_version", 0) < min_gfx:
            continue
        vram = 0
        for b in _numeric_dirs(os.path.join(nd, "mem_banks")):
            bp = parse_properties(_read(os.path.join(nd, "mem_banks", b, "properties")) or "")
            if bp.get("heap_type") in (HEAP_TYPE_FB_PUBLIC, HEAP_TYPE_FB_PRIVATE):
                vram += bp.get("size_in_bytes", 0)
        peers: List[int] = []
        link_bw = 0
        for l in _numeric_dirs(os.path.join(nd, "io_links")):
            lp = parse_properties(_read(os.path.join(nd, "io_links", l, "properties")) or "")
            if lp.get("type") == IOLINK_TYPE_XGMI:
                peers.append(lp.get("node_to", -1))
                link_bw = max(link_bw, lp.get("max_bandwidth", 0))
        render = p.get("drm_render_minor", -1)
        card = _card_for_render(root, render) if render >= 0 else None
        numa_txt = _drm_attr(root, card, render, "numa_node")
        try:
            numa = int(numa_txt) if numa_txt is not None else -1
        except ValueError:
            numa = -1
        raw.append(GpuDevice(
            node_id=int(nid), gpu_id=gpu_id, render_minor=render,
            gfx_target_version=p.get("gfx_target_version", 0), simd_count=p.get("simd_count", 0),
            num_xcc=p.get("num_xcc", 1), unique_id=p.get("unique_id", 0),
            location_id=p.get("location_id", 0), domain=p.get("domain", 0),
            vendor_id=p.get("vendor_id", 0), device_id=p.get("device_id", 0), vram_bytes=vram,
            hive_id=p.get("hive_id", 0), xgmi_peers=sorted(peers), xgmi_link_mbps=link_bw,
            card_minor=card, numa_node=numa,
            max_engine_clk_mhz=p.get("max_engine_clk_fcompute", 0),
            lds_kb=p.get("lds_size_in_kb", 0), wave_size=p.get("wave_front_size", 64) or 64,
        ))
    # partitions: agents sharing one ASIC (unique_id, else PCI location) are numbered in node order
    groups: Dict[tuple, List[GpuDevice]] = {}
    for g in raw:
        key = (g.unique_id,) if g.unique_id else (g.domain, g.location_id)
        groups.setdefault(key, []).append(g)
    for members in groups.values():
        members.sort(key=lambda d: d.node_id)
        n = len(members)
        for i, g in enumerate(members):
            g.partition_index = i
            g.partitions_on_asic = n
            head = members[0]
            cp = _drm_attr(root, head.card_minor, head.render_minor, "current_compute_partition")
            mp = _drm_attr(root, head.card_minor, head.render_minor, "current_memory_partition")
            g.compute_partition = (cp or _infer_partition(g.num_xcc, n)).upper()
            g.memory_partition = (mp or "NPS1").upper()
            if head.numa_node >= 0 and g.numa_node < 0:
                g.numa_node = head.numa_node
    raw.sort(key=lambda d: (d.numa_node if d.numa_node >= 0 else 99, d.domain, d.location_id,
                            d.partition_index))
    gen_id = int(gen.strip()) if gen and gen.strip().isdigit() else 0
    return NodeTopology(gpus=raw, cpu_nodes=cpu_nodes, generation_id=gen_id)


def _infer_partition(num_xcc: int, partitions: int) -> str:
    for name, split in PARTITION_SPLIT.items():
        if split == partitions:
            return name
    return {8: "SPX", 4: "DPX", 2: "QPX", 1: "CPX"}.get(num_xcc, "SPX")


def available_partitions(root: str, dev: GpuDevice) -> List[str]:
    txt = _drm_attr(root, dev.card_minor, dev.render_minor, "available_compute_partition")
    if not txt:
        return ["SPX"]
    return [t.strip().upper() for t in txt.split(",") if t.strip()]
