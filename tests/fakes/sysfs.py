"""Build a fake MI355X node (KFD topology + DRM class + /dev) under a temp directory.

The per-GPU ``properties`` template and the io_link / mem_bank shapes are the ones captured from
a live 8× MI355X node (tests/fixtures/mi355x_node7, tests/fixtures/mi355x_node_layout.json); only
the per-GPU identity fields (node id, render minor, PCI location, unique id, NUMA node) vary.
CPX mode splits every ASIC into 8 agents with ``num_xcc 1`` and 1/8 of the CUs and memory, each on
one of the ASIC's ``amdgpu_xcp_*`` render nodes — the layout the real driver uses.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Iterable, Optional, Sequence, Union

FIX = Path(__file__).resolve().parent.parent / "fixtures"
LAYOUT = json.loads((FIX / "mi355x_node_layout.json").read_text())
GPU_TEMPLATE = (FIX / "mi355x_node7" / "properties").read_text()
CPU_TEMPLATE = (FIX / "mi355x_node7" / "cpu_node_properties").read_text()
VRAM_BYTES = 309220868096
SPLIT = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}


def _props(template: str, **overrides) -> str:
    lines = []
    seen = set()
    for line in template.splitlines():
        parts = line.split()
        if len(parts) != 2:
            continue
        k = parts[0]
        if k in overrides:
            lines.append(f"{k} {overrides[k]}")
            seen.add(k)
        else:
            lines.append(line)
    for k, v in overrides.items():
        if k not in seen:
            lines.append(f"{k} {v}")
    return "\n".join(lines) + "\n"


def _w(path: Path, text: str) -> None:
    path.parent.mkdir(parents=True, exist_ok=True)
    path.write_text(text)


def bdf_to_location(bdf: str) -> int:
    _dom, bus, devfn = bdf.split(":")
    dev, fn = devfn.split(".")
    return (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn)


def build_node(root, n_gpus: int = 8, compute_partition: Union[str, Sequence[str]] = "SPX",
               memory_partition: Union[str, Sequence[str]] = "NPS1", hidden: Iterable[int] = (),
               gfx_target_version: int = 90500, with_dev: bool = True) -> Path:
    """Create ``root``/sys/... and ``root``/dev/...; returns ``root`` as a Path.

    ``compute_partition`` / ``memory_partition``: one mode for every ASIC, or one per ASIC (a node
    whose partition change stopped half-way).  ``hidden``: ASIC indices whose agents have an empty
    ``properties`` (what a container that was not allocated those GPUs sees).
    """
    root = Path(root)
    modes = ([compute_partition] * n_gpus if isinstance(compute_partition, str)
             else list(compute_partition))
    mems = [memory_partition] * n_gpus if isinstance(memory_partition, str) else list(memory_partition)
    topo = root / "sys/class/kfd/kfd/topology"
    drm = root / "sys/class/drm"
    devices = root / "sys/devices"
    _w(topo / "generation_id", "1\n")
    _w(topo / "system_properties", "platform_oem 0\nplatform_id 0\nplatform_rev 2\n")
    # two CPU sockets
    for cpu in range(2):
        nd = topo / "nodes" / str(cpu)
        _w(nd / "properties", _props(CPU_TEMPLATE, cpu_core_id_base=cpu * 128))
        _w(nd / "gpu_id", "0\n")
        _w(nd / "name", "\n")
    hidden = set(hidden)
    gpus = LAYOUT["gpus"][:n_gpus]
    agent_ids = []
    node_id = 2
    for a, _g in enumerate(gpus):
        ids = []
        for _p in range(SPLIT[modes[a]]):
            ids.append(node_id)
            node_id += 1
        agent_ids.append(ids)
    all_agents = [i for ids in agent_ids for i in ids]
    for a, g in enumerate(gpus):
        split = SPLIT[modes[a]]
        loc = bdf_to_location(g["bdf"])
        uid = int(g["unique_id_hex"], 16)
        pci_dir = devices / "pci0000:00" / g["bdf"]
        # PCI device attributes (shared by the card/render node of the ASIC)
        _w(pci_dir / "numa_node", f"{g['numa_node']}\n")
        _w(pci_dir / "unique_id", g["unique_id_hex"] + "\n")
        _w(pci_dir / "current_compute_partition", modes[a] + "\n")
        _w(pci_dir / "available_compute_partition", "SPX, DPX, QPX, CPX\n")
        _w(pci_dir / "current_memory_partition", mems[a] + "\n")
        _w(pci_dir / "available_memory_partition", "NPS1, NPS2\n")
        _w(pci_dir / "vendor", "0x1002\n")
        _w(pci_dir / "device", "0x75a3\n")
        _w(pci_dir / "class", "0x120000\n")          # processing accelerator
        bus = root / "sys/bus/pci/devices"
        bus.mkdir(parents=True, exist_ok=True)
        if not (bus / g["bdf"]).exists():
            os.symlink(os.path.relpath(pci_dir, bus), bus / g["bdf"])
        _w(pci_dir / "mem_info_vram_total", f"{VRAM_BYTES}\n")
        _w(pci_dir / "mem_info_vram_used", f"{(a + 1) * 1024 ** 3}\n")
        _w(pci_dir / "gpu_busy_percent", f"{10 * a}\n")
        for j in range(8):  # card/render minors: 8 per ASIC (PCI device + 7 xcp nodes)
            card = g["card"] + j
            render = g["render"] + j
            target = pci_dir if j == 0 else devices / "platform" / f"amdgpu_xcp_{a * 7 + j - 1}"
            target.mkdir(parents=True, exist_ok=True)
            for node in (f"card{card}", f"renderD{render}"):
                d = drm / node
                d.mkdir(parents=True, exist_ok=True)
                link = d / "device"
                if not link.exists():
                    os.symlink(os.path.relpath(target, d), link)
            if with_dev:
                _w(root / "dev/dri" / f"card{card}", "")
                _w(root / "dev/dri" / f"renderD{render}", "")
        for p, nid in enumerate(agent_ids[a]):
            nd = topo / "nodes" / str(nid)
            render_minor = g["render"] + (0 if split == 1 else p)
            if a in hidden:
                _w(nd / "io_links" / "0" / "properties", "type 11\n")
                continue
            _w(nd / "properties", _props(
                GPU_TEMPLATE, simd_count=1024 // split, array_count=32 // split,
                num_xcc=8 // split, gfx_target_version=gfx_target_version,
                drm_render_minor=render_minor, location_id=loc, domain=0, unique_id=uid,
                device_id=30115, vendor_id=4098))
            _w(nd / "gpu_id", f"{40000 + nid}\n")
            _w(nd / "name", "ip discovery\n")
            _w(nd / "mem_banks" / "0" / "properties",
               f"heap_type 1\nsize_in_bytes {VRAM_BYTES // split}\nflags 0\nwidth 8192\nmem_clk_max 2000\n")
            li = 0
            for peer in all_agents:
                if peer == nid:
                    continue
                _w(nd / "io_links" / str(li) / "properties",
                   f"type 11\nversion_major 0\nversion_minor 0\nnode_from {nid}\nnode_to {peer}\n"
                   f"weight 15\nmin_latency 0\nmax_latency 0\nmin_bandwidth 76000\n"
                   f"max_bandwidth 76000\nrecommended_transfer_size 0\nflags 1\n")
                li += 1
    if with_dev:
        _w(root / "dev" / "kfd", "")
    return root


def add_cpu_only_pci(root, bdf: str = "0000:c1:00.0", vendor: str = "0x1a03",
                     cls: str = "0x030000", device: str = "0x2000") -> None:
    """A PCI device that is not an MI355X (default: the BMC's ASPEED VGA) on the node."""
    root = Path(root)
    d = root / "sys/devices/pci0000:c0" / bdf
    _w(d / "vendor", vendor + "\n")
    _w(d / "class", cls + "\n")
    _w(d / "device", device + "\n")
    bus = root / "sys/bus/pci/devices"
    bus.mkdir(parents=True, exist_ok=True)
    os.symlink(os.path.relpath(d, bus), bus / bdf)


def remove_gpu(root, asic_index: int, compute_partition: str = "SPX") -> None:
    """Fault injection: make one ASIC's agents disappear (driver reset / fell off the bus)."""
    root = Path(root)
    split = SPLIT[compute_partition]
    topo = root / "sys/class/kfd/kfd/topology/nodes"
    first = 2 + asic_index * split
    for nid in range(first, first + split):
        p = topo / str(nid) / "properties"
        if p.exists():
            p.write_text("")


def set_partition(root, n_gpus: int, compute_partition: Union[str, Sequence[str]],
                  memory_partition: Union[str, Sequence[str]] = "NPS1",
                  tmp_parent: Optional[Path] = None) -> Path:
    """Re-enumerate the node in another compute partition mode (what a mode switch does)."""
    import shutil

    root = Path(root)
    shutil.rmtree(root / "sys", ignore_errors=True)
    shutil.rmtree(root / "dev", ignore_errors=True)
    return build_node(root, n_gpus=n_gpus, compute_partition=compute_partition,
                      memory_partition=memory_partition)
