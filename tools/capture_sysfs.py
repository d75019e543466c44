#!/usr/bin/env python3
"""Copy the KFD topology + DRM partition sysfs files of a real node into a plain directory tree.

sysfs attributes report a 4096-byte size whatever they hold, so archivers copy padding; read each
attribute with open().read() instead.  The output tree is what tests/fixtures/ ships as the fake
node the device plugin, labeller and kfd-probe are tested against.
"""
import os
import sys

KFD = "/sys/class/kfd/kfd/topology"


def copy_attr(src: str, dst: str) -> None:
    try:
        with open(src, "rb") as f:
            data = f.read()
    except OSError:
        return
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "wb") as f:
        f.write(data)


def main(out: str) -> int:
    for name in ("generation_id", "system_properties"):
        copy_attr(os.path.join(KFD, name), os.path.join(out, "kfd", name))
    nodes = os.path.join(KFD, "nodes")
    for n in sorted(os.listdir(nodes), key=int):
        nd = os.path.join(nodes, n)
        for attr in ("properties", "gpu_id", "name"):
            copy_attr(os.path.join(nd, attr), os.path.join(out, "kfd", "nodes", n, attr))
        for sub in ("mem_banks", "io_links", "p2p_links"):
            sd = os.path.join(nd, sub)
            if not os.path.isdir(sd):
                continue
            for b in sorted(os.listdir(sd)):
                copy_attr(os.path.join(sd, b, "properties"),
                          os.path.join(out, "kfd", "nodes", n, sub, b, "properties"))
    drm = "/sys/class/drm"
    for card in sorted(os.listdir(drm)):
        if not card.startswith(("card", "renderD")) or "-" in card:
            continue
        dev = os.path.join(drm, card, "device")
        for attr in ("current_compute_partition", "available_compute_partition",
                     "current_memory_partition", "available_memory_partition", "vendor", "device",
                     "unique_id", "numa_node", "mem_info_vram_total", "mem_info_vram_used",
                     "gpu_busy_percent", "uevent"):
            copy_attr(os.path.join(dev, attr), os.path.join(out, "drm", card, "device", attr))
        try:
            link = os.readlink(os.path.join(drm, card, "device"))
            with open(os.path.join(out, "drm", card, "device_link"), "w") as f:
                f.write(link + "\n")
        except OSError:
            pass
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sysfs"))
