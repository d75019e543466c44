"""A fake ``amdsmi`` module that replays what the real library returned on an MI355X node.

tests/fixtures/amdsmi_python_mi355x.json was captured by tools/probe_amdsmi.py on the GPU box
(serials redacted).  Every GPU of the fake node returns that record with its own BDF / UUID /
render minor, so exporter and partition-manager code paths run against real field names, units and
"N/A" placements.
"""
from __future__ import annotations

import copy
import ctypes
import enum
import json
from pathlib import Path

_FIX = json.loads((Path(__file__).resolve().parent.parent / "fixtures" / "amdsmi_python_mi355x.json").read_text())
_LAYOUT = json.loads((Path(__file__).resolve().parent.parent / "fixtures" / "mi355x_node_layout.json").read_text())
_REC = _FIX["handles"][0]


class AmdSmiComputePartitionType(enum.Enum):
    SPX = 0
    DPX = 1
    TPX = 2
    QPX = 3
    CPX = 4


class AmdSmiMemoryPartitionType(enum.Enum):
    NPS1 = 0
    NPS2 = 1
    NPS4 = 2


class Handle(ctypes.c_void_p):
    """Like amdsmi's processor handles: a c_void_p (unhashable) that also indexes our tables."""

    __hash__ = None

    def __index__(self):
        return int(self.value or 0)


class FakeAmdSmi:
    """Instances behave like the module (attributes = API functions)."""

    AmdSmiComputePartitionType = AmdSmiComputePartitionType
    AmdSmiMemoryPartitionType = AmdSmiMemoryPartitionType

    def __init__(self, n_gpus: int = 8, fail: set = ()):
        self.n = n_gpus
        self.fail = set(fail)
        self.inited = False
        self.compute = {i: "SPX" for i in range(n_gpus)}
        self.memory = {i: "NPS1" for i in range(n_gpus)}
        self.ecc_uncorrectable = {i: 0 for i in range(n_gpus)}
        self.calls = []

    def _rec(self, h, key):
        if key in self.fail:
            raise RuntimeError(f"AMDSMI_STATUS_NOT_SUPPORTED ({key})")
        return copy.deepcopy(_REC[key])

    def amdsmi_init(self, *a):
        self.inited = True

    def amdsmi_shut_down(self):
        self.inited = False

    def amdsmi_get_processor_handles(self):
        # the real library returns ctypes.c_void_p handles, which are unhashable
        return [Handle(i) for i in range(self.n)]

    def amdsmi_get_gpu_device_bdf(self, h):
        return _LAYOUT["gpus"][int(h)]["bdf"]

    def amdsmi_get_gpu_device_uuid(self, h):
        return "%08x-0000-1000-8000-%012x" % (int(h), int(_LAYOUT["gpus"][int(h)]["unique_id_hex"], 16) & 0xFFFFFFFFFFFF)

    def amdsmi_get_gpu_asic_info(self, h):
        return self._rec(h, "amdsmi_get_gpu_asic_info")

    def amdsmi_get_gpu_enumeration_info(self, h):
        r = self._rec(h, "amdsmi_get_gpu_enumeration_info")
        r["drm_render"] = _LAYOUT["gpus"][int(h)]["render"]
        r["drm_card"] = _LAYOUT["gpus"][int(h)]["card"]
        r["hip_id"] = int(h)
        return r

    def amdsmi_get_gpu_kfd_info(self, h):
        return {"kfd_id": 1000 + int(h), "node_id": 2 + int(h), "current_partition_id": 0}

    def amdsmi_get_gpu_driver_info(self, h):
        return self._rec(h, "amdsmi_get_gpu_driver_info")

    def amdsmi_get_gpu_metrics_info(self, h):
        r = self._rec(h, "amdsmi_get_gpu_metrics_info")
        r["average_gfx_activity"] = 10 * int(h)
        return r

    def amdsmi_get_power_info(self, h):
        return self._rec(h, "amdsmi_get_power_info")

    def amdsmi_get_gpu_vram_usage(self, h):
        return self._rec(h, "amdsmi_get_gpu_vram_usage")

    def amdsmi_get_gpu_total_ecc_count(self, h):
        r = self._rec(h, "amdsmi_get_gpu_total_ecc_count")
        r["uncorrectable_count"] = self.ecc_uncorrectable[int(h)]
        return r

    def amdsmi_get_gpu_compute_partition(self, h):
        return self.compute[int(h)]

    def amdsmi_get_gpu_memory_partition(self, h):
        return self.memory[int(h)]

    def amdsmi_get_gpu_process_list(self, h):
        return self._rec(h, "amdsmi_get_gpu_process_list")
