"""amd-smi backend of the partition manager (operator/partition.py): applies a compute / memory
partition mode to one ASIC through the amdsmi Python bindings.

amd-smi's memory-partition call is hive-wide and reloads the driver itself
(``memory_reloads_driver``); a compute-partition call re-enumerates that ASIC's agents.  Either way
the processor handles the session listed are invalid afterwards, so the session is shut down and
re-initialised before the next lookup, and every lookup lists the handles anew.

Kept in its own module and imported only by the ``partition-manager`` component (and its CPU
test): it is the one piece of the operator that changes a device-wide setting, and nothing that
runs on a shared GPU box (bench, validator, GPU tests) ever needs it (listed in .gpurunignore).
"""
from __future__ import annotations

from ..utils import topology as topo_mod
from .partition import PartitionError


class AmdSmiPartitionBackend:
    memory_reloads_driver = True

    def __init__(self, amdsmi_module=None):
        if amdsmi_module is None:
            import amdsmi as amdsmi_module  # noqa: N813
        self.S = amdsmi_module
        self.S.amdsmi_init()
        self._stale = False

    def _fresh(self) -> None:
        """A new session after any mode change: the old one's handles point at withdrawn agents."""
        if self._stale:
            try:
                self.S.amdsmi_shut_down()
            except Exception:  # noqa: BLE001 - the reload may already have torn it down
                pass
            self.S.amdsmi_init()
            self._stale = False

    def _handle(self, dev: topo_mod.GpuDevice):
        self._fresh()
        for h in self.S.amdsmi_get_processor_handles():
            if str(self.S.amdsmi_get_gpu_device_bdf(h)).lower() == dev.pci_bdf.lower():
                return h
        raise PartitionError(f"amd-smi has no handle for {dev.pci_bdf}")

    def set_compute(self, dev: topo_mod.GpuDevice, mode: str) -> None:
        h = self._handle(dev)
        self._stale = True
        self.S.amdsmi_set_gpu_compute_partition(h, getattr(self.S.AmdSmiComputePartitionType, mode))

    def set_memory(self, dev: topo_mod.GpuDevice, mode: str) -> None:
        h = self._handle(dev)
        self._stale = True
        self.S.amdsmi_set_gpu_memory_partition(h, getattr(self.S.AmdSmiMemoryPartitionType, mode))
