"""FakeAmdSmi plus the partition-setting calls (used only by the partition-manager CPU tests;
listed in .gpurunignore with operator/partition_amdsmi.py)."""
from fakes.amdsmi import FakeAmdSmi


class FakeAmdSmiPartitionable(FakeAmdSmi):
    def amdsmi_set_gpu_compute_partition(self, h, mode):
        self.calls.append(("compute", int(h), mode.name))
        self.compute[int(h)] = mode.name

    def amdsmi_set_gpu_memory_partition(self, h, mode):
        self.calls.append(("memory", int(h), mode.name))
        self.memory[int(h)] = mode.name
