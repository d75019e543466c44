"""FakeAmdSmi plus the partition-setting calls (used only by the partition-manager CPU tests;
listed in .gpurunignore with operator/partition_amdsmi.py).

``FakeAmdSmiHive`` follows how amdgpu applies the modes on an MI300/MI355 hive,
so the manager is tested against the hardware's semantics rather than per-handle setters:

* processor handles are per KFD agent (SPX: one per ASIC, CPX: eight) and belong to the session
  that listed them;
* ``amdsmi_set_gpu_memory_partition`` is hive-wide: EVERY ASIC changes NPS mode and the driver
  reloads — all KFD agents are withdrawn and re-created (the fake sysfs tree is rebuilt), every
  handle is invalid, and the session itself is dead until ``amdsmi_shut_down`` + ``amdsmi_init``;
* ``amdsmi_set_gpu_compute_partition`` re-partitions one ASIC: its agent count changes and its
  handles become invalid.
A stale handle or session raises, as the library does.
"""
from fakes import sysfs as fake_sysfs
from fakes.amdsmi import _LAYOUT, FakeAmdSmi, Handle


class FakeAmdSmiPartitionable(FakeAmdSmi):
    def amdsmi_set_gpu_compute_partition(self, h, mode):
        self.calls.append(("compute", int(h), mode.name))
        self.compute[int(h)] = mode.name

    def amdsmi_set_gpu_memory_partition(self, h, mode):
        self.calls.append(("memory", int(h), mode.name))
        self.memory[int(h)] = mode.name


class FakeAmdSmiHive(FakeAmdSmi):
    def __init__(self, root, n_gpus: int = 8, compute: str = "SPX", memory: str = "NPS1"):
        super().__init__(n_gpus)
        self.root = root
        self.compute = {a: compute for a in range(n_gpus)}
        self.memory = {a: memory for a in range(n_gpus)}
        self.session = 0
        self.session_alive = False
        self.asic_gen = {a: 0 for a in range(n_gpus)}
        self.reloads = 0
        self._next = 1
        self._handles = {}

    def amdsmi_init(self, *a):
        self.inited = True
        self.session += 1
        self.session_alive = True

    def amdsmi_shut_down(self):
        self.inited = False
        self.session_alive = False

    def amdsmi_get_processor_handles(self):
        if not (self.inited and self.session_alive):
            raise RuntimeError("AMDSMI_STATUS_DRV_ERR: session predates a driver reload")
        out = []
        for a in range(self.n):
            for p in range(fake_sysfs.SPLIT[self.compute[a]]):
                hid = self._next
                self._next += 1
                self._handles[hid] = (self.session, a, self.asic_gen[a], p)
                out.append(Handle(hid))
        return out

    def _asic(self, h) -> int:
        rec = self._handles.get(int(h))
        if (rec is None or not self.session_alive or rec[0] != self.session
                or rec[2] != self.asic_gen[rec[1]]):
            raise RuntimeError("AMDSMI_STATUS_INVAL: stale processor handle")
        return rec[1]

    def amdsmi_get_gpu_device_bdf(self, h):
        return _LAYOUT["gpus"][self._asic(h)]["bdf"]

    def amdsmi_set_gpu_memory_partition(self, h, mode):
        a = self._asic(h)
        self.calls.append(("memory", a, mode.name))
        for x in range(self.n):                 # hive-wide
            self.memory[x] = mode.name
            self.asic_gen[x] += 1               # every agent withdrawn and re-created
        self.reloads += 1
        self.session_alive = False              # the driver reloaded under the session
        self._sync()

    def amdsmi_set_gpu_compute_partition(self, h, mode):
        a = self._asic(h)
        self.calls.append(("compute", a, mode.name))
        self.compute[a] = mode.name
        self.asic_gen[a] += 1                   # this ASIC's agents re-enumerate
        self._sync()

    def _sync(self):
        fake_sysfs.set_partition(self.root, self.n, [self.compute[a] for a in range(self.n)],
                                 [self.memory[a] for a in range(self.n)])
