"""Partition switch on a *serving* node (BASELINE config 5; VERDICT r3 "What's missing" 2 /
"What's weak" 4): GPU pods are evicted through the Eviction API (PodDisruptionBudgets honoured),
the operator's own GPU clients (exporter, driver probe, device plugin) release their handles and
ack the pause, busy sysfs writes are retried, and the validator starts no load step meanwhile.

Fake kube-API (tests/fakes/kubeapi.py, with pods/<n>/eviction), fake MI355X sysfs tree, fake amdsmi.
"""
import errno
import json
import os
import threading
import time

import pytest

from fakes import sysfs as fake_sysfs
from fakes.amdsmi import FakeAmdSmi
from fakes.kubeapi import FakeKubeAPI
from k8s_nvidia_gpus_amd.operator import partition as pm
from k8s_nvidia_gpus_amd.operator import pause as pause_mod
from k8s_nvidia_gpus_amd.utils.kube import KubeClient
from k8s_nvidia_gpus_amd.utils.topology import read_topology


@pytest.fixture
def api():
    a = FakeKubeAPI().start()
    a.add_node("gpu-node-1", {"kubernetes.io/os": "linux", pm.LABEL_DESIRED: "CPX"})
    yield a
    a.stop()


@pytest.fixture
def client(api):
    return KubeClient(base_url=api.url)


class Backend:
    """Re-enumerates the fake sysfs like the driver; ``busy`` writes fail with EBUSY first."""

    def __init__(self, root, busy=0, guard=None):
        self.root, self.busy, self.guard = root, busy, guard
        self.applied, self.attempts = [], 0
        self.while_held = []

    def set_memory(self, dev, mode):
        self.applied.append(("memory", dev.pci_bdf, mode))

    def set_compute(self, dev, mode):
        self.attempts += 1
        if self.guard is not None:
            self.while_held.append(self.guard())
        if self.busy:
            self.busy -= 1
            raise OSError(errno.EBUSY, "Device or resource busy")
        self.applied.append(("compute", dev.pci_bdf, mode))
        if len([a for a in self.applied if a[0] == "compute"]) == 8:
            fake_sysfs.set_partition(self.root, 8, mode, "NPS1")


def _mgr(client, root, tmp_path, backend, **kw):
    args = dict(poll=0.01, pause_marker=str(tmp_path / "run/partition-in-progress"),
                ack_dir=str(tmp_path / "run/acks"), ack_components=(), sleep=lambda s: None,
                reservation=str(tmp_path / "run/validations/in-test.json"), retry_backoff=0.0)
    args.update(kw)
    return pm.PartitionManager(client, "gpu-node-1", backend, str(root), **args)


def test_serving_llm_pod_is_evicted_then_cpx_applied_on_all_asics(tmp_path, api, client):
    """The reference's LLM Deployment pod holds a GPU: a NoSchedule taint alone would never move it."""
    root = fake_sysfs.build_node(tmp_path / "r")
    api.add_pod("llm", "coder-llm-7d9f", "gpu-node-1", gpus=1)
    api.add_pod("kube-system", "cilium-abc", "gpu-node-1", gpus=0)     # no GPU: left alone
    backend = Backend(root)
    assert _mgr(client, root, tmp_path, backend).reconcile() == "applied"
    assert api.evictions == [("llm", "coder-llm-7d9f")]
    assert ("kube-system", "cilium-abc") in api.pods
    evict_posts = [r for r in api.requests if r[0] == "POST" and r[1].endswith("/eviction")]
    assert evict_posts and evict_posts[0][1] == "/api/v1/namespaces/llm/pods/coder-llm-7d9f/eviction"
    assert len([a for a in backend.applied if a[0] == "compute"]) == 8
    assert len(read_topology(str(root), 90500).gpus) == 64
    node = api.nodes["gpu-node-1"]
    assert node["metadata"]["labels"]["amd.com/gpu.compute-partition"] == "CPX"
    assert node["metadata"]["annotations"][pm.ANNOT_STATE].startswith("idle")
    assert not os.path.exists(tmp_path / "run/partition-in-progress")


def test_pdb_blocked_eviction_fails_the_change_with_the_reason(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    api.add_pod("llm", "coder-llm-7d9f", "gpu-node-1", gpus=1)
    api.pdb_blocked[("llm", "coder-llm-7d9f")] = (
        "Cannot evict pod as it would violate the pod's disruption budget.")
    backend = Backend(root)
    assert _mgr(client, root, tmp_path, backend, drain_timeout=0.05).reconcile() == "failed"
    state = api.nodes["gpu-node-1"]["metadata"]["annotations"][pm.ANNOT_STATE]
    assert state.startswith("failed") and "llm/coder-llm-7d9f" in state and "disruption budget" in state
    assert backend.applied == [] and ("llm", "coder-llm-7d9f") in api.pods
    taints = api.nodes["gpu-node-1"]["spec"].get("taints", [])
    assert not [t for t in taints if t["key"] == pm.TAINT_KEY]
    assert not os.path.exists(tmp_path / "run/partition-in-progress")


def test_ebusy_twice_then_success_is_retried_with_backoff(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    sleeps = []
    backend = Backend(root, busy=2)
    mgr = _mgr(client, root, tmp_path, backend, retry_backoff=0.5, sleep=sleeps.append)
    assert mgr.reconcile() == "applied"
    assert backend.attempts == 8 + 2
    assert [s for s in sleeps if s >= 0.5] == [0.5, 1.0]           # exponential backoff
    # a busy device that never frees up fails after applyRetries
    root2 = fake_sysfs.build_node(tmp_path / "r2")
    b2 = Backend(root2, busy=100)
    assert _mgr(client, root2, tmp_path, b2, apply_retries=3).reconcile() == "failed"
    assert b2.attempts == 4
    assert "busy" in api.nodes["gpu-node-1"]["metadata"]["annotations"][pm.ANNOT_STATE].lower()
    # a non-busy error is not retried
    root3 = fake_sysfs.build_node(tmp_path / "r3")

    class Broken(Backend):
        def set_compute(self, dev, mode):
            self.attempts += 1
            raise OSError(errno.EINVAL, "Invalid argument")
    b3 = Broken(root3)
    assert _mgr(client, root3, tmp_path, b3).reconcile() == "failed" and b3.attempts == 1


def test_operator_gpu_clients_release_their_handles_before_the_apply(tmp_path, api, client):
    """Exporter (amd-smi session), driver probe (/dev/kfd opens) and device plugin (amd-smi ECC
    session) see the pause marker, close their handles and ack; only then is the mode applied."""
    from k8s_nvidia_gpus_amd.operator.device_plugin import AmdGpuDevicePlugin, AmdSmiEccReader
    from k8s_nvidia_gpus_amd.operator.config import load_config
    from k8s_nvidia_gpus_amd.operator.exporter import AmdSmiBackend, ExporterServer, GpuCollector
    from k8s_nvidia_gpus_amd.operator.runtime import driver_ready_loop

    root = fake_sysfs.build_node(tmp_path / "r")
    marker = str(tmp_path / "run/partition-in-progress")
    acks = str(tmp_path / "run/acks")
    guard = lambda c: pause_mod.PauseGuard(c, marker=marker, ack_dir=acks)  # noqa: E731
    # exporter
    smi_exp = FakeAmdSmi()
    srv = ExporterServer(GpuCollector(AmdSmiBackend(smi_exp), "gpu-node-1", str(tmp_path / "v"),
                                      guard=guard("exporter")), port=0, host="127.0.0.1")
    # device plugin with an amd-smi ECC reader
    smi_dp = FakeAmdSmi()
    plugin = AmdGpuDevicePlugin(load_config(), root=str(root), kubelet_dir=str(tmp_path / "kd"),
                                pause_marker=marker, dev_prefix=str(root / "dev"),
                                ecc_fn=AmdSmiEccReader(smi_dp), pause_guard=guard("device-plugin"))
    plugin._ecc = plugin.health_fn.ecc_fn
    # driver readiness loop with a fake kfd-probe that records each run
    probe_log = tmp_path / "probe.log"
    probe = tmp_path / "kfd-probe"
    probe.write_text(f"#!/bin/sh\necho run >> {probe_log}\nexit 0\n")
    probe.chmod(0o755)
    stop = threading.Event()
    threads = [
        threading.Thread(target=srv.watch_pause, kwargs={"interval": 0.02, "stop_event": stop}),
        threading.Thread(target=plugin.run, kwargs={"poll": 0.02, "stop_event": stop, "health_interval": 60}),
        threading.Thread(target=driver_ready_loop,
                         args=(str(probe), 8, 90500, str(tmp_path / "v"), 0.05),
                         kwargs={"stop_event": stop, "guard": guard("driver"), "pause_poll": 0.02}),
    ]
    for t in threads:
        t.daemon = True
        t.start()

    def held():
        """Who still holds a GPU handle at the moment of the write."""
        return {"exporter": smi_exp.inited, "device-plugin": smi_dp.inited}

    runs_at_apply = []

    class B(Backend):
        def set_compute(self, dev, mode):
            runs_at_apply.append(len(probe_log.read_text().splitlines()))
            time.sleep(0.01)
            super().set_compute(dev, mode)

    backend = B(root, guard=held)
    api.add_pod("llm", "coder-llm-7d9f", "gpu-node-1", gpus=1)
    mgr = _mgr(client, root, tmp_path, backend, pause_marker=marker, ack_dir=acks,
               ack_components=pause_mod.COMPONENTS, pause_ack_timeout=10.0, sleep=time.sleep)
    try:
        time.sleep(0.15)                      # clients up and probing
        assert smi_exp.inited and smi_dp.inited
        assert mgr.reconcile() == "applied"
        time.sleep(0.3)                       # clients resume after the marker is gone
        resumed = (smi_exp.inited, smi_dp.inited)
        with srv.lock:
            paused_after = srv.collector.paused
    finally:
        stop.set()
        for t in threads:
            t.join(5)
    # at every write, no client held a handle; all three acked this pause's nonce
    assert backend.while_held and all(h == {"exporter": False, "device-plugin": False}
                                      for h in backend.while_held)
    assert len(set(runs_at_apply)) == 1       # the probe did not run during the apply
    for c in pause_mod.COMPONENTS:
        assert os.path.exists(os.path.join(acks, c))
    assert resumed == (True, True) and not paused_after
    assert len(read_topology(str(root), 90500).gpus) == 64


def test_exporter_reports_stale_while_paused(tmp_path):
    from prometheus_client import generate_latest

    from k8s_nvidia_gpus_amd.operator.exporter import AmdSmiBackend, GpuCollector, make_registry

    marker = str(tmp_path / "pause")
    g = pause_mod.PauseGuard("exporter", marker=marker, ack_dir=str(tmp_path / "acks"))
    smi = FakeAmdSmi()
    col = GpuCollector(AmdSmiBackend(smi), "n", str(tmp_path), guard=g)
    reg = make_registry(col)
    body = generate_latest(reg).decode()
    assert "amd_gpu_exporter_up 1.0" in body and "amd_gpu_exporter_paused 0.0" in body
    nonce = pause_mod.start_pause(marker)
    body = generate_latest(reg).decode()
    assert "amd_gpu_exporter_up 0.0" in body and "amd_gpu_exporter_paused 1.0" in body
    assert "amd_gpu_power_watts{" not in body and not smi.inited
    assert pause_mod.acks(nonce, str(tmp_path / "acks"), ["exporter"]) == {"exporter": True}
    pause_mod.end_pause(marker)
    body = generate_latest(reg).decode()
    assert "amd_gpu_exporter_up 1.0" in body and smi.inited and "amd_gpu_power_watts{" in body


def test_validator_defers_load_steps_during_a_partition_change(tmp_path):
    from k8s_nvidia_gpus_amd.operator.config import load_config
    from k8s_nvidia_gpus_amd.operator.validator import Validator

    root = fake_sysfs.build_node(tmp_path / "r")
    marker = tmp_path / "pause"
    pause_mod.start_pause(str(marker))
    calls = []
    cfg = load_config(text="validator: {podResourcesRequired: false}\n")
    v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", root=str(root),
                  runner=lambda argv, t: calls.append(argv) or (0, ""), pause_marker=str(marker))
    r = v.run_step("gemm")
    assert r.deferred and "partition change" in r.reason and calls == []


def test_drain_waits_for_a_running_validator_load_step(tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    res = tmp_path / "run/validations/in-test.json"
    res.parent.mkdir(parents=True)
    res.write_text(json.dumps({"nonce": "n", "device_uids": [], "expires": time.time() + 3600}))
    assert _mgr(client, root, tmp_path, Backend(root), drain_timeout=0.05).reconcile() == "failed"
    assert "validator load step" in api.nodes["gpu-node-1"]["metadata"]["annotations"][pm.ANNOT_STATE]


# ----------------------------------------------------------------------------- driver semantics
def test_amdsmi_hive_spx_nps1_to_cpx_nps2_with_handle_invalidation(tmp_path, api, client):
    """against the hardware-faithful fake (NPS hive-wide with a driver reload
    that kills the amd-smi session; a compute change invalidates that ASIC's handles) the manager
    applies NPS2 ONCE, waits for the reload, re-opens amd-smi and switches every ASIC to CPX."""
    from fakes.amdsmi_partition import FakeAmdSmiHive
    from k8s_nvidia_gpus_amd.operator.partition_amdsmi import AmdSmiPartitionBackend

    root = fake_sysfs.build_node(tmp_path / "r")
    api.nodes["gpu-node-1"]["metadata"]["labels"][pm.LABEL_MEM_DESIRED] = "NPS2"
    hive = FakeAmdSmiHive(root)
    backend = AmdSmiPartitionBackend(hive)
    assert _mgr(client, root, tmp_path, backend).reconcile() == "applied"
    mem = [c for c in hive.calls if c[0] == "memory"]
    assert hive.reloads == 1 and len(mem) == 1 and mem[0][2] == "NPS2"        # once per node
    assert sorted(c[1] for c in hive.calls if c[0] == "compute") == list(range(8))
    topo = read_topology(str(root), 90500)
    assert len(topo.gpus) == 64
    assert {(g.compute_partition, g.memory_partition) for g in topo.gpus} == {("CPX", "NPS2")}
    state = api.nodes["gpu-node-1"]["metadata"]["annotations"][pm.ANNOT_STATE]
    assert state.startswith("idle: applied CPX/NPS2") and "validator" in state
    assert _mgr(client, root, tmp_path, backend).reconcile() == "idle"


def test_amdsmi_hive_cpx_nps1_to_cpx_nps2_waits_for_64_agents(tmp_path, api, client):
    """a node already in CPX keeps CPX through the NPS reload, so the re-enumeration
    wait must expect 8 agents per ASIC (it expected one per ASIC and timed out into `failed`)."""
    from fakes.amdsmi_partition import FakeAmdSmiHive
    from k8s_nvidia_gpus_amd.operator.partition_amdsmi import AmdSmiPartitionBackend

    root = fake_sysfs.build_node(tmp_path / "r", compute_partition="CPX")
    api.nodes["gpu-node-1"]["metadata"]["labels"][pm.LABEL_MEM_DESIRED] = "NPS2"
    hive = FakeAmdSmiHive(root, compute="CPX")
    backend = AmdSmiPartitionBackend(hive)
    assert _mgr(client, root, tmp_path, backend, reenum_timeout=2).reconcile() == "applied"
    assert hive.reloads == 1 and not [c for c in hive.calls if c[0] == "compute"]
    topo = read_topology(str(root), 90500)
    assert len(topo.gpus) == 64
    assert {(g.compute_partition, g.memory_partition) for g in topo.gpus} == {("CPX", "NPS2")}
    labels = api.nodes["gpu-node-1"]["metadata"]["labels"]
    assert labels["amd.com/gpu.memory-partition"] == "NPS2"


def test_sysfs_reload_command_cpx_nps1_to_cpx_nps2(tmp_path, api, client):
    """The same CPX/NPS1 -> CPX/NPS2 change through sysfs writes plus the driver reload command."""
    root = fake_sysfs.build_node(tmp_path / "r", compute_partition="CPX")
    api.nodes["gpu-node-1"]["metadata"]["labels"][pm.LABEL_MEM_DESIRED] = "NPS2"
    backend = DriverSysfs(root)
    runs = []
    mgr = _mgr(client, root, tmp_path, backend, reload_cmd=["/host/reload-amdgpu.sh"],
               reenum_timeout=2, run_cmd=lambda argv: runs.append(argv) or backend.reload())
    assert mgr.reconcile() == "applied" and runs == [["/host/reload-amdgpu.sh"]]
    topo = read_topology(str(root), 90500)
    assert len(topo.gpus) == 64 and backend.reloads == 1
    assert {(g.compute_partition, g.memory_partition) for g in topo.gpus} == {("CPX", "NPS2")}


def test_a_per_asic_nps_loop_on_one_session_fails_on_the_faithful_fake(tmp_path):
    """What the round-4 manager did — NPS per ASIC through the session opened at start — meets a
    dead session after the first (hive-wide) reload."""
    from fakes.amdsmi_partition import FakeAmdSmiHive

    root = fake_sysfs.build_node(tmp_path / "r")
    hive = FakeAmdSmiHive(root)
    hive.amdsmi_init()
    hs = hive.amdsmi_get_processor_handles()
    hive.amdsmi_set_gpu_memory_partition(hs[0], hive.AmdSmiMemoryPartitionType.NPS2)
    with pytest.raises(RuntimeError, match="stale"):
        hive.amdsmi_set_gpu_memory_partition(hs[1], hive.AmdSmiMemoryPartitionType.NPS2)
    with pytest.raises(RuntimeError, match="reload"):
        hive.amdsmi_get_processor_handles()
    hive.amdsmi_shut_down()
    hive.amdsmi_init()
    hs = hive.amdsmi_get_processor_handles()
    hive.amdsmi_set_gpu_compute_partition(hs[2], hive.AmdSmiComputePartitionType.CPX)
    with pytest.raises(RuntimeError, match="stale"):         # that ASIC's handle is gone
        hive.amdsmi_set_gpu_compute_partition(hs[2], hive.AmdSmiComputePartitionType.SPX)
    hive.amdsmi_get_gpu_device_bdf(hs[3])                    # other ASICs' handles still valid
    assert len(hive.amdsmi_get_processor_handles()) == 7 + 8


class DriverSysfs(pm.SysfsPartitionBackend):
    """The real sysfs writes on the fake tree plus what amdgpu does with them: a compute write
    re-partitions that ASIC at once; a memory write only requests the NPS mode, which a driver
    reload (``reload``) applies to the whole hive."""

    def __init__(self, root):
        super().__init__(str(root))
        self.requested = None
        self.reloads = 0

    BDFS = [g["bdf"] for g in fake_sysfs.LAYOUT["gpus"][:8]]     # build_node's ASIC order

    def _modes(self):
        heads = {g.pci_bdf: g for g in read_topology(self.root, 90500).gpus}
        return ([heads[b].compute_partition for b in self.BDFS],
                [heads[b].memory_partition for b in self.BDFS])

    def set_compute(self, dev, mode):
        super().set_compute(dev, mode)
        c, m = self._modes()
        c[self.BDFS.index(dev.pci_bdf)] = mode
        fake_sysfs.set_partition(self.root, 8, c, m)

    def set_memory(self, dev, mode):
        path = os.path.join(self.root, "sys/class/drm", f"card{dev.card_minor}", "device",
                            "current_memory_partition")
        old = open(path).read()
        super().set_memory(dev, mode)           # the write goes through ...
        with open(path, "w") as f:              # ... but reads back the running mode until a reload
            f.write(old)
        self.requested = mode

    def reload(self):
        c, _ = self._modes()
        self.reloads += 1
        fake_sysfs.set_partition(self.root, 8, c, [self.requested] * 8)
        return 0


def test_sysfs_nps_request_ends_in_pending_reload_then_a_reload_command_completes_it(
        tmp_path, api, client):
    root = fake_sysfs.build_node(tmp_path / "r")
    api.nodes["gpu-node-1"]["metadata"]["labels"][pm.LABEL_MEM_DESIRED] = "NPS2"
    api.add_pod("llm", "coder-llm-7d9f", "gpu-node-1", gpus=1)
    backend = DriverSysfs(root)
    mgr = _mgr(client, root, tmp_path, backend, reenum_timeout=0.05)
    assert mgr.reconcile() == "pending-reload"
    node = api.nodes["gpu-node-1"]
    state = node["metadata"]["annotations"][pm.ANNOT_STATE]
    assert state.startswith("pending-reload: NPS2") and "driverReloadCommand" in state
    assert not [t for t in node["spec"].get("taints", []) if t["key"] == pm.TAINT_KEY]
    assert not os.path.exists(tmp_path / "run/partition-in-progress")
    assert {g.memory_partition for g in read_topology(str(root), 90500).gpus} == {"NPS1"}
    assert backend.requested == "NPS2" and api.evictions == [("llm", "coder-llm-7d9f")]
    # the next reconcile neither drains again nor times out: the request stands
    api.add_pod("llm", "coder-llm-new", "gpu-node-1", gpus=1)
    assert mgr.reconcile() == "pending-reload" and len(api.evictions) == 1
    # with a reload command configured the change completes
    runs = []
    mgr2 = _mgr(client, root, tmp_path, backend, reload_cmd=["/host/reload-amdgpu.sh"], reenum_timeout=5,
                run_cmd=lambda argv: runs.append(argv) or backend.reload())
    assert mgr2.reconcile() == "applied" and runs == [["/host/reload-amdgpu.sh"]]
    topo = read_topology(str(root), 90500)
    assert len(topo.gpus) == 64 and backend.reloads == 1
    assert {(g.compute_partition, g.memory_partition) for g in topo.gpus} == {("CPX", "NPS2")}


def test_validator_step_started_after_the_drain_is_waited_for(tmp_path, api, client):
    """a validator reservation that appears after the drain (between the drain and the
    write) holds the apply until it is released."""
    root = fake_sysfs.build_node(tmp_path / "r")
    res = tmp_path / "run/validations/in-test.json"
    res.parent.mkdir(parents=True)
    seen = []

    def acks(*a, **k):
        # the validator reserves right after the drain finished
        res.write_text(json.dumps({"nonce": "n", "device_uids": [], "expires": time.time() + 3600}))
        return {}

    def sleep(_s):
        seen.append(res.exists())
        if len(seen) == 3:
            res.unlink()                       # its step finished

    backend = Backend(root)
    mgr = _mgr(client, root, tmp_path, backend, sleep=sleep, ack_components=("x",))
    orig = pause_mod.acks
    pause_mod.acks = lambda nonce, d, comps: (acks(), {c: True for c in comps})[1]
    try:
        assert mgr.reconcile() == "applied"
    finally:
        pause_mod.acks = orig
    assert seen[:3] == [True, True, True] and len(backend.applied) == 8
