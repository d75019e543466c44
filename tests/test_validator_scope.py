"""Validator GPU scope: GPUs that kubelet allocated to pods are never loaded, a fully allocated node
defers the load steps (label ``deferred``, never ``true``), an unreachable kubelet fails them, a GPU
allocated between the PodResources answer and the launch is left untouched (reservation + re-read),
the device plugin gates GPUs on this boot's validation, an unchanged node re-uses its last full
pass (but a partition switch does not), and compute-partitioned (CPX) nodes validate against
per-partition floors.

kubelet's PodResources API is served by tests/fakes/podresources.py over a real unix socket; the
node is the fake MI355X sysfs tree (tests/fakes/sysfs.py) with 8 ASICs (64 CPX agents)."""
import json
import os
import time

import pytest

from fakes import sysfs as fake_sysfs
from fakes.podresources import FakePodResources
from k8s_nvidia_gpus_amd.operator.config import load_config
from k8s_nvidia_gpus_amd.operator.validator import (FINGERPRINT, IN_TEST, VALIDATED_DEVICES,
                                                    Validator, hold_loop)
from k8s_nvidia_gpus_amd.utils.topology import read_topology
from test_validator import GEMM_FP8_LOG, RCCL_8GPU, Runner


def _gemm_log(n, tflops, size=8192, dtype="bf16"):
    lines = [f"[{dtype} MFMA GEMM {size}x{size}x{size} (C = A*B^T), {n} device(s), 50 iters]"]
    for i in range(n):
        lines.append(json.dumps({"check": f"gemm_{dtype}", "device": i, "m": size, "n": size, "k": size,
                                 "tflops": tflops, "bad_samples": 0, "passed": True}))
    return "\n".join(lines + ["Test PASSED", "Done", ""])


def _pt(test, device, value, peer=-1, engine=""):
    return json.dumps({"check": "proftester", "test": test, "device": device, "peer": peer,
                       "engine": engine, "value": value, "min": value, "max": value, "unit": "GB/s",
                       "seconds": 0.01, "skipped": False, "passed": True, "note": ""})


def _node(tmp_path, mode="SPX", boot="boot-1"):
    root = fake_sysfs.build_node(tmp_path / "root", compute_partition=mode)
    (root / "proc/sys/kernel/random").mkdir(parents=True, exist_ok=True)
    (root / "proc/sys/kernel/random/boot_id").write_text(boot + "\n")
    return root


def _cfg(tmp_path, extra=""):
    sock = tmp_path / "pod-resources/kubelet.sock"
    text = (f"expectedGpusPerNode: 8\nvalidator: {{gemmMinTflops: 900, gemmFp8: false, "
            f"podResourcesSocket: {sock}, rccl: true, bandwidth: false, reserveAckSeconds: 0.2{extra}}}\n")
    return load_config(text=text), str(sock)


def _uids(root):
    return [g.device_uid for g in sorted(read_topology(str(root), 90500).gpus, key=lambda g: g.node_id)]


def _narrowed(call):
    return call[1].split("=", 1)[1].split(",") if call[0] == "env" else None


def test_allocated_gpus_are_excluded(tmp_path):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path)
    uids = _uids(root)
    pods = {("llm", "coder-llm-0"): [("amd.com/gpu", [uids[2], uids[5]])],
            ("default", "cpu-pod"): [("example.com/nic", ["x"])]}
    r = Runner({"amd-gemm-validator": (0, _gemm_log(6, 1500.0)), "rccl-allreduce-bench": (0, RCCL_8GPU)})
    with FakePodResources(sock, pods) as fake:
        v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root))
        g = v.run_step("gemm")
        rc = v.run_step("rccl")
    assert fake.calls >= 1
    assert g.passed and rc.passed
    # the GEMM ran on the 6 free agents only, by ROCr index
    assert _narrowed(r.calls[0]) == ["0", "1", "3", "4", "6", "7"]
    assert _narrowed(r.calls[1]) == ["0", "1", "3", "4", "6", "7"]
    sc = g.detail["gpu_scope"]
    assert not sc["full"] and sc["allocated"] == {uids[2]: "llm/coder-llm-0", uids[5]: "llm/coder-llm-0"}
    assert uids[2] not in sc["validated"] and len(sc["validated"]) == 6
    # a partial validation never becomes the node's fingerprint, and the node is not "validated"
    for st in ("driver", "runtime", "vectoradd", "plugin", "bandwidth", "stress"):
        (tmp_path / "m" / f"{st}-ready").write_text("1\n")
    rep = v.run_step("report")
    assert not rep.passed and rep.detail["label"] == "partial" and rep.proceed
    assert not os.path.exists(tmp_path / "m" / FINGERPRINT)
    assert not os.path.exists(tmp_path / "m" / "validator-ready")
    # only the GPUs the load steps actually ran on are validated for the plugin's gate
    assert sorted(rep.detail["validated_devices"]) == sorted(sc["validated"])


class _Kube:
    def __init__(self):
        self.labels = {}
        self.deleted = []

    def set_node_labels(self, node, labels):
        self.labels.update(labels)

    def delete_pod(self, ns, name):
        self.deleted.append((ns, name))


def _chain_markers(marker, steps=("driver", "runtime", "vectoradd", "plugin")):
    marker.mkdir(exist_ok=True)
    for st in steps:
        (marker / f"{st}-ready").write_text("1\n")


def test_fully_allocated_node_defers_and_is_not_labelled_validated(tmp_path):
    """First boot, every GPU already taken: nothing is loaded, no load step gets a -ready marker,
    the chain goes on (proceed), and the node label says "deferred" — not "true"."""
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path)
    pods = {("train", f"job-{i}"): [("amd.com/gpu", [u])] for i, u in enumerate(_uids(root))}
    r = Runner({})
    kube = _Kube()
    _chain_markers(tmp_path / "m")
    with FakePodResources(sock, pods):
        v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root), kube=kube,
                      node_name="n1")
        for step in ("gemm", "rccl"):
            res = v.run_step(step)
            assert not res.passed and res.deferred and res.proceed, step
        for step in ("stress", "bandwidth"):                # disabled in this config
            assert v.run_step(step).detail.get("skipped")
        rep = v.run_step("report")
    assert r.calls == []                                   # no GPU was touched
    d = json.loads((tmp_path / "m/gemm.json").read_text())
    assert "allocated" in d["deferred"] and d["gpu_scope"]["validated"] == []
    assert not (tmp_path / "m/gemm-ready").exists()
    assert not rep.passed and rep.detail["label"] == "deferred"
    assert kube.labels == {"amd.com/gpu.validated": "deferred"}
    assert rep.detail["validated_devices"] == []
    assert not (tmp_path / "m/validator-ready").exists()


def test_unreachable_kubelet_fails_the_step_and_the_node(tmp_path):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path)
    os.makedirs(os.path.dirname(sock))
    with open(sock, "w") as f:                              # a socket path nobody serves
        f.write("")
    r = Runner({})
    kube = _Kube()
    _chain_markers(tmp_path / "m")
    v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root), kube=kube,
                  node_name="n1")
    res = v.run_step("gemm")
    assert not res.passed and not res.deferred and "PodResources" in res.reason and r.calls == []
    assert not res.proceed                                  # the init container fails
    v.run_step("rccl")
    rep = v.run_step("report")
    assert rep.detail["label"] == "false" and kube.labels["amd.com/gpu.validated"] == "false"
    assert "gemm" in rep.detail["failed"]


def test_absent_kubelet_socket_fails_unless_not_required(tmp_path):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path)                              # socket path never created
    r = Runner({"amd-gemm-validator": (0, _gemm_log(8, 1500.0))})
    res = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root)).run_step("gemm")
    assert not res.passed and "absent" in res.reason and r.calls == []
    cfg.raw["validator"]["podResourcesRequired"] = False    # bare box (bring-up rehearsal)
    res = Validator(cfg, str(tmp_path / "m2"), bin_dir="/x", runner=r, root=str(root)).run_step("gemm")
    assert res.passed and r.calls and r.calls[0][0] != "env"


class _RacingPodResources(FakePodResources):
    """The second List answer (after the validator's reservation) shows a pod that took a GPU in
    between the first answer and the launch."""

    def __init__(self, sock, pods, late):
        super().__init__(sock, pods)
        self.late = late

    def List(self, request, context):  # noqa: N802
        if self.calls == 1:
            self.pods.update(self.late)
        return super().List(request, context)


def test_gpu_allocated_between_list_and_launch_is_left_untouched(tmp_path):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path)
    uids = _uids(root)
    seen_reservation = []

    class R(Runner):
        def __call__(self, argv, timeout):
            seen_reservation.append(json.loads((tmp_path / "m" / IN_TEST).read_text()))
            return super().__call__(argv, timeout)

    r = R({"amd-gemm-validator": (0, _gemm_log(7, 1500.0))})
    late = {("llm", "coder-llm-0"): [("amd.com/gpu", [uids[3]])]}
    with _RacingPodResources(sock, {}, late) as fake:
        v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root))
        g = v.run_step("gemm")
    assert fake.calls == 3                  # answer, reserve + re-read, after the step
    assert g.passed
    assert g.detail["reservation"]["taken_while_reserving"] == {uids[3]: "llm/coder-llm-0"}
    assert _narrowed(r.calls[0]) == ["0", "1", "2", "4", "5", "6", "7"]   # GPU 3 never loaded
    # while the GEMM ran, the reservation named exactly the GPUs under test
    assert uids[3] not in seen_reservation[0]["device_uids"] and len(seen_reservation[0]["device_uids"]) == 7
    assert not (tmp_path / "m" / IN_TEST).exists()          # released afterwards
    assert uids[3] not in g.detail["validated_devices"]


def test_plugin_gates_on_validation_and_reports_reserved_gpus_unhealthy(tmp_path):
    """First boot: the plugin advertises every GPU Unhealthy until the validator's load steps passed
    on it; during a load step the GPUs under test are Unhealthy and the plugin acks the
    reservation; after the pass exactly the validated GPUs turn Healthy."""
    import threading

    from k8s_nvidia_gpus_amd.operator import deviceplugin_api as api
    from k8s_nvidia_gpus_amd.operator.device_plugin import AmdGpuDevicePlugin, ValidationGate

    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path, ", rccl: false, reserveAckSeconds: 5")
    uids = _uids(root)
    marker = tmp_path / "m"
    marker.mkdir()
    gate = ValidationGate(str(marker), root=str(root), gate=True)
    plugin = AmdGpuDevicePlugin(cfg, root=str(root), kubelet_dir=str(tmp_path / "kd"), pause_marker=None,
                                dev_prefix=str(root / "dev"), gate=gate, ecc_fn=lambda d: 0)
    health = lambda: {d.ID: d.health for d in plugin.list_response().devices}  # noqa: E731
    assert set(health().values()) == {api.UNHEALTHY}        # nothing validated this boot yet
    stop = threading.Event()
    loop = threading.Thread(target=plugin.run, kwargs={"poll": 0.02, "stop_event": stop,
                                                        "health_interval": 60}, daemon=True)
    during = []

    class R(Runner):
        def __call__(self, argv, timeout):
            during.append(health())
            return super().__call__(argv, timeout)

    busy = {("llm", "coder-llm-0"): [("amd.com/gpu", [uids[0]])]}
    r = R({"amd-gemm-validator": (0, _gemm_log(7, 1500.0))})
    loop.start()
    try:
        with FakePodResources(sock, busy):
            v = Validator(cfg, str(marker), bin_dir="/x", runner=r, root=str(root))
            g = v.run_step("gemm")
        time.sleep(0.2)
        after = health()
    finally:
        stop.set()
        loop.join(5)
    assert g.passed and g.detail["reservation"]["acked"]
    assert all(during[0][u] == api.UNHEALTHY for u in uids[1:])
    doc = json.loads((marker / VALIDATED_DEVICES).read_text())
    assert doc["boot_id"] == "boot-1" and sorted(doc["device_uids"]) == sorted(uids[1:])
    assert after[uids[0]] == api.UNHEALTHY                   # held by a pod, never validated
    assert all(after[u] == api.HEALTHY for u in uids[1:])
    # a reboot (new boot id) closes the gate again
    (root / "proc/sys/kernel/random/boot_id").write_text("boot-2\n")
    plugin.refresh()
    assert set(health().values()) == {api.UNHEALTHY}
    # a reservation past its expiry (a crashed validator) is ignored
    (root / "proc/sys/kernel/random/boot_id").write_text("boot-1\n")
    (marker / IN_TEST).write_text(json.dumps({"nonce": "x", "device_uids": uids, "expires": time.time() - 1}))
    plugin.refresh()
    assert all(health()[u] == api.HEALTHY for u in uids[1:])


def test_hold_loop_reruns_the_chain_when_a_deferred_node_gets_a_free_gpu(tmp_path, monkeypatch):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path, ", retryDeferredSeconds: 0.01")
    uids = _uids(root)
    marker = tmp_path / "m"
    _chain_markers(marker)
    pods = {("train", f"job-{i}"): [("amd.com/gpu", [u])] for i, u in enumerate(uids)}
    kube = _Kube()
    monkeypatch.setenv("POD_NAME", "amd-gpu-validator-abc")
    monkeypatch.setenv("POD_NAMESPACE", "amd-gpu-operator")
    with FakePodResources(sock, pods):
        v = Validator(cfg, str(marker), bin_dir="/x", runner=Runner({}), root=str(root), kube=kube,
                      node_name="n1")
        for st in ("gemm", "rccl", "stress", "bandwidth"):
            v.run_step(st)
        assert v.run_step("report").detail["label"] == "deferred"
        ticks = []

        def sleep(_):
            time.sleep(0.012)                                # > retryDeferredSeconds per tick
            ticks.append(1)
            if len(ticks) == 3:                              # a job finishes: GPU 5 is free
                del pods[("train", "job-5")]
        rc = hold_loop(v, str(marker), interval=0.0, stop=lambda: len(ticks) > 10, sleep=sleep)
    assert rc == 0 and kube.deleted == [("amd-gpu-operator", "amd-gpu-validator-abc")]
    assert 3 <= len(ticks) <= 5


def test_partition_switch_invalidates_the_fingerprint(tmp_path):
    """SPX → CPX changes no boot/driver/image/config field; the agent set and partition
    mode are part of the fingerprint, so a validator restart after a switch re-runs the load steps."""
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path, ", pluginTest: false, vectorAdd: false, rccl: false")
    marker = tmp_path / "m"
    _chain_markers(marker, ("driver", "runtime"))
    with FakePodResources(sock, {}):
        r1 = Runner({"amd-gemm-validator": (0, _gemm_log(8, 1600.0))})
        v = Validator(cfg, str(marker), bin_dir="/x", runner=r1, root=str(root))
        assert v.run_step("gemm").passed and v.run_step("report").detail["full_validation"]
        fp_spx = v.fingerprint()
        # the partition manager switches every ASIC to CPX (same boot)
        import shutil

        shutil.rmtree(root / "sys")
        fake_sysfs.build_node(root, compute_partition="CPX")
        r2 = Runner({"amd-gemm-validator": (0, _gemm_log(64, 190.0, size=4096))})
        v2 = Validator(cfg, str(marker), bin_dir="/x", runner=r2, root=str(root))
        fp_cpx = v2.fingerprint()
        assert fp_cpx["boot_id"] == fp_spx["boot_id"] and fp_cpx["partition"] != fp_spx["partition"]
        assert fp_cpx["agents"] == "64" and fp_spx["agents"] == "8"
        g = v2.run_step("gemm")
        assert g.passed and "reused" not in g.detail and len(r2.calls) == 1
        assert len(g.detail["validated_devices"]) == 64


def test_unchanged_node_reuses_full_pass_and_changed_fingerprint_reruns(tmp_path):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path, ", pluginTest: false, vectorAdd: false")
    marker = tmp_path / "m"
    (marker).mkdir()
    for st in ("driver", "runtime"):
        (marker / f"{st}-ready").write_text("1\n")
    outputs = {"amd-gemm-validator": (0, _gemm_log(8, 1600.0)), "rccl-allreduce-bench": (0, RCCL_8GPU)}
    with FakePodResources(sock, {}):
        r1 = Runner(outputs)
        v = Validator(cfg, str(marker), bin_dir="/x", runner=r1, root=str(root))
        assert v.run_step("gemm").passed and v.run_step("rccl").passed
        rep = v.run_step("report")
        assert rep.passed and rep.detail["full_validation"]
        assert r1.calls and all(c[0] != "env" for c in r1.calls)   # whole node, no narrowing
        assert (marker / FINGERPRINT).exists()

        # validator pod restarted (image unchanged, same boot): nothing is loaded again
        r2 = Runner(outputs)
        v2 = Validator(cfg, str(marker), bin_dir="/x", runner=r2, root=str(root))
        g = v2.run_step("gemm")
        assert g.passed and "unchanged" in g.detail["reused"] and r2.calls == []
        assert g.detail["previous"]["aggregate_tflops"] == pytest.approx(12800.0)
        assert v2.run_step("report").detail["full_validation"]

        # reboot (new boot id) or a new operator image: a full run again
        (root / "proc/sys/kernel/random/boot_id").write_text("boot-2\n")
        r3 = Runner(outputs)
        v3 = Validator(cfg, str(marker), bin_dir="/x", runner=r3, root=str(root))
        g3 = v3.run_step("gemm")
        assert g3.passed and "reused" not in g3.detail and len(r3.calls) == 1
        os.environ["VALIDATOR_IMAGE_ID"] = "sha256:new"
        try:
            r4 = Runner(outputs)
            g4 = Validator(cfg, str(marker), bin_dir="/x", runner=r4, root=str(root)).run_step("gemm")
            assert "reused" not in g4.detail and len(r4.calls) == 1
        finally:
            del os.environ["VALIDATOR_IMAGE_ID"]


def test_cpx_validates_with_per_partition_floors(tmp_path):
    """64 CPX agents: the GEMM is sized for one 32-CU partition with a floor of 1/8 of the
    whole-GPU floor (a partition's ~190 TFLOPS passes; 90 fails), HBM floor scaled the same way,
    xGMI pair copies skipped, RCCL over one agent per ASIC."""
    root = _node(tmp_path, "CPX")
    cfg, sock = _cfg(tmp_path, ", bandwidth: true, hbmMinGBps: 4000")
    assert len(_uids(root)) == 64
    bw = "\n".join([_pt("hbm-copy", i, 700.0) for i in range(64)]
                   + [_pt("pcie-h2d", i, 50.0) for i in range(64)]
                   + [_pt("pcie-d2h", i, 50.0) for i in range(64)] + ["Test PASSED", "Done", ""])
    r = Runner({"amd-gemm-validator": (0, _gemm_log(64, 190.0, size=4096)),
                "amd-proftester": (0, bw), "rccl-allreduce-bench": (0, RCCL_8GPU)})
    with FakePodResources(sock, {}):
        v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root))
        g = v.run_step("gemm")
        b = v.run_step("bandwidth")
        rc = v.run_step("rccl")
    assert g.passed, g.reason
    assert g.detail["partition_split"] == 8 and g.detail["floor_tflops"] == pytest.approx(112.5)
    assert g.detail["size"] == 4096 and "--size" in r.calls[0] and r.calls[0][r.calls[0].index("--size") + 1] == "4096"
    assert b.passed, b.reason
    assert b.detail["floors_gbps"]["hbm-copy"] == pytest.approx(500.0)
    assert "xgmi" not in b.detail["floors_gbps"] and "xgmi_skipped" in b.detail
    assert "xgmi" not in r.calls[1][r.calls[1].index("-t") + 1]
    # RCCL: partition 0 of each ASIC (ROCr indices 0, 8, 16, ...)
    assert rc.passed and _narrowed(r.calls[2]) == [str(8 * a) for a in range(8)]

    slow = Runner({"amd-gemm-validator": (0, _gemm_log(64, 90.0, size=4096))})
    with FakePodResources(sock, {}):
        g2 = Validator(cfg, str(tmp_path / "m2"), bin_dir="/x", runner=slow, root=str(root)).run_step("gemm")
    assert not g2.passed and "below 112.5" in g2.reason


def test_index_device_ids_map_through_the_plugin_file(tmp_path):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path)
    cfg.raw["deviceIdStrategy"] = "index"
    uids = _uids(root)
    idmap = tmp_path / "ids.json"
    idmap.write_text(json.dumps({str(i): u for i, u in enumerate(uids)}))
    r = Runner({"amd-gemm-validator": (0, _gemm_log(7, 1500.0))})
    with FakePodResources(sock, {("a", "p"): [("amd.com/gpu", ["3"])]}):
        v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root),
                      device_id_map=str(idmap))
        assert v.run_step("gemm").passed
    assert _narrowed(r.calls[0]) == ["0", "1", "2", "4", "5", "6", "7"]
    # without the plugin's map an index ID cannot be placed: fail closed
    r2 = Runner({})
    with FakePodResources(sock, {("a", "p"): [("amd.com/gpu", ["3"])]}):
        res = Validator(cfg, str(tmp_path / "m3"), bin_dir="/x", runner=r2, root=str(root),
                        device_id_map=str(tmp_path / "missing.json")).run_step("gemm")
    assert not res.passed and "cannot map" in res.reason and r2.calls == []


def test_gate_opens_on_the_gemm_and_a_pending_pod_gets_its_gpu_before_rccl(tmp_path):
    """on an 8-agent node the plugin advertises the GPUs Healthy as soon as the
    per-device GEMM passed; the node-wide RCCL step waits ``gateGraceSeconds`` after the gate
    opened, a pod pending for the node is allocated GPU 0 in that window, and RCCL then reserves
    and loads only the other 7 (GPU 0 never appears in its reservation)."""
    import threading

    from k8s_nvidia_gpus_amd.operator import deviceplugin_api as api
    from k8s_nvidia_gpus_amd.operator.device_plugin import AmdGpuDevicePlugin, ValidationGate

    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path, ", rccl: true, reserveAckSeconds: 5, gateGraceSeconds: 3")
    uids = _uids(root)
    marker = tmp_path / "m"
    _chain_markers(marker, ("driver", "runtime", "vectoradd"))
    gate = ValidationGate(str(marker), root=str(root), gate=True)
    plugin = AmdGpuDevicePlugin(cfg, root=str(root), kubelet_dir=str(tmp_path / "kd"),
                                pause_marker=None, dev_prefix=str(root / "dev"), gate=gate,
                                ecc_fn=lambda d: 0)
    health = lambda: {d.ID: d.health for d in plugin.list_response().devices}  # noqa: E731
    stop = threading.Event()
    loop = threading.Thread(target=plugin.run, kwargs={"poll": 0.02, "stop_event": stop,
                                                        "health_interval": 60}, daemon=True)
    pods = {}
    seen = {}
    reservations = []

    class R(Runner):
        def __call__(self, argv, timeout):
            reservations.append(json.loads((marker / IN_TEST).read_text())["device_uids"])
            return super().__call__(argv, timeout)

    def grace_sleep(secs):
        # the grace window: the gate is open; kubelet hands GPU 0 to the pending pod
        time.sleep(0.2)
        seen["health_in_grace"] = health()
        seen["grace"] = secs
        pods[("llm", "coder-llm-0")] = [("amd.com/gpu", [uids[0]])]

    r = R({"amd-gemm-validator": (0, _gemm_log(8, 1500.0)), "rccl-allreduce-bench": (0, RCCL_8GPU)})
    loop.start()
    try:
        with FakePodResources(sock, pods):
            v = Validator(cfg, str(marker), bin_dir="/x", runner=r, root=str(root), sleep=grace_sleep)
            assert set(health().values()) == {api.UNHEALTHY}          # gate closed at boot
            g = v.run_step("gemm")
            assert g.passed and sorted(g.detail["validated_devices"]) == sorted(uids)
            rc = v.run_step("rccl")
    finally:
        stop.set()
        loop.join(5)
    assert all(seen["health_in_grace"][u] == api.HEALTHY for u in uids)   # allocatable pre-RCCL
    assert 0 < seen["grace"] <= 3
    assert rc.passed and rc.detail["reservation"]["gate_grace_waited_s"] > 0
    assert uids[0] not in reservations[-1] and len(reservations[-1]) == 7
    assert _narrowed(r.calls[-1]) == [str(i) for i in range(1, 8)]      # RCCL never touched GPU 0
    doc = json.loads((marker / VALIDATED_DEVICES).read_text())
    assert sorted(doc["device_uids"]) == sorted(uids) and doc["opened"] <= time.time()


def test_a_serving_plugin_that_never_acks_defers_the_load_step(tmp_path):
    """the plugin's registration socket accepts connections but the reservation
    is never acked (a plugin stuck in an amd-smi call) → the step is deferred and no GPU is loaded;
    without any plugin socket the step proceeds after reserveAckSeconds."""
    import socket as socketlib

    root = _node(tmp_path)
    psock = tmp_path / "dp" / "amd-gpu.sock"
    psock.parent.mkdir()
    cfg, sock = _cfg(tmp_path, f", rccl: false, reserveAckSeconds: 0.3, pluginSocket: {psock}")
    srv = socketlib.socket(socketlib.AF_UNIX, socketlib.SOCK_STREAM)
    srv.bind(str(psock))
    srv.listen(8)
    r = Runner({"amd-gemm-validator": (0, _gemm_log(8, 1500.0))})
    try:
        with FakePodResources(sock, {}):
            v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root))
            g = v.run_step("gemm")
    finally:
        srv.close()
    assert g.deferred and not g.passed and "did not ack" in g.reason
    assert g.detail["reservation"]["unacked_live_plugin"] and r.calls == []
    assert not (tmp_path / "m" / IN_TEST).exists()          # the reservation was withdrawn
    psock.unlink()                                          # no plugin at all: proceed
    with FakePodResources(sock, {}):
        g = Validator(cfg, str(tmp_path / "m2"), bin_dir="/x", runner=r, root=str(root)).run_step("gemm")
    assert g.passed and not g.detail["reservation"]["acked"] and r.calls


def test_partition_started_during_the_reservation_defers_the_step(tmp_path):
    """the pause marker appears after the first check (the partition manager drained
    while the validator reserved): the step is deferred after the reservation, nothing loads."""
    from k8s_nvidia_gpus_amd.operator import pause as pause_mod

    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path, ", rccl: false, reserveAckSeconds: 0.2")
    pause = tmp_path / "pause"

    class Racing(FakePodResources):
        def List(self, request, context):  # noqa: N802
            if self.calls == 1:                       # the re-read after the reservation
                pause_mod.start_pause(str(pause), str(tmp_path / "acks"))
            return super().List(request, context)

    r = Runner({"amd-gemm-validator": (0, _gemm_log(8, 1500.0))})
    with Racing(sock, {}):
        v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root),
                      pause_marker=str(pause))
        g = v.run_step("gemm")
    assert g.deferred and "partition change started" in g.reason and r.calls == []
    assert v.run_step("vectoradd").deferred


def test_a_pod_admitted_during_the_step_is_recorded(tmp_path):
    """The residual window: a pod kubelet admitted after the post-reservation re-read shows up in
    the step result's allocated_during_step (PodResources is read once more after the load)."""
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path, ", rccl: false, reserveAckSeconds: 0.1")
    uids = _uids(root)
    pods = {}

    class R(Runner):
        def __call__(self, argv, timeout):
            pods[("late", "pod-0")] = [("amd.com/gpu", [uids[4]])]      # admitted mid-step
            return super().__call__(argv, timeout)

    with FakePodResources(sock, pods):
        g = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", root=str(root),
                      runner=R({"amd-gemm-validator": (0, _gemm_log(8, 1500.0))})).run_step("gemm")
    assert g.passed and g.detail["allocated_during_step"] == {uids[4]: "late/pod-0"}
