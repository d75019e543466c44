"""Validator GPU scope: GPUs that kubelet allocated to pods are never loaded, a fully allocated node
defers the load steps without failing, an unchanged node re-uses its last full pass, and
compute-partitioned (CPX) nodes validate against per-partition floors.

kubelet's PodResources API is served by tests/fakes/podresources.py over a real unix socket; the
node is the fake MI355X sysfs tree (tests/fakes/sysfs.py) with 8 ASICs (64 CPX agents)."""
import json
import os

import pytest

from fakes import sysfs as fake_sysfs
from fakes.podresources import FakePodResources
from k8s_nvidia_gpus_amd.operator.config import load_config
from k8s_nvidia_gpus_amd.operator.validator import FINGERPRINT, Validator
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
            f"podResourcesSocket: {sock}, rccl: true, bandwidth: false{extra}}}\n")
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
    # a partial validation never becomes the node's fingerprint
    v.run_step("report")
    assert not os.path.exists(tmp_path / "m" / FINGERPRINT)


def test_fully_allocated_node_defers_without_failure(tmp_path):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path)
    pods = {("train", f"job-{i}"): [("amd.com/gpu", [u])] for i, u in enumerate(_uids(root))}
    r = Runner({})
    with FakePodResources(sock, pods):
        v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root))
        for step in ("gemm", "rccl", "stress", "bandwidth"):
            res = v.run_step(step)
            assert res.passed, step
    assert r.calls == []                                   # no GPU was touched
    d = json.loads((tmp_path / "m/gemm.json").read_text())
    assert "allocated" in d["deferred"] and d["gpu_scope"]["validated"] == []
    assert (tmp_path / "m/gemm-ready").exists()


def test_unreadable_kubelet_answer_fails_closed(tmp_path):
    root = _node(tmp_path)
    cfg, sock = _cfg(tmp_path)
    os.makedirs(os.path.dirname(sock))
    with open(sock, "w") as f:                              # a socket path nobody serves
        f.write("")
    r = Runner({})
    v = Validator(cfg, str(tmp_path / "m"), bin_dir="/x", runner=r, root=str(root))
    res = v.run_step("gemm")
    assert res.passed and "PodResources" in res.detail["deferred"] and r.calls == []


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
        assert g.passed and "unchanged" in g.detail["deferred"] and r2.calls == []
        assert g.detail["previous"]["aggregate_tflops"] == pytest.approx(12800.0)
        assert v2.run_step("report").detail["full_validation"]

        # reboot (new boot id) or a new operator image: a full run again
        (root / "proc/sys/kernel/random/boot_id").write_text("boot-2\n")
        r3 = Runner(outputs)
        v3 = Validator(cfg, str(marker), bin_dir="/x", runner=r3, root=str(root))
        g3 = v3.run_step("gemm")
        assert g3.passed and "deferred" not in g3.detail and len(r3.calls) == 1
        os.environ["VALIDATOR_IMAGE_ID"] = "sha256:new"
        try:
            r4 = Runner(outputs)
            g4 = Validator(cfg, str(marker), bin_dir="/x", runner=r4, root=str(root)).run_step("gemm")
            assert "deferred" not in g4.detail and len(r4.calls) == 1
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
    assert res.passed and "cannot map" in res.detail["deferred"] and r2.calls == []
