"""amd.com/gpu device plugin against a fake MI355X sysfs tree and a fake kubelet (CPU-only)."""
import json
import os
import tempfile
import threading
import time

import pytest

from fakes import sysfs as fake_sysfs
from fakes.kubelet import FakeKubelet
from k8s_nvidia_gpus_amd.operator import deviceplugin_api as api
from k8s_nvidia_gpus_amd.operator.config import load_config
from k8s_nvidia_gpus_amd.operator.device_plugin import (ANNOT_DEVICE_IDS, ANNOT_RENDER_MINORS,
                                                        AmdGpuDevicePlugin, PresenceHealth,
                                                        preferred_allocation)
from k8s_nvidia_gpus_amd.utils.topology import read_topology


@pytest.fixture
def node(tmp_path):
    return fake_sysfs.build_node(tmp_path / "root")


@pytest.fixture
def sockdir():
    # unix socket paths must stay short (108 bytes)
    d = tempfile.mkdtemp(prefix="dp", dir="/tmp")
    yield d
    for n in os.listdir(d):
        try:
            os.unlink(os.path.join(d, n))
        except OSError:
            pass
    os.rmdir(d)


def make_plugin(root, sockdir, cfg_text="", **kw):
    cfg = load_config(text=cfg_text)
    return AmdGpuDevicePlugin(cfg, root=str(root), kubelet_dir=sockdir,
                              pause_marker=os.path.join(str(root), "pause"),
                              dev_prefix=os.path.join(str(root), "dev"), **kw)


def test_enumerates_eight_mi355x(node, sockdir):
    p = make_plugin(node, sockdir)
    resp = p.list_response()
    assert len(resp.devices) == 8
    assert all(d.health == api.HEALTHY for d in resp.devices)
    ids = [d.ID for d in resp.devices]
    assert len(set(ids)) == 8 and all(i.startswith("GPU-") for i in ids)
    numa = sorted(d.topology.nodes[0].ID for d in resp.devices)
    assert numa == [0, 0, 0, 0, 1, 1, 1, 1]


def test_cpx_advertises_64_partitions(tmp_path, sockdir):
    root = fake_sysfs.build_node(tmp_path / "r", compute_partition="CPX")
    p = make_plugin(root, sockdir)
    resp = p.list_response()
    assert len(resp.devices) == 64
    assert len({d.ID for d in resp.devices}) == 64
    t = read_topology(str(root), 90500)
    assert {g.cu_count for g in t.gpus} == {32}
    assert {g.compute_partition for g in t.gpus} == {"CPX"}


def test_allocate_returns_device_specs_not_env_visibility(node, sockdir):
    p = make_plugin(node, sockdir)
    ids = [d.ID for d in p.list_response().devices][:2]
    req = api.AllocateRequest()
    req.container_requests.add(devices_ids=ids)
    resp = p.Allocate(req, None)
    (c,) = resp.container_responses
    paths = [d.container_path for d in c.devices]
    assert paths[0] == "/dev/kfd"
    renders = [x for x in paths if x.startswith("/dev/dri/renderD")]
    assert len(renders) == 2
    for d in c.devices:
        assert d.permissions == "rw"
        assert os.path.exists(d.host_path)
    assert c.annotations[ANNOT_RENDER_MINORS] == ",".join(r.split("renderD")[1] for r in renders)
    assert c.annotations[ANNOT_DEVICE_IDS] == ",".join(ids)
    for k in c.envs:
        assert "VISIBLE" not in k  # isolation never rides on a visibility env var
    assert not c.cdi_devices


def test_allocate_cdi_mode(node, sockdir):
    p = make_plugin(node, sockdir, "allocation: {mode: cdi}")
    ids = [d.ID for d in p.list_response().devices][:1]
    req = api.AllocateRequest()
    req.container_requests.add(devices_ids=ids)
    (c,) = p.Allocate(req, None).container_responses
    assert [x.name for x in c.cdi_devices] == [f"amd.com/gpu={ids[0]}"]
    assert not c.devices


def test_allocate_unknown_id_rejected(node, sockdir):
    p = make_plugin(node, sockdir)
    req = api.AllocateRequest()
    req.container_requests.add(devices_ids=["GPU-doesnotexist"])
    with pytest.raises(KeyError):
        p.Allocate(req, None)


def test_index_id_strategy(node, sockdir):
    p = make_plugin(node, sockdir, "deviceIdStrategy: index")
    assert [d.ID for d in p.list_response().devices] == [str(i) for i in range(8)]


def test_index_ids_stay_with_their_gpu_when_one_disappears(tmp_path, sockdir):
    """an index already handed to kubelet must keep naming the same physical GPU."""
    root = fake_sysfs.build_node(tmp_path / "r")
    p = make_plugin(root, sockdir, "deviceIdStrategy: index")
    before = {i: d.device_uid for i, d in p._id_map().items()}
    victim = before["0"]
    bdfs = [g["bdf"] for g in fake_sysfs.LAYOUT["gpus"]]
    gpu = next(g for g in read_topology(str(root), 90500).gpus if g.device_uid == victim)
    fake_sysfs.remove_gpu(root, bdfs.index(gpu.pci_bdf))
    assert p.refresh() is True
    after = {i: d.device_uid for i, d in p._id_map().items()}
    assert after == before
    health = {d.ID: d.health for d in p.list_response().devices}
    assert health["0"] == api.UNHEALTHY and list(health.values()).count(api.HEALTHY) == 7
    # allocation by index still resolves to the same render node as before the removal
    resp = p.container_response(["5"])
    assert resp.annotations[ANNOT_DEVICE_IDS] == before["5"]


def _pref(p, avail, must, size):
    req = api.PreferredAllocationRequest()
    req.container_requests.add(available_deviceIDs=avail, must_include_deviceIDs=must, allocation_size=size)
    return list(p.GetPreferredAllocation(req, None).container_responses[0].deviceIDs)


def test_preferred_allocation_packs_numa(node, sockdir):
    p = make_plugin(node, sockdir)
    devs = p.list_response().devices
    numa = {d.ID: d.topology.nodes[0].ID for d in devs}
    ids = [d.ID for d in devs]
    got = _pref(p, ids, [], 4)
    assert len(got) == 4 and len({numa[i] for i in got}) == 1
    # best fit: with socket 0 half used, a 2-GPU request goes to socket 0's remaining pair
    s0 = [i for i in ids if numa[i] == 0]
    avail = [i for i in ids if i not in s0[:2]]
    got2 = _pref(p, avail, [], 2)
    assert {numa[i] for i in got2} == {0}
    # must_include is honoured and the rest follows its socket
    s1 = [i for i in ids if numa[i] == 1]
    got3 = _pref(p, ids, [s1[0]], 3)
    assert got3[0] == s1[0] and {numa[i] for i in got3} == {1}


def test_preferred_allocation_packs_partitions_on_one_asic(tmp_path, sockdir):
    root = fake_sysfs.build_node(tmp_path / "r", compute_partition="CPX")
    t = read_topology(str(root), 90500)
    by_asic = {}
    for g in t.gpus:
        by_asic.setdefault(g.unique_id, []).append(g)
    # fragment: ASIC A has 3 free partitions, ASIC B has 8
    a, b = list(by_asic.values())[:2]
    avail = a[:3] + b
    got = preferred_allocation(avail, [], 3)
    assert len({g.unique_id for g in got}) == 1 and got[0].unique_id == a[0].unique_id
    got8 = preferred_allocation(avail, [], 8)
    assert {g.unique_id for g in got8} == {b[0].unique_id}


def test_health_device_disappears(tmp_path, sockdir):
    root = fake_sysfs.build_node(tmp_path / "r")
    p = make_plugin(root, sockdir)
    assert p.refresh() is False
    victim = read_topology(str(root), 90500).gpus[0]
    fake_sysfs.remove_gpu(root, [g["bdf"] for g in fake_sysfs.LAYOUT["gpus"]].index(victim.pci_bdf))
    assert p.refresh() is True
    h = {d.ID: d.health for d in p.list_response().devices}
    assert h[victim.device_uid] == api.UNHEALTHY
    assert sum(v == api.HEALTHY for v in h.values()) == 7


def test_health_ecc_threshold(node, sockdir):
    bad = read_topology(str(node), 90500).gpus[3].device_uid
    health = PresenceHealth(str(node), ecc_fn=lambda d: 5 if d.device_uid == bad else 0, ecc_threshold=1)
    p = make_plugin(node, sockdir, health_fn=health)
    h = {d.ID: d.health for d in p.list_response().devices}
    assert h[bad] == api.UNHEALTHY and list(h.values()).count(api.HEALTHY) == 7


def test_ecc_threshold_active_when_built_like_main(node, sockdir, monkeypatch):
    """the plugin as main() builds it (no health_fn) must apply
    health.eccUncorrectableThreshold through amd-smi, not only when a test injects an ecc_fn."""
    import sys

    from fakes.amdsmi import FakeAmdSmi

    smi = FakeAmdSmi()
    monkeypatch.setitem(sys.modules, "amdsmi", smi)
    p = make_plugin(node, sockdir, "health:\n  eccUncorrectableThreshold: 2\n")
    assert all(d.health == api.HEALTHY for d in p.list_response().devices)
    smi.ecc_uncorrectable[3] = 1            # below the threshold: still healthy
    assert p.refresh() is False
    smi.ecc_uncorrectable[3] = 2            # reaches it: that GPU (and only it) goes Unhealthy
    assert p.refresh() is True
    bdf3 = smi.amdsmi_get_gpu_device_bdf(3)
    bad = next(g.device_uid for g in read_topology(str(node), 90500).gpus if g.pci_bdf == bdf3)
    h = {d.ID: d.health for d in p.list_response().devices}
    assert h[bad] == api.UNHEALTHY and list(h.values()).count(api.HEALTHY) == 7


def test_ecc_disabled_without_amdsmi_is_logged(node, sockdir, monkeypatch, caplog):
    import sys

    monkeypatch.setitem(sys.modules, "amdsmi", None)   # import fails like on a node without it
    with caplog.at_level("WARNING", logger="amd-device-plugin"):
        p = make_plugin(node, sockdir)
    assert p.health_fn.ecc_fn is None
    assert any("uncorrectable-ECC health check" in r.getMessage() for r in caplog.records)


def test_pause_marker_hides_devices(node, sockdir):
    p = make_plugin(node, sockdir)
    open(os.path.join(str(node), "pause"), "w").close()
    assert p.refresh()
    assert len(p.list_response().devices) == 0
    os.unlink(os.path.join(str(node), "pause"))
    assert p.refresh()
    assert len(p.list_response().devices) == 8


def test_grpc_register_listandwatch_allocate_and_kubelet_restart(node, sockdir):
    kubelet = FakeKubelet(sockdir).start()
    p = make_plugin(node, sockdir)
    stop = threading.Event()
    t = threading.Thread(target=p.run, kwargs=dict(health_interval=0.2, poll=0.05, stop_event=stop),
                         daemon=True)
    t.start()
    try:
        assert kubelet.registered.wait(10)
        reg = kubelet.registrations[-1]
        assert reg.resource_name == "amd.com/gpu" and reg.version == "v1beta1"
        assert reg.options.get_preferred_allocation_available
        ch, stub = kubelet.plugin_stub()
        opts = stub.GetDevicePluginOptions(api.Empty(), timeout=5)
        assert opts.get_preferred_allocation_available and not opts.pre_start_required
        stream = stub.ListAndWatch(api.Empty(), timeout=20)
        first = next(stream)
        assert len(first.devices) == 8
        # a device fails -> the stream pushes an update with it Unhealthy
        fake_sysfs.remove_gpu(node, 0)
        second = next(stream)
        assert sum(d.health == api.UNHEALTHY for d in second.devices) == 1
        req = api.AllocateRequest()
        req.container_requests.add(devices_ids=[first.devices[1].ID])
        resp = stub.Allocate(req, timeout=5)
        assert len(resp.container_responses[0].devices) == 2
        stream.cancel()
        ch.close()
        # kubelet restart: sockets wiped, plugin must re-serve and re-register
        n = len(kubelet.registrations)
        kubelet.restart()
        deadline = time.time() + 10
        while len(kubelet.registrations) <= n and time.time() < deadline:
            time.sleep(0.05)
        assert len(kubelet.registrations) > n
        ch2, stub2 = kubelet.plugin_stub()
        assert len(next(stub2.ListAndWatch(api.Empty(), timeout=10)).devices) == 8
        ch2.close()
    finally:
        stop.set()
        t.join(10)
        kubelet.stop()


def test_index_id_map_file_for_the_validator(tmp_path, sockdir):
    """The plugin publishes {kubelet ID: device_uid}; the validator maps PodResources answers with it."""
    from k8s_nvidia_gpus_amd.operator.config import load_config
    from k8s_nvidia_gpus_amd.operator.device_plugin import AmdGpuDevicePlugin

    root = fake_sysfs.build_node(tmp_path / "r")
    path = tmp_path / "run/device-plugin/ids.json"
    cfg = load_config(text="deviceIdStrategy: index\n")
    p = AmdGpuDevicePlugin(cfg, root=str(root), kubelet_dir=str(sockdir), pause_marker=None,
                           health_fn=lambda devs: {d.device_uid: api.HEALTHY for d in devs},
                           id_map_path=str(path))
    m = json.loads(path.read_text())
    assert m == {i: d.device_uid for i, d in p._id_map().items()} and set(m) == {str(i) for i in range(8)}
