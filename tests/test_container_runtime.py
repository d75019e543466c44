"""amd-container-runtime (C++ OCI runtime shim) against fabricated OCI bundles, plus ASan/UBSan
builds of the host-side native tools (sanitizers on host code)."""
import json
import os
import shutil
import stat
import subprocess
from pathlib import Path

import pytest

from fakes import sysfs as fake_sysfs
from k8s_nvidia_gpus_amd.ops import build as B

REPO = Path(__file__).resolve().parent.parent
pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def _spec(minors=None, privileged=False, extra_devices=()):
    spec = {
        "ociVersion": "1.2.0",
        "process": {"args": ["/bin/sh"], "env": ["AMD_VISIBLE_DEVICES=all", "PATH=/usr/bin"],
                    "capabilities": {"bounding": ["CAP_CHOWN"] + (["CAP_SYS_ADMIN"] if privileged else [])}},
        "root": {"path": "rootfs"},
        "annotations": {"io.kubernetes.cri.container-type": "container"},
        "linux": {
            "resources": {"devices": [{"allow": False, "access": "rwm"}],
                          "memory": {"limit": 17179869184}},
            "devices": [{"path": p, "type": "c", "major": 226, "minor": m, "fileMode": 438}
                        for p, m in extra_devices],
        },
    }
    if minors is not None:
        spec["annotations"]["amd.com/gpu.render-minors"] = minors
    return spec


@pytest.fixture(scope="module")
def rt_bin():
    B.build_native(only=["amd-container-runtime"])
    return str(B.NATIVE_BIN / "amd-container-runtime")


@pytest.fixture
def env(tmp_path):
    root = fake_sysfs.build_node(tmp_path / "node")
    log = tmp_path / "rt.log"
    fake_runc = tmp_path / "runc"
    fake_runc.write_text("#!/bin/sh\necho \"$0 $*\" > \"$(dirname \"$0\")/runc.args\"\n")
    fake_runc.chmod(0o755)
    cfg = tmp_path / "config.json"
    cfg.write_text(json.dumps({"runtime": str(fake_runc), "fallback_runtimes": [], "log": str(log)}))
    e = dict(os.environ, AMD_CONTAINER_RUNTIME_CONFIG=str(cfg),
             AMD_CONTAINER_RUNTIME_DEV_ROOT=str(root))
    return e, tmp_path


def _bundle(tmp_path, spec, name="b"):
    b = tmp_path / name
    b.mkdir()
    (b / "config.json").write_text(json.dumps(spec))
    return b


def test_version(rt_bin):
    out = subprocess.run([rt_bin, "--version"], capture_output=True, text=True, check=True).stdout
    assert "amd-container-runtime" in out


def test_create_injects_exactly_the_allocated_nodes_and_execs_runc(rt_bin, env):
    e, tmp = env
    b = _bundle(tmp, _spec("136,144", extra_devices=[("/dev/dri/renderD128", 128),
                                                     ("/dev/dri/card0", 0)]))
    argv = [rt_bin, "--root", "/run/containerd/runc/k8s.io", "--log", "/x.log", "--log-format",
            "json", "create", "--bundle", str(b), "--pid-file", "/p", "ctr-1"]
    r = subprocess.run(argv, capture_output=True, text=True, env=e)
    assert r.returncode == 0, r.stderr
    spec = json.loads((b / "config.json").read_text())
    devs = {d["path"]: d for d in spec["linux"]["devices"]}
    assert set(devs) == {"/dev/kfd", "/dev/dri/renderD136", "/dev/dri/renderD144"}
    assert devs["/dev/dri/renderD136"]["major"] == 226 and devs["/dev/dri/renderD136"]["minor"] == 136
    assert devs["/dev/kfd"]["fileMode"] == 438
    rules = spec["linux"]["resources"]["devices"]
    assert rules[0] == {"allow": False, "access": "rwm"}  # deny-all kept first
    allowed = {(r["major"], r["minor"]) for r in rules[1:]}
    assert allowed == {(241, 0), (226, 136), (226, 144)}
    # everything else passed through untouched (64-bit number kept as its literal)
    assert spec["linux"]["resources"]["memory"]["limit"] == 17179869184
    assert spec["process"]["env"][0] == "AMD_VISIBLE_DEVICES=all"  # env is irrelevant to isolation
    # runc got the identical argv
    got = (tmp / "runc.args").read_text().split()
    assert got[1:] == argv[1:]
    assert "injected GPU devices" in (tmp / "rt.log").read_text()


def test_no_annotation_leaves_spec_untouched(rt_bin, env):
    e, tmp = env
    spec = _spec(None, extra_devices=[("/dev/dri/renderD128", 128)])
    b = _bundle(tmp, spec)
    before = (b / "config.json").read_text()
    r = subprocess.run([rt_bin, "create", "-b", str(b), "c"], capture_output=True, text=True, env=e)
    assert r.returncode == 0, r.stderr
    assert (b / "config.json").read_text() == before


def test_privileged_keeps_other_device_nodes(rt_bin, env):
    e, tmp = env
    b = _bundle(tmp, _spec("128", privileged=True, extra_devices=[("/dev/dri/renderD136", 136)]))
    out = subprocess.run([rt_bin, "--amd-edit-bundle", str(b)], capture_output=True, text=True,
                         env=e, check=True).stdout
    paths = [d["path"] for d in json.loads(out)["linux"]["devices"]]
    assert "/dev/dri/renderD136" in paths and "/dev/dri/renderD128" in paths


@pytest.mark.parametrize("minors,msg", [("12x", "bad render minor"), ("", "empty"),
                                        ("200", "renderD200")])
def test_bad_allocation_fails_create(rt_bin, env, minors, msg):
    e, tmp = env
    b = _bundle(tmp, _spec(minors))
    r = subprocess.run([rt_bin, "create", "--bundle=" + str(b), "c"], capture_output=True,
                       text=True, env=e)
    assert r.returncode == 1 and msg in r.stderr
    assert not (tmp / "runc.args").exists()  # runc never ran


def test_non_create_commands_pass_through(rt_bin, env):
    e, tmp = env
    r = subprocess.run([rt_bin, "--root", "/r", "state", "ctr-1"], capture_output=True, text=True, env=e)
    assert r.returncode == 0
    assert (tmp / "runc.args").read_text().split()[1:] == ["--root", "/r", "state", "ctr-1"]


def test_unicode_and_escapes_round_trip(rt_bin, env):
    e, tmp = env
    spec = _spec("128")
    spec["process"]["args"] = ["/bin/echo", "tab\there", "quote\"", "ünïcødé ✓", "\u0001"]
    b = _bundle(tmp, spec)
    out = subprocess.run([rt_bin, "--amd-edit-bundle", str(b)], capture_output=True, text=True,
                         env=e, check=True).stdout
    assert json.loads(out)["process"]["args"] == spec["process"]["args"]


@pytest.mark.slow
def test_host_tools_clean_under_asan_ubsan(tmp_path):
    """Build kfd-probe + amd-container-runtime with -fsanitize=address,undefined and run them."""
    inc = [f"-I{REPO / 'native/include'}"]
    flags = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
             "-fno-sanitize-recover=all"]
    probe = tmp_path / "kfd-probe-asan"
    rtb = tmp_path / "rt-asan"
    subprocess.run(["g++", *flags, *inc, str(REPO / "native/src/kfd_probe.cpp"),
                    str(REPO / "native/src/kfd_topology.cpp"), "-o", str(probe)], check=True)
    subprocess.run(["g++", *flags, *inc, str(REPO / "native/src/amd_container_runtime.cpp"), "-o",
                    str(rtb)], check=True)
    root = fake_sysfs.build_node(tmp_path / "n", compute_partition="CPX")
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    r = subprocess.run([str(probe), "--sysfs-root", str(root / "sys/class/kfd/kfd/topology"),
                        "--dev-root", str(root / "dev"), "--no-open", "--expect-gpus", "64"],
                       capture_output=True, text=True, env=e)
    assert r.returncode == 0, r.stderr
    b = tmp_path / "b"
    b.mkdir()
    (b / "config.json").write_text(json.dumps(_spec("128,129,130")))
    e["AMD_CONTAINER_RUNTIME_DEV_ROOT"] = str(root)
    e["AMD_CONTAINER_RUNTIME_CONFIG"] = "/nonexistent"
    r = subprocess.run([str(rtb), "--amd-edit-bundle", str(b)], capture_output=True, text=True, env=e)
    assert r.returncode == 0, r.stderr
    (b / "config.json").write_text('{"annotations": {"amd.com/gpu.render-minors": "1"}, "bad": [1,2,')
    r = subprocess.run([str(rtb), "--amd-edit-bundle", str(b)], capture_output=True, text=True, env=e)
    assert r.returncode == 1 and "JSON" in r.stderr and "AddressSanitizer" not in r.stderr
