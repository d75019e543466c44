"""ComfyUI-compatible Wan2.1 server (k8s_nvidia_gpus_amd/models/wan/server.py) on CPU with a
miniature random-init model store: the repo's own ComfyUI client (the reference's
generate_wan_t2v.py flow: /queue → /object_info preflight → /prompt → /history polling → /view)
runs end-to-end against a live uvicorn server; validation errors, savers, queue control and
path safety are checked through FastAPI's test client."""
import os
import socket
import threading
import time

import pytest
import torch
from fastapi.testclient import TestClient

from k8s_nvidia_gpus_amd.models.comfy_client import (WAN_MODELS, ComfyClient, WanJob,
                                                     build_wan_graph, run_jobs)
from k8s_nvidia_gpus_amd.models.wan.server import (Executor, create_app, node_specs,
                                                   synthetic_store, validate_graph)


@pytest.fixture(scope="module")
def store():
    return synthetic_store("cpu", tiny=True)


@pytest.fixture
def app(store, tmp_path):
    return create_app(store, str(tmp_path / "output"), ffmpeg="")


def _job(**kw):
    base = dict(prompt="a panda riding a motorbike", width=64, height=48, frames=5, steps=2,
                formats=("webp",), seed=3)
    base.update(kw)
    return WanJob(**base)


def test_object_info_lists_reference_model_files(app):
    with TestClient(app) as c:
        info = c.get("/object_info").json()
        assert info["UNETLoader"]["input"]["required"]["unet_name"][0] == [WAN_MODELS["unet"]]
        assert info["CLIPLoader"]["input"]["required"]["clip_name"][0] == [WAN_MODELS["clip"]]
        assert info["VAELoader"]["input"]["required"]["vae_name"][0] == [WAN_MODELS["vae"]]
        assert "uni_pc" in info["KSampler"]["input"]["required"]["sampler_name"][0]
        assert c.get("/object_info/KSampler").json().keys() == {"KSampler"}
        assert c.get("/queue").json() == {"queue_running": [], "queue_pending": []}


def test_validation_errors_are_comfy_shaped(app, store):
    specs = node_specs(store)
    g = build_wan_graph(_job())
    assert validate_graph(g, specs) == (None, {})
    bad = {k: dict(v, inputs=dict(v["inputs"])) for k, v in g.items()}
    ks = next(k for k, v in bad.items() if v["class_type"] == "KSampler")
    bad[ks]["inputs"]["sampler_name"] = "dpmpp_9m"
    del bad[ks]["inputs"]["steps"]
    err, node_errors = validate_graph(bad, specs)
    assert err["type"] == "prompt_outputs_failed_validation"
    types = {e["type"] for e in node_errors[ks]["errors"]}
    assert types == {"value_not_in_list", "required_input_missing"}
    with TestClient(app) as c:
        r = c.post("/prompt", json={"prompt": bad})
        assert r.status_code == 400 and ks in r.json()["node_errors"]
        r = c.post("/prompt", json={"prompt": {"1": {"class_type": "NoSuchNode", "inputs": {}}}})
        assert r.status_code == 400 and r.json()["error"]["type"] == "invalid_prompt"
        odd = build_wan_graph(_job())
        lat = next(k for k, v in odd.items() if v["class_type"] == "EmptyHunyuanLatentVideo")
        odd[lat]["inputs"]["width"] = 70
        assert c.post("/prompt", json={"prompt": odd}).status_code == 400


def test_prompt_runs_and_history_view_roundtrip(app):
    with TestClient(app) as c:
        r = c.post("/prompt", json={"prompt": build_wan_graph(_job(formats=("webp",))),
                                    "client_id": "t"})
        assert r.status_code == 200
        pid = r.json()["prompt_id"]
        assert app.state.queue.wait_idle(120)
        h = c.get(f"/history/{pid}").json()[pid]
        assert h["status"]["status_str"] == "success" and h["status"]["completed"]
        files = ComfyClient.output_files(h)
        assert len(files) == 1 and files[0]["filename"].endswith(".webp")
        v = c.get("/view", params=files[0])
        assert v.status_code == 200 and v.content[:4] == b"RIFF" and v.content[8:12] == b"WEBP"
        from PIL import Image
        import io

        im = Image.open(io.BytesIO(v.content))
        assert im.size == (64, 48) and getattr(im, "n_frames", 1) == 5
        assert c.get("/view", params={"filename": "../../etc/passwd"}).status_code == 404
        assert "wan_prompts_total{status=\"completed\"} 1" in c.get("/metrics").text


def test_image_mode_and_webm_without_ffmpeg(app):
    with TestClient(app) as c:
        pid = c.post("/prompt", json={"prompt": build_wan_graph(_job(mode="image"))}).json()["prompt_id"]
        pid2 = c.post("/prompt", json={"prompt": build_wan_graph(_job(formats=("webm",)))}).json()["prompt_id"]
        assert app.state.queue.wait_idle(120)
        h = c.get(f"/history/{pid}").json()[pid]
        pngs = ComfyClient.output_files(h)
        assert len(pngs) == 1 and pngs[0]["filename"].endswith("_00001_.png")
        h2 = c.get(f"/history/{pid2}").json()[pid2]
        assert h2["status"]["status_str"] == "error"
        err = [m for m in h2["status"]["messages"] if m[0] == "execution_error"][0][1]
        assert err["node_type"] == "SaveWEBM" and "ffmpeg" in err["exception_message"]


def test_savewebm_drives_ffmpeg(store, tmp_path):
    """SaveWEBM pipes raw RGB frames to ffmpeg (a stand-in script records the call here)."""
    fake = tmp_path / "ffmpeg"
    fake.write_text("#!/bin/sh\nfor a; do last=$a; done\ncat > \"$last\"\necho \"$@\" > \"$last.args\"\n")
    fake.chmod(0o755)
    ex = Executor(store, str(tmp_path / "out"), ffmpeg=str(fake))
    from k8s_nvidia_gpus_amd.models.wan.server import Image

    frames = torch.randint(0, 255, (3, 16, 32, 3), dtype=torch.uint8)
    ui = ex.node_SaveWEBM(Image(frames), "clips/wan", "vp9", 24, 32)["ui"]
    writes = ex.take_writes()                  # encoding runs on the encode pool
    assert [w[0] for w in writes] == ["SaveWEBM"]
    for _, _, fut in writes:
        fut.result(timeout=60)
    f = ui["images"][0]
    assert f["subfolder"] == "clips" and f["filename"] == "wan_00001_.webm"
    path = tmp_path / "out" / "clips" / f["filename"]
    assert path.stat().st_size == frames.numel()
    args = (str(path) + ".args")
    assert "libvpx-vp9" in open(args).read() and "32x16" in open(args).read()
    with pytest.raises(ValueError):
        ex._next_name("../escape", "png")


def test_queue_delete_and_interrupt(app):
    with TestClient(app) as c:
        ids = [c.post("/prompt", json={"prompt": build_wan_graph(_job(steps=6, seed=i))}).json()["prompt_id"]
               for i in range(3)]
        c.post("/queue", json={"delete": [ids[2]]})
        c.post("/interrupt")
        assert app.state.queue.wait_idle(180)
        hist = c.get("/history").json()
        assert ids[2] not in hist
        assert all(hist[i]["status"]["completed"] for i in ids[:2])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_reference_client_flow_against_live_server(app, tmp_path):
    """The repo's ComfyUI client (same flow as the reference script) against a real HTTP server."""
    import uvicorn

    port = _free_port()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    try:
        client = ComfyClient(f"http://127.0.0.1:{port}")
        assert client.wait_reachable(30)
        assert client.missing_models(WAN_MODELS) == []
        saved = run_jobs(client, [_job(seed=1), _job(seed=2)], tmp_path / "dl", poll=0.2,
                         timeout=120, log=lambda *_: None)
        assert len(saved) == 2 and all(p.stat().st_size > 0 for p in saved)
        assert (tmp_path / "dl" / "index.html").exists()
        assert saved[0].read_bytes() != saved[1].read_bytes()      # different seeds
    finally:
        server.should_exit = True
        th.join(10)
    assert os.path.isdir(tmp_path / "output")
    time.sleep(0)


def test_startup_warmup_gates_readiness(store, tmp_path):
    app = create_app(store, str(tmp_path / "out"), ffmpeg="", warmup=(64, 48, 5))
    with TestClient(app) as c:
        assert app.state.ready.wait(120)
        assert c.get("/queue").status_code == 200
        hist = c.get("/history").json()
        assert len(hist) == 1 and next(iter(hist.values()))["status"]["status_str"] == "success"


def test_encode_failure_reported_after_gpu_part(store, tmp_path):
    """A saver failing on the encode pool turns the prompt into an error entry naming the node."""
    bad = tmp_path / "ffmpeg"
    bad.write_text("#!/bin/sh\necho boom >&2\nexit 3\n")
    bad.chmod(0o755)
    app = create_app(store, str(tmp_path / "out"), ffmpeg=str(bad))
    with TestClient(app) as c:
        pid = c.post("/prompt", json={"prompt": build_wan_graph(_job(formats=("webm",)))}).json()["prompt_id"]
        assert app.state.queue.wait_idle(120)
        st = c.get(f"/history/{pid}").json()[pid]["status"]
        assert st["status_str"] == "error" and st["completed"]
        err = [m for m in st["messages"] if m[0] == "execution_error"][0][1]
        assert err["node_type"] == "SaveWEBM" and "boom" in err["exception_message"]
    assert not list((tmp_path / "out").rglob("*.webm"))        # no empty placeholder left


def test_failed_warmup_keeps_the_pod_unready(store, tmp_path, monkeypatch):
    """a warm-up job that fails (models that do not load) must not turn the pod ready."""
    from k8s_nvidia_gpus_amd.models.wan import server as WS

    def boom(self, graph, on_node=None):
        raise RuntimeError("cannot load wan2.1_t2v_1.3B_bf16.safetensors")

    monkeypatch.setattr(WS.Executor, "run", boom)
    app = create_app(store, str(tmp_path / "out"), ffmpeg="", warmup=(64, 48, 5))
    with TestClient(app) as c:
        t0 = time.time()
        while app.state.warmup_error is None and time.time() - t0 < 60:
            time.sleep(0.05)
        assert not app.state.ready.is_set()
        r = c.get("/queue")
        assert r.status_code == 503 and "warm-up failed" in r.json()["status"]
