"""Client tools: Wan2.1 ComfyUI client (fake ComfyUI server), SD batch client, isolation checker."""
import importlib.util
import json
import subprocess
import sys
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path

import pytest

from k8s_nvidia_gpus_amd.models import comfy_client as cc

REPO = Path(__file__).resolve().parent.parent


def _load(path: Path, name: str):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class FakeComfy:
    """/queue, /object_info, /prompt, /history/<id>, /view — enough of ComfyUI's HTTP API."""

    def __init__(self, models=cc.WAN_MODELS, fail=False):
        self.models = models
        self.fail = fail
        self.prompts = {}
        self.polls = 0

    def start(self):
        fake = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _json(self, obj, code=200):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                u = urllib.parse.urlparse(self.path)
                if u.path == "/queue":
                    return self._json({"queue_running": [], "queue_pending": []})
                if u.path == "/object_info":
                    return self._json({
                        "UNETLoader": {"input": {"required": {"unet_name": [[fake.models["unet"]], {}]}}},
                        "CLIPLoader": {"input": {"required": {"clip_name": [[fake.models["clip"]]]}}},
                        "VAELoader": {"input": {"required": {"vae_name": [[fake.models["vae"]]]}}}})
                if u.path.startswith("/history/"):
                    pid = u.path.split("/")[-1]
                    fake.polls += 1
                    g = fake.prompts[pid]
                    if fake.polls % 2:  # first poll: still running
                        return self._json({})
                    outs = {}
                    for nid, n in g.items():
                        if n["class_type"].startswith("Save"):
                            ext = {"SaveWEBM": "webm", "SaveAnimatedWEBP": "webp", "SaveImage": "png"}[n["class_type"]]
                            outs[nid] = {"images": [{"filename": f"{n['inputs']['filename_prefix']}_00001.{ext}",
                                                     "subfolder": "", "type": "output"}]}
                    st = {"completed": True, "status_str": "error" if fake.fail else "success",
                          "messages": ["boom"] if fake.fail else []}
                    return self._json({pid: {"status": st, "outputs": outs}})
                if u.path == "/view":
                    q = dict(urllib.parse.parse_qsl(u.query))
                    body = f"FAKE:{q['filename']}".encode()
                    self.send_response(200)
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return
                self._json({"error": "no route"}, 404)

            def do_POST(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n))
                pid = f"p{len(fake.prompts)}"
                fake.prompts[pid] = body["prompt"]
                self._json({"prompt_id": pid, "number": len(fake.prompts)})

        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return f"http://127.0.0.1:{self.httpd.server_address[1]}"

    def stop(self):
        self.httpd.shutdown()


def test_wan_graph_structure():
    g = cc.build_wan_graph(cc.WanJob(prompt="p", seed=5, formats=("webm", "webp")))
    by_type = {n["class_type"]: (nid, n) for nid, n in g.items()}
    for t in ("UNETLoader", "CLIPLoader", "VAELoader", "EmptyHunyuanLatentVideo", "KSampler",
              "VAEDecode", "SaveWEBM", "SaveAnimatedWEBP"):
        assert t in by_type, t
    ks = by_type["KSampler"][1]["inputs"]
    assert ks["seed"] == 5 and ks["sampler_name"] == "uni_pc" and ks["steps"] == 25
    assert ks["model"] == [by_type["UNETLoader"][0], 0]
    assert by_type["CLIPLoader"][1]["inputs"]["type"] == "wan"
    assert by_type["EmptyHunyuanLatentVideo"][1]["inputs"]["length"] == 16
    img = cc.build_wan_graph(cc.WanJob(prompt="p", mode="image"))
    assert "SaveImage" in {n["class_type"] for n in img.values()}
    with pytest.raises(ValueError):
        cc.build_wan_graph(cc.WanJob(prompt="p", width=500))


def test_comfy_end_to_end_with_fake_server(tmp_path):
    fake = FakeComfy()
    url = fake.start()
    try:
        client = cc.ComfyClient(url)
        assert client.reachable()
        jobs = [cc.WanJob(prompt="a <b>panda</b>", seed=s, prefix=f"wan_t2v_{i:02d}") for i, s in enumerate((1, 2), 1)]
        saved = cc.run_jobs(client, jobs, tmp_path, poll=0.01, log=lambda *a: None)
        assert [p.name for p in saved] == ["wan_t2v_01_00001.webm", "wan_t2v_02_00001.webm"]
        assert saved[0].read_bytes() == b"FAKE:wan_t2v_01_00001.webm"
        index = (tmp_path / "index.html").read_text()
        assert "<video" in index and "&lt;b&gt;panda" in index  # prompt is escaped
    finally:
        fake.stop()


def test_comfy_missing_models_and_failed_generation(tmp_path):
    fake = FakeComfy(models={"unet": "other.safetensors", "clip": cc.WAN_MODELS["clip"],
                             "vae": cc.WAN_MODELS["vae"]})
    url = fake.start()
    try:
        with pytest.raises(cc.ComfyError, match="UNETLoader"):
            cc.run_jobs(cc.ComfyClient(url), [cc.WanJob(prompt="x")], tmp_path, log=lambda *a: None)
    finally:
        fake.stop()
    fake = FakeComfy(fail=True)
    url = fake.start()
    try:
        with pytest.raises(cc.ComfyError, match="generation failed"):
            cc.run_jobs(cc.ComfyClient(url), [cc.WanJob(prompt="x")], tmp_path, poll=0.01, log=lambda *a: None)
    finally:
        fake.stop()


def test_wan_cli_unreachable_without_port_forward(tmp_path):
    mod = _load(REPO / "cluster-config/apps/llm/scripts/generate_wan_t2v.py", "wan_cli")
    assert mod.main(["--prompt", "x", "--comfy-url", "http://127.0.0.1:9", "--output-dir", str(tmp_path)]) == 1


def test_batch_generate_against_real_sd_app(tmp_path):
    """scripts/batch_generate.py → real FastAPI app (fake pipeline) over a real socket."""
    import uvicorn
    from PIL import Image

    from k8s_nvidia_gpus_amd.models.sd15_api import Settings, create_app

    class Pipe:
        def __call__(self, prompt, num_inference_steps, guidance_scale, width, height, **kw):
            return type("O", (), {"images": [Image.new("RGB", (width, height)) for _ in prompt]})()

    app = create_app(Settings(device="cpu", dtype="float32"), pipeline_factory=lambda s: Pipe())
    config = uvicorn.Config(app, host="127.0.0.1", port=0, log_level="error")
    server = uvicorn.Server(config)
    t = threading.Thread(target=server.run, daemon=True)
    t.start()
    import time

    for _ in range(200):
        if server.started:
            break
        time.sleep(0.02)
    port = server.servers[0].sockets[0].getsockname()[1]
    try:
        mod = _load(REPO / "scripts/batch_generate.py", "batch_generate")
        rc = mod.main(["a cabin", "4", "cabin", str(tmp_path), "--parallel", "4", "--seed", "3",
                       "--url", f"http://127.0.0.1:{port}/generate"])
        assert rc == 0
        assert sorted(p.name for p in tmp_path.iterdir()) == [f"cabin_0{i}.png" for i in range(1, 5)]
    finally:
        server.should_exit = True
        t.join(10)


def test_batch_generate_defaults_fixed():
    mod = _load(REPO / "scripts/batch_generate.py", "batch_generate2")
    src = (REPO / "scripts/batch_generate.py").read_text()
    assert "import traceback" in src
    import argparse

    # --steps default is 30 (the reference's help said 30 but used 40)
    p = subprocess.run([sys.executable, str(REPO / "scripts/batch_generate.py"), "--help"],
                       capture_output=True, text=True)
    assert "default: 30" in p.stdout
    assert mod.DEFAULT_URL.endswith(":30800/generate")


def _pod_log(uid, passed=True):
    probe = {"ready": True, "gpus": 1, "agents": [{"node": 2, "unique_id": uid, "render_minor": 128}]}
    tail = "Test PASSED\nDone\n" if passed else "Test FAILED\n"
    return ("pod: x\n" + json.dumps(probe) + "\n[Vector addition of 50000 elements]\n" + tail)


def test_isolation_checker():
    mod = _load(REPO / "scripts/check_isolation.py", "check_isolation")
    ok, rep = mod.check({"a": _pod_log("111"), "b": _pod_log("222")})
    assert ok, rep
    ok, rep = mod.check({"a": _pod_log("111"), "b": _pod_log("111")})
    assert not ok and any("shares GPU" in r for r in rep)
    ok, _ = mod.check({"a": _pod_log("111"), "b": _pod_log("222", passed=False)})
    assert not ok


def test_time_to_first_gpu_pod_tool():
    import time

    from fakes.kubeapi import FakeKubeAPI

    api = FakeKubeAPI().start()
    api.add_node("gpu-node-1")

    def kubelet(a, pod):
        pod["status"]["phase"] = "Succeeded"
        a.logs[(pod["metadata"]["namespace"], pod["metadata"]["name"])] = "Test PASSED\nDone\n"

    api.on_pod_created = kubelet
    threading.Timer(0.2, lambda: api.nodes["gpu-node-1"]["metadata"]["labels"].update(
        {"amd.com/gpu.validated": "true"})).start()
    try:
        mod = _load(REPO / "tools/time_to_first_gpu_pod.py", "ttfgp")
        t0 = time.time()
        rc = mod.main(["--api", api.url, "--since", str(t0), "--poll", "0.05", "--timeout", "10"])
        assert rc == 0
        assert not [k for k in api.pods if k[1].startswith("ttfgp-")]  # cleaned up
    finally:
        api.stop()
