"""SD1.5 REST service: HTTP surface, request coalescing, seeding, validation.

Most tests use a deterministic fake pipeline that records every batched call (fast, exact batch
accounting); the FastAPI app, the GPU worker and the batching logic are the real ones
(k8s_nvidia_gpus_amd/models/sd15_api.py).  The last tests serve the in-tree SD1.5 pipeline itself
(miniature config on CPU).
"""
import io
import threading
import time

import pytest
from fastapi.testclient import TestClient
from PIL import Image

from k8s_nvidia_gpus_amd.models.sd15_api import Settings, create_app


class FakePipe:
    def __init__(self, delay=0.05):
        self.calls = []
        self.delay = delay
        self.lock = threading.Lock()
        self.concurrent = 0
        self.max_concurrent = 0

    def __call__(self, prompt, num_inference_steps, guidance_scale, width, height, generator=None,
                 negative_prompt=None):
        with self.lock:
            self.concurrent += 1
            self.max_concurrent = max(self.max_concurrent, self.concurrent)
        try:
            self.calls.append(dict(prompts=list(prompt), steps=num_inference_steps, w=width, h=height,
                                   seeded=generator is not None))
            time.sleep(self.delay)
            imgs = []
            for i, p in enumerate(prompt):
                seed = generator[i].initial_seed() if generator is not None else 0
                color = (hash(p) % 256, seed % 256, num_inference_steps % 256)
                imgs.append(Image.new("RGB", (width, height), color))
            return type("Out", (), {"images": imgs})()
        finally:
            with self.lock:
                self.concurrent -= 1


@pytest.fixture
def pipe():
    return FakePipe()


@pytest.fixture
def client(pipe):
    s = Settings(device="cpu", dtype="float32", max_batch=8, batch_window_ms=30)
    app = create_app(s, pipeline_factory=lambda _s: pipe)
    with TestClient(app) as c:
        assert app.state.worker.wait_ready(5)
        yield c


def test_health_ready_and_empty_state(client):
    assert client.get("/healthz").json() == {"ok": True}
    assert client.get("/readyz").json()["ready"] is True
    assert client.get("/last").status_code == 404
    assert "No image generated yet" in client.get("/").text


def test_generate_returns_png_with_timing_header(client, pipe):
    r = client.post("/generate", json={"prompt": "a panda riding a motorbike", "steps": 30, "seed": 7})
    assert r.status_code == 200 and r.headers["content-type"] == "image/png"
    assert r.headers["X-Gen-Time"].endswith("s")
    img = Image.open(io.BytesIO(r.content))
    assert img.size == (512, 512)  # reference defaults (configmap.yaml:57-58)
    assert client.get("/last").content == r.content
    assert "data:image/png;base64," in client.get("/").text
    assert pipe.calls[0]["steps"] == 30 and pipe.calls[0]["seeded"]


def test_seed_determinism(client):
    a = client.post("/generate", json={"prompt": "x", "seed": 11}).content
    b = client.post("/generate", json={"prompt": "x", "seed": 11}).content
    c = client.post("/generate", json={"prompt": "x", "seed": 12}).content
    assert a == b and a != c


@pytest.mark.parametrize("body,code", [
    ({"prompt": "  "}, 400),
    ({"prompt": "x", "steps": 0}, 400),
    ({"prompt": "x", "steps": 10000}, 400),
    ({"prompt": "x", "width": 500}, 400),
    ({"prompt": "x", "height": 4096}, 400),
])
def test_validation(client, body, code):
    assert client.post("/generate", json=body).status_code == code


def test_concurrent_requests_are_coalesced_and_serialised(client, pipe):
    pipe.delay = 0.2
    results = {}

    def go(i):
        r = client.post("/generate", json={"prompt": f"p{i}", "steps": 20, "seed": i})
        results[i] = r

    threads = [threading.Thread(target=go, args=(i,)) for i in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(30)
    assert all(r.status_code == 200 for r in results.values())
    assert pipe.max_concurrent == 1  # the GPU pipeline is never entered concurrently
    assert len(pipe.calls) < 6  # requests arriving together shared a UNet batch
    assert max(len(c["prompts"]) for c in pipe.calls) >= 2
    assert {int(r.headers["X-Batch-Size"]) for r in results.values()} - {1}


def test_incompatible_requests_are_not_batched_together(client, pipe):
    pipe.delay = 0.2
    out = []
    ts = [threading.Thread(target=lambda s=s: out.append(client.post("/generate", json={"prompt": "q", "steps": s})))
          for s in (10, 10, 25)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    for c in pipe.calls:
        assert len({c["steps"]}) == 1
    assert sorted(c["steps"] for c in pipe.calls for _ in c["prompts"]) == [10, 10, 25]


def test_metrics_endpoint(client):
    client.post("/generate", json={"prompt": "m"})
    text = client.get("/metrics").text
    assert 'sd15_requests_total{status="ok"} 1.0' in text
    assert "sd15_batch_size_bucket" in text


def test_load_failure_surfaces_in_readyz():
    def boom(_s):
        raise RuntimeError("weights not found")

    app = create_app(Settings(device="cpu"), pipeline_factory=boom)
    with TestClient(app) as c:
        for _ in range(50):
            if app.state.worker.load_error is not None:
                break
            time.sleep(0.02)
        r = c.get("/readyz")
        assert r.status_code == 500 and "weights not found" in r.text
        assert c.post("/generate", json={"prompt": "x"}).status_code == 500


def test_native_pipeline_serves_end_to_end_on_cpu():
    """Default factory (PIPELINE=native): the in-tree SD1.5 (miniature config on CPU) behind the
    real HTTP worker — warm-up runs before ready, seeded requests are reproducible PNGs."""
    s = Settings(device="cpu", dtype="float32", model_config="tiny", warmup_batches="1,2",
                 batch_window_ms=5)
    app = create_app(s)
    with TestClient(app) as c:
        assert app.state.worker.wait_ready(120), app.state.worker.load_error
        body = {"prompt": "a cozy cabin", "steps": 3, "width": 64, "height": 64, "seed": 7}
        r1 = c.post("/generate", json=body)
        r2 = c.post("/generate", json=body)
        assert r1.status_code == 200 and r1.headers["content-type"] == "image/png"
        assert Image.open(io.BytesIO(r1.content)).size == (64, 64)
        assert r1.content == r2.content
        assert c.get("/readyz").json()["ready"] is True


def test_unknown_pipeline_kind_fails_readiness():
    app = create_app(Settings(device="cpu", dtype="float32", pipeline="onnx"))
    with TestClient(app) as c:
        for _ in range(100):
            if app.state.worker.load_error is not None:
                break
            time.sleep(0.02)
        assert c.get("/readyz").status_code == 500
