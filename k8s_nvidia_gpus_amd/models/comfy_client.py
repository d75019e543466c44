"""ComfyUI API client for Wan2.1 text-to-video / text-to-image jobs on the cluster's GPU.

Capability parity with the reference's standalone script (reference
cluster-config/apps/llm/scripts/generate_wan_t2v.py): build a ComfyUI API graph for Wan2.1
(UNETLoader / CLIPLoader(type=wan) / VAELoader / EmptyHunyuanLatentVideo / CLIPTextEncode ×2 /
KSampler / VAEDecode + WEBM / animated-WEBP / PNG savers), optionally reach the server through
``kubectl port-forward``, check the model files exist (``/object_info``), queue (``/prompt``),
poll (``/history/<id>``), download (``/view``) and write an ``index.html``.  Differences: the graph
is assembled by a small builder with generated node ids instead of a hand-numbered dict; HTTP
errors carry ComfyUI's error payload; the port-forward targets the ``wan-video-gen`` Deployment
that this repo actually ships (cluster-config/apps/comfyui — the reference's target did not exist).
"""
from __future__ import annotations

import html
import json
import os
import random
import subprocess
import time
import urllib.error
import urllib.parse
import urllib.request
from contextlib import contextmanager
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, Iterator, List, Optional

WAN_MODELS = {
    "unet": "wan2.1_t2v_1.3B_bf16.safetensors",
    "clip": "umt5_xxl_fp16.safetensors",
    "vae": "wan_2.1_vae.safetensors",
}


@dataclass
class WanJob:
    prompt: str
    negative: str = "blurry, low quality, artifacts"
    seed: int = 0
    width: int = 512
    height: int = 320
    frames: int = 16
    steps: int = 25
    cfg: float = 6.0
    sampler: str = "uni_pc"
    scheduler: str = "simple"
    denoise: float = 1.0
    mode: str = "video"              # video | image
    formats: tuple = ("webm",)       # any of webm, webp (video mode)
    fps_webm: int = 24
    fps_webp: int = 16
    prefix: str = "wan_t2v"
    models: Dict[str, str] = field(default_factory=lambda: dict(WAN_MODELS))

    def validate(self) -> None:
        if self.width % 16 or self.height % 16:
            raise ValueError("width and height must be multiples of 16 (Wan VAE)")
        if self.mode not in ("video", "image"):
            raise ValueError("mode must be 'video' or 'image'")
        if self.mode == "video" and not set(self.formats) & {"webm", "webp"}:
            raise ValueError("video mode needs at least one of webm / webp")


class GraphBuilder:
    """ComfyUI API-format graph: {node_id: {class_type, inputs}} with links as [node_id, slot]."""

    def __init__(self):
        self.nodes: Dict[str, dict] = {}
        self._next = 1

    def add(self, class_type: str, **inputs) -> List:
        nid = str(self._next)
        self._next += 1
        self.nodes[nid] = {"class_type": class_type, "inputs": inputs}
        return [nid, 0]

    def to_json(self) -> dict:
        return self.nodes


def build_wan_graph(job: WanJob) -> dict:
    job.validate()
    frames = 1 if job.mode == "image" else job.frames
    g = GraphBuilder()
    model = g.add("UNETLoader", unet_name=job.models["unet"], weight_dtype="default")
    clip = g.add("CLIPLoader", clip_name=job.models["clip"], type="wan", device="default")
    vae = g.add("VAELoader", vae_name=job.models["vae"])
    latent = g.add("EmptyHunyuanLatentVideo", width=job.width, height=job.height, length=frames,
                   batch_size=1)
    pos = g.add("CLIPTextEncode", clip=clip, text=job.prompt)
    neg = g.add("CLIPTextEncode", clip=clip, text=job.negative)
    samples = g.add("KSampler", model=model, positive=pos, negative=neg, latent_image=latent,
                    seed=job.seed, steps=job.steps, cfg=job.cfg, sampler_name=job.sampler,
                    scheduler=job.scheduler, denoise=job.denoise)
    images = g.add("VAEDecode", samples=samples, vae=vae)
    if job.mode == "image":
        g.add("SaveImage", images=images, filename_prefix=job.prefix)
    else:
        if "webp" in job.formats:
            g.add("SaveAnimatedWEBP", images=images, filename_prefix=job.prefix, fps=job.fps_webp,
                  lossless=False, quality=90, method="default")
        if "webm" in job.formats:
            g.add("SaveWEBM", images=images, filename_prefix=job.prefix, codec="vp9",
                  fps=job.fps_webm, crf=32)
    return g.to_json()


class ComfyError(RuntimeError):
    pass


class ComfyClient:
    def __init__(self, base_url: str = "http://127.0.0.1:8181", timeout: float = 30.0):
        self.base = base_url.rstrip("/")
        self.timeout = timeout
        self.client_id = f"amdk8s-{random.SystemRandom().randrange(1 << 30)}"

    def _json(self, path: str, payload=None, timeout: Optional[float] = None):
        data = json.dumps(payload).encode() if payload is not None else None
        req = urllib.request.Request(self.base + path, data=data,
                                     headers={"Content-Type": "application/json"} if data else {})
        try:
            with urllib.request.urlopen(req, timeout=timeout or self.timeout) as r:
                return json.loads(r.read().decode())
        except urllib.error.HTTPError as e:
            raise ComfyError(f"{path}: HTTP {e.code}: {e.read().decode(errors='replace')[:500]}") from None

    def reachable(self) -> bool:
        try:
            self._json("/queue", timeout=3)
            return True
        except Exception:  # noqa: BLE001
            return False

    def wait_reachable(self, timeout: float = 30.0) -> bool:
        deadline = time.time() + timeout
        while time.time() < deadline:
            if self.reachable():
                return True
            time.sleep(0.5)
        return False

    def missing_models(self, models: Dict[str, str]) -> List[str]:
        info = self._json("/object_info")

        def options(node: str, field_: str) -> List[str]:
            spec = info.get(node, {}).get("input", {}).get("required", {}).get(field_) or []
            if spec and isinstance(spec[0], list):
                return spec[0]
            return spec if isinstance(spec, list) else []

        want = [("UNETLoader", "unet_name", models["unet"]), ("CLIPLoader", "clip_name", models["clip"]),
                ("VAELoader", "vae_name", models["vae"])]
        return [f"{node}:{name}" for node, fld, name in want if name not in options(node, fld)]

    def queue(self, graph: dict) -> str:
        resp = self._json("/prompt", {"prompt": graph, "client_id": self.client_id})
        if "error" in resp:
            raise ComfyError(f"prompt rejected: {resp['error']} {resp.get('node_errors', '')}")
        pid = resp.get("prompt_id")
        if not pid:
            raise ComfyError(f"unexpected /prompt response: {resp}")
        return pid

    def wait(self, prompt_id: str, timeout: float = 3600.0, poll: float = 5.0) -> dict:
        deadline = time.time() + timeout
        while time.time() < deadline:
            hist = self._json(f"/history/{urllib.parse.quote(prompt_id)}")
            entry = hist.get(prompt_id)
            if entry:
                st = entry.get("status") or {}
                if st.get("completed"):
                    if st.get("status_str") != "success":
                        raise ComfyError(f"generation failed: {st.get('messages') or st}")
                    return entry
            time.sleep(poll)
        raise TimeoutError(f"prompt {prompt_id} not finished after {timeout}s")

    @staticmethod
    def output_files(entry: dict) -> List[dict]:
        out = []
        for node_out in (entry.get("outputs") or {}).values():
            for key in ("images", "videos", "gifs"):
                out.extend(f for f in node_out.get(key) or [] if isinstance(f, dict) and "filename" in f)
        return out

    def download(self, info: dict, dest: Path) -> Path:
        q = urllib.parse.urlencode({"filename": info["filename"], "subfolder": info.get("subfolder", ""),
                                    "type": info.get("type", "output")})
        dest.mkdir(parents=True, exist_ok=True)
        path = dest / os.path.basename(info["filename"])
        with urllib.request.urlopen(f"{self.base}/view?{q}", timeout=300) as r, open(path, "wb") as f:
            while True:
                chunk = r.read(1 << 20)
                if not chunk:
                    break
                f.write(chunk)
        return path


@contextmanager
def port_forward(namespace: str, deployment: str, local_port: int, remote_port: int = 8181) -> Iterator:
    proc = subprocess.Popen(["kubectl", "port-forward", "-n", namespace, f"deploy/{deployment}",
                             f"{local_port}:{remote_port}", "--address", "127.0.0.1"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        yield proc
    finally:
        proc.terminate()
        try:
            proc.wait(timeout=5)
        except subprocess.TimeoutExpired:
            proc.kill()


def write_index(dest: Path, prompt: str, files: List[Path]) -> Path:
    parts = ["<!doctype html><html><head><meta charset='utf-8'><title>Wan2.1 outputs</title></head><body>",
             f"<h1>Prompt</h1><p>{html.escape(prompt)}</p>"]
    for p in files:
        src = html.escape(p.name, quote=True)
        if p.suffix.lower() in (".webm", ".mp4"):
            parts.append(f"<div><video controls src='{src}' style='max-width:100%'></video></div>")
        else:
            parts.append(f"<div><img src='{src}' style='max-width:100%'></div>")
    parts.append("</body></html>")
    out = dest / "index.html"
    out.write_text("\n".join(parts), encoding="utf-8")
    return out


def run_jobs(client: ComfyClient, jobs: List[WanJob], dest: Path, check_models: bool = True,
             timeout: float = 3600.0, poll: float = 5.0, log=print) -> List[Path]:
    if check_models:
        missing = client.missing_models(jobs[0].models)
        if missing:
            raise ComfyError("ComfyUI is missing model files: " + ", ".join(missing))
    saved: List[Path] = []
    for i, job in enumerate(jobs, 1):
        log(f"[{i}/{len(jobs)}] queueing seed={job.seed}")
        entry = client.wait(client.queue(build_wan_graph(job)), timeout=timeout, poll=poll)
        files = client.output_files(entry)
        if not files:
            raise ComfyError("finished without output files")
        for f in files:
            ext = os.path.splitext(f["filename"])[1].lower().lstrip(".")
            if job.mode == "video" and ext not in job.formats:
                continue
            p = client.download(f, dest)
            saved.append(p)
            log(f"  saved {p}")
    if saved:
        write_index(dest, jobs[0].prompt, saved)
    return saved
