"""ComfyUI-compatible API server for the in-tree Wan2.1 engine (the ``wan-video-gen`` Deployment).

The reference's Wan client (reference cluster-config/apps/llm/scripts/generate_wan_t2v.py) talks to
a ComfyUI server it does not ship: ``GET /queue`` (reachability, :153-167), ``GET /object_info``
(model-file preflight, :191-221), ``POST /prompt`` with an API-format graph (:224-234),
``GET /history/<id>`` polling (:237-251) and ``GET /view`` downloads (:268-281).  This module serves
that API surface natively so the same client (and ``models/comfy_client.py``) runs against an
MI355X with no ComfyUI, no pip install at pod start and no Python-side model zoo:

* graph validation with ComfyUI-shaped errors (``{"error": {...}, "node_errors": {...}}``, 400);
* one GPU worker thread executes queued prompts in order; node outputs are memoised per prompt and
  loaded models are cached across prompts (a 1.3B DiT + 11 GB umT5 load once per pod);
* the node set the Wan text-to-video graph uses: ``UNETLoader``, ``CLIPLoader`` (type ``wan``),
  ``VAELoader``, ``EmptyHunyuanLatentVideo``, ``EmptyLatentImage``, ``CLIPTextEncode``,
  ``KSampler``, ``VAEDecode``, ``SaveImage``, ``SaveAnimatedWEBP``, ``SaveWEBM`` (VP9 through an
  ``ffmpeg`` binary when the image has one — otherwise that node fails with a clear message);
* ``/history``, ``/view`` (path-traversal safe), ``/queue`` (+ clear/delete), ``/interrupt``,
  ``/system_stats``, ``/health`` and Prometheus ``/metrics``.

Models live under ``<base>/models/{diffusion_models|unet, text_encoders|clip, vae}`` exactly like a
ComfyUI base directory, so the existing PVC layout (cluster-config/apps/comfyui) is unchanged.
"""
from __future__ import annotations

import itertools
import json
import logging
import os
import queue
import shutil
import subprocess
import threading
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch
from fastapi import Request   # module level: the route annotations are resolved from here

from . import sampler as S

log = logging.getLogger("wan.server")

MODEL_DIRS = {
    "unet": ("diffusion_models", "unet"),
    "clip": ("text_encoders", "clip"),
    "vae": ("vae",),
}


class NodeError(Exception):
    def __init__(self, node_id: str, class_type: str, message: str, kind: str = "execution_error"):
        super().__init__(message)
        self.node_id, self.class_type, self.kind = node_id, class_type, kind


class Interrupted(Exception):
    pass


# ------------------------------------------------------------------------------------------ models
class ModelStore:
    """Resolves model names under the ComfyUI base directory and caches loaded components.
    ``loaders`` maps kind → ``fn(path) -> component`` (real safetensors loaders by default;
    the tests and ``--synthetic`` substitute random-init ones)."""

    def __init__(self, base: str, device: str = "cuda", dtype: torch.dtype = torch.bfloat16,
                 loaders: Optional[Dict[str, Callable[[str], Any]]] = None,
                 listing: Optional[Dict[str, List[str]]] = None):
        self.base = base
        self.device = torch.device(device)
        self.dtype = dtype
        self._loaders = loaders or _default_loaders()
        self._listing = listing
        self._cache: Dict[Tuple[str, str], Any] = {}
        self._lock = threading.Lock()

    def names(self, kind: str) -> List[str]:
        if self._listing is not None:
            return sorted(self._listing.get(kind, []))
        out = set()
        for d in MODEL_DIRS[kind]:
            root = os.path.join(self.base, "models", d)
            if os.path.isdir(root):
                for dirpath, _, files in os.walk(root):
                    for f in files:
                        if f.endswith((".safetensors", ".sft")):
                            out.add(os.path.relpath(os.path.join(dirpath, f), root))
        return sorted(out)

    def path(self, kind: str, name: str) -> str:
        for d in MODEL_DIRS[kind]:
            root = os.path.realpath(os.path.join(self.base, "models", d))
            p = os.path.realpath(os.path.join(root, name))
            if p.startswith(root + os.sep) and os.path.exists(p):
                return p
        return name

    def get(self, kind: str, name: str):
        if name not in self.names(kind):
            raise FileNotFoundError(f"{kind} model {name!r} not found")
        with self._lock:
            key = (kind, name)
            if key not in self._cache:
                t0 = time.time()
                comp = self._loaders[kind](self.path(kind, name))
                comp = _to_device(comp, self.device, self.dtype)
                self._cache[key] = comp
                log.info("loaded %s %s in %.1f s", kind, name, time.time() - t0)
            return self._cache[key]


def _to_device(comp, device, dtype):
    if isinstance(comp, tuple):                   # (t5 encoder, tokenizer)
        return (comp[0].to(device, dtype).eval(),) + comp[1:]
    comp = comp.to(device, dtype).eval()
    if hasattr(comp, "fuse"):
        comp.fuse()
    return comp


def _default_loaders():
    from .pipeline import load_dit, load_text_encoder, load_vae

    return {"unet": load_dit, "clip": load_text_encoder, "vae": load_vae}


# ------------------------------------------------------------------------------------------- nodes
INT_MAX = 0xFFFFFFFFFFFFFFFF


def node_specs(store: ModelStore) -> Dict[str, dict]:
    """``/object_info`` entries: ComfyUI's shape ({input: {required: {name: [type|options, cfg]}},
    output, output_name, category})."""
    def spec(required, output=(), category="wan", output_node=False):
        return {"input": {"required": required}, "output": list(output),
                "output_name": list(output), "name": None, "display_name": None,
                "category": category, "output_node": output_node, "description": ""}

    specs = {
        "UNETLoader": spec({"unet_name": [store.names("unet")],
                            "weight_dtype": [["default", "bf16"]]}, ["MODEL"], "loaders"),
        "CLIPLoader": spec({"clip_name": [store.names("clip")], "type": [["wan"]],
                            "device": [["default"]]}, ["CLIP"], "loaders"),
        "VAELoader": spec({"vae_name": [store.names("vae")]}, ["VAE"], "loaders"),
        "EmptyHunyuanLatentVideo": spec({
            "width": ["INT", {"default": 848, "min": 16, "max": 8192, "step": 16}],
            "height": ["INT", {"default": 480, "min": 16, "max": 8192, "step": 16}],
            "length": ["INT", {"default": 25, "min": 1, "max": 8192, "step": 4}],
            "batch_size": ["INT", {"default": 1, "min": 1, "max": 1}]}, ["LATENT"], "latent"),
        "EmptyLatentImage": spec({
            "width": ["INT", {"default": 512, "min": 16, "max": 8192, "step": 16}],
            "height": ["INT", {"default": 512, "min": 16, "max": 8192, "step": 16}],
            "batch_size": ["INT", {"default": 1, "min": 1, "max": 1}]}, ["LATENT"], "latent"),
        "CLIPTextEncode": spec({"text": ["STRING", {"multiline": True}], "clip": ["CLIP"]},
                               ["CONDITIONING"], "conditioning"),
        "KSampler": spec({
            "model": ["MODEL"], "seed": ["INT", {"default": 0, "min": 0, "max": INT_MAX}],
            "steps": ["INT", {"default": 20, "min": 1, "max": 10000}],
            "cfg": ["FLOAT", {"default": 8.0, "min": 0.0, "max": 100.0}],
            "sampler_name": [list(S.SAMPLERS)], "scheduler": [list(S.SCHEDULERS)],
            "positive": ["CONDITIONING"], "negative": ["CONDITIONING"],
            "latent_image": ["LATENT"],
            "denoise": ["FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0}]}, ["LATENT"], "sampling"),
        "VAEDecode": spec({"samples": ["LATENT"], "vae": ["VAE"]}, ["IMAGE"], "latent"),
        "SaveImage": spec({"images": ["IMAGE"], "filename_prefix": ["STRING", {"default": "ComfyUI"}]},
                          [], "image", True),
        "SaveAnimatedWEBP": spec({
            "images": ["IMAGE"], "filename_prefix": ["STRING", {"default": "ComfyUI"}],
            "fps": ["FLOAT", {"default": 6.0, "min": 0.01, "max": 1000.0}],
            "lossless": ["BOOLEAN", {"default": True}],
            "quality": ["INT", {"default": 80, "min": 0, "max": 100}],
            "method": [["default", "fastest", "slowest"]]}, [], "image/animation", True),
        "SaveWEBM": spec({
            "images": ["IMAGE"], "filename_prefix": ["STRING", {"default": "ComfyUI"}],
            "codec": [["vp9", "av1"]], "fps": ["FLOAT", {"default": 24.0, "min": 0.01, "max": 1000.0}],
            "crf": ["FLOAT", {"default": 32.0, "min": 0, "max": 63.0}]}, [], "image/video", True),
    }
    for k, v in specs.items():
        v["name"] = v["display_name"] = k
    return specs


OUTPUT_NODES = {"SaveImage", "SaveAnimatedWEBP", "SaveWEBM"}


def validate_graph(graph: dict, specs: Dict[str, dict]) -> Tuple[Optional[dict], Dict[str, dict]]:
    """ComfyUI's validation contract: (error, node_errors); error None when the graph is runnable."""
    if not isinstance(graph, dict) or not graph:
        return {"type": "invalid_prompt", "message": "Cannot execute because the prompt is empty",
                "details": "", "extra_info": {}}, {}
    node_errors: Dict[str, dict] = {}
    outputs = []
    for nid, node in graph.items():
        errs = []
        ct = node.get("class_type") if isinstance(node, dict) else None
        if ct not in specs:
            return {"type": "invalid_prompt", "message": f"Cannot execute because node {ct} does not exist.",
                    "details": f"Node ID '#{nid}'", "extra_info": {}}, {}
        if ct in OUTPUT_NODES:
            outputs.append(nid)
        inputs = node.get("inputs") or {}
        for name, cfg in specs[ct]["input"]["required"].items():
            if name not in inputs:
                errs.append({"type": "required_input_missing", "message": "Required input is missing",
                             "details": name, "extra_info": {"input_name": name}})
                continue
            val = inputs[name]
            kind = cfg[0]
            if isinstance(val, list) and len(val) == 2 and isinstance(val[0], str):
                src = graph.get(val[0])
                if src is None or src.get("class_type") not in specs:
                    errs.append({"type": "bad_linked_input", "message": "Bad linked input",
                                 "details": f"{name}: node {val[0]} missing", "extra_info": {}})
                    continue
                outs = specs[src["class_type"]]["output"]
                if not (0 <= int(val[1]) < len(outs)) or (isinstance(kind, str) and outs[int(val[1])] != kind):
                    errs.append({"type": "return_type_mismatch", "message": "Return type mismatch",
                                 "details": f"{name}: expected {kind}", "extra_info": {}})
                continue
            if isinstance(kind, list):
                if val not in kind:
                    errs.append({"type": "value_not_in_list", "message": "Value not in list",
                                 "details": f"{name}: '{val}' not in {kind[:20]}",
                                 "extra_info": {"input_name": name, "received_value": val}})
            elif kind in ("INT", "FLOAT"):
                try:
                    num = float(val)
                except (TypeError, ValueError):
                    errs.append({"type": "invalid_input_type", "message": f"Failed to convert to {kind}",
                                 "details": name, "extra_info": {}})
                    continue
                lim = cfg[1] if len(cfg) > 1 else {}
                if "min" in lim and num < lim["min"] or "max" in lim and num > lim["max"]:
                    errs.append({"type": "value_out_of_range", "message": "Value out of range",
                                 "details": f"{name}: {val}", "extra_info": {"input_name": name}})
                step = lim.get("step")
                if kind == "INT" and step and name in ("width", "height") and int(num) % step:
                    errs.append({"type": "value_not_multiple", "message": f"must be a multiple of {step}",
                                 "details": f"{name}: {val}", "extra_info": {}})
            elif kind in ("STRING",) and not isinstance(val, str):
                errs.append({"type": "invalid_input_type", "message": "Expected a string",
                             "details": name, "extra_info": {}})
        if errs:
            node_errors[nid] = {"errors": errs, "dependent_outputs": [], "class_type": ct}
    if not outputs:
        return {"type": "prompt_no_outputs", "message": "Prompt has no outputs", "details": "",
                "extra_info": {}}, {}
    if node_errors:
        return {"type": "prompt_outputs_failed_validation",
                "message": "Prompt outputs failed validation", "details": "", "extra_info": {}}, node_errors
    return None, {}


@dataclass
class Image:
    frames: torch.Tensor     # uint8 [N, H, W, 3]


class Executor:
    """Evaluates one API-format graph: output nodes pull their inputs recursively (memoised)."""

    def __init__(self, store: ModelStore, out_dir: str, shift: float = 8.0,
                 ffmpeg: Optional[str] = None):
        self.store = store
        self.out_dir = out_dir
        self.shift = shift
        self.ffmpeg = ffmpeg if ffmpeg is not None else shutil.which("ffmpeg")
        self._counter_lock = threading.Lock()
        self.interrupt = threading.Event()
        self._runners: Dict[int, Any] = {}     # id(DiT) -> DiTRunner (HIP-graph step per shape)
        # output encoding (PNG / WEBP / ffmpeg) runs off the GPU worker: the next prompt's
        # sampling overlaps the previous prompt's CPU-side encode
        from concurrent.futures import ThreadPoolExecutor

        self.encode_pool = ThreadPoolExecutor(max_workers=2, thread_name_prefix="wan-encode")
        self._writes: List[Tuple[str, str, Any]] = []

    def _defer(self, node_class: str, fn, *args) -> None:
        self._writes.append((node_class, fn.__name__,
                             self.encode_pool.submit(_removing_on_failure(fn), *args)))

    def take_writes(self) -> List[Tuple[str, str, Any]]:
        w, self._writes = self._writes, []
        return w

    # --------------------------------------------------------------------- graph walk
    def run(self, graph: dict, on_node: Optional[Callable[[str], None]] = None) -> Dict[str, dict]:
        memo: Dict[str, tuple] = {}
        ui: Dict[str, dict] = {}

        def value(nid: str) -> tuple:
            if nid in memo:
                return memo[nid]
            if self.interrupt.is_set():
                raise Interrupted()
            node = graph[nid]
            ct = node["class_type"]
            args = {}
            for k, v in (node.get("inputs") or {}).items():
                if isinstance(v, list) and len(v) == 2 and isinstance(v[0], str):
                    args[k] = value(v[0])[int(v[1])]
                else:
                    args[k] = v
            if on_node:
                on_node(nid)
            try:
                res = getattr(self, "node_" + ct)(**args)
            except (Interrupted, NodeError):
                raise
            except Exception as e:  # noqa: BLE001 - reported per node, like ComfyUI
                raise NodeError(nid, ct, f"{type(e).__name__}: {e}") from e
            if isinstance(res, dict) and "ui" in res:
                ui[nid] = res["ui"]
                res = ()
            memo[nid] = res
            return res

        for nid, node in graph.items():
            if node["class_type"] in OUTPUT_NODES:
                value(nid)
        return ui

    # --------------------------------------------------------------------- loaders
    def node_UNETLoader(self, unet_name, weight_dtype="default"):
        return (self.store.get("unet", unet_name),)

    def node_CLIPLoader(self, clip_name, type="wan", device="default"):  # noqa: A002
        return (self.store.get("clip", clip_name),)

    def node_VAELoader(self, vae_name):
        return (self.store.get("vae", vae_name),)

    # --------------------------------------------------------------------- latents / text
    def node_EmptyHunyuanLatentVideo(self, width, height, length, batch_size=1):
        from .config import latent_frames

        t = latent_frames(int(length))
        return ({"samples": torch.zeros(int(batch_size), 16, t, int(height) // 8, int(width) // 8)},)

    def node_EmptyLatentImage(self, width, height, batch_size=1):
        return self.node_EmptyHunyuanLatentVideo(width, height, 1, batch_size)

    @torch.no_grad()
    def node_CLIPTextEncode(self, text, clip):
        enc, tok = clip[0], clip[1]
        dev = next(enc.parameters()).device
        ids = torch.tensor([tok.encode(str(text))], device=dev)
        return (enc(ids),)

    # --------------------------------------------------------------------- sampling / decode
    def node_KSampler(self, model, seed, steps, cfg, sampler_name, scheduler, positive, negative,
                      latent_image, denoise=1.0):
        from .pipeline import DiTRunner, ksample

        runner = self._runners.get(id(model))
        if runner is None:
            runner = DiTRunner(model, use_graphs=next(model.parameters()).is_cuda)
            self._runners[id(model)] = runner
        lat = latent_image["samples"]
        total = int(steps)

        def cb(i, _x0):
            if self.interrupt.is_set():
                raise Interrupted()
            log.debug("step %d/%d", i + 1, total)

        out = ksample(model, positive, negative, lat, int(seed), total, float(cfg), sampler_name,
                      scheduler, float(denoise), self.shift, cb, runner)
        return ({"samples": out.float()},)

    @torch.no_grad()
    def node_VAEDecode(self, samples, vae):
        from .pipeline import frames_uint8

        dev = next(vae.parameters()).device
        return (Image(frames_uint8(vae.decode(samples["samples"].to(dev)))),)

    # --------------------------------------------------------------------- savers
    def _next_name(self, prefix: str, ext: str) -> Tuple[str, str]:
        prefix = str(prefix).replace("\\", "/")
        sub, base = os.path.split(prefix)
        sub = os.path.normpath(sub) if sub else ""
        if sub.startswith("..") or os.path.isabs(sub):
            raise ValueError(f"filename_prefix {prefix!r} leaves the output directory")
        d = os.path.join(self.out_dir, sub)
        os.makedirs(d, exist_ok=True)
        with self._counter_lock:
            for i in itertools.count(1):
                name = f"{base}_{i:05d}_.{ext}"
                p = os.path.join(d, name)
                if not os.path.exists(p):
                    open(p, "wb").close()         # reserve the name
                    return name, sub

    def node_SaveImage(self, images: Image, filename_prefix="ComfyUI"):
        res = []
        for fr in images.frames:
            name, sub = self._next_name(filename_prefix, "png")
            self._defer("SaveImage", _write_png, fr.numpy(), os.path.join(self.out_dir, sub, name))
            res.append({"filename": name, "subfolder": sub, "type": "output"})
        return {"ui": {"images": res}}

    def node_SaveAnimatedWEBP(self, images: Image, filename_prefix="ComfyUI", fps=6.0, lossless=True,
                              quality=80, method="default"):
        meth = {"default": 4, "fastest": 0, "slowest": 6}.get(method, 4)
        name, sub = self._next_name(filename_prefix, "webp")
        self._defer("SaveAnimatedWEBP", _write_webp, images.frames.numpy(),
                    os.path.join(self.out_dir, sub, name), int(1000.0 / float(fps)), bool(lossless),
                    int(quality), meth)
        return {"ui": {"images": [{"filename": name, "subfolder": sub, "type": "output"}],
                       "animated": [True]}}

    def node_SaveWEBM(self, images: Image, filename_prefix="ComfyUI", codec="vp9", fps=24.0, crf=32.0):
        if not self.ffmpeg:
            raise RuntimeError("SaveWEBM needs an ffmpeg binary with libvpx-vp9 in the image; "
                               "use SaveAnimatedWEBP (formats=webp) on this server")
        fr = images.frames
        n, h, w, _ = fr.shape
        name, sub = self._next_name(filename_prefix, "webm")
        enc = {"vp9": "libvpx-vp9", "av1": "libaom-av1"}[codec]
        cmd = [self.ffmpeg, "-y", "-loglevel", "error", "-f", "rawvideo", "-pix_fmt", "rgb24",
               "-s", f"{w}x{h}", "-r", str(float(fps)), "-i", "-", "-c:v", enc, "-crf", str(int(crf)),
               "-b:v", "0", "-pix_fmt", "yuv420p", os.path.join(self.out_dir, sub, name)]
        self._defer("SaveWEBM", _run_ffmpeg, cmd, fr.numpy().tobytes())
        return {"ui": {"images": [{"filename": name, "subfolder": sub, "type": "output"}],
                       "animated": [True]}}


def _removing_on_failure(fn):
    """An encoder that fails leaves no truncated or placeholder file behind (the name was reserved
    with an empty file by ``Executor._next_name``)."""
    def wrapped(*args):
        path = args[1] if fn is not _run_ffmpeg else args[0][-1]
        try:
            fn(*args)
        except BaseException:
            try:
                os.remove(path)
            except OSError:
                pass
            raise
    wrapped.__name__ = fn.__name__
    return wrapped


def _write_png(arr, path: str) -> None:
    from PIL import Image as PILImage

    PILImage.fromarray(arr).save(path, compress_level=4)


def _write_webp(frames, path: str, duration_ms: int, lossless: bool, quality: int, method: int) -> None:
    from PIL import Image as PILImage

    pil = [PILImage.fromarray(f) for f in frames]
    pil[0].save(path, save_all=True, append_images=pil[1:], duration=duration_ms, lossless=lossless,
                quality=quality, method=method, loop=0)


def _run_ffmpeg(cmd: List[str], data: bytes) -> None:
    proc = subprocess.run(cmd, input=data, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    if proc.returncode != 0:
        raise RuntimeError(f"ffmpeg failed: {proc.stderr.decode(errors='replace')[-300:]}")


# ------------------------------------------------------------------------------------------- queue
@dataclass
class Job:
    number: int
    prompt_id: str
    graph: dict
    client_id: str = ""
    extra: dict = field(default_factory=dict)


class PromptQueue:
    def __init__(self, executor: Executor, max_history: int = 1000):
        self.ex = executor
        self._q: "queue.Queue[Optional[Job]]" = queue.Queue()
        self._pending: List[Job] = []
        self._running: Optional[Job] = None
        self._finalizing = 0                   # prompts whose outputs are still being encoded
        self._history: Dict[str, dict] = {}
        self._order: List[str] = []
        self._lock = threading.Lock()
        self._counter = itertools.count()
        self.max_history = max_history
        self.stats = {"completed": 0, "failed": 0, "interrupted": 0, "exec_seconds": 0.0}
        self._thread = threading.Thread(target=self._loop, daemon=True, name="wan-gpu-worker")
        self._thread.start()

    def submit(self, graph: dict, client_id: str = "", extra: Optional[dict] = None) -> Job:
        job = Job(next(self._counter), str(uuid.uuid4()), graph, client_id, extra or {})
        with self._lock:
            self._pending.append(job)
        self._q.put(job)
        return job

    def _loop(self):
        while True:
            job = self._q.get()
            if job is None:
                return
            with self._lock:
                if job not in self._pending:           # deleted while queued
                    continue
                self._pending.remove(job)
                self._running = job
            self.ex.interrupt.clear()
            t0 = time.time()
            msgs: List[list] = [["execution_start", {"prompt_id": job.prompt_id, "timestamp": int(t0 * 1000)}]]
            status, outputs, kind = "success", {}, "completed"
            try:
                outputs = self.ex.run(job.graph)
            except Interrupted:
                status, kind = "error", "interrupted"
                msgs.append(["execution_interrupted", {"prompt_id": job.prompt_id}])
            except NodeError as e:
                status, kind = "error", "failed"
                msgs.append(["execution_error", {"prompt_id": job.prompt_id, "node_id": e.node_id,
                                                 "node_type": e.class_type, "exception_message": str(e),
                                                 "exception_type": e.kind}])
                log.warning("prompt %s failed at node %s (%s): %s", job.prompt_id, e.node_id,
                            e.class_type, e)
            except Exception as e:  # noqa: BLE001 - outside any node: still one failed prompt,
                # never a dead worker thread that leaves every later prompt pending forever
                status, kind = "error", "failed"
                msgs.append(["execution_error", {"prompt_id": job.prompt_id, "node_id": "",
                                                 "node_type": "", "exception_message": repr(e),
                                                 "exception_type": type(e).__name__}])
                log.exception("prompt %s failed", job.prompt_id)
            gpu_s = time.time() - t0
            writes = self.ex.take_writes()
            with self._lock:
                self._running = None
                self._finalizing += 1
            if writes:
                threading.Thread(target=self._finalize, name="wan-finalize", daemon=True,
                                 args=(job, status, kind, outputs, msgs, t0, gpu_s, writes)).start()
            else:
                self._finalize(job, status, kind, outputs, msgs, t0, gpu_s, writes)

    def _finalize(self, job: Job, status: str, kind: str, outputs: dict, msgs: List[list],
                  t0: float, gpu_s: float, writes) -> None:
        """Wait for the prompt's output files, then publish its history entry (a client polling
        /history never sees a prompt as done before its files exist)."""
        for node_class, what, fut in writes:
            try:
                fut.result()
            except Exception as e:  # noqa: BLE001 - reported like a node failure
                if status == "success":
                    status, kind = "error", "failed"
                    msgs.append(["execution_error", {"prompt_id": job.prompt_id, "node_id": "",
                                                     "node_type": node_class,
                                                     "exception_message": f"{what}: {e}",
                                                     "exception_type": "execution_error"}])
        if status == "success":
            msgs.append(["execution_success", {"prompt_id": job.prompt_id,
                                               "timestamp": int(time.time() * 1000)}])
        dt = time.time() - t0
        # "completed" marks the prompt as final (the client then reads status_str)
        entry = {"prompt": [job.number, job.prompt_id, job.graph, job.extra, []],
                 "outputs": outputs,
                 "status": {"status_str": status, "completed": True, "messages": msgs},
                 "meta": {"execution_s": round(dt, 3), "gpu_s": round(gpu_s, 3)}}
        with self._lock:
            self.stats[kind] += 1
            self.stats["exec_seconds"] += dt
            self._history[job.prompt_id] = entry
            self._order.append(job.prompt_id)
            while len(self._order) > self.max_history:
                self._history.pop(self._order.pop(0), None)
            self._finalizing -= 1

    def queue_state(self) -> dict:
        def row(j: Job):
            return [j.number, j.prompt_id, j.graph, j.extra, []]

        with self._lock:
            return {"queue_running": [row(self._running)] if self._running else [],
                    "queue_pending": [row(j) for j in self._pending]}

    def history(self, prompt_id: Optional[str] = None, max_items: Optional[int] = None) -> dict:
        with self._lock:
            if prompt_id is not None:
                return {prompt_id: self._history[prompt_id]} if prompt_id in self._history else {}
            ids = self._order[-max_items:] if max_items else list(self._order)
            return {i: self._history[i] for i in ids}

    def clear_pending(self) -> None:
        with self._lock:
            self._pending.clear()

    def delete(self, ids: List[str]) -> None:
        with self._lock:
            self._pending = [j for j in self._pending if j.prompt_id not in ids]

    def clear_history(self, ids: Optional[List[str]] = None) -> None:
        with self._lock:
            for i in (ids if ids is not None else list(self._order)):
                self._history.pop(i, None)
                if i in self._order:
                    self._order.remove(i)

    def remaining(self) -> int:
        with self._lock:
            return len(self._pending) + (1 if self._running else 0) + self._finalizing

    def wait_idle(self, timeout: float = 60.0) -> bool:
        deadline = time.time() + timeout
        while time.time() < deadline:
            if self.remaining() == 0:
                return True
            time.sleep(0.02)
        return False


# --------------------------------------------------------------------------------------------- app
def warmup_graph(store: ModelStore, width: int = 512, height: int = 320, frames: int = 16) -> Optional[dict]:
    """A one-step job at the default size with the reference client's model files, when all three
    exist: loads the models and pays MIOpen's per-shape kernel compilation + solver search, the
    hipBLASLt heuristics and the HIP-graph capture before the pod reports ready."""
    from ..comfy_client import WanJob, build_wan_graph

    job = WanJob(prompt="warm-up", negative="", width=width, height=height, frames=frames, steps=1,
                 mode="video", formats=("webp",), prefix="_warmup/wan")
    if any(job.models[k] not in store.names(k) for k in ("unet", "clip", "vae")):
        return None
    return build_wan_graph(job)


def _freeze_tunableop() -> None:
    """With PyTorch TunableOp enabled (the Deployment sets it), GEMM tuning runs only during the
    warm-up job — the DiT's fixed shapes — and is then switched off and the table written: later
    requests use the tuned solutions, and a new prompt length (the umT5 GEMMs' M) falls back to the
    default heuristic instead of stalling the request on a tuning sweep."""
    try:
        tun = torch.cuda.tunable
        if tun.is_enabled() and tun.tuning_is_enabled():
            tun.tuning_enable(False)
            tun.write_file()
            log.info("TunableOp: tuning frozen after warm-up, results written")
    except (AttributeError, RuntimeError) as e:  # torch without TunableOp / no GPU
        log.debug("TunableOp not frozen: %s", e)


def create_app(store: ModelStore, out_dir: str, shift: float = 8.0, ffmpeg: Optional[str] = None,
               warmup: Optional[Tuple[int, int, int]] = None):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import JSONResponse, PlainTextResponse, Response

    os.makedirs(out_dir, exist_ok=True)
    ex = Executor(store, out_dir, shift, ffmpeg)
    pq = PromptQueue(ex)
    app = FastAPI(title="Wan2.1 ComfyUI-compatible API (MI355X)")
    app.state.queue = pq
    app.state.executor = ex
    ready = threading.Event()
    app.state.ready = ready
    app.state.warmup_error = None
    if warmup is not None:
        graph = warmup_graph(store, *warmup)
        if graph is None:
            log.info("warm-up skipped: the reference model files are not all present")
            _freeze_tunableop()          # no request may start a tuning sweep
            ready.set()
        else:
            job = pq.submit(graph, "warmup")

            def watch():
                while pq.history(job.prompt_id) == {}:
                    time.sleep(0.5)
                st = pq.history(job.prompt_id)[job.prompt_id]["status"]["status_str"]
                _freeze_tunableop()
                if st != "success":
                    # the models did not load / run: stay NOT ready (readiness 503) rather than
                    # take traffic that would fail
                    app.state.warmup_error = st
                    log.error("warm-up job failed (%s): the pod stays unready", st)
                    return
                log.info("warm-up finished: %s", st)
                ready.set()

            threading.Thread(target=watch, daemon=True, name="wan-warmup").start()
    else:
        _freeze_tunableop()
        ready.set()

    @app.get("/health")
    def health():
        return {"status": "ok"}

    @app.get("/queue")
    def get_queue():
        if not ready.is_set():     # readiness: 503 until the start-up warm-up job has run
            err = app.state.warmup_error
            return JSONResponse({"status": f"warm-up failed: {err}" if err else "warming up"}, 503)
        return pq.queue_state()

    @app.post("/queue")
    async def post_queue(req: Request):
        body = await req.json()
        if body.get("clear"):
            pq.clear_pending()
        if "delete" in body:
            pq.delete(list(body["delete"]))
        return {}

    @app.post("/interrupt")
    def interrupt():
        ex.interrupt.set()
        return {}

    @app.get("/object_info")
    def object_info():
        return node_specs(store)

    @app.get("/object_info/{node}")
    def object_info_node(node: str):
        specs = node_specs(store)
        return {node: specs[node]} if node in specs else {}

    @app.get("/models/{folder}")
    def models(folder: str):
        kinds = {"diffusion_models": "unet", "unet": "unet", "text_encoders": "clip",
                 "clip": "clip", "vae": "vae"}
        if folder not in kinds:
            raise HTTPException(404)
        return store.names(kinds[folder])

    @app.post("/prompt")
    async def post_prompt(req: Request):
        try:
            body = await req.json()
        except json.JSONDecodeError:
            return JSONResponse({"error": {"type": "invalid_prompt", "message": "bad JSON",
                                           "details": "", "extra_info": {}}, "node_errors": {}}, 400)
        graph = body.get("prompt")
        err, node_errors = validate_graph(graph, node_specs(store))
        if err is not None:
            return JSONResponse({"error": err, "node_errors": node_errors}, 400)
        job = pq.submit(graph, body.get("client_id", ""), body.get("extra_data") or {})
        return {"prompt_id": job.prompt_id, "number": job.number, "node_errors": {}}

    @app.get("/prompt")
    def get_prompt():
        return {"exec_info": {"queue_remaining": pq.remaining()}}

    @app.get("/history")
    def history_all(max_items: Optional[int] = None):
        return pq.history(max_items=max_items)

    @app.get("/history/{prompt_id}")
    def history_one(prompt_id: str):
        return pq.history(prompt_id)

    @app.post("/history")
    async def history_post(req: Request):
        body = await req.json()
        if body.get("clear"):
            pq.clear_history()
        if "delete" in body:
            pq.clear_history(list(body["delete"]))
        return {}

    @app.get("/view")
    def view(filename: str, subfolder: str = "", type: str = "output"):  # noqa: A002
        if type != "output":
            raise HTTPException(404, "only output files are served")
        root = os.path.realpath(out_dir)
        p = os.path.realpath(os.path.join(root, subfolder, filename))
        if not p.startswith(root + os.sep) or not os.path.isfile(p):
            raise HTTPException(404)
        media = {".png": "image/png", ".webp": "image/webp", ".webm": "video/webm"}.get(
            os.path.splitext(p)[1].lower(), "application/octet-stream")
        with open(p, "rb") as f:
            data = f.read()
        return Response(data, media_type=media,
                        headers={"Content-Disposition": f'filename="{os.path.basename(p)}"'})

    @app.get("/system_stats")
    def system_stats():
        devs = []
        if torch.cuda.is_available():
            for i in range(torch.cuda.device_count()):
                free, total = torch.cuda.mem_get_info(i)
                devs.append({"name": torch.cuda.get_device_name(i), "type": "cuda", "index": i,
                             "vram_total": total, "vram_free": free})
        return {"system": {"os": os.name, "python_version": "", "embedded_python": False,
                           "pytorch_version": torch.__version__, "backend": "in-tree Wan2.1 (gfx950)"},
                "devices": devs}

    @app.get("/metrics")
    def metrics():
        st = pq.stats
        lines = ["# TYPE wan_prompts_total counter"]
        for k in ("completed", "failed", "interrupted"):
            lines.append(f'wan_prompts_total{{status="{k}"}} {st[k]}')
        lines += ["# TYPE wan_execution_seconds_total counter",
                  f"wan_execution_seconds_total {st['exec_seconds']:.3f}",
                  "# TYPE wan_queue_remaining gauge", f"wan_queue_remaining {pq.remaining()}"]
        return PlainTextResponse("\n".join(lines) + "\n")

    return app


# ----------------------------------------------------------------------------------- synthetic mode
def synthetic_store(device: str = "cuda", tiny: bool = False) -> ModelStore:
    """Random-init components of the published architectures under the reference's file names
    (benchmarks, smoke tests, a cluster with no checkpoints yet)."""
    from ..comfy_client import WAN_MODELS
    from .config import UMT5Config, WanDiTConfig, WanVAEConfig
    from .dit import WanDiT
    from .pipeline import _ByteTokenizer
    from .t5 import UMT5Encoder

    def init(mod):
        with torch.no_grad():
            for n, p in mod.named_parameters():
                if p.dim() >= 2 and "modulation" not in n:
                    p.normal_(0.0, p[0].numel() ** -0.5)
        return mod

    dev = torch.device(device)
    dc = WanDiTConfig.tiny() if tiny else WanDiTConfig.wan21_t2v_1_3b()
    tc = UMT5Config.tiny(vocab=300) if tiny else UMT5Config.umt5_xxl()
    vc = WanVAEConfig.tiny() if tiny else WanVAEConfig.wan21()
    if tiny:
        dc = WanDiTConfig(dim=dc.dim, ffn_dim=dc.ffn_dim, freq_dim=dc.freq_dim, heads=dc.heads,
                          layers=dc.layers, text_dim=tc.dim)

    def mk(kind):
        def load(_path):
            torch.manual_seed({"unet": 0, "clip": 1, "vae": 2}[kind])
            with torch.device(dev):
                if kind == "unet":
                    return init(WanDiT(dc))
                if kind == "clip":
                    return (init(UMT5Encoder(tc)), _ByteTokenizer(tc.vocab))
                from .vae import WanVAE
                return init(WanVAE(vc))
        return load

    return ModelStore("/nonexistent", device, torch.float32 if tiny else torch.bfloat16,
                      loaders={k: mk(k) for k in ("unet", "clip", "vae")},
                      listing={k: [WAN_MODELS[k]] for k in ("unet", "clip", "vae")})


def main(argv=None) -> int:  # pragma: no cover - container entry point
    import argparse

    import uvicorn

    ap = argparse.ArgumentParser(description="ComfyUI-compatible Wan2.1 server (in-tree, MI355X)")
    ap.add_argument("--listen", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8181)
    ap.add_argument("--base-directory", default=os.environ.get("COMFY_BASE", "/data"))
    ap.add_argument("--output-directory", default=None)
    ap.add_argument("--shift", type=float, default=8.0)
    ap.add_argument("--warmup", default=os.environ.get("WAN_WARMUP", ""),
                    help="WxHxF: run one 1-step job of that size before /queue reports ready")
    ap.add_argument("--synthetic", action="store_true",
                    help="random-init weights under the reference file names (no checkpoints)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s %(message)s")
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    store = synthetic_store(dev) if a.synthetic else ModelStore(a.base_directory, dev)
    out = a.output_directory or os.path.join(a.base_directory, "output")
    warm = tuple(int(v) for v in a.warmup.lower().split("x")) if a.warmup else None
    uvicorn.run(create_app(store, out, a.shift, warmup=warm), host=a.listen, port=a.port)
    return 0


if __name__ == "__main__":  # pragma: no cover
    raise SystemExit(main())
