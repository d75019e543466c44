"""Stable Diffusion 1.5 text-to-image REST service for one MI355X (PyTorch-ROCm).

Same HTTP surface as the reference's SD15 app (reference cluster-config/apps/sd15-api/configmap.yaml:
16-121): ``GET /healthz``, ``GET /`` (HTML preview of the last image), ``GET /last`` (PNG),
``POST /generate`` (``{prompt, steps=30, guidance_scale=7.5, seed, width=512, height=512}`` → PNG
with an ``X-Gen-Time`` header).  Redesigned for a 288 GB GPU shared by concurrent clients:

* **One GPU worker, request coalescing.**  The reference calls ``pipe(...)`` from FastAPI's thread
  pool, so concurrent requests run the pipeline concurrently on one GPU (SURVEY.md §3.4 hazard).
  Here a single worker thread owns the pipeline; requests wait in a queue, and requests with the
  same (steps, guidance, width, height) that arrive together run as ONE batched UNet pass
  (``MAX_BATCH``; each keeps its own seeded generator, so outputs match an unbatched run).
  Batching the UNet is what fills 256 CUs: a single 64×64 latent with CFG is batch 2.
* **No memory-saving slicing by default.**  ``enable_attention_slicing`` / ``enable_vae_slicing``
  exist for 6-8 GB consumer cards (reference configmap.yaml:42-43); on 288 GB they only cost time.
  Both stay switchable (``ATTENTION_SLICING`` / ``VAE_SLICING``).
* **Readiness separate from liveness.**  The model loads in the background; ``/readyz`` is 503
  until it is on the GPU, ``/healthz`` answers immediately (the reference loads at import time, so
  the pod is unreachable while weights download).
* ``_LAST_IMAGE`` is read and written under one lock (the reference reads it unlocked).
* ``/metrics``: Prometheus counters/histograms for requests, latency and batch size.

* **In-tree model, no diffusers.**  The default pipeline is this repository's SD1.5
  (``k8s_nvidia_gpus_amd/models/sd15``: HIP GroupNorm / attention / fused epilogues, the UNet pass
  replayed from a HIP graph), loading the same checkpoint files from ``MODEL_DIR``.  Before the pod
  reports ready it warms up every batch size in ``WARMUP_BATCHES`` (MIOpen solver search + graph
  capture happen then, not on the first user request).  ``PIPELINE=diffusers`` keeps the upstream
  library path for images that ship diffusers.

``create_app(pipeline_factory=...)`` takes the pipeline constructor so tests run the whole HTTP +
batching path on CPU with a fake or a miniature in-tree pipeline.
"""
from __future__ import annotations

import base64
import io
import logging
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional

logger = logging.getLogger("sd15-api")

DEFAULT_MODEL_ID = "stable-diffusion-v1-5/stable-diffusion-v1-5"


def _env_bool(name: str, default: bool) -> bool:
    v = os.getenv(name)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


@dataclass
class Settings:
    model_id: str = DEFAULT_MODEL_ID
    dtype: str = "float16"            # float16 | bfloat16 | float32
    device: str = "cuda"              # torch's name for the HIP device on ROCm
    attention_slicing: bool = False
    vae_slicing: bool = False
    vae_cpu: bool = False
    max_batch: int = 8
    batch_window_ms: float = 15.0     # how long the worker waits to coalesce compatible requests
    max_steps: int = 150
    max_side: int = 2048
    queue_limit: int = 256
    request_timeout_s: float = 600.0
    pipeline: str = "native"          # native (in-tree SD1.5) | diffusers
    model_dir: str = ""               # diffusers-layout checkpoint directory (native pipeline)
    scheduler: str = "pndm"           # pndm | ddim | euler (native pipeline)
    hip_graphs: bool = True
    warmup_batches: str = "1"         # batch sizes captured before /readyz turns green
    model_config: str = "sd15"        # sd15 | tiny (tests)

    @classmethod
    def from_env(cls) -> "Settings":
        return cls(
            model_id=os.getenv("MODEL_ID", DEFAULT_MODEL_ID),
            dtype=os.getenv("TORCH_DTYPE", "float16"),
            device=os.getenv("DEVICE", "cuda"),
            attention_slicing=_env_bool("ATTENTION_SLICING", False),
            vae_slicing=_env_bool("VAE_SLICING", False),
            vae_cpu=_env_bool("VAE_CPU", False),
            max_batch=int(os.getenv("MAX_BATCH", "8")),
            batch_window_ms=float(os.getenv("BATCH_WINDOW_MS", "15")),
            max_steps=int(os.getenv("MAX_STEPS", "150")),
            max_side=int(os.getenv("MAX_SIDE", "2048")),
            queue_limit=int(os.getenv("QUEUE_LIMIT", "256")),
            request_timeout_s=float(os.getenv("REQUEST_TIMEOUT_S", "600")),
            pipeline=os.getenv("PIPELINE", "native"),
            model_dir=os.getenv("MODEL_DIR", ""),
            scheduler=os.getenv("SCHEDULER", "pndm"),
            hip_graphs=_env_bool("HIP_GRAPHS", True),
            warmup_batches=os.getenv("WARMUP_BATCHES", "1"),
            model_config=os.getenv("MODEL_CONFIG", "sd15"),
        )


def load_native_pipeline(settings: Settings):
    """In-tree SD1.5 (``models/sd15``) on the ROCm device; random-init weights without MODEL_DIR."""
    from k8s_nvidia_gpus_amd.models.sd15.pipeline import load_native_pipeline as _load

    return _load(settings)


def load_pipeline(settings: Settings):
    if settings.pipeline == "diffusers":
        return load_diffusers_pipeline(settings)
    if settings.pipeline != "native":
        raise ValueError(f"PIPELINE={settings.pipeline!r} (native | diffusers)")
    return load_native_pipeline(settings)


def load_diffusers_pipeline(settings: Settings):
    """Production pipeline: diffusers SD1.5 on the ROCm device."""
    import torch
    from diffusers import StableDiffusionPipeline  # only present in the serving image

    dtype = getattr(torch, settings.dtype)
    use_gpu = torch.cuda.is_available() and settings.device.startswith("cuda")
    if not use_gpu:
        dtype = torch.float32
    pipe = StableDiffusionPipeline.from_pretrained(settings.model_id, torch_dtype=dtype)
    if settings.attention_slicing:
        pipe.enable_attention_slicing()
    if settings.vae_slicing:
        pipe.enable_vae_slicing()
    pipe.set_progress_bar_config(disable=True)
    if use_gpu:
        pipe = pipe.to(settings.device)
        if settings.vae_cpu:
            pipe.vae.to("cpu")
        logger.info("loaded %s on %s (%s)", settings.model_id,
                    torch.cuda.get_device_name(0), dtype)
    else:
        logger.warning("no GPU visible: running %s on CPU", settings.model_id)
    return pipe


def _make_generator(seed: Optional[int], device: str):
    if seed is None:
        return None
    import torch

    dev = device if (device.startswith("cuda") and torch.cuda.is_available()) else "cpu"
    return torch.Generator(device=dev).manual_seed(int(seed))


@dataclass
class _Job:
    prompt: str
    steps: int
    guidance: float
    width: int
    height: int
    seed: Optional[int]
    negative_prompt: Optional[str] = None
    done: threading.Event = field(default_factory=threading.Event)
    png: Optional[bytes] = None
    image: Any = None                 # PIL image from the GPU worker; PNG-encoded by the request thread
    error: Optional[BaseException] = None
    batch_size: int = 0
    t_enqueue: float = field(default_factory=time.time)

    def key(self):
        return (self.steps, round(self.guidance, 4), self.width, self.height)


class GenerationWorker:
    """Owns the pipeline; runs queued jobs one batch at a time on the GPU."""

    def __init__(self, settings: Settings, pipeline_factory: Callable[[Settings], Any]):
        self.settings = settings
        self._factory = pipeline_factory
        self._pipe = None
        self._load_error: Optional[BaseException] = None
        self._q: "queue.Queue[_Job]" = queue.Queue(maxsize=settings.queue_limit)
        self._stop = threading.Event()
        self._ready = threading.Event()
        self._thread = threading.Thread(target=self._run, name="sd15-gpu-worker", daemon=True)
        self.batches_run = 0
        self.images_done = 0

    # -- lifecycle --
    def start(self) -> None:
        self._thread.start()

    def stop(self, timeout: float = 5.0) -> None:
        self._stop.set()
        self._thread.join(timeout)

    @property
    def ready(self) -> bool:
        return self._ready.is_set()

    @property
    def load_error(self) -> Optional[BaseException]:
        return self._load_error

    def wait_ready(self, timeout: Optional[float] = None) -> bool:
        return self._ready.wait(timeout)

    def submit(self, job: _Job) -> None:
        self._q.put_nowait(job)  # raises queue.Full → HTTP 503

    def queue_depth(self) -> int:
        return self._q.qsize()

    # -- worker loop --
    def _run(self) -> None:
        try:
            self._pipe = self._factory(self.settings)
            self._warmup()
        except BaseException as e:  # noqa: BLE001 - surfaced through /readyz
            logger.exception("pipeline load failed")
            self._load_error = e
            return
        self._ready.set()
        pending: List[_Job] = []
        while not self._stop.is_set():
            if not pending:
                try:
                    pending.append(self._q.get(timeout=0.2))
                except queue.Empty:
                    continue
            # coalesce: take everything already queued, wait briefly for stragglers
            deadline = time.time() + self.settings.batch_window_ms / 1000.0
            while True:
                try:
                    pending.append(self._q.get_nowait())
                except queue.Empty:
                    if time.time() >= deadline:
                        break
                    time.sleep(0.001)
            head = pending[0].key()
            batch = [j for j in pending if j.key() == head][: self.settings.max_batch]
            ids = {id(j) for j in batch}
            pending = [j for j in pending if id(j) not in ids]
            self._run_batch(batch)

    def _warmup(self) -> None:
        """Run each WARMUP_BATCHES size once at the default request shape (2 steps): the native
        pipeline captures its HIP graph per batch size and MIOpen picks its solvers here, so the
        first real request of that size runs at steady-state speed."""
        sizes = [int(x) for x in str(self.settings.warmup_batches).split(",") if x.strip()]
        if not sizes or not getattr(self._pipe, "native_pipeline", False):
            return
        for b in sizes:
            t0 = time.time()
            self._pipe(["warmup"] * b, num_inference_steps=2, guidance_scale=7.5, width=512,
                       height=512, output_type="latent")
            logger.info("warm-up batch %d: %.2fs", b, time.time() - t0)

    def _run_batch(self, batch: List[_Job]) -> None:
        import contextlib

        j0 = batch[0]
        gens = [_make_generator(j.seed, self.settings.device) for j in batch]
        kwargs = dict(
            prompt=[j.prompt for j in batch],
            num_inference_steps=j0.steps,
            guidance_scale=j0.guidance,
            width=j0.width,
            height=j0.height,
        )
        if any(j.negative_prompt for j in batch):
            kwargs["negative_prompt"] = [j.negative_prompt or "" for j in batch]
        if any(g is not None for g in gens):
            # unseeded requests in a seeded batch get a fresh random seed each
            import random

            kwargs["generator"] = [g if g is not None else
                                   _make_generator(random.getrandbits(63), self.settings.device)
                                   for g in gens]
        try:
            ctx = contextlib.nullcontext()
            try:
                import torch

                if torch.cuda.is_available() and self.settings.device.startswith("cuda") \
                        and self.settings.dtype != "float32" \
                        and not getattr(self._pipe, "native_pipeline", False):
                    ctx = torch.autocast(device_type="cuda", dtype=getattr(torch, self.settings.dtype))
            except ImportError:  # pragma: no cover - torch is always in the serving image
                pass
            with ctx:
                images = self._pipe(**kwargs).images
            if len(images) != len(batch):
                raise RuntimeError(f"pipeline returned {len(images)} images for {len(batch)} prompts")
            # PNG encoding (~25 ms per 512² image) happens in each request's own thread, not here:
            # the GPU worker moves straight on to the next coalesced batch
            for j, img in zip(batch, images):
                j.image = img
                j.batch_size = len(batch)
        except BaseException as e:  # noqa: BLE001 - delivered to every waiting request
            logger.exception("generation failed")
            for j in batch:
                j.error = e
        finally:
            self.batches_run += 1
            self.images_done += len(batch)
            for j in batch:
                j.done.set()


try:
    from pydantic import BaseModel

    class GenReq(BaseModel):
        """Request body of POST /generate (same fields and defaults as the reference's GenReq)."""

        prompt: str
        steps: Optional[int] = 30
        guidance_scale: Optional[float] = 7.5
        seed: Optional[int] = None
        width: Optional[int] = 512
        height: Optional[int] = 512
        negative_prompt: Optional[str] = None
except ImportError:  # pragma: no cover - pydantic ships with fastapi in the serving image
    GenReq = None


def create_app(settings: Optional[Settings] = None,
               pipeline_factory: Optional[Callable[[Settings], Any]] = None):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import HTMLResponse, PlainTextResponse, Response

    try:
        import prometheus_client as prom
    except ImportError:  # pragma: no cover
        prom = None

    settings = settings or Settings.from_env()
    worker = GenerationWorker(settings, pipeline_factory or load_pipeline)
    state = {"last": None}
    last_lock = threading.Lock()

    registry = prom.CollectorRegistry() if prom else None
    if prom:
        m_req = prom.Counter("sd15_requests_total", "generate requests", ["status"], registry=registry)
        m_lat = prom.Histogram("sd15_generate_seconds", "end-to-end generate latency",
                               buckets=(0.25, 0.5, 1, 2, 4, 8, 16, 32, 64, 128), registry=registry)
        m_batch = prom.Histogram("sd15_batch_size", "images per GPU batch",
                                 buckets=(1, 2, 4, 8, 16, 32), registry=registry)
        prom.Gauge("sd15_queue_depth", "queued requests", registry=registry).set_function(
            worker.queue_depth)

    app = FastAPI(title="SD1.5 API (MI355X)")
    app.state.worker = worker
    app.state.settings = settings

    @app.on_event("startup")
    def _startup():
        worker.start()

    @app.on_event("shutdown")
    def _shutdown():
        worker.stop()

    @app.get("/healthz")
    def healthz():
        return {"ok": True}

    @app.get("/readyz")
    def readyz():
        if worker.load_error is not None:
            raise HTTPException(500, f"model load failed: {worker.load_error}")
        if not worker.ready:
            raise HTTPException(503, "model loading")
        return {"ready": True, "model": settings.model_id}

    @app.get("/", response_class=HTMLResponse)
    def index():
        with last_lock:
            last = state["last"]
        if last is None:
            return ("<h1>SD1.5 on MI355X</h1><p>No image generated yet. "
                    "POST /generate to create one.</p>")
        b64 = base64.b64encode(last).decode("ascii")
        return ("<html><head><title>SD1.5</title></head><body style='font-family:sans-serif'>"
                "<h1>Latest image</h1>"
                f"<img src='data:image/png;base64,{b64}' alt='latest image' style='max-width:90vw'/>"
                "</body></html>")

    @app.get("/last")
    def last_image():
        with last_lock:
            last = state["last"]
        if last is None:
            raise HTTPException(404, "No image generated yet")
        return Response(content=last, media_type="image/png")

    @app.get("/metrics")
    def metrics():
        if not prom:
            raise HTTPException(404, "prometheus_client missing")
        return PlainTextResponse(prom.generate_latest(registry).decode(),
                                 media_type=prom.CONTENT_TYPE_LATEST)

    @app.post("/generate")
    def generate(req: GenReq):
        prompt = (req.prompt or "").strip()
        steps = req.steps if req.steps is not None else 30
        guidance = req.guidance_scale if req.guidance_scale is not None else 7.5
        width = req.width if req.width is not None else 512
        height = req.height if req.height is not None else 512
        if not prompt:
            raise HTTPException(400, "prompt is required")
        if not 1 <= steps <= settings.max_steps:
            raise HTTPException(400, f"steps must be in [1, {settings.max_steps}]")
        for name, v in (("width", width), ("height", height)):
            if v % 8 or not 64 <= v <= settings.max_side:
                raise HTTPException(400, f"{name} must be a multiple of 8 in [64, {settings.max_side}]")
        if worker.load_error is not None:
            raise HTTPException(500, "model failed to load")
        job = _Job(prompt=prompt, steps=steps, guidance=float(guidance), width=width,
                   height=height, seed=req.seed, negative_prompt=req.negative_prompt)
        t0 = time.time()
        try:
            worker.submit(job)
        except queue.Full:
            if prom:
                m_req.labels("busy").inc()
            raise HTTPException(503, "queue full")
        if not job.done.wait(settings.request_timeout_s):
            if prom:
                m_req.labels("timeout").inc()
            raise HTTPException(504, "generation timed out")
        if job.error is not None:
            if prom:
                m_req.labels("error").inc()
            raise HTTPException(500, f"generation failed: {job.error}")
        if job.png is None:
            buf = io.BytesIO()
            job.image.save(buf, format="PNG")
            job.png = buf.getvalue()
            job.image = None
        latency = time.time() - t0
        with last_lock:
            state["last"] = job.png
        if prom:
            m_req.labels("ok").inc()
            m_lat.observe(latency)
            m_batch.observe(job.batch_size)
        logger.info("generated %dx%d steps=%d batch=%d in %.2fs", width, height, steps,
                    job.batch_size, latency)
        return Response(content=job.png, media_type="image/png",
                        headers={"X-Gen-Time": f"{latency:.2f}s",
                                 "X-Batch-Size": str(job.batch_size)})

    return app


def main() -> None:  # pragma: no cover - container entry point
    import uvicorn

    logging.basicConfig(level=logging.INFO)
    uvicorn.run(create_app(), host="0.0.0.0", port=int(os.getenv("PORT", "8000")))


if __name__ == "__main__":  # pragma: no cover
    main()
