"""Stable Diffusion 1.5 model family, in-tree and MI355X-native (see ``pipeline.py``)."""
from .config import SD15, SD15Config, tiny  # noqa: F401
from .pipeline import StableDiffusion, UNetRunner, load_native_pipeline  # noqa: F401
