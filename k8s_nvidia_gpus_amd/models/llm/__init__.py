"""In-tree Qwen2 (Qwen2.5-7B-Instruct Q4_K_M GGUF) inference engine and llama-server-compatible
API for MI355X — the model family behind the reference's ``llm`` app (reference
cluster-config/apps/llm/deployment.yaml)."""
from .config import LLMConfig, QWEN25_7B, tiny  # noqa: F401
