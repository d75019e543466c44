set -euo pipefail
timeout -k 10 300 python -u tools/debug/llm_batch_debug.py
