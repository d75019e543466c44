set -euo pipefail
timeout -k 10 120 tools/debug/attn_phases
