set -euo pipefail
timeout -k 10 120 tools/debug/gemv_probe
Q8=1 timeout -k 10 120 tools/debug/gemv_probe
