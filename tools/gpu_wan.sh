#!/usr/bin/env bash
# GPU pass for the Wan2.1 family: kernel/model numerics, T2V-1.3B bench, rocprofv3 kernel stats.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT="${OUT:-gpurun_out/wan}"
mkdir -p "$OUT"
echo "== pytest wan gpu"
timeout -k 10 600 python -u -m pytest tests/test_wan_gpu.py -x -v -s -p no:warnings --timeout 300 --timeout-method thread > "$OUT/pytest_wan.log" 2>&1 || { tail -60 "$OUT/pytest_wan.log"; exit 1; }
tail -3 "$OUT/pytest_wan.log"
echo "== wan bench"
timeout -k 10 900 python -u tools/wan_bench.py ${WAN_ARGS:-} --out "$OUT/wan_bench.json" > "$OUT/wan_bench.log" 2>&1 || { tail -30 "$OUT/wan_bench.log"; exit 1; }
tail -5 "$OUT/wan_bench.log"
if [[ "${PROFILE:-1}" == 1 ]]; then
  echo "== rocprof wan"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o wan --output-format csv -- python3 tools/wan_bench.py --arms native --iters 3 --warmup 1 --no-e2e > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
  find "$OUT/prof" -name "*kernel_stats.csv" -exec head -25 {} \;
fi
echo "== done"
