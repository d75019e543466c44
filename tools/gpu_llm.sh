#!/usr/bin/env bash
# GPU pass for the LLM engine: kernel/engine numerics, Qwen2.5-7B decode bench, rocprofv3 stats.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT="${OUT:-gpurun_out/llm}"
mkdir -p "$OUT"
echo "== pytest llm gpu"
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -v -p no:warnings --timeout 200 --timeout-method thread > "$OUT/pytest_llm.log" 2>&1 || { tail -60 "$OUT/pytest_llm.log"; exit 1; }
tail -3 "$OUT/pytest_llm.log"
echo "== llm bench"
timeout -k 10 600 python -u tools/llm_bench.py --gemv --kernels --out "$OUT/llm_bench.json" > "$OUT/llm_bench.log" 2>&1 || { tail -30 "$OUT/llm_bench.log"; exit 1; }
grep -v '^{' "$OUT/llm_bench.log" | tail -20
if [[ "${PROFILE:-1}" == 1 ]]; then
  echo "== rocprof llm"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o llm --output-format csv -- python3 tools/llm_bench.py --steps 32 --tokens 1 --prompt 128 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
  find "$OUT/prof" -name "*kernel_stats.csv" -exec head -16 {} \;
fi
echo "== done"
