#!/usr/bin/env bash
# One GPU-box pass: GPU pytest (kernels + operator components on real hardware), bench.py,
# native validators + amd-proftester, GEMM A/B vs hipBLASLt, rocprofv3 kernel stats of the bench.
# Each GPU step has its own time limit; the first failure ends the call.  OUT=gpurun_out/<dir>.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT="${OUT:-gpurun_out/session}"
mkdir -p "$OUT"
export AMDK8S_EVIDENCE_DIR="$OUT/evidence"
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:warnings --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "== bench.py (defaults)"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== native validator (bf16 + fp8) + proftester"
timeout -k 10 300 native/bin/amd-gemm-validator --size 8192 --iters 50 --json > "$OUT/gemm_validator_bf16.log" 2>&1
timeout -k 10 300 native/bin/amd-gemm-validator --dtype fp8 --size 8192 --iters 50 --json > "$OUT/gemm_validator_fp8.log" 2>&1
grep -h '"check"' "$OUT"/gemm_validator_*.log
timeout -k 10 300 native/bin/amd-proftester --json > "$OUT/proftester_all.log" 2>&1
grep -v '^{' "$OUT/proftester_all.log"
if [[ "${AB:-1}" == 1 ]]; then
  echo "== GEMM A/B vs hipBLASLt"
  timeout -k 10 300 python tools/gemm_ab.py --sizes 8192 16384 > "$OUT/gemm_ab.txt" 2>&1
  tail -8 "$OUT/gemm_ab.txt"
fi
if [[ "${PROFILE:-1}" == 1 ]]; then
  echo "== rocprofv3 kernel stats"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
  find "$OUT/prof" -name "*kernel_stats.csv" -exec head -5 {} \;
fi
echo "== done"
