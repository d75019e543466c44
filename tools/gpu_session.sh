#!/usr/bin/env bash
# One GPU-box pass: GPU pytest (kernels + operator components on real hardware), bench.py,
# rocprofv3 kernel stats of the bench. Each GPU step has its own time limit; first failure ends it.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/session
export AMDK8S_EVIDENCE_DIR=gpurun_out/session/evidence
echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:warnings > gpurun_out/session/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/session/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/session/pytest_gpu.log
echo "== bench.py (defaults)"
timeout -k 10 600 python bench.py > gpurun_out/session/bench.json 2> gpurun_out/session/bench.err || { cat gpurun_out/session/bench.err | tail -20; exit 1; }
cat gpurun_out/session/bench.json
echo "== native validator (bf16 + fp8)"
timeout -k 10 300 native/bin/amd-gemm-validator --size 8192 --iters 50 --json > gpurun_out/session/gemm_validator_bf16.log 2>&1
timeout -k 10 300 native/bin/amd-gemm-validator --dtype fp8 --size 8192 --iters 50 --json > gpurun_out/session/gemm_validator_fp8.log 2>&1
grep -h '"check"' gpurun_out/session/gemm_validator_*.log
if [[ "${PROFILE:-1}" == 1 ]]; then
  echo "== rocprofv3 kernel stats"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/session/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/session/prof.log 2>&1 || { tail -20 gpurun_out/session/prof.log; exit 1; }
  find gpurun_out/session/prof -name "*kernel_stats.csv" -exec head -5 {} \;
fi
echo "== done"
