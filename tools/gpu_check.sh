#!/usr/bin/env bash
# One GPU-box pass: GPU tests, native validators, bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; steps are chained so the first failure ends the call.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
STEP="${1:-all}"
run() { echo "=== $*" ; }
if [[ "$STEP" == all || "$STEP" == tests ]]; then
  run pytest -m gpu
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -5 gpurun_out/pytest_gpu.log
fi
if [[ "$STEP" == all || "$STEP" == native ]]; then
  run native tools
  timeout -k 10 120 native/bin/amd-vectoradd --json --bandwidth 3000000000 | tee gpurun_out/vectoradd.log
  timeout -k 10 300 native/bin/amd-gemm-validator --size 8192 --iters 50 --json | tee gpurun_out/gemm_validator.log
  timeout -k 10 120 native/bin/rccl-allreduce-bench -b 1M -e 256M -f 4 --json | tee gpurun_out/rccl.log
fi
if [[ "$STEP" == all || "$STEP" == bench ]]; then
  run bench
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 | tee gpurun_out/bench.json
fi
if [[ "$STEP" == all || "$STEP" == prof ]]; then
  run rocprofv3
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
echo "=== gpu_check done"
