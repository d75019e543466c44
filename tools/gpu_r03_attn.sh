#!/bin/bash
# Round 3: attn_d128 correctness (GPU tests) then the attention probe sweep.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_sd15_gpu.py -k "attention" > gpurun_out/r03/attn_tests.log 2>&1 || { tail -40 gpurun_out/r03/attn_tests.log; exit 1; }
tail -5 gpurun_out/r03/attn_tests.log
timeout -k 10 300 python -u tools/attn_probe.py > gpurun_out/r03/attn_probe.log 2>&1 || { tail -30 gpurun_out/r03/attn_probe.log; exit 1; }
grep -v '^{' gpurun_out/r03/attn_probe.log
