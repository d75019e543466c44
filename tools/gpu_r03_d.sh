#!/bin/bash
# Round 3 session D: GEMM epilogue kernels after the read/MFMA interleave + the w4a wide-projection
# path (tests, probe), then the Wan CFG step at 2560 and 32 760 tokens.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r03/d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_epi_gpu.py > $OUT/gemm_epi_tests.log 2>&1 || { tail -40 $OUT/gemm_epi_tests.log; exit 1; }
tail -2 $OUT/gemm_epi_tests.log
timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_epi_probe.log 2>&1 || { tail -20 $OUT/gemm_epi_probe.log; exit 1; }
grep -v '^{' $OUT/gemm_epi_probe.log | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
  --out $OUT/wan_bench_2560.json > $OUT/wan_bench_2560.log 2>&1 || { tail -20 $OUT/wan_bench_2560.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560.log
AMDK8S_GEMM_WIDE=epi timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
  --out $OUT/wan_bench_2560_nowide.json > $OUT/wan_bench_2560_nowide.log 2>&1 || { tail -20 $OUT/wan_bench_2560_nowide.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560_nowide.log
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --no-e2e --width 832 --height 480 \
  --frames 81 --iters 3 --warmup 1 --out $OUT/wan_bench_32760.json > $OUT/wan_bench_32760.log 2>&1 \
  || { tail -20 $OUT/wan_bench_32760.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_32760.log
