#!/bin/bash
# Round 3 session B: fused-epilogue GEMM (tests vs fp32, probe vs hipBLASLt on the DiT shapes),
# then the Wan CFG step with the new GEMM + attention (A/B: AMDK8S_WAN_GEMM=torch keeps hipBLASLt).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r03/b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_sd15_gpu.py -k attention > $OUT/attn_tests.log 2>&1 || { tail -40 $OUT/attn_tests.log; exit 1; }
tail -2 $OUT/attn_tests.log
ATTN_VARIANTS=0,2 timeout -k 10 300 python -u tools/attn_probe.py > $OUT/attn_probe.log 2>&1 || { tail -20 $OUT/attn_probe.log; exit 1; }
grep -v '^{' $OUT/attn_probe.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gemm_epi_gpu.py > $OUT/gemm_epi_tests.log 2>&1 || { tail -40 $OUT/gemm_epi_tests.log; exit 1; }
tail -3 $OUT/gemm_epi_tests.log
timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_epi_probe.log 2>&1 || { tail -20 $OUT/gemm_epi_probe.log; exit 1; }
grep -v '^{' $OUT/gemm_epi_probe.log
timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph,native --no-e2e \
  --out $OUT/wan_bench_2560.json > $OUT/wan_bench_2560.log 2>&1 || { tail -20 $OUT/wan_bench_2560.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560.log
AMDK8S_WAN_GEMM=torch timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
  --out $OUT/wan_bench_2560_blt.json > $OUT/wan_bench_2560_blt.log 2>&1 || { tail -20 $OUT/wan_bench_2560_blt.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560_blt.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_wan_gpu.py > $OUT/pytest_wan.log 2>&1 || { tail -40 $OUT/pytest_wan.log; exit 1; }
tail -2 $OUT/pytest_wan.log
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --no-e2e --width 832 --height 480 \
  --frames 81 --iters 3 --warmup 1 --out $OUT/wan_bench_32760.json > $OUT/wan_bench_32760.log 2>&1 \
  || { tail -20 $OUT/wan_bench_32760.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_32760.log
