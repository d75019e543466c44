#!/bin/bash
# Round 3 session E: the wave-grid GEMM family (256x128 / 128x128 / 128x64 / 64x64 tiles) and the
# w4a bias / GELU / gated-residual / fp16 epilogues — GPU tests, SD1.5 + Wan shape probes, then
# the SD1.5 UNet pass and the Wan CFG step at 2560 and 32 760 tokens.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_epi_gpu.py > $OUT/gemm_epi_tests.log 2>&1 || { tail -40 $OUT/gemm_epi_tests.log; exit 1; }
tail -2 $OUT/gemm_epi_tests.log
MODE=sd timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_probe_sd.log 2>&1 || { tail -20 $OUT/gemm_probe_sd.log; exit 1; }
grep -v '^{' $OUT/gemm_probe_sd.log | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_probe_wan.log 2>&1 || { tail -20 $OUT/gemm_probe_wan.log; exit 1; }
grep -v '^{' $OUT/gemm_probe_wan.log | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_sd15_gpu.py tests/test_wan_gpu.py > $OUT/pytest_models.log 2>&1 || { tail -40 $OUT/pytest_models.log; exit 1; }
tail -2 $OUT/pytest_models.log
timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 --miopen-find \
  --out $OUT/sd15_bench.json > $OUT/sd15_bench.log 2>&1 || { tail -20 $OUT/sd15_bench.log; exit 1; }
grep -E "unet|e2e" $OUT/sd15_bench.log
timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
  --out $OUT/wan_bench_2560.json > $OUT/wan_bench_2560.log 2>&1 || { tail -20 $OUT/wan_bench_2560.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560.log
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --no-e2e --width 832 --height 480 \
  --frames 81 --iters 3 --warmup 1 --out $OUT/wan_bench_32760.json > $OUT/wan_bench_32760.log 2>&1 \
  || { tail -20 $OUT/wan_bench_32760.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_32760.log
