#!/bin/bash
# Round 3 session I: planner v2 (unsplit 160+-WG grids, split target 192) — GEMM tests, SD1.5
# UNet pass + e2e + steady-state profile, SD GEMM probe.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_epi_gpu.py > $OUT/gemm_epi_tests.log 2>&1 || { tail -40 $OUT/gemm_epi_tests.log; exit 1; }
tail -2 $OUT/gemm_epi_tests.log
timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 --miopen-find \
  --out $OUT/sd15_bench.json > $OUT/sd15_bench.log 2>&1 || { tail -20 $OUT/sd15_bench.log; exit 1; }
grep -E "unet|e2e" $OUT/sd15_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_sd15 -o sd15 -- \
  python3 tools/steady_prof.py sd15-unet --iters 20 > $OUT/prof_sd15.log 2>&1 || { tail -20 $OUT/prof_sd15.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_sd15 -name '*.db' | head -1) --after-gap-ms 200 --per 20 \
  --top 60 > $OUT/sd15_unet_steady_kernels.txt && head -40 $OUT/sd15_unet_steady_kernels.txt
