#!/bin/bash
# Round 3 session H: split-K via per-split workspace slices + the joint tile/split planner; conv
# probe (hand conv under every (tile, split) vs MIOpen per SD1.5 shape), SD GEMM probe, SD1.5 and
# Wan (stacked fp32 modulations, no Cijk) benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/h
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_epi_gpu.py > $OUT/gemm_epi_tests.log 2>&1 || { tail -40 $OUT/gemm_epi_tests.log; exit 1; }
tail -2 $OUT/gemm_epi_tests.log
timeout -k 10 500 python -u tools/conv_probe.py > $OUT/conv_probe.log 2>&1 || { tail -20 $OUT/conv_probe.log; exit 1; }
grep -v '^{' $OUT/conv_probe.log | grep -v amdgpu.ids
MODE=sd timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_probe_sd.log 2>&1 || { tail -20 $OUT/gemm_probe_sd.log; exit 1; }
grep -v '^{' $OUT/gemm_probe_sd.log | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_wan_gpu.py > $OUT/pytest_wan.log 2>&1 || { tail -40 $OUT/pytest_wan.log; exit 1; }
tail -2 $OUT/pytest_wan.log
timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
  --out $OUT/wan_bench_2560.json > $OUT/wan_bench_2560.log 2>&1 || { tail -20 $OUT/wan_bench_2560.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560.log
timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 --miopen-find \
  --out $OUT/sd15_bench.json > $OUT/sd15_bench.log 2>&1 || { tail -20 $OUT/sd15_bench.log; exit 1; }
grep -E "unet|e2e" $OUT/sd15_bench.log
