#!/bin/bash
# Round 3 session C: SD1.5 with the hand-written GEMM + 32x32x16 attention (GPU tests, UNet-pass
# bench with the hipBLASLt A/B, end-to-end img/s), then steady-state rocprofv3 kernel profiles of
# one SD1.5 UNet CFG pass and one Wan2.1 CFG DiT step (kernel trace only; no counters).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/c
mkdir -p $OUT
timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_epi_probe_w4a.log 2>&1 || { tail -20 $OUT/gemm_epi_probe_w4a.log; exit 1; }
grep -v '^{' $OUT/gemm_epi_probe_w4a.log | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_sd15_gpu.py > $OUT/pytest_sd15.log 2>&1 || { tail -40 $OUT/pytest_sd15.log; exit 1; }
tail -2 $OUT/pytest_sd15.log
timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 --miopen-find \
  --out $OUT/sd15_bench.json > $OUT/sd15_bench.log 2>&1 || { tail -20 $OUT/sd15_bench.log; exit 1; }
grep -E "unet|e2e" $OUT/sd15_bench.log
AMDK8S_SD_GEMM=torch timeout -k 10 400 python -u tools/sd15_bench.py --arms native-graph --batches "" \
  --miopen-find --out $OUT/sd15_bench_blt.json > $OUT/sd15_bench_blt.log 2>&1 || { tail -20 $OUT/sd15_bench_blt.log; exit 1; }
grep -E "unet" $OUT/sd15_bench_blt.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_sd15 -o sd15 -- \
  python3 tools/steady_prof.py sd15-unet --iters 20 > $OUT/prof_sd15.log 2>&1 || { tail -20 $OUT/prof_sd15.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_sd15 -name '*.db' | head -1) --after-gap-ms 200 --per 20 \
  --top 40 > $OUT/sd15_unet_steady_kernels.txt && head -25 $OUT/sd15_unet_steady_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_wan -o wan -- \
  python3 tools/steady_prof.py wan-step --iters 5 > $OUT/prof_wan.log 2>&1 || { tail -20 $OUT/prof_wan.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_wan -name '*.db' | head -1) --after-gap-ms 200 --per 5 \
  --top 40 > $OUT/wan_step_steady_kernels.txt && head -25 $OUT/wan_step_steady_kernels.txt
