#!/bin/bash
# Round 3 session AL: single-launch GroupNorm only for sets up to 64 KB (16² and 8² levels) — SD1.5 GPU tests (both forms),
# UNet pass A/B over AMDK8S_GN_FUSED, steady-state UNet kernel profile of the default.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/al
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_sd15_gpu.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_sd15.log 2>&1 || { tail -60 $OUT/pytest_sd15.log; exit 1; }
tail -2 $OUT/pytest_sd15.log
for f in 0 1; do
  AMDK8S_GN_FUSED=$f timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 --miopen-find \
    --out $OUT/sd15_bench_gnf$f.json > $OUT/sd15_bench_gnf$f.log 2>&1 || { tail -20 $OUT/sd15_bench_gnf$f.log; exit 1; }
  echo "AMDK8S_GN_FUSED=$f"; grep -E "unet|e2e" $OUT/sd15_bench_gnf$f.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_sd15 -o sd15 -- \
  python3 tools/steady_prof.py sd15-unet --iters 20 > $OUT/prof_sd15.log 2>&1 || { tail -20 $OUT/prof_sd15.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_sd15 -name '*.db' | head -1) --after-gap-ms 200 --per 20 \
  --top 40 > $OUT/sd15_unet_steady_kernels.txt && head -14 $OUT/sd15_unet_steady_kernels.txt | cut -c1-150
