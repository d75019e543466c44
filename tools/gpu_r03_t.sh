#!/bin/bash
# Round 3 session T: steady-state kernel profiles of the final tree — LLM decode (T=1), SD1.5 UNet
# pass, Wan CFG step — for profiles/.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/t
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_llm -o llm --output-format csv -- \
  python3 tools/llm_bench.py --steps 32 --tokens 1 --prompt 128 > $OUT/prof_llm.log 2>&1 || { tail -20 $OUT/prof_llm.log; exit 1; }
find $OUT/prof_llm -name "*kernel_stats.csv" -exec cp {} $OUT/llm_kernel_stats.csv \;
head -22 $OUT/llm_kernel_stats.csv | cut -c1-180
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_sd15 -o sd15 -- \
  python3 tools/steady_prof.py sd15-unet --iters 20 > $OUT/prof_sd15.log 2>&1 || { tail -20 $OUT/prof_sd15.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_sd15 -name '*.db' | head -1) --after-gap-ms 200 --per 20 \
  --top 60 > $OUT/sd15_unet_steady_kernels.txt && head -12 $OUT/sd15_unet_steady_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_wan -o wan -- \
  python3 tools/steady_prof.py wan-step --iters 5 > $OUT/prof_wan.log 2>&1 || { tail -20 $OUT/prof_wan.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_wan -name '*.db' | head -1) --after-gap-ms 200 --per 5 \
  --top 60 > $OUT/wan_step_steady_kernels.txt && head -12 $OUT/wan_step_steady_kernels.txt
