#!/bin/bash
# Round 3 session U: Wan2.1 end-to-end job (umT5 encode + 25 steps + VAE decode) and the 14B DiT
# CFG step with the round-3 kernels.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/u
mkdir -p $OUT
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --t5 \
  --out $OUT/wan_bench_e2e.json > $OUT/wan_bench_e2e.log 2>&1 || { tail -20 $OUT/wan_bench_e2e.log; exit 1; }
grep '\[wan_bench\]' $OUT/wan_bench_e2e.log | tail -6
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --no-e2e --model 14b --iters 5 --warmup 2 \
  --out $OUT/wan14b_step.json > $OUT/wan14b_step.log 2>&1 || { tail -20 $OUT/wan14b_step.log; exit 1; }
grep '\[wan_bench\]' $OUT/wan14b_step.log | tail -3
