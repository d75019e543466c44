#!/bin/bash
# Round 3: Wan GPU tests, then the CFG-step benchmark at the reference defaults (2560 tokens) and at
# 832x480x81 (32 760 tokens).
set -o pipefail
cd "$(dirname "$0")/.."
OUT="${OUT:-gpurun_out/r03/wan}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q -p no:warnings --timeout 200 --timeout-method thread \
  tests/test_wan_gpu.py > "$OUT/pytest_wan.log" 2>&1 || { tail -40 "$OUT/pytest_wan.log"; exit 1; }
tail -2 "$OUT/pytest_wan.log"
timeout -k 10 400 python -u tools/wan_bench.py --arms native-graph,native --no-e2e \
  --out "$OUT/wan_bench_2560.json" > "$OUT/wan_bench_2560.log" 2>&1 || { tail -20 "$OUT/wan_bench_2560.log"; exit 1; }
grep '\[wan_bench\] native' "$OUT/wan_bench_2560.log"
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --no-e2e --width 832 --height 480 \
  --frames 81 --iters 3 --warmup 1 --out "$OUT/wan_bench_32760.json" > "$OUT/wan_bench_32760.log" 2>&1 \
  || { tail -20 "$OUT/wan_bench_32760.log"; exit 1; }
grep '\[wan_bench\] native' "$OUT/wan_bench_32760.log"
