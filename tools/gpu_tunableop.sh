#!/usr/bin/env bash
# PyTorch TunableOp over the Wan2.1 DiT GEMM shapes: tune once (all hipBLASLt / rocBLAS solutions per
# shape), then measure the CFG step with the tuned table.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT="${OUT:-gpurun_out/tunable}"
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/wan_bench.py --arms native --no-e2e --iters 5 --warmup 2 > "$OUT/base.log" 2>&1
tail -1 "$OUT/base.log" | cut -c1-400
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME="$OUT/tunableop_results%d.csv" \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 \
  timeout -k 10 600 python -u tools/wan_bench.py --arms native --no-e2e --iters 2 --warmup 1 > "$OUT/tune.log" 2>&1
tail -1 "$OUT/tune.log" | cut -c1-400
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME="$OUT/tunableop_results%d.csv" \
  timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph,native --no-e2e --iters 10 --warmup 3 > "$OUT/tuned.log" 2>&1
tail -1 "$OUT/tuned.log" | cut -c1-400
ls "$OUT"
