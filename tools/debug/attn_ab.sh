#!/usr/bin/env bash
# A/B of prompt-attention builds (ab/<name>.so from tools/build_ab_lib.sh, "default" = in-tree):
# the auto plan at each case, every variant twice in alternating order (box drift shows up).
set -uo pipefail
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out/attn_ab}
mkdir -p "$OUT"
CASES=${CASES:-"512:0 512:31488 2048:0 8192:0"}
for rep in 1 2; do
  for v in ${VARIANTS:-default}; do
    if [[ $v == default ]]; then lib=""; else lib="$PWD/ab/$v.so"; fi
    AMDK8S_KERNEL_LIB=$lib SWEEP_AUTO_ONLY=1 SWEEP_ITERS=50 timeout -k 10 120 \
      python3 tools/debug/prefill_attn_sweep.py $CASES > "$OUT/${v}_$rep.log" 2>&1 || exit 1
    echo "== $v rep $rep"; grep '^{' "$OUT/${v}_$rep.log" | cut -c1-150
  done
done
