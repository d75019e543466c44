#!/usr/bin/env bash
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT="${OUT:-gpurun_out/wan3}"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_wan_gpu.py -x -q -p no:warnings --timeout 200 --timeout-method thread > "$OUT/pytest_wan.log" 2>&1 || { tail -40 "$OUT/pytest_wan.log"; exit 1; }
tail -2 "$OUT/pytest_wan.log"
timeout -k 10 400 python -u tools/wan_vae_prof.py > "$OUT/vae.log" 2>&1 || { tail -20 "$OUT/vae.log"; exit 1; }
cat "$OUT/vae.log" | grep decode
timeout -k 10 600 python -u tools/wan_bench.py --t5 --arms native --out "$OUT/wan_bench_t5.json" > "$OUT/wan_bench_t5.log" 2>&1 || { tail -20 "$OUT/wan_bench_t5.log"; exit 1; }
tail -1 "$OUT/wan_bench_t5.log"
