#!/bin/bash
# Round 3 session R: same-box A/B of the attention loop versions (VER 1 = round-3 kernel, VER 2 =
# unmasked full tiles + pointer loads + packed softmax arithmetic), alternating runs; Wan / SD steps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/r
mkdir -p $OUT
AMDK8S_ATTN_VER=2 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_sd15_gpu.py tests/test_wan_gpu.py > $OUT/pytest_models_v2.log 2>&1 || { tail -40 $OUT/pytest_models_v2.log; exit 1; }
tail -2 $OUT/pytest_models_v2.log
for rep in 1 2; do
  for v in 1 2; do
    AMDK8S_ATTN_VER=$v ATTN_VARIANTS=2 timeout -k 10 300 python -u tools/attn_probe.py > $OUT/attn_probe_v${v}_$rep.log 2>&1 || { tail -20 $OUT/attn_probe_v${v}_$rep.log; exit 1; }
    echo "ver=$v rep=$rep"; grep -E "v2_qt8" $OUT/attn_probe_v${v}_$rep.log | grep -v '^{'
  done
done
for v in 1 2 1 2; do
  AMDK8S_ATTN_VER=$v timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
    --out $OUT/wan_bench_v$v.json > $OUT/wan_bench_v$v.log 2>&1 || { tail -20 $OUT/wan_bench_v$v.log; exit 1; }
  echo "ver=$v"; grep '\[wan_bench\] native' $OUT/wan_bench_v$v.log
done
for v in 1 2; do
  AMDK8S_ATTN_VER=$v timeout -k 10 400 python -u tools/sd15_bench.py --arms native-graph --batches "" --miopen-find \
    --out $OUT/sd15_bench_v$v.json > $OUT/sd15_bench_v$v.log 2>&1 || { tail -20 $OUT/sd15_bench_v$v.log; exit 1; }
  echo "ver=$v"; grep -E "unet" $OUT/sd15_bench_v$v.log
done
