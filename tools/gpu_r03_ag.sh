#!/bin/bash
# Round 3 session AG: prefill A/B (SDPA GQA path on the cache slabs vs repeat_interleave), then
# the round-end rehearsal of the tree: every GPU test, smoke(), bench.py, LLM decode + T=1 profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ag
mkdir -p $OUT
for g in 0 1; do
  AMDK8S_LLM_PREFILL_GQA=$g timeout -k 10 300 python -u tools/llm_bench.py --tokens 1 --steps 32 \
    --out $OUT/llm_bench_gqa$g.json > $OUT/llm_bench_gqa$g.log 2>&1 || { tail -30 $OUT/llm_bench_gqa$g.log; exit 1; }
  echo "prefill_gqa=$g"; grep -E "prefill" $OUT/llm_bench_gqa$g.log | grep -v '^{'
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-300
timeout -k 10 400 python -u tools/llm_bench.py --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 \
  || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_t1 -o llm -- \
  python3 tools/steady_prof.py llm-decode --tokens 1 --iters 64 --warmup 8 > $OUT/prof_t1.log 2>&1 \
  || { tail -20 $OUT/prof_t1.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_t1 -name '*.db' | head -1) --after-gap-ms 200 \
  --per 64 --top 30 > $OUT/llm_decode_t1_kernels.txt && head -12 $OUT/llm_decode_t1_kernels.txt | cut -c1-150
# kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1): does the per-kernel floor move?
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 300 python -u tools/llm_bench.py --steps 96 \
    --out gpurun_out/r03/ag/llm_bench_devkernarg$k.json > gpurun_out/r03/ag/llm_bench_devkernarg$k.log 2>&1 \
    || { tail -30 gpurun_out/r03/ag/llm_bench_devkernarg$k.log; exit 1; }
  echo "HIP_FORCE_DEV_KERNARG=$k"; grep -E "decode|prefill" gpurun_out/r03/ag/llm_bench_devkernarg$k.log | grep -v '^{'
done
# older GEMV knobs re-measured on the current kernels (tools/gpu_r03_ah.sh)
OUT=gpurun_out/r03/ah
mkdir -p $OUT
for cfg in "2 0" "4 0" "2 1" "4 1"; do
  set -- $cfg
  AMDK8S_LLM_REGX_T=$1 AMDK8S_LLM_LONGROW=$2 timeout -k 10 300 python -u tools/llm_bench.py --steps 96 \
    --out $OUT/llm_bench_rx$1_lr$2.json > $OUT/llm_bench_rx$1_lr$2.log 2>&1 || { tail -30 $OUT/llm_bench_rx$1_lr$2.log; exit 1; }
  echo "regx_t=$1 longrow=$2"; grep -E "decode" $OUT/llm_bench_rx$1_lr$2.log | grep -v '^{'
done
