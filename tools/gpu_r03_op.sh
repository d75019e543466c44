#!/bin/bash
# Round 3 sessions O+P combined (pool congested): see tools/gpu_r03_o.sh and tools/gpu_r03_p.sh.
# and row sums — tests, probe, PMC, SD1.5 + Wan benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/o
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_epi_gpu.py > $OUT/gemm_epi_tests.log 2>&1 || { tail -40 $OUT/gemm_epi_tests.log; exit 1; }
tail -2 $OUT/gemm_epi_tests.log
TOKENS=2560 timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_probe_wan.log 2>&1 || { tail -20 $OUT/gemm_probe_wan.log; exit 1; }
grep -v '^{' $OUT/gemm_probe_wan.log | grep -v amdgpu.ids
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_sd15_gpu.py tests/test_wan_gpu.py > $OUT/pytest_models.log 2>&1 || { tail -40 $OUT/pytest_models.log; exit 1; }
tail -2 $OUT/pytest_models.log
ATTN_VARIANTS=2 timeout -k 10 300 python -u tools/attn_probe.py > $OUT/attn_probe.log 2>&1 || { tail -20 $OUT/attn_probe.log; exit 1; }
grep -v '^{' $OUT/attn_probe.log | grep -v amdgpu.ids
export ATTN_ONLY=wan_self ATTN_VARIANTS=2
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY \
  -d $OUT/attn_pmc/p1 -o p1 --output-format csv -- python3 tools/attn_probe.py > $OUT/attn_pmc_p1.log 2>&1 || { tail -20 $OUT/attn_pmc_p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_ADDR_CONFLICT SQ_CYCLES GRBM_GUI_ACTIVE \
  -d $OUT/attn_pmc/p2 -o p2 --output-format csv -- python3 tools/attn_probe.py > $OUT/attn_pmc_p2.log 2>&1 || { tail -20 $OUT/attn_pmc_p2.log; exit 1; }
unset ATTN_ONLY ATTN_VARIANTS
PMC_MATCH=attn python3 tools/pmc_summary.py "$OUT/attn_pmc/**/*counter_collection.csv" > $OUT/attn_pmc_summary.txt && grep -E "attn_m32|VALU insts per|bank conflicts per|duration" $OUT/attn_pmc_summary.txt
timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
  --out $OUT/wan_bench_2560.json > $OUT/wan_bench_2560.log 2>&1 || { tail -20 $OUT/wan_bench_2560.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560.log
timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 --miopen-find \
  --out $OUT/sd15_bench.json > $OUT/sd15_bench.log 2>&1 || { tail -20 $OUT/sd15_bench.log; exit 1; }
grep -E "unet|e2e" $OUT/sd15_bench.log
OUT=gpurun_out/r03/p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
for lr in 0 1; do
  AMDK8S_LLM_LONGROW=$lr timeout -k 10 400 python -u tools/llm_bench.py --gemv --out $OUT/llm_bench_lr$lr.json \
    > $OUT/llm_bench_lr$lr.log 2>&1 || { tail -30 $OUT/llm_bench_lr$lr.log; exit 1; }
  echo "longrow=$lr"; grep -v '^{' $OUT/llm_bench_lr$lr.log | grep -E "decode|prefill"
done
