#!/bin/bash
# Round 3 session J: Wan CFG-step steady-state kernel profile (library GEMMs left?), PMC passes over
# the 32x32x16 flash-attention kernel at the Wan self-attention shape, LLM tests + bench (prefill
# GEMMs on the hand kernels).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/j
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_wan -o wan -- \
  python3 tools/steady_prof.py wan-step --iters 5 > $OUT/prof_wan.log 2>&1 || { tail -20 $OUT/prof_wan.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_wan -name '*.db' | head -1) --after-gap-ms 200 --per 5 \
  --top 60 > $OUT/wan_step_steady_kernels.txt && head -30 $OUT/wan_step_steady_kernels.txt
export ATTN_ONLY=wan_self ATTN_VARIANTS=2
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY \
  -d $OUT/attn_pmc/p1 -o p1 --output-format csv -- python3 tools/attn_probe.py > $OUT/attn_pmc_p1.log 2>&1 || { tail -20 $OUT/attn_pmc_p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_ADDR_CONFLICT SQ_CYCLES GRBM_GUI_ACTIVE \
  -d $OUT/attn_pmc/p2 -o p2 --output-format csv -- python3 tools/attn_probe.py > $OUT/attn_pmc_p2.log 2>&1 || { tail -20 $OUT/attn_pmc_p2.log; exit 1; }
unset ATTN_ONLY ATTN_VARIANTS
PMC_MATCH=attn python3 tools/pmc_summary.py "$OUT/attn_pmc/**/*counter_collection.csv" > $OUT/attn_pmc_summary.txt && cat $OUT/attn_pmc_summary.txt
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
timeout -k 10 600 python -u tools/llm_bench.py --kernels --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -v '^{' $OUT/llm_bench.log | tail -8
timeout -k 10 600 python -u tools/wan_serve_bench.py > $OUT/wan_serve.log 2>&1 || { tail -30 $OUT/wan_serve.log; exit 1; }
grep -v "^\[wan_serve_bench\] [0-9]* s$" $OUT/wan_serve.log | tail -15
