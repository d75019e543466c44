#!/usr/bin/env bash
# PMC passes over the w4 ablation binaries (tools/gemm_w4_ablate.hip) and hipBLASLt, to split a
# K-tile's cycles between MFMA, fragment reads and tile staging (counters with --kernel-trace
# only, per pool rules). Usage: tools/gemm_pmc_abl.sh "0 1 2 3" (ablation masks).
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SHAPE="${SHAPE:-8192 8192 8192}"
CTRS1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
CTRS2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for abl in ${1:-0 1 2 3}; do
  out=gpurun_out/pmc_abl/a${abl}
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $CTRS1 -d $out/p1 -o p1 \
    --output-format csv -- tools/w4abl$abl $SHAPE > /dev/null 2>&1
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $CTRS2 -d $out/p2 -o p2 \
    --output-format csv -- tools/w4abl$abl $SHAPE > /dev/null 2>&1
  echo "== ablate=$abl"; python3 tools/pmc_summary.py "$out/**/*counter_collection.csv"
done
if [ "${BLT:-1}" = 1 ]; then
  out=gpurun_out/pmc_abl/blt
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $CTRS1 -d $out/p1 -o p1 --output-format csv -- \
    python3 tools/gemm_arm.py --arm blt --shape "${SHAPE// /x}" --iters 20 > /dev/null 2>&1
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $CTRS2 -d $out/p2 -o p2 --output-format csv -- \
    python3 tools/gemm_arm.py --arm blt --shape "${SHAPE// /x}" --iters 20 > /dev/null 2>&1
  echo "== blt"; python3 tools/pmc_summary.py "$out/**/*counter_collection.csv"
fi
