#!/bin/bash
# Round 3 session AB: round-end rehearsal of the current tree (every GPU test, smoke(), bench.py)
# + the LLM decode with the new defaults (split attention, norms in the GEMV prologues) and a GEMV
# decomposition sweep including grids that are whole multiples of the 256 CUs.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/ab
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-300
timeout -k 10 600 python -u tools/llm_bench.py --gemv --gemv-sweep4 --gemv-cases gate_up,down_q4k,down_q6k,o_proj \
  --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -E "decode|prefill" $OUT/llm_bench.log | grep -v '^{'
