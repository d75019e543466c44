#!/bin/bash
# Round 3 session F: fast GELU epilogues + tile threshold (GEMM tests, probes), Wan CFG step at
# 2560 / 32 760 tokens, SD1.5 UNet pass + steady-state kernel profile, LLM decode (V loads issued
# with the K loads in the split-context attention) tests + bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03/f
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_epi_gpu.py > $OUT/gemm_epi_tests.log 2>&1 || { tail -40 $OUT/gemm_epi_tests.log; exit 1; }
tail -2 $OUT/gemm_epi_tests.log
timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_probe_wan.log 2>&1 || { tail -20 $OUT/gemm_probe_wan.log; exit 1; }
grep -v '^{' $OUT/gemm_probe_wan.log | grep -v amdgpu.ids
MODE=sd timeout -k 10 300 python -u tools/gemm_epi_probe.py > $OUT/gemm_probe_sd.log 2>&1 || { tail -20 $OUT/gemm_probe_sd.log; exit 1; }
grep sum $OUT/gemm_probe_sd.log
timeout -k 10 300 python -u tools/wan_bench.py --arms native-graph --no-e2e \
  --out $OUT/wan_bench_2560.json > $OUT/wan_bench_2560.log 2>&1 || { tail -20 $OUT/wan_bench_2560.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_2560.log
timeout -k 10 500 python -u tools/wan_bench.py --arms native-graph --no-e2e --width 832 --height 480 \
  --frames 81 --iters 3 --warmup 1 --out $OUT/wan_bench_32760.json > $OUT/wan_bench_32760.log 2>&1 \
  || { tail -20 $OUT/wan_bench_32760.log; exit 1; }
grep '\[wan_bench\] native' $OUT/wan_bench_32760.log
timeout -k 10 500 python -u tools/sd15_bench.py --arms native-graph --batches 1,8 --miopen-find \
  --out $OUT/sd15_bench.json > $OUT/sd15_bench.log 2>&1 || { tail -20 $OUT/sd15_bench.log; exit 1; }
grep -E "unet|e2e" $OUT/sd15_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_sd15 -o sd15 -- \
  python3 tools/steady_prof.py sd15-unet --iters 20 > $OUT/prof_sd15.log 2>&1 || { tail -20 $OUT/prof_sd15.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_sd15 -name '*.db' | head -1) --after-gap-ms 200 --per 20 \
  --top 40 > $OUT/sd15_unet_steady_kernels.txt && head -30 $OUT/sd15_unet_steady_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_wan -o wan -- \
  python3 tools/steady_prof.py wan-step --iters 5 > $OUT/prof_wan.log 2>&1 || { tail -20 $OUT/prof_wan.log; exit 1; }
python3 tools/rocpd_summary.py $(find $OUT/prof_wan -name '*.db' | head -1) --after-gap-ms 200 --per 5 \
  --top 40 > $OUT/wan_step_steady_kernels.txt && head -25 $OUT/wan_step_steady_kernels.txt
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -x -q -p no:warnings --timeout 200 \
  --timeout-method thread > $OUT/pytest_llm.log 2>&1 || { tail -60 $OUT/pytest_llm.log; exit 1; }
tail -2 $OUT/pytest_llm.log
timeout -k 10 600 python -u tools/llm_bench.py --kernels --out $OUT/llm_bench.json > $OUT/llm_bench.log 2>&1 || { tail -30 $OUT/llm_bench.log; exit 1; }
grep -v '^{' $OUT/llm_bench.log | tail -20
