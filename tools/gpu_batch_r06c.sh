# round-6 GPU batch C: library-kernel shares of the SD1.5 / Wan request paths (csv stats only),
# ffn_down one-pass vs two-pass at 5-8 tokens, the narrow-N GEMM plan in the prefill
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_epi_gpu.py tests/test_llm_prefill_attn_gpu.py > gpurun_out/c_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/llm_prefill_gemm_probe.py --m 512 --only qkv,o --quick > gpurun_out/c_gemm512.log 2>&1 &&
timeout -k 10 300 python -u tools/llm_bench.py --tokens 5,6,7,8 > gpurun_out/c_onepass.log 2>&1 &&
AMDK8S_DOWN_ONEPASS=0 timeout -k 10 300 python -u tools/llm_bench.py --tokens 5,6,7,8 > gpurun_out/c_twopass.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sdprof -o sd -- python3 $R/tools/sd15_bench.py --arms "" --batches 1 > $R/gpurun_out/c_sd_e2e.log 2>&1 &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/wanprof -o wan -- python3 $R/tools/wan_bench.py --arms native-graph --iters 1 --warmup 1 --t5 > $R/gpurun_out/c_wan_e2e.log 2>&1
rc=$?
find /tmp/sdprof /tmp/wanprof -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/ \; 2>/dev/null
ls -R /tmp/sdprof | head -20 > $R/gpurun_out/c_prof_listing.txt 2>&1
exit $rc
