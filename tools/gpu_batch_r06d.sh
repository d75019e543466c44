# round-6 GPU batch D: numerics of the CLIP / causal / ffn_down changes, the Infinity-Cache policy
# of the two-launch ffn_down, steady-state library shares of SD1.5 and Wan (kernel traces)
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sd15_gpu.py tests/test_llm_gpu.py -k "causal or clip or batched_decode or eight_token or split_k or batch_invariant or mfma_gemv_vs_fp32 or native_prefill or chunked or prefill_many" > gpurun_out/d_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/llm_bench.py --tokens 1,4,5,6,7,8 > gpurun_out/d_temporal.log 2>&1 &&
AMDK8S_SPLIT_TEMPORAL=0 timeout -k 10 300 python -u tools/llm_bench.py --tokens 6,8 > gpurun_out/d_nt.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sdprof -o sd -- python3 $R/tools/sd15_bench.py --arms "" --batches 1 > $R/gpurun_out/d_sd_e2e.log 2>&1 &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/wanprof -o wan -- python3 $R/tools/wan_bench.py --arms "" --t5 > $R/gpurun_out/d_wan_e2e.log 2>&1
rc=$?
for f in /tmp/sdprof/sd_kernel_trace.csv /tmp/wanprof/wan_kernel_trace.csv /tmp/sdprof/sd_kernel_stats.csv /tmp/wanprof/wan_kernel_stats.csv; do [ -f $f ] && gzip -c $f > $R/gpurun_out/d_$(basename $f).gz; done
exit $rc
