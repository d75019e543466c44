R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_llm_prefill_attn_gpu.py tests/test_gemm_epi_gpu.py tests/test_llm_gpu.py -k "prefill_attention or w4a_partial or split_k or batch_invariant or batched_decode or eight_token or mfma_gemv_vs_fp32" > gpurun_out/t1.log 2>&1 &&
timeout -k 10 300 python -u tools/llm_bench.py --tokens 1,4,5,8 > gpurun_out/llm_onepass.log 2>&1 &&
AMDK8S_DOWN_ONEPASS=0 timeout -k 10 300 python -u tools/llm_bench.py --tokens 5,8 > gpurun_out/llm_twopass.log 2>&1 &&
for m in 128 256 512 1024; do timeout -k 10 200 python -u tools/llm_prefill_gemm_probe.py --m $m --only qkv,o > gpurun_out/gemm_$m.log 2>&1 || exit 1; done &&
timeout -k 10 120 python -u tools/debug/prefill_attn_sweep.py 512:3072 512:31488 64:8192 1:31488 > gpurun_out/pa_sweep2.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/sdprof -o sd -- python3 $R/tools/sd15_bench.py --arms "" --batches 1 > $R/gpurun_out/sd_e2e.log 2>&1 &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d /tmp/wanprof -o wan -- python3 $R/tools/wan_bench.py --arms native-graph --iters 1 --warmup 1 --t5 > $R/gpurun_out/wan_e2e.log 2>&1
rc=$?
find /tmp/sdprof /tmp/wanprof -name "*stats.csv" -exec cp {} $R/gpurun_out/ \; 2>/dev/null
exit $rc
