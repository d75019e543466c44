# round-6 GPU batch F: zigzag causal order (numerics + sweep), 512 / 32k prefill, the server with
# 8 streaming clients and a 30k-token prompt admitted next to 7 streams
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_llm_prefill_attn_gpu.py tests/test_llm_gpu.py -k "prefill" > gpurun_out/f_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/debug/prefill_attn_sweep.py 512:0 2048:0 8192:0 512:31488 > gpurun_out/f_sweep.log 2>&1 &&
timeout -k 10 200 python -u tools/llm_bench.py --prompt 512 --tokens "" > gpurun_out/f_prefill512.log 2>&1 &&
timeout -k 10 300 python -u tools/llm_bench.py --prompt 32000 --ctx 32256 --tokens "" > gpurun_out/f_prefill32k.log 2>&1 &&
timeout -k 10 600 python -u tools/llm_serve_bench.py --clients 8 --admit 8 --long-prompt 30000 --admit-gen 1024 --ctx-size 32768 --out gpurun_out/f_serve.json > gpurun_out/f_serve.log 2>&1
