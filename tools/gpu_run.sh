#!/usr/bin/env bash
# The one GPU-box session runner (replaces the per-session gpu_r0*_*.sh scripts).
#
#   tools/gpu_run.sh <name> <step> [<step> ...]     → writes gpurun_out/<name>/...
#
# Steps (run in order; each GPU step has its own time limit; the first failure ends the call):
#   tests            pytest -m gpu (what the driver runs at round end)
#   tests:<expr>     pytest -m gpu -k <expr>
#   smoke            __graft_entry__.smoke()
#   driver           python3 bench.py --gpus 1 --steps 20 --warmup 5   (the driver's exact command)
#   driver-notel     the same with --no-telemetry
#   bench            bench.py defaults (K=200 / W=20)
#   native           amd-vectoradd, amd-gemm-validator (bf16 + fp8), amd-proftester
#   llm[:<tokens>]   tools/llm_bench.py (decode T list, default 1,2,3,4) + prefill
#   llm-ctx:<n>      tools/llm_bench.py decode T = 1,4,8 after an n-token prompt (long-context decode)
#   bringup          operator bring-up rehearsal with the shipped ConfigMap config: gated + ungated
#                    time-to-first-GPU-pod (python -m k8s_nvidia_gpus_amd.operator bringup)
#   prefill-gemm[:M,..]  tools/llm_prefill_gemm_probe.py --quick (planner pick, w4a plain, hipBLASLt)
#   attn-probe       tools/debug/prefill_attn_probe.py (chunked-prefill attention formulations)
#   serve[:<args>]   tools/llm_serve_bench.py: the server under 1/4/8 streaming clients + a long-prompt
#                    admission (args: comma-separated, '=' for spaces, e.g. serve:--clients=8,--gen=256)
#   gemv[:<cases>]   tools/llm_bench.py --gemv: cold-weight GEMV decomposition sweep, T = 1 and 4
#   prof-bench       rocprofv3 --kernel-trace --stats of the driver's bench command
#   prof-llm[:<T>[:<prompt>]]   rocprofv3 kernel trace of steady LLM decode at T tokens → per-kernel summary
#   prof-prefill     the same for a 512-token prompt prefill
#   pmc-llm[:<T>]    tools/llm_pmc.sh: PMC passes (busy / VALU / wait shares, HBM bytes) at T tokens
#   sd15 / wan       tools/sd15_bench.py / tools/wan_bench.py
#   env:VAR=VALUE    export VAR for the following steps (A/B knobs)
#
# Usage from the container:  gpurun --timeout 900 -- tools/gpu_run.sh r04a tests smoke driver bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
NAME="${1:?usage: tools/gpu_run.sh <name> <step>...}"
shift
OUT="gpurun_out/$NAME"
mkdir -p "$OUT"

fail() { echo "!! step '$1' failed (exit $2); log tail:"; tail -40 "$3"; exit 1; }
jsonline() { grep '^{' "$1" | tail -1 | cut -c1-"${2:-400}"; }

for step in "$@"; do
  echo "== $step ($(date +%T))"
  case "$step" in
    tests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || fail "$step" $? "$OUT/pytest_gpu.log"
      tail -1 "$OUT/pytest_gpu.log" ;;
    tests:*)
      expr="${step#tests:}"
      log="$OUT/pytest_gpu_${expr//[^A-Za-z0-9_]/_}.log"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "$expr" --timeout 300 \
        --timeout-method thread -p no:cacheprovider > "$log" 2>&1 || fail "$step" $? "$log"
      tail -1 "$log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || fail "$step" $? "$OUT/smoke.log"
      tail -1 "$OUT/smoke.log" ;;
    driver|driver-notel)
      extra=""; [[ "$step" == driver-notel ]] && extra="--no-telemetry"
      n=$(ls "$OUT"/"$step"_*.log 2>/dev/null | wc -l)
      log="$OUT/${step}_$n.log"
      timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 $extra > "$log" 2>&1 \
        || fail "$step" $? "$log"
      jsonline "$log" 600 ;;
    bench)
      n=$(ls "$OUT"/bench_*.log 2>/dev/null | wc -l)
      timeout -k 10 400 python3 bench.py > "$OUT/bench_$n.log" 2>&1 || fail "$step" $? "$OUT/bench_$n.log"
      jsonline "$OUT/bench_$n.log" 600 ;;
    native)
      timeout -k 10 120 native/bin/amd-vectoradd > "$OUT/vectoradd.log" 2>&1 || fail "$step" $? "$OUT/vectoradd.log"
      tail -2 "$OUT/vectoradd.log"
      timeout -k 10 300 native/bin/amd-gemm-validator --size 8192 --iters 50 --json \
        > "$OUT/gemm_validator_bf16.log" 2>&1 || fail "$step" $? "$OUT/gemm_validator_bf16.log"
      timeout -k 10 300 native/bin/amd-gemm-validator --dtype fp8 --size 8192 --iters 50 --json \
        > "$OUT/gemm_validator_fp8.log" 2>&1 || fail "$step" $? "$OUT/gemm_validator_fp8.log"
      grep -h '"check"' "$OUT"/gemm_validator_*.log | cut -c1-300
      timeout -k 10 300 native/bin/amd-proftester --json > "$OUT/proftester.log" 2>&1 \
        || fail "$step" $? "$OUT/proftester.log"
      grep -v '^{' "$OUT/proftester.log" | tail -8 ;;
    llm|llm:*)
      toks="1,2,3,4,8"; [[ "$step" == llm:* ]] && toks="${step#llm:}"
      n=$(ls "$OUT"/llm_bench_*.json 2>/dev/null | wc -l)
      timeout -k 10 500 python -u tools/llm_bench.py --tokens "$toks" --out "$OUT/llm_bench_$n.json" \
        > "$OUT/llm_bench_$n.log" 2>&1 || fail "$step" $? "$OUT/llm_bench_$n.log"
      grep -E "decode|prefill" "$OUT/llm_bench_$n.log" | grep -v '^{' ;;
    gemv|gemv:*)
      cases="qkv,o_proj,gate_up,gate_up_q8,down_q4k,down_q6k,lm_head"; [[ "$step" == gemv:* ]] && cases="${step#gemv:}"
      n=$(ls "$OUT"/gemv_*.json 2>/dev/null | wc -l)
      timeout -k 10 600 python -u tools/llm_bench.py --tokens "" --prompt 64 --gemv --gemv-sweep4 \
        --gemv-cases "$cases" --out "$OUT/gemv_$n.json" > "$OUT/gemv_$n.log" 2>&1 || fail "$step" $? "$OUT/gemv_$n.log"
      grep "'gemv'" "$OUT/gemv_$n.log" | sort -t: -k8 | tail -40 | cut -c1-200 ;;
    prof-bench)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o bench --output-format csv \
        -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/prof_bench.log" 2>&1 \
        || fail "$step" $? "$OUT/prof_bench.log"
      find "$OUT/prof_bench" -name "*kernel_stats.csv" -exec head -6 {} \; | cut -c1-200 ;;
    llm-ctx:*)
      np="${step#llm-ctx:}"
      timeout -k 10 500 python -u tools/llm_bench.py --tokens 1,4,8 --prompt "$np" --out "$OUT/llm_ctx_$np.json" \
        > "$OUT/llm_ctx_$np.log" 2>&1 || fail "$step" $? "$OUT/llm_ctx_$np.log"
      grep -E "decode|prefill" "$OUT/llm_ctx_$np.log" | grep -v '^{' ;;
    serve|serve:*)
      extra=""; [[ "$step" == serve:* ]] && extra="${step#serve:}"; extra="${extra//,/ }"
      extra="${extra//=/ }"
      n=$(ls "$OUT"/serve_*.json 2>/dev/null | wc -l)
      # shellcheck disable=SC2086
      timeout -k 10 900 python -u tools/llm_serve_bench.py $extra --server-log "$OUT/serve_server_$n.log" \
        --out "$OUT/serve_$n.json" > "$OUT/serve_$n.log" 2>&1 || fail "$step" $? "$OUT/serve_$n.log"
      grep -E "^(concurrency|admit|server ready)" "$OUT/serve_$n.log" | cut -c1-900 ;;
    bringup)
      # the shipped operator config (ConfigMap), narrowed to this box's GPU count
      python3 - "$OUT/operator.yaml" <<'PYEOF'
import sys, yaml
cm = yaml.safe_load(open("cluster-config/apps/amd-gpu-operator/config.yaml"))
cfg = yaml.safe_load(cm["data"]["operator.yaml"])
import torch
cfg["expectedGpusPerNode"] = torch.cuda.device_count()
open(sys.argv[1], "w").write(yaml.safe_dump(cfg))
PYEOF
      timeout -k 10 600 python3 -m k8s_nvidia_gpus_amd.operator bringup --config "$OUT/operator.yaml" \
        --workdir "$OUT/bringup_work" > "$OUT/bringup.log" 2>&1 || fail "$step" $? "$OUT/bringup.log"
      grep -v '^{' "$OUT/bringup.log" | tail -24; grep '^{' "$OUT/bringup.log" | tail -1 > "$OUT/bringup.json"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('time_to_first_gpu_pod_s', d['time_to_first_gpu_pod_s'], 'time_to_validated_s', d['time_to_validated_s'])" "$OUT/bringup.json" ;;
    prefill-gemm|prefill-gemm:*)
      ms="512"; [[ "$step" == prefill-gemm:* ]] && ms="${step#prefill-gemm:}"
      for m in ${ms//,/ }; do
        timeout -k 10 300 python -u tools/llm_prefill_gemm_probe.py --m "$m" --quick \
          --out "$OUT/prefill_gemm_$m.json" > "$OUT/prefill_gemm_$m.log" 2>&1 || fail "$step" $? "$OUT/prefill_gemm_$m.log"
        grep "^{" "$OUT/prefill_gemm_$m.log" | cut -c1-220
      done ;;
    prefill-many)
      timeout -k 10 400 python -u tools/debug/prefill_many_probe.py > "$OUT/prefill_many_probe.log" 2>&1 \
        || fail "$step" $? "$OUT/prefill_many_probe.log"
      grep '^{' "$OUT/prefill_many_probe.log" ;;
    attn-probe)
      timeout -k 10 300 python -u tools/debug/prefill_attn_probe.py > "$OUT/prefill_attn_probe.log" 2>&1 \
        || fail "$step" $? "$OUT/prefill_attn_probe.log"
      cut -c1-200 "$OUT/prefill_attn_probe.log" ;;
    prof-llm|prof-llm:*)
      t=1; np=512; [[ "$step" == prof-llm:* ]] && t="${step#prof-llm:}"
      [[ "$t" == *:* ]] && { np="${t#*:}"; t="${t%%:*}"; }
      tag="t${t}_p${np}"
      timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d "$OUT/prof_llm_$tag" -o llm \
        -- python3 tools/steady_prof.py llm-decode --tokens "$t" --prompt "$np" --iters 20 --warmup 5 > "$OUT/prof_llm_$tag.log" 2>&1 \
        || fail "$step" $? "$OUT/prof_llm_$tag.log"
      db=$(find "$OUT/prof_llm_$tag" -name '*.db' | head -1)
      python3 tools/rocpd_summary.py "$db" --after-gap-ms 200 --per 20 --top 30 > "$OUT/llm_decode_${tag}_kernels.txt" \
        && head -24 "$OUT/llm_decode_${tag}_kernels.txt" | cut -c1-170 ;;
    prof-prefill)
      timeout -k 10 400 rocprofv3 --kernel-trace --output-format rocpd -d "$OUT/prof_prefill" -o prefill \
        -- python3 tools/steady_prof.py llm-prefill --iters 10 --warmup 3 > "$OUT/prof_prefill.log" 2>&1 \
        || fail "$step" $? "$OUT/prof_prefill.log"
      db=$(find "$OUT/prof_prefill" -name '*.db' | head -1)
      python3 tools/rocpd_summary.py "$db" --after-gap-ms 200 --per 10 --top 30 > "$OUT/llm_prefill_kernels.txt" \
        && head -30 "$OUT/llm_prefill_kernels.txt" | cut -c1-170 ;;
    pmc-llm|pmc-llm:*)
      t=1; [[ "$step" == pmc-llm:* ]] && t="${step#pmc-llm:}"
      OUT="$OUT/llm_pmc_t$t" TOKENS=$t timeout -k 10 400 tools/llm_pmc.sh > "$OUT/llm_pmc_t$t.txt" 2>&1 \
        || fail "$step" $? "$OUT/llm_pmc_t$t.txt"
      cut -c1-200 "$OUT/llm_pmc_t$t.txt" | tail -14 ;;
    sd15)
      timeout -k 10 600 python -u tools/sd15_bench.py > "$OUT/sd15.log" 2>&1 || fail "$step" $? "$OUT/sd15.log"
      tail -5 "$OUT/sd15.log" ;;
    wan)
      timeout -k 10 900 python -u tools/wan_bench.py > "$OUT/wan.log" 2>&1 || fail "$step" $? "$OUT/wan.log"
      tail -5 "$OUT/wan.log" ;;
    env:*)
      kv="${step#env:}"; export "${kv?}"; echo "   export $kv" ;;
    *)
      echo "unknown step '$step'"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
