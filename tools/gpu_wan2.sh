#!/usr/bin/env bash
# Wan GPU pass 2: server test, bench with the umT5-xxl encoder, warm VAE decode kernel profile.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT="${OUT:-gpurun_out/wan2}"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_wan_gpu.py -x -q -p no:warnings --timeout 200 --timeout-method thread > "$OUT/pytest_wan.log" 2>&1 || { tail -40 "$OUT/pytest_wan.log"; exit 1; }
tail -2 "$OUT/pytest_wan.log"
timeout -k 10 300 python -u tools/attn_probe.py > "$OUT/attn_probe.log" 2>&1 || { tail -20 "$OUT/attn_probe.log"; exit 1; }
tail -1 "$OUT/attn_probe.log" | cut -c1-300
timeout -k 10 600 python -u tools/sd15_bench.py --out "$OUT/sd15.json" > "$OUT/sd15.log" 2>&1 || { tail -20 "$OUT/sd15.log"; exit 1; }
tail -1 "$OUT/sd15.log" | cut -c1-300
timeout -k 10 600 python -u tools/wan_bench.py --t5 --arms native,torch --out "$OUT/wan_bench_t5.json" > "$OUT/wan_bench_t5.log" 2>&1 || { tail -20 "$OUT/wan_bench_t5.log"; exit 1; }
tail -1 "$OUT/wan_bench_t5.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/vaeprof" -o vae --output-format csv -- python3 tools/wan_vae_prof.py > "$OUT/vaeprof.log" 2>&1 || { tail -20 "$OUT/vaeprof.log"; exit 1; }
grep decode "$OUT/vaeprof.log"
echo done
