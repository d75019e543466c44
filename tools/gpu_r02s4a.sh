set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02s4a; mkdir -p $OUT
export AMDK8S_EVIDENCE_DIR="$OUT/evidence"
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:warnings --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo "== bench"
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "== sd15"
timeout -k 10 400 python -u tools/sd15_bench.py --out $OUT/sd15.json > $OUT/sd15.log 2>&1 || { tail -30 $OUT/sd15.log; exit 1; }
tail -8 $OUT/sd15.log
echo "== rocprof sd15"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_sd15 -o sd15 --output-format csv -- python3 tools/sd15_bench.py --arms native-graph --batches 1 --iters 10 > $OUT/prof_sd15.log 2>&1 || { tail -20 $OUT/prof_sd15.log; exit 1; }
find $OUT/prof_sd15 -name "*kernel_stats.csv" -exec head -25 {} \;
