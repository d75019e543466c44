# A/B of bench.py's process groups on one GPU: A plain single process; B torchrun-launched with
# the shipped setup (gloo timing group, RCCL created after the timed windows); N torchrun with
# RCCL from the start (AMDK8S_BENCH_PG=nccl, round-5 behaviour); then A and B again.
set -o pipefail
C="--gpus 1 --steps 100 --warmup 10 --no-fp8 --no-telemetry"
run() { echo "== $1"; shift; timeout -k 10 120 "$@" 2>/dev/null | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['launcher'], d.get('process_group_backend'), d.get('allreduce_backend'), d.get('allreduce_busbw_gbps'), d.get('end_barrier_ms'))"; }
run A python3 bench.py $C --no-allreduce &&
run B python3 bench.py $C --launcher torchrun &&
AMDK8S_BENCH_PG=nccl run N python3 bench.py $C --launcher torchrun &&
run A2 python3 bench.py $C --no-allreduce &&
run B2 python3 bench.py $C --launcher torchrun
