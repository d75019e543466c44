# Is the ~3 % lower GEMM rate of a torchrun-launched bench.py (1 rank) the launcher, the RCCL
# process group, or run-to-run drift?  A: plain, B: torchrun + RCCL, C: torchrun + gloo group,
# D: plain with RCCL initialised by hand (TORCHELASTIC_RUN_ID set, no agent process), A again.
set -o pipefail
C="--gpus 1 --steps 100 --warmup 10 --no-fp8 --no-allreduce --no-telemetry"
run() { echo "== $1"; shift; timeout -k 10 120 "$@" 2>/dev/null | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['launcher'], d.get('process_group_backend'), d.get('end_barrier_ms'))"; }
run A python3 bench.py $C &&
run B python3 bench.py $C --launcher torchrun &&
AMDK8S_BENCH_PG=gloo run C python3 bench.py $C --launcher torchrun &&
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 TORCHELASTIC_RUN_ID=probe run D python3 bench.py $C &&
run A2 python3 bench.py $C &&
run B2 python3 bench.py $C --launcher torchrun
