set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/kprof; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p -o k --output-format csv -- python3 tools/llm_bench.py --layers 2 --steps 8 --tokens 1 --prompt 64 --kernels > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/kprof/p/**/k_kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
by = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    if any(k in n for k in ('attn', 'rmsnorm', 'rope', 'combine', 'dequant_kernel')):
        by[n[:60]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for n, v in by.items():
    v = sorted(v)
    print(n, len(v), 'min', v[0], 'med', v[len(v)//2], 'max', v[-1])
# attention durations in launch order (last 300 of them = the --kernels loop: pos 100/1000/4000)
att = [(int(r['Start_Timestamp']), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, r.get('Grid_Size_Y', r.get('Grid_Size', '')), r.get('Workgroup_Size', '')) for r in rows if 'attn_decode' in r['Kernel_Name']]
att.sort()
for i in range(0, len(att), max(1, len(att)//30)):
    print('attn', i, att[i][1:])
print(list(rows[0].keys()))
PY
