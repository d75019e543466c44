#!/usr/bin/env bash
# Capture what a real MI355X node exposes (KFD sysfs topology, DRM nodes, amd-smi views) so the
# CPU-side fakes in tests/fixtures mirror real hardware, and A/B the in-tree GEMM against
# torch.matmul (hipBLASLt) in ONE process on the same random data.
# Runs on the GPU box under gpurun; every GPU step has its own time limit.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/facts
mkdir -p "$OUT"

# --- host facts (no GPU work) ---
T=/sys/class/kfd/kfd/topology
if [[ -d $T ]]; then
  ( cd "$T" && find . -maxdepth 4 -type f \( -name properties -o -name gpu_id -o -name name \
      -o -name generation_id -o -name system_properties \) -print0 |
      tar --null -cf - -T - 2>/dev/null ) > "$OUT/kfd_topology.tar" || true
fi
ls -la /dev/kfd /dev/dri > "$OUT/dev_nodes.txt" 2>&1 || true
ls -la /dev/dri/by-path > "$OUT/dri_by_path.txt" 2>&1 || true
for c in /sys/class/drm/card*/device; do
  [[ -e $c/current_compute_partition ]] || continue
  echo "$c $(cat $c/current_compute_partition 2>/dev/null) $(cat $c/current_memory_partition 2>/dev/null) avail=$(cat $c/available_compute_partition 2>/dev/null)"
done > "$OUT/partitions.txt" 2>&1 || true
uname -r > "$OUT/uname.txt"; cat /sys/module/amdgpu/version >> "$OUT/uname.txt" 2>/dev/null || true
cat /opt/rocm/.info/version >> "$OUT/uname.txt" 2>/dev/null || true

# --- amd-smi (read-only queries) ---
timeout -k 5 60 amd-smi static --json > "$OUT/amdsmi_static.json" 2> "$OUT/amdsmi_static.err" || true
timeout -k 5 60 amd-smi metric --json > "$OUT/amdsmi_metric.json" 2> "$OUT/amdsmi_metric.err" || true
timeout -k 5 60 amd-smi list --json > "$OUT/amdsmi_list.json" 2> "$OUT/amdsmi_list.err" || true
timeout -k 5 60 amd-smi topology --json > "$OUT/amdsmi_topology.json" 2> "$OUT/amdsmi_topology.err" || true
timeout -k 5 60 python3 tools/probe_amdsmi.py > "$OUT/amdsmi_python.json" 2> "$OUT/amdsmi_python.err" || true

# --- GEMM A/B: in-tree kernel vs torch.matmul, interleaved rounds, one process ---
timeout -k 10 300 python3 tools/gemm_ab.py --sizes 4096 8192 --rounds 5 > "$OUT/gemm_ab.txt" 2>&1
echo "facts captured under $OUT"
