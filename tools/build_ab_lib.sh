#!/usr/bin/env bash
# A/B variant of the kernel library: every object as built in-tree, except one translation unit
# recompiled with extra -D flags, linked to ab/<name>.so (load it with AMDK8S_KERNEL_LIB=...).
#   tools/build_ab_lib.sh <name> <source.hip> [-DFOO=1 ...]
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
python3 -m k8s_nvidia_gpus_amd.ops.build kernels > /dev/null
objdir=build/obj
mkdir -p ab/obj_$name
stem=$(basename "$src" .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -Wno-unused-result \
  "$@" -Ik8s_nvidia_gpus_amd/ops/csrc -c "$src" -o ab/obj_$name/$stem.o
objs=$(ls $objdir/*.o | grep -v "/$stem.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs ab/obj_$name/$stem.o -o ab/$name.so
rm -rf ab/obj_$name
echo "ab/$name.so"
