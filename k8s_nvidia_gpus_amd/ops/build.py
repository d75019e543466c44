"""In-tree build driver for every native artefact of the stack.

Two kinds of output, both built IN-TREE so they travel with the repository snapshot:

* ``k8s_nvidia_gpus_amd/ops/_lib/libamdk8s_kernels.so`` — the hand-written gfx950 HIP kernels
  (bf16 MFMA GEMM, vectorAdd, …) behind a small C ABI that Python reaches through ``ctypes``
  after ``import torch`` (so the process has exactly one HIP runtime: the soname
  ``libamdhip64.so.7`` already loaded by torch satisfies the library's dependency).
* ``native/bin/*`` — standalone executables used by the operator DaemonSets / validator pods:
  ``amd-vectoradd`` (reference-compatible stdout protocol), ``amd-gemm-validator``,
  ``amd-proftester`` (per-pipe load generator: tensor / HBM / fp32 / fp64 / PCIe / xGMI),
  ``rccl-allreduce-bench``, ``kfd-probe`` and ``amd-container-runtime`` (the runc wrapper containerd
  runs for RuntimeClass ``amd``; it injects the allocated /dev/kfd + render nodes as an OCI hook would).

The reference has no in-tree native code at all (its GPU code lives in pulled images
such as ``nvcr.io/nvidia/k8s/cuda-sample:vectoradd`` — reference README.md:283); these are the
MI355X-native replacements listed in SURVEY.md §7.2.

Everything targets gfx950 only (``--offload-arch=gfx950``); there is no other backend.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional, Sequence

PKG_DIR = Path(__file__).resolve().parent
REPO_ROOT = PKG_DIR.parent.parent
CSRC_DIR = PKG_DIR / "csrc"
LIB_DIR = PKG_DIR / "_lib"
OBJ_DIR = REPO_ROOT / "build" / "obj"
NATIVE_DIR = REPO_ROOT / "native"
NATIVE_BIN = NATIVE_DIR / "bin"

ROCM_PATH = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = os.environ.get("HIPCC", str(ROCM_PATH / "bin" / "hipcc"))
CXX = os.environ.get("CXX_HOST", "g++")
OFFLOAD_ARCH = "gfx950"

KERNEL_LIB_NAME = "libamdk8s_kernels.so"
KERNEL_LIB = LIB_DIR / KERNEL_LIB_NAME

HIP_FLAGS = [
    f"--offload-arch={OFFLOAD_ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
]

# per-translation-unit extra flags of the kernel library (A/B builds: AMDK8S_HIP_DEFINES)
FILE_FLAGS: dict = {}


@dataclass
class NativeTarget:
    """One standalone executable under native/bin."""

    name: str
    sources: List[str]
    compiler: str  # "hipcc" (device code) or "cxx" (host-only C++)
    libs: List[str] = field(default_factory=list)
    extra_flags: List[str] = field(default_factory=list)


NATIVE_TARGETS: List[NativeTarget] = [
    NativeTarget("amd-vectoradd", ["native/src/amd_vectoradd.hip",
                                   "k8s_nvidia_gpus_amd/ops/csrc/vector_add.hip"], "hipcc"),
    NativeTarget("amd-gemm-validator", ["native/src/amd_gemm_validator.hip",
                                        "k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950.hip",
                                        "k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950_w4.hip",
                                        "k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950_w4a.hip",
                                        "k8s_nvidia_gpus_amd/ops/csrc/gemm_fp8_gfx950.hip",
                                        "k8s_nvidia_gpus_amd/ops/csrc/gemm_fp8_gfx950_f8a.hip",
                                        "k8s_nvidia_gpus_amd/ops/csrc/fill.hip"], "hipcc"),
    NativeTarget("amd-proftester", ["native/src/amd_proftester.hip",
                                    "k8s_nvidia_gpus_amd/ops/csrc/loadgen.hip",
                                    "k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950_w4a.hip",
                                    "k8s_nvidia_gpus_amd/ops/csrc/gemm_fp8_gfx950_f8a.hip",
                                    "k8s_nvidia_gpus_amd/ops/csrc/fill.hip"], "hipcc",
                 libs=["-lpthread"]),
    NativeTarget("rccl-allreduce-bench", ["native/src/rccl_allreduce_bench.hip"], "hipcc",
                 libs=["-lrccl", "-lpthread"]),
    NativeTarget("kfd-probe", ["native/src/kfd_probe.cpp", "native/src/kfd_topology.cpp"], "cxx"),
    NativeTarget("amd-container-runtime", ["native/src/amd_container_runtime.cpp"], "cxx",
                 extra_flags=["-static-libstdc++", "-static-libgcc"]),
]


def _run(cmd: Sequence[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(cmd), flush=True)
    proc = subprocess.run(list(cmd), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"command failed ({proc.returncode}): {' '.join(cmd)}\n{proc.stdout}")


def _stale(output: Path, inputs: Sequence[Path]) -> bool:
    if not output.exists():
        return True
    t = output.stat().st_mtime
    return any(p.stat().st_mtime > t for p in inputs)


def kernel_sources() -> List[Path]:
    return sorted(CSRC_DIR.glob("*.hip"))


def _headers() -> List[Path]:
    return (sorted(CSRC_DIR.glob("*.h")) + sorted(CSRC_DIR.glob("*.inc"))
            + sorted((NATIVE_DIR / "include").glob("*.h*")))


def build_kernel_library(force: bool = False, verbose: bool = False, jobs: int = 4) -> Path:
    """Compile csrc/*.hip (one translation unit per kernel family) and link the shared library."""
    srcs = kernel_sources()
    if not srcs:
        raise RuntimeError(f"no HIP sources under {CSRC_DIR}")
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    hdrs = _headers()
    objs = []
    todo = []
    for s in srcs:
        o = OBJ_DIR / (s.stem + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            todo.append((s, o))

    def compile_one(pair):
        s, o = pair
        _run([HIPCC, *HIP_FLAGS, *FILE_FLAGS.get(s.name, []), f"-I{CSRC_DIR}", "-c", str(s), "-o",
              str(o)], verbose)

    if todo:
        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(compile_one, todo))
    if force or todo or _stale(KERNEL_LIB, objs):
        tmp = KERNEL_LIB.with_suffix(".so.tmp")
        _run([HIPCC, f"--offload-arch={OFFLOAD_ARCH}", "-shared", "-fPIC", *map(str, objs),
              "-o", str(tmp)], verbose)
        os.replace(tmp, KERNEL_LIB)  # atomic: a concurrent loader never sees a half-written .so
    return KERNEL_LIB


def build_native(force: bool = False, verbose: bool = False, jobs: int = 4,
                 only: Optional[Sequence[str]] = None) -> List[Path]:
    NATIVE_BIN.mkdir(parents=True, exist_ok=True)
    hdrs = _headers()
    outs = []
    todo = []
    for t in NATIVE_TARGETS:
        if only and t.name not in only:
            continue
        out = NATIVE_BIN / t.name
        srcs = [REPO_ROOT / s for s in t.sources]
        outs.append(out)
        if force or _stale(out, srcs + hdrs):
            todo.append((t, srcs, out))

    def build_one(item):
        t, srcs, out = item
        inc = [f"-I{NATIVE_DIR / 'include'}", f"-I{CSRC_DIR}"]
        if t.compiler == "hipcc":
            cmd = [HIPCC, *HIP_FLAGS, *inc, *t.extra_flags, *map(str, srcs), "-o", str(out),
                   f"-L{ROCM_PATH / 'lib'}", f"-Wl,-rpath,{ROCM_PATH / 'lib'}", *t.libs]
        else:
            cmd = [CXX, "-O2", "-std=c++17", "-Wall", "-Wextra", *inc, *t.extra_flags,
                   *map(str, srcs), "-o", str(out), *t.libs]
        _run(cmd, verbose)

    if todo:
        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(build_one, todo))
    return outs


def build_all(force: bool = False, verbose: bool = False, jobs: int = 4) -> None:
    build_kernel_library(force=force, verbose=verbose, jobs=jobs)
    build_native(force=force, verbose=verbose, jobs=jobs)


def toolchain_available() -> bool:
    return shutil.which(HIPCC) is not None or Path(HIPCC).exists()


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="build the gfx950 kernels and native tools in-tree")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("what", nargs="*", default=["all"], help="all | kernels | native | <target>")
    args = ap.parse_args(argv)
    what = set(args.what)
    if "all" in what:
        build_all(args.force, args.verbose, args.jobs)
    else:
        if "kernels" in what:
            build_kernel_library(args.force, args.verbose, args.jobs)
            what.discard("kernels")
        if "native" in what:
            build_native(args.force, args.verbose, args.jobs)
            what.discard("native")
        if what:
            build_native(args.force, args.verbose, args.jobs, only=sorted(what))
    print(f"built: {KERNEL_LIB} and native tools under {NATIVE_BIN}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
