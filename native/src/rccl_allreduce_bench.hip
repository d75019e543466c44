// rccl-allreduce-bench — RCCL all-reduce bandwidth + correctness over xGMI, one pod × N GPUs.
//
// BASELINE.json config 4 ("Pod requesting amd.com/gpu:8 runs RCCL all-reduce bandwidth test over
// xGMI"); the reference leaves the multi-GPU-pod case as "TBD" (reference README.md:389-391) and
// has no collective call sites at all.  Single process drives every GPU the device
// plugin allocated (ncclCommInitAll + group calls), nccl-tests style:
//
//   size  count  type  time(us)  algbw(GB/s)  busbw(GB/s)  #wrong
//
// busbw = algbw · 2(n−1)/n (ring all-reduce traffic per rank).  On MI355X each GPU has 7 xGMI links
// of ~153 GB/s; a ring uses one outgoing link per hop, so RCCL reaches beyond one link only by
// spreading channels over several rings — report what is measured, not the aggregate link rate.
// Correctness: rank r contributes (r+1) in every element; after the sum every element must be
// n(n+1)/2 (exact in bf16 for n ≤ 8 and in fp32 always).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "amdk8s_native.h"

#define RCCL_CHECK(expr)                                                                       \
  do {                                                                                         \
    ncclResult_t _r = (expr);                                                                  \
    if (_r != ncclSuccess) {                                                                   \
      std::fprintf(stderr, "RCCL error %s at %s:%d: %s\n", ncclGetErrorString(_r), __FILE__,   \
                   __LINE__, #expr);                                                           \
      std::exit(3);                                                                            \
    }                                                                                          \
  } while (0)

namespace {

__global__ void fill_f32(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ void count_wrong_f32(const float* p, size_t n, float expect, unsigned long long* bad) {
  unsigned long long local = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    local += (p[i] != expect);
  if (local) atomicAdd(bad, local);
}

struct Options {
  size_t min_bytes = 8;
  size_t max_bytes = (size_t)1 << 30;
  int factor = 4;
  int iters = 20;
  int warmup = 5;
  int ngpus = 0;  // 0 = all visible
  bool json = false;
};

size_t parse_size(const char* s) {
  char* end = nullptr;
  double v = std::strtod(s, &end);
  std::string suf = end ? end : "";
  if (suf == "K" || suf == "k") v *= 1024;
  else if (suf == "M" || suf == "m") v *= 1024 * 1024;
  else if (suf == "G" || suf == "g") v *= 1024.0 * 1024 * 1024;
  return (size_t)v;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
      return argv[++i];
    };
    if (a == "-b" || a == "--minbytes") o.min_bytes = parse_size(next());
    else if (a == "-e" || a == "--maxbytes") o.max_bytes = parse_size(next());
    else if (a == "-f" || a == "--stepfactor") o.factor = std::atoi(next());
    else if (a == "-n" || a == "--iters") o.iters = std::atoi(next());
    else if (a == "-w" || a == "--warmup") o.warmup = std::atoi(next());
    else if (a == "-g" || a == "--ngpus") o.ngpus = std::atoi(next());
    else if (a == "--json") o.json = true;
    else {
      std::printf("usage: rccl-allreduce-bench [-b MIN] [-e MAX] [-f FACTOR] [-n ITERS] "
                  "[-w WARMUP] [-g NGPUS] [--json]\n");
      return a == "-h" || a == "--help" ? 0 : 2;
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    std::fprintf(stderr, "No HIP device visible to this container\n");
    return 1;
  }
  const int n = o.ngpus > 0 ? std::min(o.ngpus, ndev) : ndev;
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  RCCL_CHECK(ncclCommInitAll(comms.data(), n, devs.data()));
  int ver = 0;
  ncclGetVersion(&ver);

  std::vector<float*> buf(n);
  std::vector<hipStream_t> st(n);
  std::vector<unsigned long long*> dbad(n);
  const size_t max_count = std::max<size_t>(1, o.max_bytes / sizeof(float));
  for (int i = 0; i < n; ++i) {
    AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
    AMDK8S_HIP_CHECK(hipMalloc(&buf[i], max_count * sizeof(float)));
    AMDK8S_HIP_CHECK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    AMDK8S_HIP_CHECK(hipMalloc(&dbad[i], sizeof(unsigned long long)));
  }
  std::printf("# rccl-allreduce-bench: %d GPU(s), RCCL %d, in-place float sum, %d iters\n", n, ver,
              o.iters);
  std::printf("# %12s %12s %6s %10s %12s %12s %8s\n", "size(B)", "count", "type", "time(us)",
              "algbw(GB/s)", "busbw(GB/s)", "#wrong");
  double peak_bus = 0, peak_alg = 0;
  size_t peak_size = 0;
  unsigned long long total_bad = 0;
  const float expect = (float)n * (n + 1) / 2.0f;
  for (size_t bytes = o.min_bytes; bytes <= o.max_bytes; bytes *= (size_t)o.factor) {
    const size_t count = std::max<size_t>(1, bytes / sizeof(float));
    // correctness pass
    for (int i = 0; i < n; ++i) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
      hipLaunchKernelGGL(fill_f32, dim3(1024), dim3(256), 0, st[i], buf[i], count, (float)(i + 1));
      AMDK8S_HIP_CHECK(hipMemsetAsync(dbad[i], 0, sizeof(unsigned long long), st[i]));
    }
    RCCL_CHECK(ncclGroupStart());
    for (int i = 0; i < n; ++i)
      RCCL_CHECK(ncclAllReduce(buf[i], buf[i], count, ncclFloat, ncclSum, comms[i], st[i]));
    RCCL_CHECK(ncclGroupEnd());
    unsigned long long bad = 0;
    for (int i = 0; i < n; ++i) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
      hipLaunchKernelGGL(count_wrong_f32, dim3(1024), dim3(256), 0, st[i], buf[i], count, expect,
                         dbad[i]);
      unsigned long long b = 0;
      AMDK8S_HIP_CHECK(hipMemcpyAsync(&b, dbad[i], sizeof(b), hipMemcpyDeviceToHost, st[i]));
      AMDK8S_HIP_CHECK(hipStreamSynchronize(st[i]));
      bad += b;
    }
    total_bad += bad;
    // timed passes (values grow; only bandwidth matters here)
    auto launch = [&]() {
      RCCL_CHECK(ncclGroupStart());
      for (int i = 0; i < n; ++i)
        RCCL_CHECK(ncclAllReduce(buf[i], buf[i], count, ncclFloat, ncclSum, comms[i], st[i]));
      RCCL_CHECK(ncclGroupEnd());
    };
    for (int w = 0; w < o.warmup; ++w) launch();
    for (int i = 0; i < n; ++i) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
      AMDK8S_HIP_CHECK(hipStreamSynchronize(st[i]));
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < o.iters; ++it) launch();
    for (int i = 0; i < n; ++i) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
      AMDK8S_HIP_CHECK(hipStreamSynchronize(st[i]));
    }
    const double us =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() /
        o.iters;
    const double algbw = (double)count * sizeof(float) / (us * 1e-6) / 1e9;
    const double busbw = n > 1 ? algbw * 2.0 * (n - 1) / n : algbw;
    if (busbw > peak_bus) {
      peak_bus = busbw;
      peak_alg = algbw;
      peak_size = count * sizeof(float);
    }
    std::printf("  %12zu %12zu %6s %10.1f %12.2f %12.2f %8llu\n", count * sizeof(float), count,
                "float", us, algbw, busbw, bad);
    if (bytes > o.max_bytes / (size_t)o.factor) break;
  }
  std::printf("# peak busbw %.2f GB/s (algbw %.2f GB/s) at %zu bytes on %d GPU(s)\n", peak_bus,
              peak_alg, peak_size, n);
  if (o.json)
    std::printf("{\"check\": \"rccl_allreduce\", \"ngpus\": %d, \"peak_busbw_gbps\": %.2f, "
                "\"peak_algbw_gbps\": %.2f, \"peak_bytes\": %zu, \"wrong\": %llu, \"passed\": %s}\n",
                n, peak_bus, peak_alg, peak_size, total_bad, total_bad == 0 ? "true" : "false");
  for (int i = 0; i < n; ++i) {
    ncclCommDestroy(comms[i]);
    hipFree(buf[i]);
    hipFree(dbad[i]);
    hipStreamDestroy(st[i]);
  }
  if (total_bad) {
    std::printf("Test FAILED\n");
    return 1;
  }
  std::printf("Test PASSED\nDone\n");
  return 0;
}
