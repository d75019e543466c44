// amd-proftester — per-pipe load generator and bandwidth probe for MI355X nodes.
//
// The AMD counterpart of NVIDIA's dcgmproftester, which the reference's GPU operator ships as the
// DCGM profiling load (BASELINE.json names it as the comparison point).  Each
// dcgmproftester target field becomes a test driven by a hand-written gfx950 kernel or a copy engine:
//
//   field  dcgmproftester target        test here      what runs
//   1004   tensor pipe active           tensor         bf16 MFMA GEMM 8192³ (gemm_bf16_gfx950_w4a.hip)
//   1004*  (fp8 tensor)                 tensor-fp8     fp8 e4m3 MFMA GEMM   (gemm_fp8_gfx950_f8a.hip)
//   1005   DRAM active                  hbm-copy       nt 16-B/lane streaming copy (loadgen.hip);
//                                       hbm-read, hbm-write   the read-only / write-only forms
//   1006   FP64 pipe active             fp64           v_mfma_f64_16x16x4_f64 chains (loadgen.hip)
//   1007   FP32 pipe active             fp32           v_pk_fma_f32 chains (loadgen.hip)
//   1008   FP16 pipe active             tensor-fp16    fp16 MFMA GEMM: the w4a loop on
//                                                      v_mfma_f32_16x16x32_f16 (gemm_bf16_gfx950_w4a.hip)
//   1009   PCIe TX bytes                pcie-d2h       hipMemcpyAsync device → pinned host
//   1010   PCIe RX bytes                pcie-h2d       hipMemcpyAsync pinned host → device
//   1011/2 NVLink TX/RX bytes           xgmi           every ordered GPU pair over xGMI: SDMA peer
//                                                      copy and the copy kernel pulling from the
//                                                      peer; then every GPU pulling from all peers
//                                                      at once (aggregate per-GPU link bandwidth)
//
// Every device visible to the container runs its tests in its own host thread, started together
// (like amd-gemm-validator).  `--duration S` turns a test into a sustained load of S seconds
// (dcgmproftester -d) and reports the mean and the min/max of 100 ms windows, so an exporter or
// Prometheus rule can be checked against a known load.  Output: one human line per result, one
// JSON line with --json, then "Test PASSED" / "Done" (or "Test FAILED") like amd-vectoradd.
// Copies are integrity-checked (sampled 64 KiB windows compared on the host).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "amdk8s_native.h"

namespace {

using Clock = std::chrono::steady_clock;

struct Options {
  std::vector<std::string> tests;
  int device = -1;
  double duration_s = 0;         // 0 = timed measurement, > 0 = sustained load
  size_t hbm_bytes = 2ull << 30; // per buffer: far past the 256 MiB Infinity Cache
  size_t pcie_bytes = 256ull << 20;
  size_t xgmi_bytes = 256ull << 20;
  int gemm_size = 8192;
  int iters = 20;
  double settle_ms = 200;
  bool json = false;
};

struct Result {
  std::string test;
  int device = -1;
  int peer = -1;                 // xgmi: source device of a pair (-1 = all peers)
  std::string engine;            // xgmi/pcie: "sdma" | "kernel"
  std::string unit;
  double value = 0, min = 0, max = 0;
  double seconds = 0;
  bool passed = false, skipped = false;
  std::string note;  // fixed ASCII text without quotes (safe inside the JSON line)
};

std::mutex g_out_mu;
std::vector<Result> g_results;

void emit(const Result& r) {
  std::lock_guard<std::mutex> g(g_out_mu);
  g_results.push_back(r);
}

// Barrier for the per-device threads: every device starts each test together.
class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    const int gen = gen_.load();
    if (count_.fetch_add(1) + 1 == n_) {
      count_.store(0);
      gen_.fetch_add(1);
    } else {
      while (gen_.load() == gen) std::this_thread::yield();
    }
  }

 private:
  const int n_;
  std::atomic<int> count_{0};
  std::atomic<int> gen_{0};
};

// Runs `launch` (one unit of work moving/computing `amount`) and returns amount / second:
// settle → warmup → either `iters` timed units (hipEvent) or, with a duration, a sustained loop
// sampled in ~100 ms windows.
struct Rate {
  double mean = 0, min = 0, max = 0, seconds = 0;
};

Rate measure(hipStream_t s, const std::function<void()>& launch, double amount, const Options& o) {
  // settle: the power-management transient after a load step (bench.py settle())
  const auto t0 = Clock::now();
  for (int n = 0; n < 4000; ++n) {
    launch();
    if ((n & 3) == 3) {
      AMDK8S_HIP_CHECK(hipStreamSynchronize(s));
      if (std::chrono::duration<double, std::milli>(Clock::now() - t0).count() >= o.settle_ms) break;
    }
  }
  AMDK8S_HIP_CHECK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  AMDK8S_HIP_CHECK(hipEventCreate(&e0));
  AMDK8S_HIP_CHECK(hipEventCreate(&e1));
  Rate r;
  if (o.duration_s <= 0) {
    AMDK8S_HIP_CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < o.iters; ++i) launch();
    AMDK8S_HIP_CHECK(hipEventRecord(e1, s));
    AMDK8S_HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    AMDK8S_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    r.seconds = ms * 1e-3;
    r.mean = r.min = r.max = amount * o.iters / r.seconds;
  } else {
    // sustained: windows of launches sized to ~100 ms each
    int per_window = 1;
    double total_amount = 0, total_s = 0;
    r.min = 1e300;
    const auto end = Clock::now() + std::chrono::duration<double>(o.duration_s);
    while (Clock::now() < end) {
      AMDK8S_HIP_CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per_window; ++i) launch();
      AMDK8S_HIP_CHECK(hipEventRecord(e1, s));
      AMDK8S_HIP_CHECK(hipEventSynchronize(e1));
      float ms = 0;
      AMDK8S_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double rate = amount * per_window / (ms * 1e-3);
      if (ms >= 50) {  // only full windows count toward min/max
        r.min = std::min(r.min, rate);
        r.max = std::max(r.max, rate);
      }
      total_amount += amount * per_window;
      total_s += ms * 1e-3;
      if (ms < 100) per_window = std::max(per_window + 1, (int)(per_window * 100.0 / std::max(ms, 1.f)));
    }
    r.seconds = total_s;
    r.mean = total_s > 0 ? total_amount / total_s : 0;
    if (r.min > r.max) r.min = r.max = r.mean;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return r;
}

Result from_rate(const std::string& test, int dev, const std::string& unit, const Rate& r,
                 double scale) {
  Result out;
  out.test = test;
  out.device = dev;
  out.unit = unit;
  out.value = r.mean * scale;
  out.min = r.min * scale;
  out.max = r.max * scale;
  out.seconds = r.seconds;
  out.passed = out.value > 0;
  return out;
}

// Compares `windows` sampled 64 KiB windows of two device buffers on the host.
bool same_bytes(const void* a, int dev_a, const void* b, int dev_b, size_t bytes, int windows = 8) {
  const size_t w = std::min<size_t>(64 << 10, bytes);
  std::vector<char> ha(w), hb(w);
  for (int i = 0; i < windows; ++i) {
    const size_t off = (bytes - w) / std::max(1, windows - 1) * i / 16 * 16;
    AMDK8S_HIP_CHECK(hipSetDevice(dev_a));
    AMDK8S_HIP_CHECK(hipMemcpy(ha.data(), (const char*)a + off, w, hipMemcpyDeviceToHost));
    AMDK8S_HIP_CHECK(hipSetDevice(dev_b));
    AMDK8S_HIP_CHECK(hipMemcpy(hb.data(), (const char*)b + off, w, hipMemcpyDeviceToHost));
    if (std::memcmp(ha.data(), hb.data(), w) != 0) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------------------------
// per-device tests
// ------------------------------------------------------------------------------------------------
void test_hbm(const std::string& test, int dev, const Options& o, hipStream_t s, int cus) {
  const size_t bytes = o.hbm_bytes / 16 * 16;
  void *src = nullptr, *dst = nullptr;
  uint32_t* sink = nullptr;
  AMDK8S_HIP_CHECK(hipMalloc(&src, bytes));
  AMDK8S_HIP_CHECK(hipMalloc(&dst, bytes));
  AMDK8S_HIP_CHECK(hipMalloc(&sink, 64));
  // initialise both buffers with the toggling write pattern (never zeros)
  AMDK8S_HIP_CHECK((hipError_t)amdk8s_hbm_stream(1, nullptr, src, (long)bytes, cus, 0, sink, s));
  AMDK8S_HIP_CHECK(hipMemsetAsync(dst, 0, bytes, s));
  const int mode = test == "hbm-read" ? 0 : test == "hbm-write" ? 1 : 2;
  const double moved = mode == 2 ? 2.0 * bytes : (double)bytes;
  auto launch = [&] {
    AMDK8S_HIP_CHECK((hipError_t)amdk8s_hbm_stream(mode, src, dst, (long)bytes, cus, 0, sink, s));
  };
  const Rate r = measure(s, launch, moved, o);
  Result res = from_rate(test, dev, "GB/s", r, 1e-9);
  if (mode == 2) {
    AMDK8S_HIP_CHECK(hipStreamSynchronize(s));
    res.passed = res.passed && same_bytes(src, dev, dst, dev, bytes);
    if (!res.passed) res.note = "copy verification failed";
  }
  emit(res);
  hipFree(src);
  hipFree(dst);
  hipFree(sink);
}

void test_flops(const std::string& test, int dev, const Options& o, hipStream_t s, int cus) {
  void* sink = nullptr;
  AMDK8S_HIP_CHECK(hipMalloc(&sink, 64));
  const bool f64 = test == "fp64";
  const int blocks = cus * 8;                  // 32 waves per CU = 8 per SIMD
  const int iters = f64 ? 3000 : 20000;        // ~10 ms per launch
  const double flop = f64 ? amdk8s_fp64_mfma_flop(blocks, iters) : amdk8s_fp32_fma_flop(blocks, iters);
  auto launch = [&] {
    const int rc = f64 ? amdk8s_fp64_mfma(blocks, iters, (double*)sink, s)
                       : amdk8s_fp32_fma(blocks, iters, (float*)sink, s);
    AMDK8S_HIP_CHECK((hipError_t)rc);
  };
  Options lo = o;
  lo.iters = std::max(3, o.iters / 4);
  emit(from_rate(test, dev, "TFLOPS", measure(s, launch, flop, lo), 1e-12));
  hipFree(sink);
}

int tensor_gemm(const std::string& test, const void* A, const void* B, void* C, int n, hipStream_t s) {
  if (test == "tensor-fp8") return amdk8s_gemm_fp8_nt_f8a(A, B, C, n, n, n, n, n, n, s);
  if (test == "tensor-fp16") return amdk8s_gemm_f16_nt_w4a(A, B, C, n, n, n, n, n, n, s);
  return amdk8s_gemm_bf16_nt_w4a(A, B, C, n, n, n, n, n, n, s);
}

__global__ void bf16_to_f16(uint16_t* p, long n) {  // reinterpret the bf16 fill as fp16 data
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float f = __uint_as_float((uint32_t)p[i] << 16);
    const _Float16 h = (_Float16)f;
    p[i] = *reinterpret_cast<const uint16_t*>(&h);
  }
}

void test_tensor(const std::string& test, int dev, const Options& o, hipStream_t s) {
  const bool fp8 = test == "tensor-fp8";
  const size_t S = o.gemm_size, esz = fp8 ? 1 : 2;
  void *A, *B, *C;
  AMDK8S_HIP_CHECK(hipMalloc(&A, S * S * esz));
  AMDK8S_HIP_CHECK(hipMalloc(&B, S * S * esz));
  AMDK8S_HIP_CHECK(hipMalloc(&C, S * S * 2));
  auto fill = fp8 ? amdk8s_fill_uniform_fp8 : amdk8s_fill_uniform_bf16;
  AMDK8S_HIP_CHECK((hipError_t)fill(A, (long)(S * S), 11 + dev, -1.f, 1.f, s));
  AMDK8S_HIP_CHECK((hipError_t)fill(B, (long)(S * S), 12 + dev, -1.f, 1.f, s));
  if (test == "tensor-fp16") {
    hipLaunchKernelGGL(bf16_to_f16, dim3(4096), dim3(256), 0, s, (uint16_t*)A, (long)(S * S));
    hipLaunchKernelGGL(bf16_to_f16, dim3(4096), dim3(256), 0, s, (uint16_t*)B, (long)(S * S));
  }
  const int n = (int)S;
  Result res;
  int rc = tensor_gemm(test, A, B, C, n, s);
  if (rc != 0) {
    res.test = test;
    res.device = dev;
    res.note = "GEMM shape rejected (size must be a multiple of 256)";
    emit(res);
  } else {
    auto launch = [&] { AMDK8S_HIP_CHECK((hipError_t)tensor_gemm(test, A, B, C, n, s)); };
    emit(from_rate(test, dev, "TFLOPS", measure(s, launch, 2.0 * S * S * S, o), 1e-12));
  }
  hipFree(A);
  hipFree(B);
  hipFree(C);
}

void test_pcie(const std::string& test, int dev, const Options& o, hipStream_t s, int cus) {
  const size_t bytes = o.pcie_bytes / 16 * 16;
  void *host = nullptr, *devbuf = nullptr;
  uint32_t* sink = nullptr;
  AMDK8S_HIP_CHECK(hipHostMalloc(&host, bytes, hipHostMallocDefault));
  AMDK8S_HIP_CHECK(hipMalloc(&devbuf, bytes));
  AMDK8S_HIP_CHECK(hipMalloc(&sink, 64));
  for (size_t i = 0; i < bytes / 4; ++i) ((uint32_t*)host)[i] = (uint32_t)(i * 2654435761u);
  AMDK8S_HIP_CHECK((hipError_t)amdk8s_hbm_stream(1, nullptr, devbuf, (long)bytes, cus, 0, sink, s));
  const bool h2d = test == "pcie-h2d";
  auto launch = [&] {
    if (h2d) AMDK8S_HIP_CHECK(hipMemcpyAsync(devbuf, host, bytes, hipMemcpyHostToDevice, s));
    else AMDK8S_HIP_CHECK(hipMemcpyAsync(host, devbuf, bytes, hipMemcpyDeviceToHost, s));
  };
  Options lo = o;
  lo.settle_ms = 0;
  Result res = from_rate(test, dev, "GB/s", measure(s, launch, (double)bytes, lo), 1e-9);
  res.engine = "sdma";
  // integrity: after the last copy the two sides hold the same bytes
  AMDK8S_HIP_CHECK(hipStreamSynchronize(s));
  std::vector<char> back(std::min<size_t>(bytes, 1 << 20));
  AMDK8S_HIP_CHECK(hipMemcpy(back.data(), devbuf, back.size(), hipMemcpyDeviceToHost));
  if (std::memcmp(back.data(), host, back.size()) != 0) {
    res.passed = false;
    res.note = "host/device contents differ after the copy";
  }
  emit(res);
  hipHostFree(host);
  hipFree(devbuf);
  hipFree(sink);
}

// ------------------------------------------------------------------------------------------------
// xGMI: needs every device at once, so it runs on the main thread after the per-device tests.
// ------------------------------------------------------------------------------------------------
void test_xgmi(const std::vector<int>& devs, const Options& o) {
  if (devs.size() < 2) {
    Result r;
    r.test = "xgmi";
    r.device = devs.empty() ? -1 : devs[0];
    r.skipped = true;
    r.passed = true;
    r.note = "needs >= 2 GPUs in the allocation";
    emit(r);
    return;
  }
  const size_t bytes = o.xgmi_bytes / 16 * 16;
  const int n = (int)devs.size();
  std::vector<void*> src(n), dst(n);
  std::vector<hipStream_t> st(n);
  std::vector<uint32_t*> sink(n);
  std::vector<int> cus(n);
  for (int i = 0; i < n; ++i) {
    AMDK8S_HIP_CHECK(hipSetDevice(devs[i]));
    hipDeviceProp_t p;
    AMDK8S_HIP_CHECK(hipGetDeviceProperties(&p, devs[i]));
    cus[i] = p.multiProcessorCount;
    // one destination slot per possible source so the all-pairs phase has no write sharing
    AMDK8S_HIP_CHECK(hipMalloc(&src[i], bytes));
    AMDK8S_HIP_CHECK(hipMalloc(&dst[i], bytes * n));
    AMDK8S_HIP_CHECK(hipMalloc(&sink[i], 64));
    AMDK8S_HIP_CHECK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    AMDK8S_HIP_CHECK((hipError_t)amdk8s_hbm_stream(1, nullptr, src[i], (long)bytes, cus[i], 0, sink[i], st[i]));
    for (int j = 0; j < n; ++j) {
      if (j == i) continue;
      int can = 0;
      AMDK8S_HIP_CHECK(hipDeviceCanAccessPeer(&can, devs[i], devs[j]));
      if (can) {
        const hipError_t e = hipDeviceEnablePeerAccess(devs[j], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) AMDK8S_HIP_CHECK(e);
        (void)hipGetLastError();
      }
    }
    AMDK8S_HIP_CHECK(hipStreamSynchronize(st[i]));
  }
  Options lo = o;
  lo.settle_ms = 0;
  lo.duration_s = 0;
  lo.iters = std::max(3, o.iters / 2);
  // 1) each ordered pair alone: SDMA peer copy and the copy kernel on the destination pulling
  for (int d = 0; d < n; ++d) {
    for (int s = 0; s < n; ++s) {
      if (s == d) continue;
      int can = 0;
      AMDK8S_HIP_CHECK(hipDeviceCanAccessPeer(&can, devs[d], devs[s]));
      for (const char* engine : {"sdma", "kernel"}) {
        Result r;
        r.test = "xgmi";
        r.device = devs[d];
        r.peer = devs[s];
        r.engine = engine;
        r.unit = "GB/s";
        if (!can && std::string(engine) == "kernel") {
          r.skipped = true;
          r.passed = true;
          r.note = "no peer access";
          emit(r);
          continue;
        }
        AMDK8S_HIP_CHECK(hipSetDevice(devs[d]));
        void* out = (char*)dst[d] + (size_t)s * bytes;
        auto launch = [&] {
          if (std::string(engine) == "sdma")
            AMDK8S_HIP_CHECK(hipMemcpyPeerAsync(out, devs[d], src[s], devs[s], bytes, st[d]));
          else
            AMDK8S_HIP_CHECK((hipError_t)amdk8s_hbm_stream(2, src[s], out, (long)bytes, cus[d], 0,
                                                           sink[d], st[d]));
        };
        const Rate rate = measure(st[d], launch, (double)bytes, lo);
        r.value = r.min = r.max = rate.mean * 1e-9;
        r.seconds = rate.seconds;
        AMDK8S_HIP_CHECK(hipStreamSynchronize(st[d]));
        r.passed = r.value > 0 && same_bytes(src[s], devs[s], out, devs[d], bytes, 4);
        if (!r.passed) r.note = "peer copy verification failed";
        emit(r);
      }
    }
  }
  // 2) every GPU pulls from every peer at once with the copy kernel (one launch per peer on its
  //    own stream): the aggregate inbound xGMI bandwidth per GPU with all links busy.
  std::vector<std::vector<hipStream_t>> ps(n, std::vector<hipStream_t>(n));
  for (int d = 0; d < n; ++d) {
    AMDK8S_HIP_CHECK(hipSetDevice(devs[d]));
    for (int s = 0; s < n; ++s)
      if (s != d) AMDK8S_HIP_CHECK(hipStreamCreateWithFlags(&ps[d][s], hipStreamNonBlocking));
  }
  const int reps = std::max(3, o.iters / 2);
  auto round = [&](int count) {
    for (int it = 0; it < count; ++it)
      for (int d = 0; d < n; ++d) {
        AMDK8S_HIP_CHECK(hipSetDevice(devs[d]));
        for (int s = 0; s < n; ++s)
          if (s != d)
            AMDK8S_HIP_CHECK((hipError_t)amdk8s_hbm_stream(
                2, src[s], (char*)dst[d] + (size_t)s * bytes, (long)bytes,
                std::max(1, cus[d] / (n - 1)), 0, sink[d], ps[d][s]));
      }
    for (int d = 0; d < n; ++d) {
      AMDK8S_HIP_CHECK(hipSetDevice(devs[d]));
      AMDK8S_HIP_CHECK(hipDeviceSynchronize());
    }
  };
  round(1);
  const auto t0 = Clock::now();
  round(reps);
  const double secs = std::chrono::duration<double>(Clock::now() - t0).count();
  for (int d = 0; d < n; ++d) {
    Result r;
    r.test = "xgmi";
    r.device = devs[d];
    r.peer = -1;
    r.engine = "kernel-all-peers";
    r.unit = "GB/s";
    r.value = r.min = r.max = (double)bytes * (n - 1) * reps / secs * 1e-9;
    r.seconds = secs;
    r.passed = r.value > 0;
    emit(r);
  }
  for (int d = 0; d < n; ++d) {
    AMDK8S_HIP_CHECK(hipSetDevice(devs[d]));
    for (int s = 0; s < n; ++s)
      if (s != d) hipStreamDestroy(ps[d][s]);
    hipStreamDestroy(st[d]);
    hipFree(src[d]);
    hipFree(dst[d]);
    hipFree(sink[d]);
  }
}

const char* kAllTests[] = {"tensor", "tensor-fp16", "tensor-fp8", "hbm-read", "hbm-write", "hbm-copy",
                           "fp32", "fp64", "pcie-h2d", "pcie-d2h", "xgmi"};

std::string resolve(const std::string& t) {
  // dcgmproftester field IDs → tests
  if (t == "1004") return "tensor";
  if (t == "1008") return "tensor-fp16";
  if (t == "1005") return "hbm-copy";
  if (t == "1006") return "fp64";
  if (t == "1007") return "fp32";
  if (t == "1009") return "pcie-d2h";
  if (t == "1010") return "pcie-h2d";
  if (t == "1011" || t == "1012") return "xgmi";
  return t;
}

void run_device(int dev, const Options& o, Barrier* bar) {
  AMDK8S_HIP_CHECK(hipSetDevice(dev));
  hipDeviceProp_t p;
  AMDK8S_HIP_CHECK(hipGetDeviceProperties(&p, dev));
  hipStream_t s;
  AMDK8S_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (const auto& t : o.tests) {
    if (t == "xgmi") continue;
    bar->wait();
    if (t.rfind("tensor", 0) == 0) test_tensor(t, dev, o, s);
    else if (t.rfind("hbm-", 0) == 0) test_hbm(t, dev, o, s, p.multiProcessorCount);
    else if (t == "fp32" || t == "fp64") test_flops(t, dev, o, s, p.multiProcessorCount);
    else if (t.rfind("pcie-", 0) == 0) test_pcie(t, dev, o, s, p.multiProcessorCount);
  }
  hipStreamDestroy(s);
}

size_t parse_size(const char* s) {
  char* end = nullptr;
  double v = std::strtod(s, &end);
  const std::string suf = end ? end : "";
  if (suf == "K" || suf == "k") v *= 1024;
  else if (suf == "M" || suf == "m") v *= 1024.0 * 1024;
  else if (suf == "G" || suf == "g") v *= 1024.0 * 1024 * 1024;
  return (size_t)v;
}

void usage() {
  std::printf(
      "usage: amd-proftester [-t TEST[,TEST...]|FIELD] [--device D] [--duration S] [--iters N]\n"
      "                      [--hbm-bytes B] [--pcie-bytes B] [--xgmi-bytes B] [--gemm-size S]\n"
      "                      [--settle-ms MS] [--json] [--list]\n"
      "tests: tensor tensor-fp16 tensor-fp8 hbm-read hbm-write hbm-copy fp32 fp64 pcie-h2d pcie-d2h xgmi all\n"
      "dcgmproftester field IDs: 1004 1005 1006 1007 1008 1009 1010 1011 1012\n");
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  std::string tests = "all";
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "-t" || a == "--test") tests = next();
    else if (a == "--device" || a == "-i") o.device = std::atoi(next());
    else if (a == "--duration" || a == "-d") o.duration_s = std::atof(next());
    else if (a == "--iters") o.iters = std::max(1, std::atoi(next()));
    else if (a == "--hbm-bytes") o.hbm_bytes = parse_size(next());
    else if (a == "--pcie-bytes") o.pcie_bytes = parse_size(next());
    else if (a == "--xgmi-bytes") o.xgmi_bytes = parse_size(next());
    else if (a == "--gemm-size") o.gemm_size = std::atoi(next());
    else if (a == "--settle-ms") o.settle_ms = std::atof(next());
    else if (a == "--json") o.json = true;
    else if (a == "--list") {
      for (const char* t : kAllTests) std::printf("%s\n", t);
      return 0;
    } else {
      usage();
      return a == "-h" || a == "--help" ? 0 : 2;
    }
  }
  size_t pos = 0;
  while (pos <= tests.size()) {
    const size_t c = tests.find(',', pos);
    const std::string t = resolve(tests.substr(pos, c == std::string::npos ? std::string::npos : c - pos));
    if (t == "all") o.tests.insert(o.tests.end(), std::begin(kAllTests), std::end(kAllTests));
    else if (std::find(std::begin(kAllTests), std::end(kAllTests), t) != std::end(kAllTests))
      o.tests.push_back(t);
    else {
      std::fprintf(stderr, "unknown test '%s'\n", t.c_str());
      usage();
      return 2;
    }
    if (c == std::string::npos) break;
    pos = c + 1;
  }
  if (o.hbm_bytes < 16 || o.pcie_bytes < 16 || o.xgmi_bytes < 16 || o.gemm_size <= 0) {
    usage();
    return 2;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    std::fprintf(stderr, "No HIP device visible to this container\n");
    return 1;
  }
  std::vector<int> devs;
  for (int d = 0; d < ndev; ++d)
    if (o.device < 0 || o.device == d) devs.push_back(d);
  if (devs.empty()) {
    std::fprintf(stderr, "device %d not visible (%d devices)\n", o.device, ndev);
    return 1;
  }
  std::printf("[amd-proftester: %zu device(s), %s]\n", devs.size(),
              o.duration_s > 0 ? "sustained load" : "timed measurement");
  Barrier bar((int)devs.size());
  std::vector<std::thread> th;
  for (int d : devs) th.emplace_back(run_device, d, std::cref(o), &bar);
  for (auto& t : th) t.join();
  if (std::find(o.tests.begin(), o.tests.end(), "xgmi") != o.tests.end()) test_xgmi(devs, o);

  bool ok = true;
  for (const auto& r : g_results) {
    ok = ok && r.passed;
    if (r.skipped) std::printf("%-10s device %d: skipped (%s)\n", r.test.c_str(), r.device, r.note.c_str());
    else {
      std::printf("%-10s device %d", r.test.c_str(), r.device);
      if (r.peer >= 0) std::printf(" <- %d", r.peer);
      if (!r.engine.empty()) std::printf(" [%s]", r.engine.c_str());
      std::printf(": %.1f %s", r.value, r.unit.c_str());
      if (o.duration_s > 0) std::printf(" (min %.1f, max %.1f over %.1f s)", r.min, r.max, r.seconds);
      std::printf("%s%s\n", r.note.empty() ? "" : "  ", r.note.c_str());
    }
    if (o.json)
      std::printf("{\"check\": \"proftester\", \"test\": \"%s\", \"device\": %d, \"peer\": %d, "
                  "\"engine\": \"%s\", \"value\": %.3f, \"min\": %.3f, \"max\": %.3f, \"unit\": \"%s\", "
                  "\"seconds\": %.4f, \"skipped\": %s, \"passed\": %s, \"note\": \"%s\"}\n",
                  r.test.c_str(), r.device, r.peer, r.engine.c_str(), r.value, r.min, r.max,
                  r.unit.c_str(), r.seconds, r.skipped ? "true" : "false",
                  r.passed ? "true" : "false", r.note.c_str());
  }
  if (!ok) {
    std::printf("Test FAILED\n");
    return 1;
  }
  std::printf("Test PASSED\nDone\n");
  return 0;
}
