// amd-vectoradd — the validator's functional GPU probe (HIP, gfx950).
//
// Replaces the reference's `nvcr.io/nvidia/k8s/cuda-sample:vectoradd` Job (reference
// README.md:264-299) with the same stdout protocol, so the same log checks work:
//
//   [Vector addition of 50000 elements]
//   Copy input data from the host memory to the HIP device
//   HIP kernel launch with 196 blocks of 256 threads
//   Copy output data from the HIP device to the host memory
//   Test PASSED
//   Done
//
// Differences by design:
//   * it runs on EVERY device visible to the container (the device plugin decides which ones),
//     printing one protocol block per device and one final "Done"; with one device the output is
//     byte-identical in structure to the reference sample;
//   * `--json` appends one machine-readable line per device (name, PCI bus, elapsed);
//   * `--bandwidth BYTES` additionally runs the 16-B-per-lane streaming form and reports GB/s.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "amdk8s_native.h"

namespace {

struct Options {
  int elements = 50000;
  bool json = false;
  long bw_bytes = 0;
  int only_device = -1;
};

void usage() {
  std::printf(
      "usage: amd-vectoradd [--elements N] [--device I] [--json] [--bandwidth BYTES]\n");
}

bool run_device(int dev, const Options& o, int ndev) {
  AMDK8S_HIP_CHECK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  AMDK8S_HIP_CHECK(hipGetDeviceProperties(&prop, dev));
  if (ndev > 1)
    std::printf("[device %d: %s (%s), PCI %04x:%02x:%02x]\n", dev, prop.name, prop.gcnArchName,
                prop.pciDomainID, prop.pciBusID, prop.pciDeviceID);
  const int n = o.elements;
  std::printf("[Vector addition of %d elements]\n", n);
  std::vector<float> ha(n), hb(n), hc(n);
  std::mt19937 rng(1234 + dev);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  for (int i = 0; i < n; ++i) {
    ha[i] = U(rng);
    hb[i] = U(rng);
  }
  float *da = nullptr, *db = nullptr, *dc = nullptr;
  const size_t bytes = sizeof(float) * (size_t)n;
  auto t0 = std::chrono::steady_clock::now();
  AMDK8S_HIP_CHECK(hipMalloc(&da, bytes));
  AMDK8S_HIP_CHECK(hipMalloc(&db, bytes));
  AMDK8S_HIP_CHECK(hipMalloc(&dc, bytes));
  std::printf("Copy input data from the host memory to the HIP device\n");
  AMDK8S_HIP_CHECK(hipMemcpy(da, ha.data(), bytes, hipMemcpyHostToDevice));
  AMDK8S_HIP_CHECK(hipMemcpy(db, hb.data(), bytes, hipMemcpyHostToDevice));
  std::printf("HIP kernel launch with %d blocks of %d threads\n", amdk8s_vector_add_blocks(n), 256);
  int rc = amdk8s_vector_add_f32(da, db, dc, n, nullptr);
  if (rc != 0) {
    std::fprintf(stderr, "Failed to launch vectorAdd kernel (error %d)\n", rc);
    return false;
  }
  AMDK8S_HIP_CHECK(hipDeviceSynchronize());
  std::printf("Copy output data from the HIP device to the host memory\n");
  AMDK8S_HIP_CHECK(hipMemcpy(hc.data(), dc, bytes, hipMemcpyDeviceToHost));
  auto t1 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) {
    if (std::fabs(ha[i] + hb[i] - hc[i]) > 1e-5f) {
      std::fprintf(stderr, "Result verification failed at element %d!\n", i);
      return false;
    }
  }
  std::printf("Test PASSED\n");
  double gbps = 0.0;
  if (o.bw_bytes > 0) {
    long nb = (o.bw_bytes / 3 / 16) * 4;  // three arrays, multiple of 4 floats
    float *ba, *bb, *bc;
    AMDK8S_HIP_CHECK(hipMalloc(&ba, nb * 4));
    AMDK8S_HIP_CHECK(hipMalloc(&bb, nb * 4));
    AMDK8S_HIP_CHECK(hipMalloc(&bc, nb * 4));
    AMDK8S_HIP_CHECK(hipMemset(ba, 0, nb * 4));
    AMDK8S_HIP_CHECK(hipMemset(bb, 0, nb * 4));
    hipEvent_t e0, e1;
    AMDK8S_HIP_CHECK(hipEventCreate(&e0));
    AMDK8S_HIP_CHECK(hipEventCreate(&e1));
    const int cus = prop.multiProcessorCount;
    for (int w = 0; w < 3; ++w) amdk8s_vector_add_f32_bw(ba, bb, bc, nb, cus, nullptr);
    const int iters = 20;
    AMDK8S_HIP_CHECK(hipEventRecord(e0, nullptr));
    for (int it = 0; it < iters; ++it) amdk8s_vector_add_f32_bw(ba, bb, bc, nb, cus, nullptr);
    AMDK8S_HIP_CHECK(hipEventRecord(e1, nullptr));
    AMDK8S_HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    AMDK8S_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    gbps = (double)nb * 12.0 * iters / (ms * 1e-3) / 1e9;
    std::printf("Streaming vectorAdd: %.1f GB/s over %.2f GiB\n", gbps,
                nb * 12.0 / (1024.0 * 1024 * 1024));
    hipFree(ba);
    hipFree(bb);
    hipFree(bc);
  }
  if (o.json) {
    const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    std::printf(
        "{\"check\": \"vectoradd\", \"device\": %d, \"name\": \"%s\", \"arch\": \"%s\", "
        "\"pci\": \"%04x:%02x:%02x.0\", \"elements\": %d, \"blocks\": %d, \"threads\": 256, "
        "\"elapsed_ms\": %.3f, \"stream_gbps\": %.1f, \"passed\": true}\n",
        dev, prop.name, prop.gcnArchName, prop.pciDomainID, prop.pciBusID, prop.pciDeviceID, n,
        amdk8s_vector_add_blocks(n), ms, gbps);
  }
  hipFree(da);
  hipFree(db);
  hipFree(dc);
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&](const char* what) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", what);
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--elements") o.elements = std::atoi(next("--elements"));
    else if (a == "--device") o.only_device = std::atoi(next("--device"));
    else if (a == "--json") o.json = true;
    else if (a == "--bandwidth") o.bw_bytes = std::atol(next("--bandwidth"));
    else if (a == "-h" || a == "--help") { usage(); return 0; }
    else { usage(); return 2; }
  }
  if (o.elements <= 0) { usage(); return 2; }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) {
    std::fprintf(stderr, "No HIP device visible to this container (%s)\n",
                 e == hipSuccess ? "0 devices" : hipGetErrorString(e));
    return 1;
  }
  bool ok = true;
  for (int d = 0; d < ndev; ++d) {
    if (o.only_device >= 0 && d != o.only_device) continue;
    ok = run_device(d, o, o.only_device >= 0 ? 1 : ndev) && ok;
  }
  if (!ok) {
    std::printf("Test FAILED\n");
    return 1;
  }
  std::printf("Done\n");
  return 0;
}
