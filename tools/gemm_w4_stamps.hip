// Diagnostic: per-K-tile s_memtime stamps of the w4 GEMM (one block = one CU's tile) to see whether
// stalls are uniform over K or grow as CUs drift apart. Not part of the product build.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DAMDK8S_W4_STAMPS tools/gemm_w4_stamps.hip \
//     k8s_nvidia_gpus_amd/ops/csrc/fill.hip -o /tmp/w4stamps && /tmp/w4stamps 4096 4096 16384
#include "../k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950_w4.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
extern "C" int amdk8s_fill_uniform_bf16(void* dst, long n, unsigned long long seed, float lo, float hi,
                                        hipStream_t stream);
int main(int argc, char** argv) {
  int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096,
      K = argc > 3 ? atoi(argv[3]) : 16384;
  void *A, *B, *C;
  hipMalloc(&A, (size_t)M * K * 2); hipMalloc(&B, (size_t)N * K * 2); hipMalloc(&C, (size_t)M * N * 2);
  amdk8s_fill_uniform_bf16(A, (long)M * K, 1, -1, 1, nullptr);
  amdk8s_fill_uniform_bf16(B, (long)N * K, 2, -1, 1, nullptr);
  const int T = K / 64, nwg = (M / 256) * (N / 256);
  unsigned long long* d;
  hipMalloc(&d, (size_t)nwg * T * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_w4_stamps), &d, sizeof(d));
  hipMemcpyToSymbol(HIP_SYMBOL(g_w4_stamp_stride), &T, sizeof(T));
  for (int i = 0; i < 20; ++i) amdk8s_gemm_bf16_nt_w4(A, B, C, M, N, K, K, K, N, nullptr);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h((size_t)nwg * T);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  // per K-tile: median over blocks of (stamp[t+1]-stamp[t]); and spread of block progress
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < nwg; ++b) t0 = std::min(t0, h[(size_t)b * T]);
  printf("# K-tile  median_dt  p90_dt  max_dt  spread(max-min start)  [s_memtime ticks]\n");
  for (int t = 0; t + 1 < T; t += (T > 64 ? T / 32 : 1)) {
    std::vector<long long> dt, st;
    for (int b = 0; b < nwg; ++b) {
      dt.push_back((long long)(h[(size_t)b * T + t + 1] - h[(size_t)b * T + t]));
      st.push_back((long long)(h[(size_t)b * T + t] - t0));
    }
    std::sort(dt.begin(), dt.end()); std::sort(st.begin(), st.end());
    printf("%6d %10lld %8lld %8lld %12lld\n", t, dt[dt.size() / 2], dt[dt.size() * 9 / 10], dt.back(),
           st.back() - st.front());
  }
  return 0;
}
