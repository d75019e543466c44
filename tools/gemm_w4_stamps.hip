// Diagnostic: per-K-tile s_memtime stamps of the w4 GEMM (wave 0 of every block) at four points of
// each K-tile — start, K-half 0 done, past the barrier, K-half 1 done — to see where a K-tile's
// cycles go (MFMA phases vs the vmcnt/barrier wait). Not part of the product build.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DAMDK8S_W4_STAMPS tools/gemm_w4_stamps.hip \
//     k8s_nvidia_gpus_amd/ops/csrc/fill.hip -o /tmp/w4stamps && /tmp/w4stamps 4096 4096 16384
// Stamps the INTERLEAVED schedule (the launcher is forced to it: AMDK8S_W4_SCHEDULE=interleaved).
#include "../k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950_w4.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
extern "C" int amdk8s_fill_uniform_bf16(void* dst, long n, unsigned long long seed, float lo, float hi,
                                        hipStream_t stream);

static long long median(std::vector<long long> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  setenv("AMDK8S_W4_SCHEDULE", "interleaved", 1);
  int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096,
      K = argc > 3 ? atoi(argv[3]) : 16384;
  void *A, *B, *C;
  hipMalloc(&A, (size_t)M * K * 2); hipMalloc(&B, (size_t)N * K * 2); hipMalloc(&C, (size_t)M * N * 2);
  amdk8s_fill_uniform_bf16(A, (long)M * K, 1, -1, 1, nullptr);
  amdk8s_fill_uniform_bf16(B, (long)N * K, 2, -1, 1, nullptr);
  const int T = K / 64, nwg = (M / 256) * (N / 256), stride = 4 * T;
  unsigned long long* d;
  hipMalloc(&d, (size_t)nwg * stride * 8);
  hipMemset(d, 0, (size_t)nwg * stride * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_w4_stamps), &d, sizeof(d));
  hipMemcpyToSymbol(HIP_SYMBOL(g_w4_stamp_stride), &stride, sizeof(stride));
  for (int i = 0; i < 20; ++i) amdk8s_gemm_bf16_nt_w4(A, B, C, M, N, K, K, K, N, nullptr);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h((size_t)nwg * stride);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  auto at = [&](int b, int t, int s) { return (long long)h[(size_t)b * stride + t * 4 + s]; };
  printf("# %dx%dx%d  schedule=%s  [s_memtime ticks = shader cycles, medians over blocks]\n", M, N, K,
         "interleaved");
  printf("# K-tile   total  khalf0  wait+barrier  khalf1   (ideal per K-half: 64 MFMA x 16 = 1024)\n");
  std::vector<long long> all_tot, all_a, all_w, all_b;
  for (int t = 1; t + 2 < T; ++t) {
    std::vector<long long> tot, a, w, b;
    for (int blk = 0; blk < nwg; ++blk) {
      tot.push_back(at(blk, t + 1, 0) - at(blk, t, 0));
      a.push_back(at(blk, t, 1) - at(blk, t, 0));
      w.push_back(at(blk, t, 2) - at(blk, t, 1));
      b.push_back(at(blk, t, 3) - at(blk, t, 2));
    }
    all_tot.insert(all_tot.end(), tot.begin(), tot.end());
    all_a.insert(all_a.end(), a.begin(), a.end());
    all_w.insert(all_w.end(), w.begin(), w.end());
    all_b.insert(all_b.end(), b.begin(), b.end());
    if (t % (T > 64 ? T / 16 : 4) == 1)
      printf("%8d %7lld %7lld %13lld %7lld\n", t, median(tot), median(a), median(w), median(b));
  }
  printf("%8s %7lld %7lld %13lld %7lld\n", "all", median(all_tot), median(all_a), median(all_w),
         median(all_b));
  return 0;
}
