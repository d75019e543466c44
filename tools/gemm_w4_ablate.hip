// Diagnostic: what each ingredient of the w4 GEMM main loop costs. Built once per ablation mask
// (-DAMDK8S_W4_ABLATE=bits, see gemm_bf16_gfx950_w4.hip); results are wrong by design, only the
// time is reported. Not part of the product build.
//   for m in 0 1 2 3 4 7; do hipcc --offload-arch=gfx950 -O3 -std=c++17 -DAMDK8S_W4_ABLATE=$m \
//     tools/gemm_w4_ablate.hip k8s_nvidia_gpus_amd/ops/csrc/fill.hip -o /tmp/w4abl$m; done
#include "../k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950_w4.hip"
#include <cstdio>
#include <cstdlib>
extern "C" int amdk8s_fill_uniform_bf16(void* dst, long n, unsigned long long seed, float lo, float hi,
                                        hipStream_t stream);
int main(int argc, char** argv) {
  setenv("AMDK8S_W4_SCHEDULE", "interleaved", 1);  // the ablation bits apply to this schedule
  const int M = argc > 1 ? atoi(argv[1]) : 8192, N = argc > 2 ? atoi(argv[2]) : 8192,
            K = argc > 3 ? atoi(argv[3]) : 8192;
  void *A, *B, *C;
  if (hipMalloc(&A, (size_t)M * K * 2) || hipMalloc(&B, (size_t)N * K * 2) ||
      hipMalloc(&C, (size_t)M * N * 2))
    return 1;
  amdk8s_fill_uniform_bf16(A, (long)M * K, 1, -1, 1, nullptr);
  amdk8s_fill_uniform_bf16(B, (long)N * K, 2, -1, 1, nullptr);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 30; ++i) amdk8s_gemm_bf16_nt_w4(A, B, C, M, N, K, K, K, N, nullptr);
  const int iters = 50;
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0, nullptr);
    for (int i = 0; i < iters; ++i) amdk8s_gemm_bf16_nt_w4(A, B, C, M, N, K, K, K, N, nullptr);
    hipEventRecord(e1, nullptr);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  const double tf = 2.0 * M * N * K * iters / (best * 1e-3) / 1e12;
  printf("ablate=%d schedule=%s %dx%dx%d %.1f TFLOPS\n", AMDK8S_W4_ABLATE,
         "interleaved", M, N, K, tf);
  return 0;
}
