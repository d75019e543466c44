// Probe: pair GEMV (Qwen2.5-7B gate|up shape) full kernel vs a loads-only variant of the same
// pipeline — separates streaming from compute/latency.  Includes the production kernels.
#include "../../k8s_nvidia_gpus_amd/ops/csrc/llm_decode.hip"
#include <cstdio>
#include <cstdlib>

namespace {
template <int MODE, int U>
__global__ void __launch_bounds__(512) loads_only(GemvArgs a, uint32_t* sink) {
  const int K = a.K, nb = K >> 8;
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 7, bl = lane >> 3;
  const int nst = (nb + 8 * U - 1) / (8 * U);
  const int r0 = blockIdx.x * a.rows_per_wg + wave;
  const int r1 = min(a.N, blockIdx.x * a.rows_per_wg + a.rows_per_wg);
  const int nrows = r0 < r1 ? (r1 - r0 + W - 1) / W : 0;
  const int items = nrows * nst;
  Blk<kQ4K> A[U], A1[U];
  uint32_t acc = 0;
  for (int it = 0; it < items; ++it) {
    load_stage<kQ4K, MODE, U>(a, r0 + (it / nst) * W, (it % nst) * 8 * U, nb, sub, bl, A, A1);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= A[u].q.x ^ A[u].q.w ^ A[u].sm ^ A1[u].q.y ^ A1[u].dd;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}
// full compute, but activations in registers (loaded once per wave) instead of LDS per block
template <int U>
__global__ void __launch_bounds__(512) regx(GemvArgs a) {
  const int K = a.K, nb = K >> 8;
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 7, bl = lane >> 3;
  const int r0 = blockIdx.x * a.rows_per_wg + wave;
  const int r1 = min(a.N, blockIdx.x * a.rows_per_wg + a.rows_per_wg);
  uint4 xl[U], xh[U]; float2 dxv[U]; float sxl[U], sxh[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    xl[u] = make_uint4(lane, u, 1, 2); xh[u] = make_uint4(u, lane, 3, 4);
    dxv[u] = make_float2(0.01f * lane, 0.02f); sxl[u] = 0.1f; sxh[u] = 0.2f;
  }
  Blk<kQ4K> A[U], A1[U];
  for (int row = r0; row < r1; row += W) {
    load_stage<kQ4K, kPair, U>(a, row, 0, nb, sub, bl, A, A1);
    float acc = 0.f, acc1 = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (bl + 8 * u >= nb) continue;
      const Blk<kQ4K>* bb[2] = {&A[u], &A1[u]};
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const Blk<kQ4K>& r = *bb[m];
        const float d = h2f(r.dd & 0xffffu), dmin = h2f(r.dd >> 16);
        const uint32_t sc0 = r.sm & 0xffu, sc1 = (r.sm >> 8) & 0xffu;
        const uint32_t m0 = (r.sm >> 16) & 0xffu, m1 = r.sm >> 24;
        const uint32_t q[4] = {r.q.x, r.q.y, r.q.z, r.q.w};
        int il = 0, ih = 0;
        il = dot4(q[0] & 0x0f0f0f0fu, xl[u].x, il); il = dot4(q[1] & 0x0f0f0f0fu, xl[u].y, il);
        il = dot4(q[2] & 0x0f0f0f0fu, xl[u].z, il); il = dot4(q[3] & 0x0f0f0f0fu, xl[u].w, il);
        ih = dot4((q[0] >> 4) & 0x0f0f0f0fu, xh[u].x, ih); ih = dot4((q[1] >> 4) & 0x0f0f0f0fu, xh[u].y, ih);
        ih = dot4((q[2] >> 4) & 0x0f0f0f0fu, xh[u].z, ih); ih = dot4((q[3] >> 4) & 0x0f0f0f0fu, xh[u].w, ih);
        float v = d * sc0 * dxv[u].x * il + d * sc1 * dxv[u].y * ih - dmin * m0 * sxl[u] - dmin * m1 * sxh[u];
        if (m == 0) acc += v; else acc1 += v;
      }
    }
    acc = wave_sum(acc); acc1 = wave_sum(acc1);
    if (lane == 0) a.out[row] = acc / (1.f + __expf(-acc)) * acc1;
  }
}
}  // namespace

int main() {
  const int N = 18944, K = 3584, nb = K / 256;
  uint8_t *q0, *q1; int8_t *s0, *s1; uint16_t *d0, *d1; float *xf, *out; uint32_t* sink;
  hipMalloc(&q0, (size_t)N * nb * 128); hipMalloc(&q1, (size_t)N * nb * 128);
  hipMalloc(&s0, (size_t)N * nb * 16); hipMalloc(&s1, (size_t)N * nb * 16);
  hipMalloc(&d0, (size_t)N * nb * 4); hipMalloc(&d1, (size_t)N * nb * 4);
  hipMalloc(&xf, K * 4); hipMalloc(&out, N * 4); hipMalloc(&sink, 4096);
  hipMemset(q0, 1, (size_t)N * nb * 128); hipMemset(q1, 1, (size_t)N * nb * 128);
  hipMemset(s0, 1, (size_t)N * nb * 16); hipMemset(s1, 1, (size_t)N * nb * 16);
  hipMemset(d0, 0, (size_t)N * nb * 4); hipMemset(d1, 0, (size_t)N * nb * 4);
  hipMemset(xf, 0, K * 4);
  int8_t* x8; float *dxp, *sxp;
  hipMalloc(&x8, K); hipMalloc(&dxp, K / 32 * 4); hipMalloc(&sxp, K / 16 * 4);
  hipMemset(x8, 1, K); hipMemset(dxp, 0, K / 8); hipMemset(sxp, 0, K / 4);
  GemvArgs a{};
  a.w0 = {q0, nullptr, s0, d0}; a.w1 = {q1, nullptr, s1, d1};
  a.xf = xf; a.ldx = K; a.norm_w = nullptr; a.eps = 1e-6f; a.out = out; a.ldo = N; a.N = N; a.K = K;
  a.T = 1;
  const bool q8 = getenv("Q8") != nullptr;
  if (q8) { a.xf = nullptr; a.x8 = x8; a.dx = dxp; a.sx = sxp; }
  printf("input %s\n", q8 ? "Q8" : "fp32");
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = 2.0 * N * nb * (128 + 16 + 4);
  for (int rows : {4, 8, 16, 32}) {
    for (int waves : {4, 8}) {
      a.rows_per_wg = rows;
      const int grid = (N + rows - 1) / rows;
      const size_t lds = (size_t)(nb * 288 + (K >> 5) * 4 + (K >> 4) * 4) + 16 * 4;
      float ms_full, ms_ld;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        for (int i = 0; i < 50; ++i)
          hipLaunchKernelGGL((qgemv_kernel<kQ4K, 1, kPair>), dim3(grid), dim3(waves * 64), lds, 0, a);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms_full, e0, e1);
        hipEventRecord(e0);
        for (int i = 0; i < 50; ++i)
          hipLaunchKernelGGL((loads_only<kPair, 2>), dim3(grid), dim3(waves * 64), 0, 0, a, sink);
        hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms_ld, e0, e1);
      }
      float ms_rx;
      hipEventRecord(e0);
      for (int i = 0; i < 50; ++i)
        hipLaunchKernelGGL((regx<2>), dim3(grid), dim3(waves * 64), 0, 0, a);
      hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms_rx, e0, e1);
      printf("rows %2d waves %d: full %.2f us (%.0f GB/s)  loads-only %.2f us (%.0f GB/s)  reg-x compute %.2f us\n", rows, waves,
             ms_full / 50 * 1e3, bytes / (ms_full / 50 * 1e-3) / 1e9, ms_ld / 50 * 1e3,
             bytes / (ms_ld / 50 * 1e-3) / 1e9, ms_rx / 50 * 1e3);
    }
  }
  return 0;
}
