// Microbenchmark: what one LDS-DMA piece (1 KiB per wave-instruction) costs a one-wave-per-SIMD
// MFMA stream, by source footprint (L2-resident vs streamed from HBM) and by what shares the
// MFMA gaps with it (ds_read_b128). Shaped like the w4 GEMM: 256 blocks × 4 waves, 64 MFMAs per
// iteration in 16 groups of 4, one raw barrier + vmcnt per iteration, 2 × 64 KiB LDS ring.
// Not part of the product build.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dma_issue_bench.hip -o /tmp/dmab && /tmp/dmab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void lds_void;

// DPG: DMA pieces per group (0, 1, 2); RPG: ds_read_b128 per group (0, 1); EVERY: DMA only in
// every EVERY-th group; ROFF: byte offset of the reads inside their 1-KiB slot (bank phase)
template <int DPG, int RPG, int EVERY = 1, int ROFF = 0, int DIST = 3>
__global__ void __launch_bounds__(256, 1)
bench(const char* __restrict__ src, size_t span, int iters, unsigned long long* out, float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[131072];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  f32x4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0, 0, 0, 0};
  bf16x8 fa[8], fb[4];
  for (int i = 0; i < 8; ++i)
    for (int e = 0; e < 8; ++e) {
      fa[i][e] = (__bf16)(0.01f * (float)((lane * 7 + i * 3 + e) % 17) - 0.08f);
      fb[i % 4][e] = (__bf16)(0.01f * (float)((lane * 5 + i * 11 + e) % 13) - 0.06f);
    }
  // each block streams its own region so the footprint = 256 blocks × per-block span
  const size_t blk_off = (size_t)blockIdx.x * span;
  size_t pos = 0;
  unsigned long long t0 = 0;
  for (int it = 0; it < iters; ++it) {
    if (it == 2) t0 = __builtin_amdgcn_s_memtime();
    char* ring = lds + (it & 1) * 65536;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[g % 4 * 4 + m]) : "v"(fb[m]), "v"(fa[g % 8]) : "memory");
      if (RPG) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(lds + ((it + 1) & 1) * 65536 +
                                                           g * 4096 + wave * 1024 + ((lane * 16 + ROFF) & 1023));
        fa[(g + DIST) % 8] = v;  // consumed DIST groups (4·DIST MFMAs) later
      }
#pragma unroll
      for (int d = 0; d < (g % EVERY == 0 ? DPG : 0); ++d) {
        const size_t o = (blk_off + ((pos + (size_t)(g * DPG + d) * 4096 + wave * 1024) & (span - 1))) + lane * 16;
        __builtin_amdgcn_global_load_lds((const void*)(src + o),
                                         (lds_void*)(ring + (g * DPG + d) % 16 * 4096 + wave * 1024),
                                         16, 0, 0);
      }
    }
    pos = (pos + 16 * DPG * 4096) & (span - 1);
    // the previous iteration's pieces must have landed (one iteration of lead, as in the GEMM)
    if (DPG == 1 && EVERY == 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    else if (DPG == 1) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
    else if (DPG == 2) asm volatile("s_waitcnt vmcnt(32) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x] = t1 - t0;
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  float s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.f) sink[tid] = s;
}

template <int DPG, int RPG, int EVERY = 1, int ROFF = 0, int DIST = 3>
static void run(const char* src, size_t span, const char* label) {
  const int iters = 400, blocks = 256;
  unsigned long long* d;
  float* sink;
  hipMalloc(&d, blocks * 8);
  hipMalloc(&sink, 1024 * 4);
  std::vector<unsigned long long> h(blocks);
  double best = 1e30;
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL((bench<DPG, RPG, EVERY, ROFF, DIST>), dim3(blocks), dim3(256), 0, nullptr, src, span, iters, d, sink);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), d, blocks * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    best = std::min(best, (double)h[blocks / 2] / (iters - 2));
  }
  const double bytes_per_clk = DPG * 16 / EVERY * 4096.0 / best;  // per CU
  printf("%-24s DMA/grp=%d every=%d reads/grp=%d dist=%d roff=%3d span/blk=%4zu KiB: %6.0f cyc/iter "
         "(MFMA floor 1024), %5.1f B/clk/CU\n", label, DPG, EVERY, RPG, DIST, ROFF, span >> 10, best,
         bytes_per_clk);
  hipFree(d);
  hipFree(sink);
}

int main() {
  const size_t big = (size_t)4 << 20;  // 4 MiB per block × 256 = 1 GiB: streamed from HBM
  char* src;
  if (hipMalloc(&src, big * 256 + 65536)) return 1;
  hipMemset(src, 0, big * 256 + 65536);
  run<0, 0>(src, 65536, "mfma only");
  run<0, 1>(src, 65536, "reads");
  run<0, 1, 1, 0, 7>(src, 65536, "reads d7");
  run<1, 0>(src, 65536, "dma L2");
  run<1, 1>(src, 65536, "dma+reads L2");
  run<1, 1, 1, 0, 1>(src, 65536, "dma+reads L2 d1");
  run<1, 1, 1, 0, 5>(src, 65536, "dma+reads L2 d5");
  run<1, 1, 1, 0, 7>(src, 65536, "dma+reads L2 d7");
  run<1, 1, 2, 0, 7>(src, 65536, "dma/2+reads L2 d7");
  run<1, 1, 1, 0, 7>(src, (size_t)1 << 18, "dma+reads 256K d7");
  return 0;
}
