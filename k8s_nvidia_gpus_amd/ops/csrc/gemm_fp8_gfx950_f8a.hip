// Hand-scheduled fp8 (OCP e4m3) MFMA GEMM for MI355X (gfx950): the validator's second precision with
// its whole K-loop as generated assembly (tools/gen_gemm_f8a_kloop.py → *_kloop.inc).
//
//   C[M,N] (bf16) = A[M,K] (fp8 e4m3, row-major) · B[N,K]ᵀ (fp8 e4m3, row-major), fp32 accumulation.
//
// Geometry, LDS image, DMA pieces, tile order and epilogue are those of the bf16 w4a kernel
// (gemm_bf16_gfx950_w4a.hip); a K-tile is 128 fp8 deep (the same 128 B per row) and the math is
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 scales, as in the hipcc-scheduled fp8 kernel
// (gemm_fp8_gfx950.hip) whose results it reproduces bit for bit. The K-loop (B fragments
// double-buffered by K-tile parity, each A fragment re-read in place after its last MFMA, two
// barriers per K-tile) is documented in the generator.
//
// Shape contract (host-checked): M % 256 == 0, N % 256 == 0, K % 128 == 0, lda/ldb % 16 == 0,
// ldc % 8 == 0, 16-B aligned base pointers, 256·lda and 256·ldb < 2³¹ (32-bit panel offsets).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gemm_fp8_gfx950_f8a_kloop.inc"

#include "tile_order.h"

namespace {

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 128;                      // fp8 elements = bytes per row per K-tile
constexpr int NT = 256;
constexpr int HALF_BYTES = 128 * BK;         // 128 rows × 128 B
constexpr int C_STRIDE = BN * 2 + 16;        // padded epilogue row (matches the generator)
constexpr int LDS_BYTES = BM * C_STRIDE;     // 135168 ≥ 2 × 64 KiB K-tile buffers
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

}  // namespace

template <int SCHED>
__global__ void __launch_bounds__(NT, 1)
amdk8s_gemm_fp8_nt_256x256_f8a(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                int ldc, int order, int nt_store) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1;  // A half this wave reads
  const int wc = wave & 1;   // B half

  // ---- block → tile: per-partition XCD corners of super-blocks, or GROUP_M order (tile_order.h) ----
  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  int m0, n0;
  {
    int tm, tn;
    amdk8s::block_tile(bid, tiles_m, tiles_n, order, GROUP_M, tm, tn);  // tile_order.h
    m0 = tm * BM;
    n0 = tn * BN;
  }

  // ---- operands of the generated body (register map in tools/gen_gemm_w4a_kloop.py) ----
  const uint32_t lda_b = (uint32_t)lda, ldb_b = (uint32_t)ldb;
  const int drow = wave * 8 + (lane >> 3);
  const int dchunk = (lane & 7) ^ ((drow >> 1) & 7);
  const uint32_t a_voff = (uint32_t)drow * lda_b + dchunk * 16;
  const uint32_t b_voff = (uint32_t)drow * ldb_b + dchunk * 16;
  const int frow = lane & 15;
  const int fq = lane >> 4;
  const uint32_t fo0 = frow * 128 + (((0 + fq) ^ (frow >> 1)) << 4);
  const uint32_t fo1 = frow * 128 + (((4 + fq) ^ (frow >> 1)) << 4);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)lds;
  const uint32_t ra0 = lds0 + wr * HALF_BYTES + fo0;
  const uint32_t ra1 = lds0 + wr * HALF_BYTES + fo1;
  const uint32_t rb0 = lds0 + (2 + wc) * HALF_BYTES + fo0;
  const uint32_t rb1 = lds0 + (2 + wc) * HALF_BYTES + fo1;
  const uint32_t cbase = lds0 + (wr * 128 + frow) * C_STRIDE + (wc * 128 + fq * 4) * 2;
  const uint32_t dma_lds = lds0 + wave * 1024;
  const uint64_t a_addr = (uint64_t)(uintptr_t)A + (uint64_t)m0 * lda_b;
  const uint64_t b_addr = (uint64_t)(uintptr_t)B + (uint64_t)n0 * ldb_b;
  const uint32_t a_lo = (uint32_t)a_addr, a_hi = (uint32_t)(a_addr >> 32);
  const uint32_t b_lo = (uint32_t)b_addr, b_hi = (uint32_t)(b_addr >> 32);
  const uint32_t nrec_a = 256u * lda_b, nrec_b = 256u * ldb_b;
  const int T = K / BK;

#define AMDK8S_F8A_OPERANDS                                                                \
  : "s"(T), "s"(a_lo), "s"(a_hi), "s"(nrec_a), "s"(b_lo), "s"(b_hi), "s"(nrec_b), "s"(lda_b),  \
    "s"(ldb_b), "s"(dma_lds), "v"(ra0), "v"(ra1), "v"(rb0), "v"(rb1), "v"(a_voff), "v"(b_voff), \
    "v"(cbase)                                                                                 \
  : AMDK8S_F8A_CLOBBERS
  static_assert(AMDK8S_F8A_NUM_SCHEDULES == 2, "one branch per generated schedule");
  if constexpr (SCHED == 0) asm volatile(AMDK8S_F8A_ASM_0 : AMDK8S_F8A_OPERANDS);
  else asm volatile(AMDK8S_F8A_ASM_1 : AMDK8S_F8A_OPERANDS);
#undef AMDK8S_F8A_OPERANDS
  __syncthreads();  // every wave's quarter of the bf16 C image is in LDS

  // ---- 16-B coalesced stores of the 256×256 bf16 tile ----
  char* cbase_g = reinterpret_cast<char*>(C) + ((size_t)m0 * ldc + n0) * 2;
  const size_t ldc_b = (size_t)ldc * 2;
#pragma unroll 4
  for (int it = 0; it < BM * BN * 2 / (NT * 16); ++it) {
    const int row = it * 8 + (tid >> 5);
    const int ch = tid & 31;
    const u32x4 v = *reinterpret_cast<const u32x4*>(lds + row * C_STRIDE + ch * 16);
    u32x4* dst = reinterpret_cast<u32x4*>(cbase_g + row * ldc_b + ch * 16);
    if (nt_store)  // C streams out (nt: no L2/MALL retention) — the caches stay with A and B
      asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(dst), "v"(v) : "memory");
    else
      *dst = v;
  }
}

extern "C" int amdk8s_gemm_fp8_nt_f8a(const void* A, const void* B, void* C, int M, int N, int K,
                                      int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  if (lda % 16 || ldb % 16 || ldc % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return (int)hipErrorInvalidValue;
  if (256ull * (unsigned long long)(lda > ldb ? lda : ldb) >= (1ull << 31))
    return (int)hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  // partition-aware tile order (tile_order.h): XCD corners of super-blocks, or GROUP_M order
  const int sb = amdk8s::tile_order_arg(M / BM, N / BN);
  // non-temporal C stores (AMDK8S_GEMM_NT_STORE=0 turns them off for A/B runs)
  const char* ntenv = getenv("AMDK8S_GEMM_NT_STORE");
  const int nt = !(ntenv && ntenv[0] == '0');
  // K-loop schedule: the generator's default, or AMDK8S_F8A_SCHEDULE=<name> for A/B runs
  int sched = AMDK8S_F8A_DEFAULT_SCHEDULE;
  if (const char* e = getenv("AMDK8S_F8A_SCHEDULE")) {
    static const char* const names[] = AMDK8S_F8A_SCHEDULE_NAMES;
    for (int i = 0; i < AMDK8S_F8A_NUM_SCHEDULES; ++i)
      if (!strcmp(e, names[i])) sched = i;
  }
  const uint8_t* a = (const uint8_t*)A;
  const uint8_t* b = (const uint8_t*)B;
  uint16_t* c = (uint16_t*)C;
  if (sched == 1)
    hipLaunchKernelGGL(amdk8s_gemm_fp8_nt_256x256_f8a<1>, dim3(nwg), dim3(NT), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc, sb, nt);
  else
    hipLaunchKernelGGL(amdk8s_gemm_fp8_nt_256x256_f8a<0>, dim3(nwg), dim3(NT), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc, sb, nt);
  return (int)hipGetLastError();
}
