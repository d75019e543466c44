// Hand-written fp8 (OCP e4m3) MFMA GEMM for MI355X (gfx950): the validator's second precision.
//
//   C[M,N] (bf16) = A[M,K] (fp8 e4m3, row-major) · B[N,K]ᵀ (fp8 e4m3, row-major), fp32 accumulation.
//
// Same block geometry and data path as the bf16 w4 kernel (gemm_bf16_gfx950_w4.hip): 256×256 block
// tile, 4 waves (2 M × 2 N) of 128×128, one wave per SIMD, accumulators pinned in AGPRs by asm
// MFMAs, two 64 KiB LDS buffers filled by `buffer_load_dwordx4 … lds` with the same 16-B XOR
// swizzle, super-block / XCD-remapped tile order.  A K-tile is 128 fp8 deep = 128 B per row, so the
// LDS image, the DMA pieces and the fragment reads are byte-for-byte those of a 64-deep bf16 tile.
// The math is `v_mfma_scale_f32_16x16x128_f8f6f4` with unit E8M0 block scales (0x7F = 2⁰), which
// runs 2× the bf16 rate: one MFMA takes the two 16-B chunks the bf16 kernel reads per K-half
// (chunks fq and 4+fq of row frow) as one 32-B operand.  Which k lands in which lane only has to
// agree between A and B — it does, they share the read pattern — so the dot product is exact.
//
// Schedule per K-tile t (64 MFMAs per wave = 16 groups of 4; buffer cur = t & 1):
//   top: lgkmcnt(0) + barrier #1 → every wave holds tile t's fragments in registers, so cur is free;
//   groups 0-7: the 16 DMA pieces of tile t+2 into cur, two per group (after MFMAs 1 and 3);
//   after group 7: vmcnt(16) (tile t+1, issued a whole tile earlier, landed for this wave) +
//     barrier #2 (for every wave);
//   groups 8-15: the 32 fragment reads of tile t+1 from the other buffer into the other register
//     set, one per MFMA gap, in first-use order (b[0..3], a[0], b[4..7], a[1..7]).
// Past the end the DMA is clamped to tile T-1 (identical bytes into a buffer nobody reads again).
//
// Shape contract (host-checked): M % 256 == 0, N % 256 == 0, K % 256 == 0, lda/ldb % 16 == 0,
// ldc % 8 == 0, 16-B aligned base pointers, 256-row panels within 32-bit buffer offsets.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "tile_order.h"

namespace {

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 128;                      // fp8 elements = bytes per row per K-tile
constexpr int NT = 256;
constexpr int HALF_BYTES = 128 * BK;         // 128 rows × 128 B
constexpr int TILE_BYTES = 4 * HALF_BYTES;   // A0 A1 B0 B1 = 64 KiB
constexpr int C_STRIDE = BN * 2 + 16;
constexpr int LDS_BYTES = BM * C_STRIDE;     // 135168 ≥ 2 × TILE_BYTES
static_assert(LDS_BYTES >= 2 * TILE_BYTES, "LDS too small");
constexpr int GROUP_M = 8;

__device__ __forceinline__ void barrier_raw() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ i32x4 lds_read16(const char* p) {
  return *reinterpret_cast<const i32x4*>(__builtin_assume_aligned(p, 16));
}

}  // namespace

__global__ void __launch_bounds__(NT, 1)
amdk8s_gemm_fp8_nt_256x256(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                           uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                           int ldc, int order) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1;
  const int wc = wave & 1;

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

  // ---- LDS-DMA: piece p (0..15): j = p >> 2 (32-row stripe), h = (p >> 1) & 1, p & 1: A/B;
  //      wave w fills rows j*32 + w*8 .. +8 of half h; lane l: row l>>3, swizzled chunk ----
  const uint32_t lda_b = (uint32_t)lda, ldb_b = (uint32_t)ldb;
  const int drow = wave * 8 + (lane >> 3);
  const int dchunk = (lane & 7) ^ ((drow >> 1) & 7);
  const uint32_t a_voff = (uint32_t)drow * lda_b + dchunk * 16;
  const uint32_t b_voff = (uint32_t)drow * ldb_b + dchunk * 16;
  const __amdgpu_buffer_rsrc_t rsrc_a = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(A) + (size_t)m0 * lda_b, (short)0, (int)(256u * lda_b), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_b = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(B) + (size_t)n0 * ldb_b, (short)0, (int)(256u * ldb_b), 0x00020000);
  auto dma_piece = [&](int t, int p) {
    const int j = p >> 2, h = (p >> 1) & 1;
    char* dst = lds + (t & 1) * TILE_BYTES + wave * 1024 + j * 4096;
    const uint32_t rows = (uint32_t)(j * 32 + h * 128);
    if ((p & 1) == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void*)(dst + h * HALF_BYTES), 16, a_voff,
                                               rows * lda_b + (uint32_t)t * BK, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_b, (lds_void*)(dst + (2 + h) * HALF_BYTES), 16,
                                               b_voff, rows * ldb_b + (uint32_t)t * BK, 0, 0);
  };

  // ---- fragment reads: lane (frow, fq) takes chunks fq and 4+fq of row frow of each 16-row block
  const int frow = lane & 15;
  const int fq = lane >> 4;
  const int fo0 = frow * 128 + (((0 + fq) ^ (frow >> 1)) << 4);
  const int fo1 = frow * 128 + (((4 + fq) ^ (frow >> 1)) << 4);
  const int a_off = wr * HALF_BYTES;
  const int b_off = 2 * HALF_BYTES + wc * HALF_BYTES;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = K / BK;
  const int unit_scale = 0x7f7f7f7f;  // E8M0 2^0 in every byte

  // Fragment sets: (alo/ahi/blo/bhi)0 and …1 alternate by tile parity (the loop is unrolled by two,
  // so every index is static); the 16-B halves lo = chunk fq, hi = chunk 4+fq.
  i32x4 alo0[8], ahi0[8], blo0[8], bhi0[8], alo1[8], ahi1[8], blo1[8], bhi1[8];
  // r-th 16-B read of a tile (r = 2x + half, x in first-use order b[0..3], a[0], b[4..7], a[1..7])
#define AMDK8S_F8_READ(ALO, AHI, BLO, BHI, BUF, R)                                       \
  {                                                                                      \
    const int x_ = (R) >> 1;                                                             \
    const int fo_ = ((R) & 1) ? fo1 : fo0;                                               \
    if (x_ < 4) ((R) & 1 ? BHI : BLO)[x_] = lds_read16((BUF) + b_off + x_ * 2048 + fo_); \
    else if (x_ == 4) ((R) & 1 ? AHI : ALO)[0] = lds_read16((BUF) + a_off + fo_);        \
    else if (x_ < 9)                                                                     \
      ((R) & 1 ? BHI : BLO)[x_ - 1] = lds_read16((BUF) + b_off + (x_ - 1) * 2048 + fo_); \
    else ((R) & 1 ? AHI : ALO)[x_ - 8] = lds_read16((BUF) + a_off + (x_ - 8) * 2048 + fo_); \
  }
#define AMDK8S_F8_MFMA1(ALO, AHI, BLO, BHI, I, J)                                        \
  {                                                                                      \
    const i32x8 fa_ = __builtin_shufflevector(ALO[I], AHI[I], 0, 1, 2, 3, 4, 5, 6, 7);   \
    const i32x8 fb_ = __builtin_shufflevector(BLO[J], BHI[J], 0, 1, 2, 3, 4, 5, 6, 7);   \
    asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]" \
                 : "+a"(acc[I][J]) : "v"(fb_), "v"(fa_), "v"(unit_scale) : "memory");    \
  }

  // ---- prologue: tiles 0, 1 in flight; tile 0's fragments into set 0 ----
#pragma unroll
  for (int p = 0; p < 16; ++p) dma_piece(0, p);
#pragma unroll
  for (int p = 0; p < 16; ++p) dma_piece(min(1, T - 1), p);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  barrier_raw();
#pragma unroll
  for (int r = 0; r < 32; ++r) AMDK8S_F8_READ(alo0, ahi0, blo0, bhi0, lds, r)

  // One K-tile on set C reading tile TT+1 into set N.
#define AMDK8S_F8_TILE(TT, CALO, CAHI, CBLO, CBHI, NALO, NAHI, NBLO, NBHI)               \
  {                                                                                      \
    const int t_ = (TT);                                                                 \
    const char* nxt = lds + ((t_ + 1) & 1) * TILE_BYTES;                                 \
    const int td = min(t_ + 2, T - 1);                                                   \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                   \
    barrier_raw(); /* every wave holds tile t in registers: its buffer may be restaged */ \
    _Pragma("unroll") for (int g = 0; g < 16; ++g) {                                     \
      _Pragma("unroll") for (int q = 0; q < 4; ++q) {                                    \
        AMDK8S_F8_MFMA1(CALO, CAHI, CBLO, CBHI, g >> 1, (g & 1) * 4 + q)                 \
        if (g < 8 && (q & 1)) dma_piece(td, 2 * g + (q >> 1));                           \
        if (g >= 8) AMDK8S_F8_READ(NALO, NAHI, NBLO, NBHI, nxt, (g - 8) * 4 + q)         \
      }                                                                                  \
      if (g == 7) {                                                                      \
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); /* tile t+1 landed (wave) */   \
        barrier_raw();                                    /* ... for every wave */       \
      }                                                                                  \
    }                                                                                    \
  }

  for (int t = 0; t < T; t += 2) {  // T even (host: K % 256 == 0)
    AMDK8S_F8_TILE(t, alo0, ahi0, blo0, bhi0, alo1, ahi1, blo1, bhi1)
    AMDK8S_F8_TILE(t + 1, alo1, ahi1, blo1, bhi1, alo0, ahi0, blo0, bhi0)
    // pad the MFMA → v_accvgpr hazard on the loop-exit edge inside the last iteration
    if (t + 2 >= T) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
    }
  }
#undef AMDK8S_F8_TILE
#undef AMDK8S_F8_READ
#undef AMDK8S_F8_MFMA1

  // ---- epilogue (as in the bf16 kernels) ----
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = wr * 128 + i * 16 + frow;
      const int n = wc * 128 + j * 16 + fq * 4;
      *reinterpret_cast<bf16x4*>(lds + m * C_STRIDE + n * 2) =
          __builtin_convertvector(acc[i][j], bf16x4);
    }
  __syncthreads();
  char* cbase = reinterpret_cast<char*>(C) + ((size_t)m0 * ldc + n0) * 2;
  const size_t ldc_b = (size_t)ldc * 2;
#pragma unroll 4
  for (int it = 0; it < BM * BN * 2 / (NT * 16); ++it) {
    const int row = it * 8 + (tid >> 5);
    const int ch = tid & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(lds + row * C_STRIDE + ch * 16);
    *reinterpret_cast<uint4*>(cbase + row * ldc_b + ch * 16) = v;
  }
}

extern "C" int amdk8s_gemm_fp8_nt(const void* A, const void* B, void* C, int M, int N, int K,
                                  int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (M % BM || N % BN || K % (2 * BK)) return (int)hipErrorInvalidValue;
  if (lda % 16 || ldb % 16 || ldc % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return (int)hipErrorInvalidValue;
  if (256ull * (unsigned long long)(lda > ldb ? lda : ldb) >= (1ull << 31))
    return (int)hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  // partition-aware tile order (tile_order.h): XCD corners of super-blocks, or GROUP_M order
  const int sb = amdk8s::tile_order_arg(M / BM, N / BN);
  hipLaunchKernelGGL(amdk8s_gemm_fp8_nt_256x256, dim3(nwg), dim3(NT), 0, stream,
                     (const uint8_t*)A, (const uint8_t*)B, (uint16_t*)C, M, N, K, lda, ldb, ldc, sb);
  return (int)hipGetLastError();
}

// out[s] = Σ_k A[m_s,k]·B[n_s,k] in fp32 for a list of sample coordinates (fp8 decoded by
// v_cvt_f32_fp8, independent of the MFMA path).
extern "C" __global__ void amdk8s_gemm_fp8_nt_sample_ref(const uint8_t* __restrict__ A,
                                                         const uint8_t* __restrict__ B,
                                                         const int* __restrict__ coords,
                                                         float* __restrict__ out, int nsamples,
                                                         int K, int lda, int ldb) {
  const int s = blockIdx.x;
  if (s >= nsamples) return;
  const int m = coords[2 * s], n = coords[2 * s + 1];
  float sum = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float a = __builtin_amdgcn_cvt_f32_fp8((int)A[(size_t)m * lda + k], 0);
    const float b = __builtin_amdgcn_cvt_f32_fp8((int)B[(size_t)n * ldb + k], 0);
    sum = fmaf(a, b, sum);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_down(sum, off, 64);
  __shared__ float part[16];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < (int)(blockDim.x + 63) / 64; ++w) tot += part[w];
    out[s] = tot;
  }
}

extern "C" int amdk8s_gemm_fp8_nt_sample_check(const void* A, const void* B, const int* coords,
                                               float* out, int nsamples, int K, int lda, int ldb,
                                               hipStream_t stream) {
  if (nsamples <= 0) return 0;
  hipLaunchKernelGGL(amdk8s_gemm_fp8_nt_sample_ref, dim3(nsamples), dim3(256), 0, stream,
                     (const uint8_t*)A, (const uint8_t*)B, coords, out, nsamples, K, lda, ldb);
  return (int)hipGetLastError();
}
