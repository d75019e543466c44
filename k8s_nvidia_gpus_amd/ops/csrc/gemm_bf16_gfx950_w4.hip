// Hand-written bf16 MFMA GEMM for MI355X (gfx950), ONE wave per SIMD variant.
//
//   C[M,N] (bf16) = A[M,K] (bf16, row-major) · B[N,K]ᵀ (bf16, row-major), fp32 accumulation.
//
// Same 256×256×64 block tile as gemm_bf16_gfx950.hip, but 256 threads = 4 waves (2 M × 2 N), each
// wave owning a 128×128 output sub-tile (8×8 tiles of v_mfma_f32_16x16x32_bf16, 256 accumulator
// registers per lane, pinned in AGPRs by asm MFMAs).  Why: per 64-deep K-tile the 8-wave 128×64
// decomposition reads 192 KiB of LDS fragments per block, this one 128 KiB (each A/B fragment
// feeds 8 MFMAs instead of 4/8).  The price is that no partner wave hides latency, so the wave
// software-pipelines itself.  The LDS holds two full K-tiles (2 × 64 KiB) filled by LDS-DMA with
// the source-side XOR swizzle of gemm_bf16_gfx950.hip; two schedules share everything else:
//
//   REGION (default): each operand's half of an LDS buffer is restaged as soon as every wave has
//     read it, so the DMA pieces spread over both K-halves (three barriers per tile); reads and DMA
//     pieces go one per MFMA gap; the next tile's fragments are never drained at the tile boundary
//     (hipcc's counted lgkmcnt waits sit at their first use).  Ties INTERLEAVED where A + B sit in
//     the Infinity Cache, +4…34 % where they stream from MALL/HBM (profiles/r01_session3/,
//     docs/gemm_tuning.md).
//   INTERLEAVED: K-half 0's 64 MFMAs run while K-half 1's 16 fragments are read; barrier; K-half
//     1's MFMAs run while the next tile's K-half 0 is read AND tile t+2's 16 DMA pieces are issued
//     (1 read + 1 global_load_lds per 4 MFMAs).  One vmcnt(0) + barrier per tile.  Fallback for
//     panels past 32-bit buffer offsets; A/B reference.
//
// Shape contract (host-checked): M % 256 == 0, N % 256 == 0, K % 64 == 0, lda/ldb/ldc % 8 == 0,
// 16-B aligned base pointers.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "tile_order.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 64;
constexpr int NT = 256;
constexpr int HALF_BYTES = 128 * BK * 2;     // 128 rows × 128 B
constexpr int TILE_BYTES = 4 * HALF_BYTES;   // A0 A1 B0 B1 = 64 KiB
constexpr int C_STRIDE = BN * 2 + 16;        // padded epilogue row
constexpr int LDS_BYTES = BM * C_STRIDE;     // 135168 ≥ 2 × TILE_BYTES
static_assert(LDS_BYTES >= 2 * TILE_BYTES, "LDS too small");
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void barrier_raw() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ bf16x8 lds_read16(const char* p) {
  return *reinterpret_cast<const bf16x8*>(__builtin_assume_aligned(p, 16));
}

}  // namespace

// K-loop schedules (template argument SCHED)
constexpr int SCHED_INTERLEAVED = 0;
constexpr int SCHED_REGION = 1;

template <int SCHED>
__global__ void __launch_bounds__(NT, 1)
amdk8s_gemm_bf16_nt_256x256_w4(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                               uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                               int ldc, int order) {
  constexpr bool BUFFER_DMA = SCHED == SCHED_REGION;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1;  // A half this wave reads (rows wr*128..)
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

  // ---- LDS-DMA sources: piece j of wave w fills rows (j*4+w)*8 .. +8 of a 128-row half ----
  // Wave-uniform bases + one 32-bit per-lane offset per operand; the LDS image is lane-linear per
  // piece, so the XOR swizzle is applied on the source chunk (dchunk) and undone on the read.
  const uint32_t lda_b = (uint32_t)lda * 2, ldb_b = (uint32_t)ldb * 2;
  const int drow = wave * 8 + (lane >> 3);                  // row inside the 32-row stripe
  const int dchunk = (lane & 7) ^ ((drow >> 1) & 7);        // logical chunk for physical lane&7
  const char* a_base = reinterpret_cast<const char*>(A) + (size_t)m0 * lda_b;
  const char* b_base = reinterpret_cast<const char*>(B) + (size_t)n0 * ldb_b;
  const uint32_t a_voff = (uint32_t)drow * lda_b + dchunk * 16;
  const uint32_t b_voff = (uint32_t)drow * ldb_b + dchunk * 16;

  // ---- fragment read offsets ----
  const int frow = lane & 15;
  const int fq = lane >> 4;
  const int fo0 = frow * 128 + (((0 + fq) ^ (frow >> 1)) << 4);   // K-half 0: chunks 0..3
  const int fo1 = frow * 128 + (((4 + fq) ^ (frow >> 1)) << 4);   // K-half 1: chunks 4..7
  const int a_off = wr * HALF_BYTES;
  const int b_off = 2 * HALF_BYTES + wc * HALF_BYTES;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int T = K / BK;

  // piece p (0..15) of K-tile t: j = p >> 2 (32-row stripe), h = (p >> 1) & 1 (half), p & 1: A/B.
  // REGION issues it as buffer_load … lds (row offset in an SGPR soffset, one lane-offset VGPR per
  // operand: its 128 fragment VGPRs leave no room for 16 per-piece 64-bit addresses).
  const __amdgpu_buffer_rsrc_t rsrc_a = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(a_base), (short)0, (int)(256u * lda_b), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_b = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(b_base), (short)0, (int)(256u * ldb_b), 0x00020000);
  auto dma_piece = [&](int t, int p) {
    const int j = p >> 2, h = (p >> 1) & 1;
    char* dst = lds + (t & 1) * TILE_BYTES + wave * 1024 + j * 4096;
    const uint32_t rows = (uint32_t)(j * 32 + h * 128);
    if (BUFFER_DMA) {
      if ((p & 1) == 0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void*)(dst + h * HALF_BYTES), 16,
                                                 a_voff, rows * lda_b + (uint32_t)t * (BK * 2), 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_b, (lds_void*)(dst + (2 + h) * HALF_BYTES),
                                                 16, b_voff, rows * ldb_b + (uint32_t)t * (BK * 2),
                                                 0, 0);
    } else if ((p & 1) == 0) {
      const char* src = a_base + (size_t)t * BK * 2 + (rows * lda_b + a_voff);
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + h * HALF_BYTES), 16, 0, 0);
    } else {
      const char* src = b_base + (size_t)t * BK * 2 + (rows * ldb_b + b_voff);
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (2 + h) * HALF_BYTES), 16,
                                       0, 0);
    }
  };
  auto dma_tile = [&](int t) {
#pragma unroll
    for (int p = 0; p < 16; ++p) dma_piece(t, p);
  };

  // MFMAs as inline asm with the accumulator pinned in AGPRs ("+a"): the compiler's own MFMA
  // lowering rotates the 256 accumulators between AGPRs and VGPRs every K-tile (hundreds of
  // v_accvgpr moves per iteration). The "memory" clobber pins program order, so the interleave
  // below is exactly what is emitted. MFMA→MFMA on the same accumulator needs no wait states;
  // the epilogue pads the MFMA→VALU hazard itself.
#define AMDK8S_W4_MFMA1(I, J, FA, FB)                                                   \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"                                \
               : "+a"(acc[I][J]) : "v"(FB[J]), "v"(FA[I]) : "memory")
#define AMDK8S_W4_MFMA4(G, FA, FB)                                                      \
  AMDK8S_W4_MFMA1((G) >> 1, ((G) & 1) * 4 + 0, FA, FB);                                 \
  AMDK8S_W4_MFMA1((G) >> 1, ((G) & 1) * 4 + 1, FA, FB);                                 \
  AMDK8S_W4_MFMA1((G) >> 1, ((G) & 1) * 4 + 2, FA, FB);                                 \
  AMDK8S_W4_MFMA1((G) >> 1, ((G) & 1) * 4 + 3, FA, FB)


  if constexpr (SCHED == SCHED_REGION) {
    // All four fragment sets are register-resident (128 VGPRs): a0/b0 = K-half 0, a1/b1 = K-half 1.
    // Per K-tile t (buffer cur = t & 1, tile t+2 restaged into it):
    //   K-half 0 on (a0, b0): groups 0-4 read b1 and a1[0] of tile t; lgkmcnt(0) + barrier #1 after
    //     group 5 → every wave is done with cur's B region; groups 6-12 read a1[1..7], groups 6-13
    //     issue the 8 B pieces of tile t+2 (one per group);
    //   K-half 1 on (a1, b1): lgkmcnt(0) + barrier #2 after group 1 → cur's A region is free; the 8
    //     A pieces go out in groups 2-9; vmcnt(16) (tile t+1, issued a whole tile earlier, landed
    //     for this wave) + barrier #3 (for every wave) after group 9; groups 10-15 read a0/b0 of
    //     tile t+1 from the other buffer, in first-use order, with no drain at the tile boundary.
    // Past the end the DMA is clamped to tile T-1 (it re-stages identical bytes into a region no
    // read needs any more) and the reads of "tile T" fetch unused bytes, so the body has no
    // branches and the accumulators only ever flow through it: a peeled tail made hipcc permute
    // the accumulators between AGPRs right behind asm MFMAs it cannot see (0.4 % wrong outputs at
    // 768×256×1024 in an earlier schedule), so the exit edge is padded inside the last iteration.
    bf16x8 a0[8], b0[8], a1[8], b1[8];
    // x-th fragment read of a K-half in first-use order: b[0..3], a[0], b[4..7], a[1..7]
    auto read_k0 = [&](const char* buf, int x) {
      if (x < 4) b0[x] = lds_read16(buf + b_off + x * 2048 + fo0);
      else if (x == 4) a0[0] = lds_read16(buf + a_off + fo0);
      else if (x < 9) b0[x - 1] = lds_read16(buf + b_off + (x - 1) * 2048 + fo0);
      else a0[x - 8] = lds_read16(buf + a_off + (x - 8) * 2048 + fo0);
    };
    auto read_k1 = [&](const char* buf, int x) {
      if (x < 4) b1[x] = lds_read16(buf + b_off + x * 2048 + fo1);
      else if (x == 4) a1[0] = lds_read16(buf + a_off + fo1);
      else if (x < 9) b1[x - 1] = lds_read16(buf + b_off + (x - 1) * 2048 + fo1);
      else a1[x - 8] = lds_read16(buf + a_off + (x - 8) * 2048 + fo1);
    };
    // at(k): the MFMA of a group after which its k-th kind of op is issued — one op per MFMA gap
    // (an MFMA leaves ≈8 issue cycles of slack; bundling a group's reads + DMA behind its 4th
    // MFMA cost 2.3-3.2 % on the streaming shapes, profiles/r01_session3/sweep_fine.txt)
    auto at = [](int k) { return k; };
    dma_tile(0);
    dma_tile(min(1, T - 1));
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    barrier_raw();
#pragma unroll
    for (int x = 0; x < 16; ++x) read_k0(lds, x);

    for (int t = 0; t < T; ++t) {
      const char* cur = lds + (t & 1) * TILE_BYTES;
      const char* nxt = lds + ((t + 1) & 1) * TILE_BYTES;
      const int td = min(t + 2, T - 1);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          AMDK8S_W4_MFMA1(g >> 1, (g & 1) * 4 + q, a0, b0);
          if (q == at(0)) {
            if (g < 4) read_k1(cur, 2 * g);
            if (g == 4) read_k1(cur, 8);                 // b1[7]
            if (g >= 6 && g < 13) read_k1(cur, g + 3);   // a1[1..7]
          }
          if (q == at(2) && g < 4) read_k1(cur, 2 * g + 1);
          if (q == at(1) && g >= 6 && g < 14) dma_piece(td, 2 * (g - 6) + 1);  // odd pieces: B
          if (q == 3 && g == 5) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier_raw();  // the B region of cur is free (every b1 read is done)
          }
        }
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          AMDK8S_W4_MFMA1(g >> 1, (g & 1) * 4 + q, a1, b1);
          if (q == at(1) && g >= 2 && g < 10) dma_piece(td, 2 * (g - 2));  // even pieces: A
          if (g >= 10) {  // 16 next-tile reads over groups 10-15: 2, 3, 3, 2, 3, 3
            const int x0 = (g - 10) * 16 / 6, x1 = (g - 9) * 16 / 6;
            if (q == at(0)) read_k0(nxt, x0);
            if (q == at(2) && x0 + 1 < x1) read_k0(nxt, x0 + 1);
            if (q == at(3) && x0 + 2 < x1) read_k0(nxt, x0 + 2);
          }
          if (q == 3 && g == 1) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            barrier_raw();  // the A region of cur is free
          }
          if (q == 3 && g == 9) {
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile t+1 landed (this wave)
            barrier_raw();                                       // ... for every wave
          }
        }
      }
      if (t + 1 >= T) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
      }
    }
  } else {
    // B fragments double-buffered by K-half; A fragments single-buffered: row I's next-K-half
    // fragment is read into fa[I] as soon as row I's 8 MFMAs of the current K-half are issued.
    bf16x8 fa[8], fb0[8], fb1[8];

    // one K-half of MFMAs on (FA, FB), reading the next K-half (FA in place, NB) from BUF+FO
    // (READ) and issuing DMA piece g of tile TD after every 4 MFMAs (DMA)
#define AMDK8S_W4_PHASE(FA, FB, NB, BUF, FO, READ, DMA, TD)                             \
  _Pragma("unroll") for (int g = 0; g < 16; ++g) {                                      \
    AMDK8S_W4_MFMA4(g, FA, FB);                                                         \
    if (READ) {                                                                         \
      if (g & 1) FA[g >> 1] = lds_read16((BUF) + a_off + (g >> 1) * 2048 + (FO));      \
      else NB[g >> 1] = lds_read16((BUF) + b_off + (g >> 1) * 2048 + (FO));             \
    }                                                                                   \
    if (DMA) dma_piece(TD, g);                                                          \
  }

    // ---- prologue: tiles 0 (and 1) in flight; K-half 0 of tile 0 into registers ----
    dma_tile(0);
    if (T > 1) {
      dma_tile(1);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier_raw();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      fa[i] = lds_read16(lds + a_off + i * 2048 + fo0);
      fb0[i] = lds_read16(lds + b_off + i * 2048 + fo0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    // One K-tile: K-half 0 on (fa, fb0) while K-half 1 is read; barrier; K-half 1 on (fa, fb1)
    // while K-half 0 of the next tile is read and (DMA) the tile after next is staged.
    // NEXT: a next tile exists; DMA: tile t+2 exists.  Peeled so the steady loop has no branches.
#define AMDK8S_W4_TILE(NEXT, DMA)                                                       \
  {                                                                                     \
    const char* cur = lds + (t & 1) * TILE_BYTES;                                       \
    const char* nxt = lds + ((t + 1) & 1) * TILE_BYTES;                                 \
    AMDK8S_W4_PHASE(fa, fb0, fb1, cur, fo1, true, false, t)                             \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                  \
    if (NEXT) {                                                                         \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* tile t+1 landed */            \
      barrier_raw();                                                                    \
      AMDK8S_W4_PHASE(fa, fb1, fb0, nxt, fo0, true, DMA, t + 2)                         \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                \
    } else {                                                                            \
      AMDK8S_W4_PHASE(fa, fb1, fb0, nxt, fo0, false, false, t)                          \
    }                                                                                   \
  }

    int t = 0;
    for (; t + 2 < T; ++t) AMDK8S_W4_TILE(true, true)
    if (t + 1 < T) {
      AMDK8S_W4_TILE(true, false)
      ++t;
    }
    AMDK8S_W4_TILE(false, false)
#undef AMDK8S_W4_TILE
#undef AMDK8S_W4_PHASE
  }
#undef AMDK8S_W4_MFMA1
#undef AMDK8S_W4_MFMA4

  // ---- epilogue: acc → bf16 → padded LDS image → 16-B coalesced stores ----
  // MFMA D → VALU read hazard (asm MFMAs hipcc cannot see): the pads must sit between the last
  // MFMA and the first v_accvgpr_read. Every accumulator is then "redefined" by an empty asm
  // after the pads, so no read of it (nor a register-allocation copy) can be placed above them.
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // REGION re-stages clamped tiles at the end
  __syncthreads();  // every wave done with the last K-tile's LDS (and its DMAs) before overwrite
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

// Schedule choice: REGION (ties INTERLEAVED where A + B sit in the Infinity Cache, +4…34 % where
// they stream from MALL/HBM); INTERLEAVED when a 256-row panel needs offsets past 2 GiB, or with
// AMDK8S_W4_SCHEDULE=interleaved (A/B runs).
extern "C" int amdk8s_gemm_bf16_nt_w4(const void* A, const void* B, void* C, int M, int N, int K,
                                      int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return (int)hipErrorInvalidValue;
  // the REGION schedule addresses each 256-row panel with a 32-bit buffer offset
  const bool panel_fits = 256ull * (unsigned long long)(lda > ldb ? lda : ldb) * 2 < (1ull << 31);
  const int nwg = (M / BM) * (N / BN);
  // super-block order whenever the tile grid allows it (AMDK8S_W4_SUPERBLOCK=0 turns it off for
  // A/B runs): +8-10 % at 8192³ and 16384²×4096 in SPX (docs/gemm_tuning.md); partition-aware tile order (tile_order.h): XCD corners of super-blocks, or GROUP_M order
  const int sb = amdk8s::tile_order_arg(M / BM, N / BN);
  const char* schenv = getenv("AMDK8S_W4_SCHEDULE");
  const bool region = panel_fits && !(schenv && schenv[0] == 'i');
  const uint16_t* a = (const uint16_t*)A;
  const uint16_t* b = (const uint16_t*)B;
  uint16_t* c = (uint16_t*)C;
  if (region)
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4<SCHED_REGION>, dim3(nwg), dim3(NT), 0, stream,
                       a, b, c, M, N, K, lda, ldb, ldc, sb);
  else
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4<SCHED_INTERLEAVED>, dim3(nwg), dim3(NT), 0,
                       stream, a, b, c, M, N, K, lda, ldb, ldc, sb);
  return (int)hipGetLastError();
}
