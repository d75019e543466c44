// Hand-written bf16 MFMA GEMM for MI355X (gfx950), ONE wave per SIMD variant.
//
//   C[M,N] (bf16) = A[M,K] (bf16, row-major) · B[N,K]ᵀ (bf16, row-major), fp32 accumulation.
//
// Same 256×256×64 block tile as gemm_bf16_gfx950.hip, but 256 threads = 4 waves (2 M × 2 N), each
// wave owning a 128×128 output sub-tile (8×8 tiles of v_mfma_f32_16x16x32_bf16, 256 accumulator
// registers per lane).  Why: per 64-deep K-tile the 8-wave 128×64 decomposition reads 192 KiB of
// LDS fragments per block, this one 128 KiB (each A/B fragment feeds 8 MFMAs instead of 4/8) — a
// third less LDS traffic and fewer instructions per MFMA, which on a DVFS-limited chip turns into
// clock (MI355X_MICROARCH.md "DVFS give-back").  The price is that no partner wave hides latency, so
// the wave software-pipelines itself:
//
//   * fragments are double-buffered by K-half (2 × 64 VGPRs): the 64 MFMAs of one K-half run while
//     the 16 ds_read_b128 of the next K-half are in flight (interleaved 1 read : 4 MFMAs with
//     sched_group_barrier);
//   * the LDS holds two full K-tiles (2 × 64 KiB, LDS-DMA with the source-side XOR swizzle of
//     gemm_bf16_gfx950.hip); tile t+2's 16 global_load_lds per thread are issued during tile t's
//     second K-half, interleaved 1 DMA : 4 MFMAs, right after the one barrier per K-tile;
//   * one `s_waitcnt vmcnt(0)` + raw s_barrier per K-tile: it retires tile t+1 (issued a whole
//     K-tile earlier) for every wave AND certifies every wave finished reading buffer t&1, which
//     the DMA of tile t+2 then overwrites.
//
// Shape contract (host-checked): M % 256 == 0, N % 256 == 0, K % 64 == 0, lda/ldb/ldc % 8 == 0,
// 16-B aligned base pointers.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

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

// Timing-only ablations (tools/gemm_w4_ablate.hip; results are WRONG): bit 0 drops the in-loop
// tile staging, bit 1 the in-loop fragment reads, bit 2 the per-K-tile barrier, bit 3 the
// per-K-tile vmcnt(0).
#ifndef AMDK8S_W4_ABLATE
#define AMDK8S_W4_ABLATE 0
#endif

#ifdef AMDK8S_W4_STAMPS
// Diagnostic build only (tools/gemm_w4_stamps.hip): s_memtime of wave 0 at 4 points of every K-tile
// (0 start, 1 K-half 0 done, 2 past the barrier, 3 K-half 1 done); stride = 4 × K-tiles.
__device__ unsigned long long* g_w4_stamps;
__device__ int g_w4_stamp_stride;
#define AMDK8S_W4_STAMP(T, SLOT)                                                            \
  if (tid == 0 && (T) * 4 + (SLOT) < g_w4_stamp_stride)                                     \
    g_w4_stamps[(size_t)blockIdx.x * g_w4_stamp_stride + (T) * 4 + (SLOT)] =                \
        __builtin_amdgcn_s_memtime();
#else
#define AMDK8S_W4_STAMP(T, SLOT)
#endif

__device__ __forceinline__ void barrier_raw() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ bf16x8 lds_read16(const char* p) {
  return *reinterpret_cast<const bf16x8*>(__builtin_assume_aligned(p, 16));
}

}  // namespace

// MODE 0: tiles staged by LDS-DMA with global_load_lds (64-bit per-lane address per piece);
// MODE 2: the same DMA as buffer_load_dwordx4 … lds — one 32-bit lane offset for every piece, the
// piece's row offset in an SGPR soffset, no per-piece address VALU; MODE 1: staged through 64
// VGPRs (global_load_dwordx4 → ds_write_b128 of the same lane-linear image), two phases of lead;
// MODE 3: MODE 0 with the next K-half's B fragments read first (all by mid-phase, A fragments as
// their rows retire) and no lgkmcnt(0) at the K-tile boundary (hipcc's counted waits instead).
template <int MODE>
__global__ void __launch_bounds__(NT, 1)
amdk8s_gemm_bf16_nt_256x256_w4(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
               uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc,
               int superblock) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  constexpr bool REG = MODE == 1;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1;  // A half this wave reads (rows wr*128..)
  const int wc = wave & 1;   // B half

  // ---- block → tile: bijective XCD remap, then GROUP_M-grouped order ----
  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  int wgid;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  int m0, n0;
  if (superblock) {
    // Round-major 16×16-tile super-blocks: the 256 tiles in flight at once (one per CU) form a
    // 4096×4096 block of C whose A/B panels (128 MiB at K = 8192) stay in the Infinity Cache; XCD x
    // owns a 4(M)×8(N) corner of it. Super-blocks are walked in snake order so consecutive rounds
    // share a panel set. Host guarantees tiles_m % 16 == tiles_n % 16 == 0.
    const int xcd = bid & 7, i = bid >> 3;
    const int round = i >> 5, j = i & 31;
    const int sb_n_count = tiles_n >> 4;
    const int sbm = round / sb_n_count;
    int sbn = round - sbm * sb_n_count;
    if (sbm & 1) sbn = sb_n_count - 1 - sbn;
    m0 = (sbm * 16 + (xcd >> 1) * 4 + (j & 3)) * BM;
    n0 = (sbn * 16 + (xcd & 1) * 8 + (j >> 2)) * BN;
  } else {
    const int group = wgid / (GROUP_M * tiles_n);
    const int first_m = group * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    const int in_group = wgid - group * GROUP_M * tiles_n;
    m0 = (first_m + in_group % gsz) * BM;
    n0 = (in_group / gsz) * BN;
  }

  // ---- LDS-DMA sources: instr j of wave w fills rows (j*4+w)*8 .. +8 of a 128-row half ----
  // Wave-uniform 64-bit bases (SGPRs) + one 32-bit per-lane offset per operand, so every DMA
  // address is saddr + voffset and no per-instruction 64-bit VGPR address stays live.
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

  // B fragments double-buffered by K-half; A fragments single-buffered: row I's next-K-half
  // fragment is read into fa[I] as soon as row I's 8 MFMAs of the current K-half are issued.
  bf16x8 fa[8], fb0[8], fb1[8];

  const int T = K / BK;

  // piece p (0..15) of K-tile t: j = p >> 2 (32-row stripe), h = (p >> 1) & 1 (half), p & 1: A/B
  // MODE 2 descriptors: the block's 256-row A / B panels (wave-uniform inputs only)
  const __amdgpu_buffer_rsrc_t rsrc_a = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(a_base), (short)0, (int)(256u * lda_b), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_b = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(b_base), (short)0, (int)(256u * ldb_b), 0x00020000);
  auto dma_piece = [&](int t, int p) {
    const int j = p >> 2, h = (p >> 1) & 1;
    char* dst = lds + (t & 1) * TILE_BYTES + wave * 1024 + j * 4096;
    if (MODE == 2) {
      const uint32_t rows = (uint32_t)(j * 32 + h * 128);
      if ((p & 1) == 0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void*)(dst + h * HALF_BYTES), 16, a_voff,
                                                 rows * lda_b + (uint32_t)t * (BK * 2), 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_b, (lds_void*)(dst + (2 + h) * HALF_BYTES), 16,
                                                 b_voff, rows * ldb_b + (uint32_t)t * (BK * 2), 0, 0);
      return;
    }
    if ((p & 1) == 0) {
      const char* src = a_base + (size_t)t * BK * 2 + (uint32_t)(j * 32 + h * 128) * lda_b + a_voff;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + h * HALF_BYTES), 16, 0, 0);
    } else {
      const char* src = b_base + (size_t)t * BK * 2 + (uint32_t)(j * 32 + h * 128) * ldb_b + b_voff;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (2 + h) * HALF_BYTES), 16, 0, 0);
    }
  };
  auto dma_tile = [&](int t) {
#pragma unroll
    for (int p = 0; p < 16; ++p) dma_piece(t, p);
  };
  // register staging: the same piece → S[p] (16 B/lane), later written lane-linearly to LDS
  u32x4 S[16];
  auto stage_load = [&](int t, int p) {
    const int j = p >> 2, h = (p >> 1) & 1;
    const char* src = (p & 1) == 0
        ? a_base + (size_t)t * BK * 2 + ((uint32_t)(j * 32 + h * 128) * lda_b + a_voff)
        : b_base + (size_t)t * BK * 2 + ((uint32_t)(j * 32 + h * 128) * ldb_b + b_voff);
    S[p] = *reinterpret_cast<const u32x4*>(__builtin_assume_aligned(src, 16));
  };
  auto stage_write = [&](int t, int p) {
    const int j = p >> 2, h = (p >> 1) & 1;
    char* dst = lds + (t & 1) * TILE_BYTES + wave * 1024 + j * 4096 +
                ((p & 1) ? (2 + h) : h) * HALF_BYTES + lane * 16;
    *reinterpret_cast<u32x4*>(__builtin_assume_aligned(dst, 16)) = S[p];
  };


#define AMDK8S_W4_READ(FA, FB, BUF, FO)                                     \
  _Pragma("unroll") for (int i = 0; i < 8; ++i) {                           \
    FA[i] = lds_read16((BUF) + a_off + i * 2048 + (FO));                    \
    FB[i] = lds_read16((BUF) + b_off + i * 2048 + (FO));                    \
  }
  // MFMAs as inline asm with the accumulator pinned in AGPRs ("+a"): the compiler's own MFMA
  // lowering rotates the 256 accumulators between AGPRs and VGPRs every K-tile (hundreds of
  // v_accvgpr moves per iteration). The "memory" clobber pins program order, so the interleave
  // below (1 ds_read [+ 1 LDS-DMA] per 4 MFMAs) is exactly what is emitted. MFMA→MFMA on the same
  // accumulator needs no wait states; the epilogue pads the MFMA→VALU hazard itself.
#define AMDK8S_W4_MFMA1(I, J, FA, FB)                                                   \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"                                \
               : "+a"(acc[I][J]) : "v"(FB[J]), "v"(FA[I]) : "memory")
#define AMDK8S_W4_MFMA4(G, FA, FB)                                                      \
  AMDK8S_W4_MFMA1((G) >> 1, ((G) & 1) * 4 + 0, FA, FB);                                 \
  AMDK8S_W4_MFMA1((G) >> 1, ((G) & 1) * 4 + 1, FA, FB);                                 \
  AMDK8S_W4_MFMA1((G) >> 1, ((G) & 1) * 4 + 2, FA, FB);                                 \
  AMDK8S_W4_MFMA1((G) >> 1, ((G) & 1) * 4 + 3, FA, FB)
  // one K-half of MFMAs on (FA, FB) with the next fragment set (NA, NB) read from BUF+FO
  // (READ) and one DMA piece per 4 MFMAs (DMA)
// REG staging: every other group writes S[PB + g/2] (tile TW) to LDS when W, then reloads it
// with the same piece of tile TL when L (TL clamped to the last tile: a harmless re-read).
#define AMDK8S_W4_PHASE(FA, FB, NB, BUF, FO, READ, DMA, TD, W, TW, L, TL, PB)           \
  _Pragma("unroll") for (int g = 0; g < 16; ++g) {                                      \
    AMDK8S_W4_MFMA4(g, FA, FB);                                                         \
    if ((READ) && !(AMDK8S_W4_ABLATE & 2)) {                                            \
      if (MODE == 3) {                                                                  \
        if (g < 8) NB[g] = lds_read16((BUF) + b_off + g * 2048 + (FO));                 \
        if (g & 1) FA[g >> 1] = lds_read16((BUF) + a_off + (g >> 1) * 2048 + (FO));     \
      } else if (g & 1) {                                                               \
        FA[g >> 1] = lds_read16((BUF) + a_off + (g >> 1) * 2048 + (FO));                \
      } else {                                                                          \
        NB[g >> 1] = lds_read16((BUF) + b_off + (g >> 1) * 2048 + (FO));                \
      }                                                                                 \
    }                                                                                   \
    if (!REG && (DMA) && !(AMDK8S_W4_ABLATE & 1)) dma_piece(TD, g);                     \
    if (REG && (g & 1) && !(AMDK8S_W4_ABLATE & 1)) {                                    \
      if (W) stage_write(TW, (PB) + (g >> 1));                                          \
      if (L) stage_load(min((TL), T - 1), (PB) + (g >> 1));                             \
    }                                                                                   \
  }

  // ---- prologue: tiles 0 (and 1) in flight; K-half 0 of tile 0 into registers ----
  if (REG) {
    // buf0 = tile 0, buf1 = tile 1 pieces 0..7; S[8..15] = tile 1 pieces 8..15 (written in tile
    // 0's first K-half), S[0..7] = tile 2 pieces 0..7 (written in tile 0's second K-half)
#pragma unroll
    for (int p = 0; p < 16; ++p) stage_load(0, p);
#pragma unroll
    for (int p = 0; p < 16; ++p) stage_write(0, p);
#pragma unroll
    for (int p = 0; p < 16; ++p) stage_load(min(1, T - 1), p);
#pragma unroll
    for (int p = 0; p < 8; ++p) stage_write(1, p);
#pragma unroll
    for (int p = 0; p < 8; ++p) stage_load(min(2, T - 1), p);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else {
    dma_tile(0);
    if (T > 1) {
      dma_tile(1);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  barrier_raw();
  AMDK8S_W4_READ(fa, fb0, lds, fo0)
  if (MODE != 3) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // One K-tile: K-half 0 on (fa0, fb0) while K-half 1 is read; barrier; K-half 1 on (fa1, fb1)
  // while K-half 0 of the next tile is read and (DMA) the tile after next is staged.
  // NEXT: a next tile exists; DMA: tile t+2 exists.  Peeled so the steady loop has no branches.
#define AMDK8S_W4_TILE(NEXT, DMA)                                                 \
  {                                                                                   \
    const char* cur = lds + (t & 1) * TILE_BYTES;                                     \
    const char* nxt = lds + ((t + 1) & 1) * TILE_BYTES;                               \
    AMDK8S_W4_STAMP(t, 0)                                                             \
    AMDK8S_W4_PHASE(fa, fb0, fb1, cur, fo1, true, false, t,                           \
                    NEXT, t + 1, DMA, t + 2, 8)                                       \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                \
    AMDK8S_W4_STAMP(t, 1)                                                             \
    if (NEXT) {                                                                       \
      if (!REG && !(AMDK8S_W4_ABLATE & 8))                                            \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* tile t+1 landed */        \
      if (!(AMDK8S_W4_ABLATE & 4)) barrier_raw();                                     \
      AMDK8S_W4_STAMP(t, 2)                                                           \
      AMDK8S_W4_PHASE(fa, fb1, fb0, nxt, fo0, true, DMA, t + 2,                       \
                      DMA, t + 2, DMA, t + 3, 0)                                      \
      if (MODE != 3) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");               \
      AMDK8S_W4_STAMP(t, 3)                                                           \
    } else {                                                                          \
      AMDK8S_W4_PHASE(fa, fb1, fb0, nxt, fo0, false, false, t,                        \
                      false, t, false, t, 0)                                          \
    }                                                                                 \
  }

  int t = 0;
  for (; t + 2 < T; ++t) AMDK8S_W4_TILE(true, true)
  if (t + 1 < T) {
    AMDK8S_W4_TILE(true, false)
    ++t;
  }
  AMDK8S_W4_TILE(false, false)
#undef AMDK8S_W4_TILE
#undef AMDK8S_W4_READ
#undef AMDK8S_W4_MFMA1
#undef AMDK8S_W4_MFMA4
#undef AMDK8S_W4_PHASE

  // ---- epilogue: acc → bf16 → padded LDS image → 16-B coalesced stores ----
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");  // MFMA D → VALU read hazard (asm MFMAs)
  __syncthreads();  // every wave done with the last K-tile's LDS before it is overwritten
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

extern "C" int amdk8s_gemm_bf16_nt_w4(const void* A, const void* B, void* C, int M, int N, int K,
                                      int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return (int)hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  // 16×16-tile super-block order whenever the tile grid allows it (AMDK8S_W4_SUPERBLOCK=0 turns
  // it off for A/B runs): +8-10 % at 8192³ and 16384²×4096 (docs/gemm_tuning.md)
  const char* sbenv = getenv("AMDK8S_W4_SUPERBLOCK");
  const int sb = (M / BM) % 16 == 0 && (N / BN) % 16 == 0 && !(sbenv && sbenv[0] == '0');
  const char* menv = getenv("AMDK8S_W4_MODE");
  const int mode = menv ? atoi(menv) : 0;
  if (mode == 1)
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4<1>, dim3(nwg), dim3(NT), 0, stream,
                       (const uint16_t*)A, (const uint16_t*)B, (uint16_t*)C, M, N, K, lda, ldb, ldc, sb);
  else if (mode == 3)
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4<3>, dim3(nwg), dim3(NT), 0, stream,
                       (const uint16_t*)A, (const uint16_t*)B, (uint16_t*)C, M, N, K, lda, ldb, ldc, sb);
  else if (mode == 2)
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4<2>, dim3(nwg), dim3(NT), 0, stream,
                       (const uint16_t*)A, (const uint16_t*)B, (uint16_t*)C, M, N, K, lda, ldb, ldc, sb);
  else
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4<0>, dim3(nwg), dim3(NT), 0, stream,
                       (const uint16_t*)A, (const uint16_t*)B, (uint16_t*)C, M, N, K, lda, ldb, ldc, sb);
  return (int)hipGetLastError();
}
