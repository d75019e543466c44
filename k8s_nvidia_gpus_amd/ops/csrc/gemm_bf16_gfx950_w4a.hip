// Hand-scheduled bf16 MFMA GEMM for MI355X (gfx950): the w4 kernel (gemm_bf16_gfx950_w4.hip) with
// its whole K-loop as generated assembly.
//
//   C[M,N] (bf16) = A[M,K] (bf16, row-major) · B[N,K]ᵀ (bf16, row-major), fp32 accumulation.
//
// Same geometry, LDS image and REGION op placement as w4 (256×256×64 block tile, 4 waves of
// 128×128, v_mfma_f32_16x16x32_bf16 into 256 AGPRs, two 64 KiB LDS-DMA buffers with the
// source-side XOR swizzle, one op per MFMA gap, three barriers per K-tile). What changes is who
// writes the instruction stream: tools/gen_gemm_w4a_kloop.py emits the prologue DMA, the K-loop
// (unrolled over the two buffer parities) and the accumulator → bf16 → LDS C-image conversion with
// every register explicit. hipcc's version of the same loop carries ≈ 27 more non-MFMA instructions
// per K-tile than hipBLASLt's assembly kernel of this geometry (counted lgkmcnt waits that also
// count LDS-DMA, s_mov m0 + s_nop pairs, per-piece SALU address math); here the DMA source advances
// by one 64-bit rsrc add per operand per K-tile, M0 is set one MFMA ahead of its DMA, and the
// lgkmcnt before each MFMA is the exact in-order count (docs/gemm_tuning.md, session 4).
//
// Shape contract (host-checked): M % 256 == 0, N % 256 == 0, K % 64 == 0, lda/ldb/ldc % 8 == 0,
// 16-B aligned base pointers, 256·lda·2 and 256·ldb·2 < 2³¹ (32-bit panel offsets).
//
// Epilogue variants (amdk8s_gemm_w4a_epi, the DiT / UNet projections; bf16 or fp16): any M — the
// last row panel's buffer descriptor covers only its valid rows, so the DMA reads zeros past M and
// those rows are not stored — and the 16-B store pass adds the bias and optionally applies
// tanh-GELU to each C value (fp32 maths on the 16-bit-rounded product), or (RESID) folds the
// product into an fp32 residual stream in place, x += gate · (C + bias), the DiT's gated update
// (the same bf16-rounded product an nn.Linear would hand to that update).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gemm_bf16_gfx950_w4a_kloop.inc"

#include "tile_order.h"

namespace {

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 64;
constexpr int NT = 256;
constexpr int HALF_BYTES = 128 * BK * 2;     // 128 rows × 128 B
constexpr int C_STRIDE = BN * 2 + 16;        // padded epilogue row (matches the generator)
constexpr int LDS_BYTES = BM * C_STRIDE;     // 135168 ≥ 2 × 64 KiB K-tile buffers
#ifndef AMDK8S_W4_GROUP_M
#define AMDK8S_W4_GROUP_M 8
#endif
// A/B knob (build-time).  At M = 32000 (a 32k prompt) 4 and 16 are within 1-2 % of 8 on q|k|v,
// o_proj and gate|up, better and worse by shape (profiles/r06/gemm32k_group_m/)
constexpr int GROUP_M = AMDK8S_W4_GROUP_M;

typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

}  // namespace

// SCHED: generated K-loop schedule; SCHED == kF16 runs the default schedule on fp16 operands
// (v_mfma_f32_16x16x32_f16, fp16 C) — same fragment layout, LDS image and cycles as bf16.
constexpr int kF16 = 16;

constexpr int kEpiNone = 0, kEpiBias = 1, kEpiBiasGelu = 2, kEpiResid = 3, kEpiSwiGLU = 4;

// Two 16-bit C values of one dword → fp32 (bf16, or fp16 under the kF16 schedule).
template <bool H>
__device__ __forceinline__ float w4a_lo(uint32_t v) {
  if constexpr (H) return (float)__builtin_bit_cast(_Float16, (uint16_t)(v & 0xffffu));
  else return __uint_as_float(v << 16);
}
template <bool H>
__device__ __forceinline__ float w4a_hi(uint32_t v) {
  if constexpr (H) return (float)__builtin_bit_cast(_Float16, (uint16_t)(v >> 16));
  else return __uint_as_float(v & 0xffff0000u);
}
template <bool H>
__device__ __forceinline__ uint32_t w4a_pack(float lo, float hi) {
  if constexpr (H) {
    const __attribute__((ext_vector_type(2))) _Float16 p = {(_Float16)lo, (_Float16)hi};
    return __builtin_bit_cast(uint32_t, p);
  } else {
    const __attribute__((ext_vector_type(2))) __bf16 p = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, p);
  }
}

// RESID operands (fp32 residual stream and optional per-sample gate rows).
struct W4aResid {
  float* x;
  const float* gate;
  int ldx, rows_per_gate, gate_stride;
};

// silu(g) · u of the 16-bit-rounded gate and up products, exactly as the LLM prefill's separate
// swiglu_f16 pass computes it from the stored gate|up tensor (llm_prefill.hip), so fusing it
// changes no bits
__device__ __forceinline__ float w4a_swiglu(float g, float u) { return g / (1.f + __expf(-g)) * u; }

__device__ __forceinline__ float w4a_gelu_tanh(float v) {
  // 0.5 v (1 + tanh(√(2/π)(v + 0.044715 v³))) = v · sigmoid(2u) = v / (1 + 2^t), t = −2u·log2 e:
  // one v_exp_f32 and one v_rcp_f32 (no IEEE division sequence — the epilogue is VALU-bound)
  const float t = v * fmaf(-0.10294324f, v * v, -2.3022082f);
  return v * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(t));
}

template <int SCHED, int EPI = kEpiNone>
__global__ void __launch_bounds__(NT, 1)
amdk8s_gemm_bf16_nt_256x256_w4a(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                int ldc, int order, int nt_store,
                                const uint16_t* __restrict__ bias = nullptr,
                                W4aResid resid = W4aResid{}, int ksplit = 1,
                                long slice_stride = 0) {
  constexpr bool H = SCHED == kF16;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1;  // A half this wave reads
  const int wc = wave & 1;   // B half

  // ---- block → tile: per-partition XCD corners of super-blocks, or GROUP_M order (tile_order.h) ----
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  // split-K (the partial last wave of amdk8s_gemm_w4a_hybrid): ksplit adjacent workgroups share
  // one tile, each a contiguous range of its K-tiles, writing a 16-bit partial tile to its slice
  const int ks = ksplit > 1 ? ksplit : 1;
  const int bid = blockIdx.x / ks, slice = blockIdx.x - bid * ks;
  int m0, n0;
  {
    int tm, tn;
    amdk8s::block_tile(bid, tiles_m, tiles_n, order, GROUP_M, tm, tn);  // tile_order.h
    m0 = tm * BM;
    n0 = tn * BN;
  }
  if (ks > 1) C += slice * slice_stride;

  // ---- operands of the generated body (register map in tools/gen_gemm_w4a_kloop.py) ----
  const uint32_t lda_b = (uint32_t)lda * 2, ldb_b = (uint32_t)ldb * 2;
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
  const int t_all = K / BK;
  const int t_lo = slice * t_all / ks;
  const uint64_t a_addr = (uint64_t)(uintptr_t)A + (uint64_t)m0 * lda_b + (uint64_t)t_lo * BK * 2;
  const uint64_t b_addr = (uint64_t)(uintptr_t)B + (uint64_t)n0 * ldb_b + (uint64_t)t_lo * BK * 2;
  const uint32_t a_lo = (uint32_t)a_addr, a_hi = (uint32_t)(a_addr >> 32);
  const uint32_t b_lo = (uint32_t)b_addr, b_hi = (uint32_t)(b_addr >> 32);
  // the last row panel's descriptor ends at row M: the DMA reads zeros past it (M tail)
  const uint32_t nrec_a = (uint32_t)min(BM, M - m0) * lda_b, nrec_b = 256u * ldb_b;
  const int T = (slice + 1) * t_all / ks - t_lo;

#define AMDK8S_W4A_OPERANDS                                                                \
  : "s"(T), "s"(a_lo), "s"(a_hi), "s"(nrec_a), "s"(b_lo), "s"(b_hi), "s"(nrec_b), "s"(lda_b),  \
    "s"(ldb_b), "s"(dma_lds), "v"(ra0), "v"(ra1), "v"(rb0), "v"(rb1), "v"(a_voff), "v"(b_voff), \
    "v"(cbase)                                                                                 \
  : AMDK8S_W4A_CLOBBERS
  static_assert(AMDK8S_W4A_NUM_SCHEDULES == 3, "one branch per generated schedule");
  if constexpr (SCHED == kF16) asm volatile(AMDK8S_W4A_F16_ASM : AMDK8S_W4A_OPERANDS);
  else if constexpr (SCHED == 0) asm volatile(AMDK8S_W4A_ASM_0 : AMDK8S_W4A_OPERANDS);
  else if constexpr (SCHED == 1) asm volatile(AMDK8S_W4A_ASM_1 : AMDK8S_W4A_OPERANDS);
  else asm volatile(AMDK8S_W4A_ASM_2 : AMDK8S_W4A_OPERANDS);
#undef AMDK8S_W4A_OPERANDS
  __syncthreads();  // every wave's quarter of the bf16 C image is in LDS

  // ---- 16-B coalesced stores of the 256×256 bf16 tile ----
  const size_t ldc_b = (size_t)ldc * 2;
  const int rows_valid = min(BM, M - m0);
  if constexpr (EPI == kEpiSwiGLU) {
    // B rows come tile-interleaved (each 256-row tile: 128 gate rows, then the same 128 up rows):
    // columns c and c + 128 of the C image are the gate and up of output column n0 / 2 + c, so the
    // tile stores 256 × 128 outputs, silu(gate) · up, and the 2F-wide product never leaves LDS
    char* obase = reinterpret_cast<char*>(C) + ((size_t)m0 * ldc + n0 / 2) * 2;
#pragma unroll 4
    for (int it = 0; it < BM * (BN / 2) * 2 / (NT * 16); ++it) {
      const int row = it * 16 + (tid >> 4);
      const int ch = tid & 15;
      const u32x4 g = *reinterpret_cast<const u32x4*>(lds + row * C_STRIDE + ch * 16);
      const u32x4 u = *reinterpret_cast<const u32x4*>(lds + row * C_STRIDE + (ch + 16) * 16);
      if (row >= rows_valid) continue;
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = w4a_pack<H>(w4a_swiglu(w4a_lo<H>(g[e]), w4a_lo<H>(u[e])),
                           w4a_swiglu(w4a_hi<H>(g[e]), w4a_hi<H>(u[e])));
      u32x4* dst = reinterpret_cast<u32x4*>(obase + row * ldc_b + ch * 16);
      if (nt_store) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(dst), "v"(o) : "memory");
      else *dst = o;
    }
    return;
  }
  char* cbase_g = reinterpret_cast<char*>(C) + ((size_t)m0 * ldc + n0) * 2;
  float bv[8];
  if constexpr (EPI != kEpiNone) {   // this thread's 8 columns are the same in every row it stores
    u32x4 braw = {0u, 0u, 0u, 0u};
    if (EPI != kEpiResid || bias) braw = *reinterpret_cast<const u32x4*>(bias + n0 + (tid & 31) * 8);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bv[2 * e] = w4a_lo<H>(braw[e]);
      bv[2 * e + 1] = w4a_hi<H>(braw[e]);
    }
  }
#pragma unroll 4
  for (int it = 0; it < BM * BN * 2 / (NT * 16); ++it) {
    const int row = it * 8 + (tid >> 5);
    const int ch = tid & 31;
    u32x4 v = *reinterpret_cast<const u32x4*>(lds + row * C_STRIDE + ch * 16);
    if (row >= rows_valid) continue;
    if constexpr (EPI == kEpiResid) {
      // 8 fp32 columns of x (and of the row's gate): two 16-B loads each, one read-modify-write
      const int gm = m0 + row, gn = n0 + ch * 8;
      f32x4* xp = reinterpret_cast<f32x4*>(resid.x + (size_t)gm * resid.ldx + gn);
      f32x4 x0 = xp[0], x1 = xp[1];
      f32x4 g0 = {1.f, 1.f, 1.f, 1.f}, g1 = g0;
      if (resid.gate) {
        const f32x4* gp = reinterpret_cast<const f32x4*>(
            resid.gate + (size_t)(gm / resid.rows_per_gate) * resid.gate_stride + gn);
        g0 = gp[0];
        g1 = gp[1];
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        x0[2 * e] += (w4a_lo<H>(v[e]) + bv[2 * e]) * g0[2 * e];
        x0[2 * e + 1] += (w4a_hi<H>(v[e]) + bv[2 * e + 1]) * g0[2 * e + 1];
        x1[2 * e] += (w4a_lo<H>(v[e + 2]) + bv[2 * e + 4]) * g1[2 * e];
        x1[2 * e + 1] += (w4a_hi<H>(v[e + 2]) + bv[2 * e + 5]) * g1[2 * e + 1];
      }
      xp[0] = x0;
      xp[1] = x1;
      continue;
    }
    if constexpr (EPI != kEpiNone) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float lo = w4a_lo<H>(v[e]) + bv[2 * e];
        float hi = w4a_hi<H>(v[e]) + bv[2 * e + 1];
        if constexpr (EPI == kEpiBiasGelu) {
          lo = w4a_gelu_tanh(lo);
          hi = w4a_gelu_tanh(hi);
        }
        v[e] = w4a_pack<H>(lo, hi);
      }
    }
    u32x4* dst = reinterpret_cast<u32x4*>(cbase_g + row * ldc_b + ch * 16);
    if (nt_store)  // C streams out (nt: no L2/MALL retention) — the caches stay with A and B
      asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(dst), "v"(v) : "memory");
    else
      *dst = v;
  }
}

namespace {
int launch_w4a(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
               hipStream_t stream, bool f16) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return (int)hipErrorInvalidValue;
  // each 256-row panel is addressed with 32-bit buffer offsets
  if (256ull * (unsigned long long)(lda > ldb ? lda : ldb) * 2 >= (1ull << 31))
    return (int)hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  // partition-aware tile order (tile_order.h): XCD corners of super-blocks, or GROUP_M order
  const int sb = amdk8s::tile_order_arg(M / BM, N / BN);
  // non-temporal C stores (AMDK8S_GEMM_NT_STORE=0 turns them off for A/B runs)
  const char* ntenv = getenv("AMDK8S_GEMM_NT_STORE");
  const int nt = !(ntenv && ntenv[0] == '0');
  // K-loop schedule: the generator's default, or AMDK8S_W4A_SCHEDULE=<name> for A/B runs (bf16)
  int sched = AMDK8S_W4A_DEFAULT_SCHEDULE;
  if (const char* e = getenv("AMDK8S_W4A_SCHEDULE")) {
    static const char* const names[] = AMDK8S_W4A_SCHEDULE_NAMES;
    for (int i = 0; i < AMDK8S_W4A_NUM_SCHEDULES; ++i)
      if (!strcmp(e, names[i])) sched = i;
  }
  if (f16) sched = kF16;
  const uint16_t* a = (const uint16_t*)A;
  const uint16_t* b = (const uint16_t*)B;
  uint16_t* c = (uint16_t*)C;
  if (sched == kF16)
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4a<kF16>, dim3(nwg), dim3(NT), 0, stream, a, b,
                       c, M, N, K, lda, ldb, ldc, sb, nt, nullptr, W4aResid{}, 1, 0L);
  else if (sched == 1)
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4a<1>, dim3(nwg), dim3(NT), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc, sb, nt, nullptr, W4aResid{}, 1, 0L);
  else if (sched == 2)
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4a<2>, dim3(nwg), dim3(NT), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc, sb, nt, nullptr, W4aResid{}, 1, 0L);
  else
    hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256_w4a<0>, dim3(nwg), dim3(NT), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc, sb, nt, nullptr, W4aResid{}, 1, 0L);
  return (int)hipGetLastError();
}
}  // namespace

// Any M >= 1 (N % 256 == 0, K % 64 == 0); epi 0 = plain, 1 = + bias, 2 = gelu_tanh(+ bias),
// 3 = x[m, n] += gate[m / rows_per_gate, n] · (C + bias) (fp32 x, C not written; bias / gate may
// be null), 4 = SwiGLU of tile-interleaved gate|up rows (C [M, N / 2], bias unused).
// dtype 1 = bf16, 0 = fp16 (operands, bias, C).
extern "C" int amdk8s_gemm_w4a_epi(int epi, int dtype, const void* A, const void* B, void* C,
                                   const void* bias, float* x, const float* gate, int M, int N,
                                   int K, int lda, int ldb, int ldc, int ldx, int rows_per_gate,
                                   int gate_stride, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || N % BN || K % BK) return (int)hipErrorInvalidValue;
  if (epi < kEpiNone || epi > kEpiSwiGLU) return (int)hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || lda < K || ldb < K) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)bias) & 15) return (int)hipErrorInvalidValue;
  if (epi == kEpiResid) {
    if (!x || ldx % 4 || ldx < N || ((uintptr_t)x & 15)) return (int)hipErrorInvalidValue;
    if (gate && (rows_per_gate <= 0 || gate_stride % 4 || ((uintptr_t)gate & 15)))
      return (int)hipErrorInvalidValue;
  } else if (epi == kEpiSwiGLU) {
    if (!C || ldc % 8 || ldc < N / 2 || ((uintptr_t)C & 15)) return (int)hipErrorInvalidValue;
  } else {
    if (!C || ldc % 8 || ldc < N || ((uintptr_t)C & 15)) return (int)hipErrorInvalidValue;
    if (epi != kEpiNone && !bias) return (int)hipErrorInvalidValue;
  }
  if (256ull * (unsigned long long)(lda > ldb ? lda : ldb) * 2 >= (1ull << 31))
    return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = N / BN;
  const int sb = amdk8s::tile_order_arg(tm, tn);
  const uint16_t* a = (const uint16_t*)A;
  const uint16_t* b = (const uint16_t*)B;
  const uint16_t* bs = (const uint16_t*)bias;
  uint16_t* c = (uint16_t*)C;
  const W4aResid r{x, gate, ldx, rows_per_gate > 0 ? rows_per_gate : M, gate_stride};
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(tm * tn), dim3(NT), 0, stream, a, b, c, M, N, K, lda, ldb, ldc,
                       sb, 0, bs, r, 1, 0L);
  };
  constexpr int S = AMDK8S_W4A_DEFAULT_SCHEDULE;
  if (dtype == 0) {
    if (epi == kEpiBias) launch(amdk8s_gemm_bf16_nt_256x256_w4a<kF16, kEpiBias>);
    else if (epi == kEpiBiasGelu) launch(amdk8s_gemm_bf16_nt_256x256_w4a<kF16, kEpiBiasGelu>);
    else if (epi == kEpiResid) launch(amdk8s_gemm_bf16_nt_256x256_w4a<kF16, kEpiResid>);
    else if (epi == kEpiSwiGLU) launch(amdk8s_gemm_bf16_nt_256x256_w4a<kF16, kEpiSwiGLU>);
    else launch(amdk8s_gemm_bf16_nt_256x256_w4a<kF16, kEpiNone>);
  } else {
    if (epi == kEpiBias) launch(amdk8s_gemm_bf16_nt_256x256_w4a<S, kEpiBias>);
    else if (epi == kEpiBiasGelu) launch(amdk8s_gemm_bf16_nt_256x256_w4a<S, kEpiBiasGelu>);
    else if (epi == kEpiResid) launch(amdk8s_gemm_bf16_nt_256x256_w4a<S, kEpiResid>);
    else if (epi == kEpiSwiGLU) launch(amdk8s_gemm_bf16_nt_256x256_w4a<S, kEpiSwiGLU>);
    else launch(amdk8s_gemm_bf16_nt_256x256_w4a<S, kEpiNone>);
  }
  return (int)hipGetLastError();
}

extern "C" int amdk8s_gemm_bf16_nt_w4a(const void* A, const void* B, void* C, int M, int N, int K,
                                       int lda, int ldb, int ldc, hipStream_t stream) {
  return launch_w4a(A, B, C, M, N, K, lda, ldb, ldc, stream, false);
}

// fp16 operands and fp16 output (fp32 accumulation), same shape contract as the bf16 entry.
extern "C" int amdk8s_gemm_f16_nt_w4a(const void* A, const void* B, void* C, int M, int N, int K,
                                      int lda, int ldb, int ldc, hipStream_t stream) {
  return launch_w4a(A, B, C, M, N, K, lda, ldb, ldc, stream, true);
}

// ---------------------------------------------------------------- partial last wave (hybrid)
// A grid of 256×256 tiles that fills the chip 1 < waves < 2 times (the LLM's gate|up prefill
// GEMM at 512 tokens: 2 × 148 = 296 tiles on 256 CUs, one workgroup per CU) runs its second round
// with 40 of 256 CUs busy.  The hybrid runs whole waves of tiles as usual (the first na columns),
// and the remaining columns' tiles split over K across the idle CUs: ksplit workgroups per tile
// write 16-bit partial tiles to a workspace, and a finalize pass sums them in fp32 (+ bias).

template <bool H>
__global__ void __launch_bounds__(256)
w4a_splitk_finalize(const uint16_t* __restrict__ ws, int S, long slice_stride, int M, int Nb,
                    uint16_t* __restrict__ C, int ldc, const uint16_t* __restrict__ bias) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // one 8-column group
  const int groups = Nb >> 3;
  if (i >= (long)M * groups) return;
  const int m = (int)(i / groups), c = (int)(i - (long)m * groups) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(ws + s * slice_stride + (long)m * Nb + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] += w4a_lo<H>(v[e]);
      acc[2 * e + 1] += w4a_hi<H>(v[e]);
    }
  }
  u32x4 o;
  if (bias) {
    const u32x4 b = *reinterpret_cast<const u32x4*>(bias + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] += w4a_lo<H>(b[e]);
      acc[2 * e + 1] += w4a_hi<H>(b[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = w4a_pack<H>(acc[2 * e], acc[2 * e + 1]);
  *reinterpret_cast<u32x4*>(C + (long)m * ldc + c) = o;
}

// The same for SwiGLU (tile-interleaved gate|up, see kEpiSwiGLU): output column group c of the
// rest is gate column (c / 128) · 256 + c % 128 and up column + 128; each sum is rounded to 16 bits
// (what the plain finalize stores) before silu(gate) · up.
template <bool H>
__global__ void __launch_bounds__(256)
w4a_splitk_finalize_swiglu(const uint16_t* __restrict__ ws, int S, long slice_stride, int M,
                           int Nb, uint16_t* __restrict__ C, int ldc) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // one 8-column output group
  const int groups = Nb >> 4;
  if (i >= (long)M * groups) return;
  const int m = (int)(i / groups), oc = (int)(i - (long)m * groups) * 8;
  const int gc = (oc >> 7) * 256 + (oc & 127);
  float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, u[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const u32x4 vg = *reinterpret_cast<const u32x4*>(ws + s * slice_stride + (long)m * Nb + gc);
    const u32x4 vu = *reinterpret_cast<const u32x4*>(ws + s * slice_stride + (long)m * Nb + gc + 128);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      g[2 * e] += w4a_lo<H>(vg[e]);
      g[2 * e + 1] += w4a_hi<H>(vg[e]);
      u[2 * e] += w4a_lo<H>(vu[e]);
      u[2 * e + 1] += w4a_hi<H>(vu[e]);
    }
  }
  u32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t gr = w4a_pack<H>(g[2 * e], g[2 * e + 1]), ur = w4a_pack<H>(u[2 * e], u[2 * e + 1]);
    o[e] = w4a_pack<H>(w4a_swiglu(w4a_lo<H>(gr), w4a_lo<H>(ur)),
                       w4a_swiglu(w4a_hi<H>(gr), w4a_hi<H>(ur)));
  }
  *reinterpret_cast<u32x4*>(C + (long)m * ldc + oc) = o;
}

// Split-K residual finalize: x[m, n] += Σ_s partial_s[m, n] (+ bias), fp32 sums of the 16-bit
// partial tiles in slice order, straight into the fp32 residual stream.
template <bool H>
__global__ void __launch_bounds__(256)
w4a_splitk_finalize_resid(const uint16_t* __restrict__ ws, int S, long slice_stride, int M, int N,
                          float* __restrict__ x, int ldx, const uint16_t* __restrict__ bias) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // one 8-column group
  const int groups = N >> 3;
  if (i >= (long)M * groups) return;
  const int m = (int)(i / groups), c = (int)(i - (long)m * groups) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(ws + s * slice_stride + (long)m * N + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] += w4a_lo<H>(v[e]);
      acc[2 * e + 1] += w4a_hi<H>(v[e]);
    }
  }
  if (bias) {
    const u32x4 b = *reinterpret_cast<const u32x4*>(bias + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] += w4a_lo<H>(b[e]);
      acc[2 * e + 1] += w4a_hi<H>(b[e]);
    }
  }
  f32x4* xp = reinterpret_cast<f32x4*>(x + (long)m * ldx + c);
  f32x4 x0 = xp[0], x1 = xp[1];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    x0[e] += acc[e];
    x1[e] += acc[4 + e];
  }
  xp[0] = x0;
  xp[1] = x1;
}

// The same with the next RMSNorm fused (the LLM prefill: o_proj → ffn_norm, ffn_down → the next
// layer's attn_norm): one workgroup per row (N % 8 == 0, N <= 8192), 8-column chunks tid + 256 u.
// x is updated exactly as w4a_splitk_finalize_resid does, and y = fp16(x · r · w) with the sum of
// squares in rmsnorm_f16's order (llm_prefill.hip), so the bits equal the two-pass path.
template <bool H>
__global__ void __launch_bounds__(256)
w4a_splitk_finalize_resid_norm(const uint16_t* __restrict__ ws, int S, long slice_stride, int N,
                               float* __restrict__ x, int ldx, const uint16_t* __restrict__ bias,
                               const float* __restrict__ nw, float eps, uint16_t* __restrict__ y,
                               int ldy) {
  constexpr int CH = 4;
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x, nch = N >> 3;
  float* xr = x + (long)m * ldx;
  float e[CH][8];
#pragma unroll
  for (int u = 0; u < CH; ++u) {
    const int c = tid + 256 * u;
    if (c >= nch) break;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(ws + s * slice_stride + (long)m * N + c * 8);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += w4a_lo<H>(v[q]);
        acc[2 * q + 1] += w4a_hi<H>(v[q]);
      }
    }
    if (bias) {
      const u32x4 b = *reinterpret_cast<const u32x4*>(bias + c * 8);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += w4a_lo<H>(b[q]);
        acc[2 * q + 1] += w4a_hi<H>(b[q]);
      }
    }
    f32x4* xp = reinterpret_cast<f32x4*>(xr + c * 8);
    f32x4 x0 = xp[0], x1 = xp[1];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      x0[q] += acc[q];
      x1[q] += acc[4 + q];
    }
    xp[0] = x0;
    xp[1] = x1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      e[u][q] = x0[q];
      e[u][4 + q] = x1[q];
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < CH; ++u)
    if (tid + 256 * u < nch) {
#pragma unroll
      for (int i = 0; i < 8; ++i) ss = __fmaf_rn(e[u][i], e[u][i], ss);
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float r = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)N + eps);
  uint16_t* yr = y + (long)m * ldy;
#pragma unroll
  for (int u = 0; u < CH; ++u) {
    const int c = tid + 256 * u;
    if (c >= nch) break;
    const f32x4 wa = *reinterpret_cast<const f32x4*>(nw + c * 8);
    const f32x4 wb = *reinterpret_cast<const f32x4*>(nw + c * 8 + 4);
    const float ww[8] = {wa[0], wa[1], wa[2], wa[3], wb[0], wb[1], wb[2], wb[3]};
    u32x4 pk;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const _Float16 lo = (_Float16)(e[u][2 * i] * r * ww[2 * i]);
      const _Float16 hi = (_Float16)(e[u][2 * i + 1] * r * ww[2 * i + 1]);
      pk[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) |
              ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
    }
    *reinterpret_cast<u32x4*>(yr + c * 8) = pk;
  }
}

// The hybrid's plan: na = columns run as whole waves (a multiple of 256, possibly 0 — then the
// plain kernel is the better choice) and ks = K slices per tile of the rest; ks = 1: no hybrid.
extern "C" void amdk8s_gemm_w4a_hybrid_plan(int M, int N, int K, int cus, int* na, int* ks) {
  const int tm = (M + BM - 1) / BM, tn = N / BN, tiles = tm * tn, T = K / BK;
  *na = N;
  *ks = 1;
  // only a grid of 1 < waves < 2: with more whole waves the partial one is a small share, and the
  // sub-grid's tile order costs more than it saves (M = 3584: 809 vs 759 us, profiles/r05)
  if (N % BN || cus <= 0 || tiles <= cus || tiles >= 2 * cus) return;
  const int full = tiles / cus * cus;             // tiles of the whole waves
  const int tn_a = full / tm;                     // whole columns inside them
  const int rest = (tn - tn_a) * tm;
  if (tn_a <= 0 || rest <= 0 || rest * 2 > cus) return;   // last wave at least half full: plain
  int s = cus / rest;
  s = s < T / 8 ? s : T / 8;                      // >= 8 K-tiles per slice (the ring's depth)
  // each slice's partial tile is rounded to 16 bits before the fp32 sum: at most 8 of them (the
  // caller runs the hybrid for fp16 only — 11 mantissa bits — never bf16)
  s = s < 8 ? s : 8;
  if (s < 2) return;
  *na = tn_a * BN;
  *ks = s;
}

// C[M, N] = A·Bᵀ (+ bias) with the partial last wave split over K (see above); ws: ks × M × (N - na)
// 16-bit elements (dtype as the operands).  epi 0 = plain, 1 = + bias, 4 = SwiGLU (C [M, N / 2]).
extern "C" int amdk8s_gemm_w4a_hybrid(int epi, int dtype, const void* A, const void* B, void* C,
                                      const void* bias, int M, int N, int K, int lda, int ldb,
                                      int ldc, int na, int ks, void* ws, long ws_elems,
                                      hipStream_t stream) {
  if (epi != kEpiNone && epi != kEpiBias && epi != kEpiSwiGLU) return (int)hipErrorInvalidValue;
  if (M <= 0 || N % BN || K % BK || na % BN || na <= 0 || na >= N || ks < 2) return (int)hipErrorInvalidValue;
  const int nb = N - na;
  if ((long)ks * M * nb > ws_elems || !ws || ((uintptr_t)ws & 15)) return (int)hipErrorInvalidValue;
  if (K / BK < ks) return (int)hipErrorInvalidValue;
  int rc = amdk8s_gemm_w4a_epi(epi, dtype, A, B, C, bias, nullptr, nullptr, M, na, K, lda, ldb, ldc,
                               0, 0, 0, stream);
  if (rc) return rc;
  if (lda % 8 || ldb % 8 || ldc % 8 || ((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15)
    return (int)hipErrorInvalidValue;
  const int tm = (M + BM - 1) / BM, tn = nb / BN;
  const int sb = amdk8s::tile_order_arg(tm, tn);
  const uint16_t* a = (const uint16_t*)A;
  const uint16_t* b = (const uint16_t*)B + (size_t)na * ldb;
  uint16_t* w = (uint16_t*)ws;
  const long stride = (long)M * nb;
  constexpr int S = AMDK8S_W4A_DEFAULT_SCHEDULE;
  if (dtype == 0)
    hipLaunchKernelGGL((amdk8s_gemm_bf16_nt_256x256_w4a<kF16, kEpiNone>), dim3(tm * tn * ks), dim3(NT),
                       0, stream, a, b, w, M, nb, K, lda, ldb, nb, sb, 0, nullptr, W4aResid{}, ks,
                       stride);
  else
    hipLaunchKernelGGL((amdk8s_gemm_bf16_nt_256x256_w4a<S, kEpiNone>), dim3(tm * tn * ks), dim3(NT),
                       0, stream, a, b, w, M, nb, K, lda, ldb, nb, sb, 0, nullptr, W4aResid{}, ks,
                       stride);
  rc = (int)hipGetLastError();
  if (rc) return rc;
  if (epi == kEpiSwiGLU) {
    const long og = (long)M * (nb / 16);
    uint16_t* c = (uint16_t*)C + na / 2;
    if (dtype == 0)
      hipLaunchKernelGGL(w4a_splitk_finalize_swiglu<true>, dim3((unsigned)((og + 255) / 256)),
                         dim3(256), 0, stream, w, ks, stride, M, nb, c, ldc);
    else
      hipLaunchKernelGGL(w4a_splitk_finalize_swiglu<false>, dim3((unsigned)((og + 255) / 256)),
                         dim3(256), 0, stream, w, ks, stride, M, nb, c, ldc);
    return (int)hipGetLastError();
  }
  const long groups = (long)M * (nb / 8);
  const uint16_t* bs = epi == kEpiBias ? (const uint16_t*)bias + na : nullptr;
  uint16_t* c = (uint16_t*)C + na;
  if (dtype == 0)
    hipLaunchKernelGGL(w4a_splitk_finalize<true>, dim3((unsigned)((groups + 255) / 256)), dim3(256),
                       0, stream, w, ks, stride, M, nb, c, ldc, bs);
  else
    hipLaunchKernelGGL(w4a_splitk_finalize<false>, dim3((unsigned)((groups + 255) / 256)), dim3(256),
                       0, stream, w, ks, stride, M, nb, c, ldc, bs);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- split-K over every tile
// A 256×256 grid far below the chip (the LLM prefill's q|k|v, o_proj and ffn_down at 512 tokens:
// 36 / 28 / 28 tiles on 256 CUs) otherwise runs on the smaller wave-grid tiles at a fraction of
// this kernel's rate.  Here every tile splits over K: ks workgroups per tile each run a contiguous
// range of its K-tiles into a 16-bit partial tile (fp16 only, like the hybrid: at most 8 roundings
// at 11 mantissa bits), and a finalize pass sums the slices in fp32 in slice order and applies the
// epilogue (store / + bias / += into the fp32 residual stream / SwiGLU).
// A/B sweeps: amdk8s_gemm_w4a_splitk_set_ks(k) pins the slice count of every shape the planner
// takes (k >= 2, capped at the K-tile count), 0 = the planner's.
static int g_splitk_pin = 0;
extern "C" void amdk8s_gemm_w4a_splitk_set_ks(int k) { g_splitk_pin = k > 0 ? k : 0; }

extern "C" void amdk8s_gemm_w4a_splitk_plan(int M, int N, int K, int cus, int* ks) {
  *ks = 1;
  if (M < 256 || N % BN || K % BK || cus <= 0) return;
  if (g_splitk_pin >= 2) {
    const int tiles = ((M + BM - 1) / BM) * (N / BN);
    if (tiles * 4 < cus * 3) *ks = g_splitk_pin < K / BK ? g_splitk_pin : K / BK;
    return;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN), T = K / BK;
  if (tiles * 4 >= cus * 3) return;               // the plain grid fills >= 3/4 of the chip
  int s = cus / tiles;
  s = s < T / 6 ? s : T / 6;                      // >= 6 K-tiles per slice (ring fill + drain)
  s = s < 8 ? s : 8;
  // and only when the split grid fills >= 3/4 of the chip: at 256 tokens o_proj / ffn_down (14
  // tiles x 8 = 112 workgroups) lost to the wave-grid family, 24.6 / 60.4 vs 22.5 / 54.6 us
  // (profiles/r06/prefill_gemm_256_splitk_sweep.log)
  if (s >= 2 && tiles * s * 4 >= cus * 3) *ks = s;
}

// norm_w (epi 3 only, may be null): also y[m] = fp16(rmsnorm(x[m]) · norm_w) of the updated rows
// (y [M][ldy], N <= 8192), the prefill's next RMSNorm in the same pass.
extern "C" int amdk8s_gemm_w4a_splitk(int epi, int dtype, const void* A, const void* B, void* C,
                                      const void* bias, float* x, int M, int N, int K, int lda,
                                      int ldb, int ldc, int ldx, int ks, void* ws, long ws_elems,
                                      const float* norm_w, float eps, void* y, int ldy,
                                      hipStream_t stream) {
  if (epi != kEpiNone && epi != kEpiBias && epi != kEpiResid && epi != kEpiSwiGLU)
    return (int)hipErrorInvalidValue;
  if (M <= 0 || N <= 0 || N % BN || K % BK || ks < 2 || K / BK < ks) return (int)hipErrorInvalidValue;
  if ((long)ks * M * N > ws_elems || !ws || ((uintptr_t)ws & 15)) return (int)hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || lda < K || ldb < K) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)bias) & 15) return (int)hipErrorInvalidValue;
  if (256ull * (unsigned long long)(lda > ldb ? lda : ldb) * 2 >= (1ull << 31))
    return (int)hipErrorInvalidValue;
  if (epi == kEpiResid) {
    if (!x || ldx % 4 || ldx < N || ((uintptr_t)x & 15)) return (int)hipErrorInvalidValue;
    if (norm_w && (dtype != 0 || N > 8192 || !y || ldy % 8 || ldy < N ||
                   (((uintptr_t)y | (uintptr_t)norm_w) & 15)))
      return (int)hipErrorInvalidValue;
  } else {
    if (norm_w) return (int)hipErrorInvalidValue;
    const int w = epi == kEpiSwiGLU ? N / 2 : N;
    if (!C || ldc % 8 || ldc < w || ((uintptr_t)C & 15)) return (int)hipErrorInvalidValue;
    if (epi == kEpiBias && !bias) return (int)hipErrorInvalidValue;
  }
  const int tm = (M + BM - 1) / BM, tn = N / BN;
  const int sb = amdk8s::tile_order_arg(tm, tn);
  const uint16_t* a = (const uint16_t*)A;
  const uint16_t* b = (const uint16_t*)B;
  uint16_t* w = (uint16_t*)ws;
  const long stride = (long)M * N;
  constexpr int S = AMDK8S_W4A_DEFAULT_SCHEDULE;
  if (dtype == 0)
    hipLaunchKernelGGL((amdk8s_gemm_bf16_nt_256x256_w4a<kF16, kEpiNone>), dim3(tm * tn * ks), dim3(NT),
                       0, stream, a, b, w, M, N, K, lda, ldb, N, sb, 0, nullptr, W4aResid{}, ks, stride);
  else
    hipLaunchKernelGGL((amdk8s_gemm_bf16_nt_256x256_w4a<S, kEpiNone>), dim3(tm * tn * ks), dim3(NT),
                       0, stream, a, b, w, M, N, K, lda, ldb, N, sb, 0, nullptr, W4aResid{}, ks, stride);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  const uint16_t* bs = epi == kEpiBias || epi == kEpiResid ? (const uint16_t*)bias : nullptr;
  uint16_t* c = (uint16_t*)C;
  const unsigned g8 = (unsigned)(((long)M * (N / 8) + 255) / 256);
  const unsigned g16 = (unsigned)(((long)M * (N / 16) + 255) / 256);
  if (epi == kEpiResid && norm_w) {
    hipLaunchKernelGGL(w4a_splitk_finalize_resid_norm<true>, dim3(M), dim3(256), 0, stream, w, ks,
                       stride, N, x, ldx, bs, norm_w, eps, (uint16_t*)y, ldy);
  } else if (epi == kEpiResid) {
    if (dtype == 0)
      hipLaunchKernelGGL(w4a_splitk_finalize_resid<true>, dim3(g8), dim3(256), 0, stream, w, ks,
                         stride, M, N, x, ldx, bs);
    else
      hipLaunchKernelGGL(w4a_splitk_finalize_resid<false>, dim3(g8), dim3(256), 0, stream, w, ks,
                         stride, M, N, x, ldx, bs);
  } else if (epi == kEpiSwiGLU) {
    if (dtype == 0)
      hipLaunchKernelGGL(w4a_splitk_finalize_swiglu<true>, dim3(g16), dim3(256), 0, stream, w, ks,
                         stride, M, N, c, ldc);
    else
      hipLaunchKernelGGL(w4a_splitk_finalize_swiglu<false>, dim3(g16), dim3(256), 0, stream, w, ks,
                         stride, M, N, c, ldc);
  } else {
    if (dtype == 0)
      hipLaunchKernelGGL(w4a_splitk_finalize<true>, dim3(g8), dim3(256), 0, stream, w, ks, stride, M,
                         N, c, ldc, bs);
    else
      hipLaunchKernelGGL(w4a_splitk_finalize<false>, dim3(g8), dim3(256), 0, stream, w, ks, stride, M,
                         N, c, ldc, bs);
  }
  return (int)hipGetLastError();
}
