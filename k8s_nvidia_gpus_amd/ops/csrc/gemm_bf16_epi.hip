// bf16 / fp16 MFMA GEMM + implicit-GEMM 3×3 convolution with fused epilogues, for the diffusion
// transformer / UNet projections and the UNet / VAE convolutions (gfx950).
//
//   Y = A · Bᵀ (+ bias)            A [M, K] activations (row-major, lda) — or, for a convolution,
//                                  the NHWC input gathered per 3×3 tap (zero rows for padding,
//                                  stride 2, or a nearest-2× upsample folded into the addressing)
//                                  B [N, K] nn.Linear weight / [Cout, 3·3·Cin] packed conv weight
//   epilogue (fp32 accumulators, one pass, no extra kernel):
//     EPI_STORE   out[m, n] = 16bit(Y)
//     EPI_GELU    out[m, n] = 16bit(gelu_tanh(Y))                     (DiT / text-embedding FFN-in)
//     EPI_RESID   x[m, n]  += Y · gate[m / rows_per_gate, n]          (fp32 residual stream, in place;
//                                                                      gate = AdaLN gate or none)
//     EPI_ADD     out[m, n] = 16bit(Y) + r[m, n]                      (UNet conv2 + shortcut)
//   split-K (grids that cannot fill the chip): each split writes its fp32 partial tile to its own
//   workspace slice; splitk_finalize sums the slices in a fixed order and applies the epilogue.
//
// The validator GEMMs (gemm_bf16_gfx950*.hip) use 256×256 tiles; the Wan2.1 DiT at the reference
// defaults (512×320×16 frames → 2×2560 token rows with CFG, generate_wan_t2v.py:305-312) has
// N = 1536 for four of its six projections, where 256×256 tiles make only 120 workgroups for 256
// CUs.  This kernel's block tile is a WM × WN grid of waves, each wave a 64×64 output block, so the
// tile is (64·WM) × (64·WN): 256×128 (8 waves) for the DiT (240 workgroups there, 1400 for the
// 8960-wide FFN), and 128×128 / 128×64 / 64×64 for the SD1.5 UNet's narrow (N = 320) and short
// (M = 2·16², 2·8² token rows at the deep levels) projections, where a 256×128 grid would leave
// most of the 256 CUs idle.  The host picks the largest tile whose grid still covers the CUs.
//
//   * each wave: 4×4 tiles of v_mfma_f32_16x16x32_bf16 (weight fragment as the A operand, so a
//     lane's 4 accumulators are 4 consecutive output columns of one row);
//   * A and B K-tiles (BK = 64) staged HBM→LDS by LDS-DMA (global_load_lds_dwordx4; 6 per thread
//     per K-tile at 256×128) into a 3-deep ring: one barrier per K-tile, the DMA of K-tile t+2
//     issued right after it and retired by a counted `s_waitcnt vmcnt` two iterations later —
//     the loop never drains the DMA queue;
//   * XOR-swizzled 128-B LDS rows (16-B chunk c of row r at c ^ ((r >> 1) & 7)), applied to the DMA
//     SOURCE address (LDS-DMA writes lane-linearly), so every ds_read_b128 fragment read is
//     conflict-free;
//   * M / N tails: rows ≥ M (columns ≥ N) are loaded as clamped copies of row M−1 (weight row N−1)
//     and never stored, so any token count and any N % 8 == 0 runs unpadded (K % 64 == 0);
//   * bf16 (Wan DiT) or fp16 (the SD1.5 service) operands and output, fp32 accumulation;
//   * epilogue through the idle LDS ring: fp32 (residual) or bf16 rows staged, then 16-B coalesced
//     loads/stores of whole rows; bias and tanh-GELU in fp32 registers before the conversion;
//   * XCD-aware bijective block remap + GROUP_M tile order (neighbouring tiles share A / B panels in
//     one XCD's L2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BK = 64;
constexpr int NSTAGE = 3;
constexpr int GROUP_M = 8;

// Tile geometry of a WM × WN wave grid, each wave a (64·TM) × (64·TN) block.
template <int WM, int WN, int TM = 1, int TN = 1>
struct Geo {
  static constexpr int BM = 64 * WM * TM, BN = 64 * WN * TN, NW = WM * WN, NT = 64 * NW;
  static constexpr int A_STAGE = BM * BK * 2, B_STAGE = BN * BK * 2;
  static constexpr int STAGE = A_STAGE + B_STAGE;
  static constexpr int RING = NSTAGE * STAGE;
  static constexpr int LA = BM / 8 / NW, LB = BN / 8 / NW;   // DMA wave-instructions per operand
  static constexpr int CF_STRIDE = BN * 4 + 16;              // fp32 epilogue row
  static constexpr int CB_STRIDE = BN * 2 + 16;              // bf16 / fp16 epilogue row
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "DMA rows must split evenly");
  static_assert(BM * CF_STRIDE <= RING, "fp32 epilogue image must fit the ring");
};

enum Epi { EPI_STORE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_ADD = 3,
           EPI_PARTIAL = 4 };   // split-K: this split's fp32 partial tile into its workspace slice

// Implicit-GEMM 3×3 convolution (pad 1) over NHWC activations: the A "row" of output pixel m at
// K-tile t is the 64-channel slice t % (Cin/64) of input pixel (tap t / (Cin/64)) — a 128-B run
// of the NHWC tensor, or a zero row where the tap falls in the padding.
enum ConvMode { CONV_NONE = 0, CONV_S1 = 1, CONV_S2 = 2, CONV_UP2 = 3 };

struct Args {
  const uint16_t* A;
  const uint16_t* B;
  const uint16_t* bias;   // [N] bf16 / fp16 (operand dtype) or null
  uint16_t* out;          // bf16 / fp16 output (STORE / GELU / ADD)
  float* x;               // fp32 residual stream (RESID)
  const float* gate;      // [M / rows_per_gate][gate_stride] fp32 or null (RESID)
  const uint16_t* r;      // [M][ldr] 16-bit addend (ADD: out = Y + bias + r; may alias out)
  int M, N, K, lda, ldb, ldo, ldx, rows_per_gate, gate_stride, ldr;
  int splits;             // K split across `splits` workgroups per tile (EPI_PARTIAL), else 1
  float* ws;              // [splits][M][N] fp32 split-K workspace (EPI_PARTIAL)
  // convolution geometry (CONV != CONV_NONE): input [batch][Hin][Win][Cin], output Hout × Wout
  int Hin, Win, Hout, Wout, Cin;
};

// 128 B of zeros: the LDS-DMA source of padding rows.
__device__ __attribute__((aligned(16))) uint4 g_zero_row[8];

__device__ __forceinline__ void barrier_raw() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ bf16x8 lds_read16(const char* p) {
  return *reinterpret_cast<const bf16x8*>(__builtin_assume_aligned(p, 16));
}

template <bool F16>
__device__ __forceinline__ f32x4 mfma16(const bf16x8 a, const bf16x8 b, const f32x4 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <bool F16>
__device__ __forceinline__ float h2f(uint16_t v) {
  if constexpr (F16) return (float)__builtin_bit_cast(_Float16, v);
  else return __uint_as_float((uint32_t)v << 16);
}

template <bool F16>
__device__ __forceinline__ uint2 pack4(f32x4 v) {
  if constexpr (F16) return __builtin_bit_cast(uint2, __builtin_convertvector(v, f16x4));
  else return __builtin_bit_cast(uint2, __builtin_convertvector(v, bf16x4));
}

__device__ __forceinline__ float gelu_tanh(float v) {
  // 0.5 v (1 + tanh(√(2/π)(v + 0.044715 v³))) = v · sigmoid(2u) = v / (1 + 2^t), t = −2u·log2 e:
  // one v_exp_f32 and one v_rcp_f32 (no IEEE division sequence — the epilogue is VALU-bound)
  const float t = v * fmaf(-0.10294324f, v * v, -2.3022082f);
  return v * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(t));
}

template <int EPI, bool F16, int WM, int WN, int CONV = CONV_NONE, int TM = 1, int TN = 1>
__global__ void __launch_bounds__(64 * WM * WN) gemm_epi_kernel(const Args a) {
  using G = Geo<WM, WN, TM, TN>;
  constexpr int MI = 4 * TM, NJ = 4 * TN;       // 16×16 accumulator blocks per wave
  constexpr int BM = G::BM, BN = G::BN, NW = G::NW, NT = G::NT, LA = G::LA, LB = G::LB;
  constexpr int A_STAGE = G::A_STAGE, STAGE = G::STAGE;
  constexpr int CF_STRIDE = G::CF_STRIDE, CB_STRIDE = G::CB_STRIDE;
  __shared__ __attribute__((aligned(16))) char lds[G::RING];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN;  // (64·TM)-row block
  const int wn = wave % WN;  // (64·TN)-column block

  // ---- block → tile: bijective XCD remap, then GROUP_M order ----
  const int tiles_m = (a.M + BM - 1) / BM;
  const int tiles_n = (a.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int wgid, split = 0;
  {
    const int tot = nwg * a.splits;
    const int bid = blockIdx.x, xcd = bid & 7, q = tot >> 3, r = tot & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    if (EPI == EPI_PARTIAL) {
      split = wgid / nwg;
      wgid -= split * nwg;
    }
  }
  const int group = wgid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * GROUP_M * tiles_n;
  const int m0 = (first_m + in_group % gsz) * BM;
  const int n0 = (in_group / gsz) * BN;

  // ---- LDS-DMA sources: wave-instruction q covers 8 rows; lane → row q*8 + lane/8, physical chunk
  //      lane%8 holds logical chunk (lane%8) ^ ((row >> 1) & 7) ----
  const size_t lda_b = (size_t)a.lda * 2, ldb_b = (size_t)a.ldb * 2;
  const char* a_src[LA];
  const char* b_src[LB];
  // convolution: per A row, the output pixel's coordinates and (stride 1 / 2) the taps that land
  // inside the input; a_src = input pixel (y·s, x·s) (or the image base for UP2) + this lane's chunk
  int cv_yx[CONV ? LA : 1], cv_mask[CONV ? LA : 1];
  const char* zsrc = reinterpret_cast<const char*>(g_zero_row) + (lane & 7) * 16;
  const size_t cin_b = (size_t)a.Cin * 2;
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    const int q = j * NW + wave, row = q * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int grow = min(m0 + row, a.M - 1);     // M tail: clamped rows, never stored
    if constexpr (CONV == CONV_NONE) {
      a_src[j] = reinterpret_cast<const char*>(a.A) + (size_t)grow * lda_b + c * 16;
    } else {
      const int hw = a.Hout * a.Wout;
      const int img = grow / hw, rem = grow - img * hw;
      const int y = rem / a.Wout, x = rem - y * a.Wout;
      cv_yx[j] = (y << 16) | x;
      if constexpr (CONV == CONV_UP2) {
        a_src[j] = reinterpret_cast<const char*>(a.A) + (size_t)img * a.Hin * a.Win * cin_b + c * 16;
        cv_mask[j] = 0;
      } else {
        constexpr int S = CONV == CONV_S2 ? 2 : 1;
        int mask = 0;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int iy = y * S + tap / 3 - 1, ix = x * S + tap % 3 - 1;
          if ((unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win) mask |= 1 << tap;
        }
        cv_mask[j] = mask;
        a_src[j] = reinterpret_cast<const char*>(a.A) +
                   ((size_t)(img * a.Hin + y * S) * a.Win + x * S) * cin_b + c * 16;
      }
    }
  }
  const int cpt = a.Cin >> 6;                    // K-tiles per tap
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int q = j * NW + wave, row = q * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int gn = min(n0 + row, a.N - 1);       // N tail: clamped weight rows, never stored
    b_src[j] = reinterpret_cast<const char*>(a.B) + (size_t)gn * ldb_b + c * 16;
  }
  // K-tiles [t0, t0 + T) of this workgroup (all of K unless split)
  const int Ttot = a.K / BK;
  const int t0 = (int)((long)Ttot * split / a.splits);
  const int T = (int)((long)Ttot * (split + 1) / a.splits) - t0;
  auto stage = [&](int i) {                      // ring slot i % NSTAGE ← absolute K-tile t0 + i
    const int t = t0 + i;
    char* sa = lds + (i % NSTAGE) * STAGE;
    char* sb = sa + A_STAGE;
    const size_t kb = (size_t)t * BK * 2;
    if constexpr (CONV == CONV_NONE) {
#pragma unroll
      for (int j = 0; j < LA; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + kb),
                                         (lds_void*)(sa + (j * NW + wave) * 1024), 16, 0, 0);
    } else {
      const int tap = t / cpt, cc = t - tap * cpt;  // uniform
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const long toff = (long)(dy * a.Win + dx) * (long)cin_b + cc * 128;
#pragma unroll
      for (int j = 0; j < LA; ++j) {
        const char* src;
        if constexpr (CONV == CONV_UP2) {       // nearest 2× upsample folded into the addressing
          const int iy = (cv_yx[j] >> 16) + dy, ix = (cv_yx[j] & 0xffff) + dx;
          const bool ok = (unsigned)iy < (unsigned)a.Hout && (unsigned)ix < (unsigned)a.Wout;
          src = ok ? a_src[j] + ((long)(iy >> 1) * a.Win + (ix >> 1)) * (long)cin_b + cc * 128 : zsrc;
        } else {
          src = ((cv_mask[j] >> tap) & 1) ? a_src[j] + toff : zsrc;
        }
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (lds_void*)(sa + (j * NW + wave) * 1024), 16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < LB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(b_src[j] + kb),
                                       (lds_void*)(sb + (j * NW + wave) * 1024), 16, 0, 0);
  };

  // ---- fragment read offsets: row (lane & 15) of a 16-row block, logical chunk 4·kk + lane/16 ----
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = fr >> 1;
  const int foff0 = fr * 128 + (((0 + fq) ^ sw) << 4);
  const int foff1 = fr * 128 + (((4 + fq) ^ sw) << 4);
  const int a_wave = wm * 64 * TM * 128;
  const int b_wave = wn * 64 * TN * 128;

  f32x4 acc[MI][NJ];   // [m 16-block][n 16-block]
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0);
  if (T > 1) stage(1);
  for (int t = 0; t < T; ++t) {
    if (t + 1 < T) wait_vmcnt<LA + LB>(); else wait_vmcnt<0>();
    barrier_raw();                       // K-tile t landed for every wave; t−1's reads are done
    if (t + 2 < T) stage(t + 2);         // into the buffer K-tile t−1 used
    const char* sa = lds + (t % NSTAGE) * STAGE + a_wave;
    const char* sb = lds + (t % NSTAGE) * STAGE + A_STAGE + b_wave;
    // the first half's 8 fragment reads, then the second half's 8 issued between the first half's
    // MFMAs (explicit order, pinned by sched_barrier: the reads' latency hides under MFMAs)
    bf16x8 af[2][MI], bw[2][NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bw[0][j] = lds_read16(sb + j * 2048 + foff0);
#pragma unroll
    for (int i = 0; i < MI; ++i) af[0][i] = lds_read16(sa + i * 2048 + foff0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[0][j] = mfma16<F16>(bw[0][j], af[0][0], acc[0][j]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NJ; ++j) bw[1][j] = lds_read16(sb + j * 2048 + foff1);
#pragma unroll
    for (int i = 0; i < MI; ++i) af[1][i] = lds_read16(sa + i * 2048 + foff1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 1; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16<F16>(bw[0][j], af[0][i], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16<F16>(bw[1][j], af[1][i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (EPI == EPI_PARTIAL) {     // split-K: plain 16-B stores of the fp32 partial tile
    float* slice = a.ws + (size_t)split * a.M * a.N;   // (no atomics, no zeroing: deterministic)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int m = m0 + wm * 64 * TM + 16 * i + fr, n = n0 + wn * 64 * TN + 16 * j + 4 * fq;
        if (m < a.M && n < a.N)                 // N % 8 == 0: a lane's 4 columns all in or out
          *reinterpret_cast<f32x4*>(slice + (size_t)m * a.N + n) = acc[i][j];
      }
    return;
  }
  barrier_raw();                         // every wave is done with the ring: reuse it for C

  // ---- epilogue: lane holds C[m0 + wm·64TM + 16i + fr][n0 + wn·64TN + 16j + 4fq + 0..3] ----
  float bias[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[j][e] = 0.f;
  if (a.bias) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * 64 * TN + 16 * j + 4 * fq;
      if (n < a.N) {                    // N % 4 == 0: a lane's 4 columns are all in or all out
        const uint2 bv = *reinterpret_cast<const uint2*>(a.bias + n);
        bias[j][0] = h2f<F16>((uint16_t)(bv.x & 0xffffu));
        bias[j][1] = h2f<F16>((uint16_t)(bv.x >> 16));
        bias[j][2] = h2f<F16>((uint16_t)(bv.y & 0xffffu));
        bias[j][3] = h2f<F16>((uint16_t)(bv.y >> 16));
      }
    }
  }
  if constexpr (EPI == EPI_RESID) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int m = wm * 64 * TM + 16 * i + fr, n = wn * 64 * TN + 16 * j + 4 * fq;
        f32x4 v = acc[i][j];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bias[j][e];
        *reinterpret_cast<f32x4*>(lds + m * CF_STRIDE + n * 4) = v;
      }
    __syncthreads();
    // BM rows × BN fp32: BN/4 threads per row (16 B each)
    constexpr int TPR = BN / 4, RPP = NT / TPR;
#pragma unroll 4
    for (int it = 0; it < BM / RPP; ++it) {
      const int row = it * RPP + tid / TPR, col = (tid % TPR) * 4;
      const int gm = m0 + row;
      if (gm < a.M && n0 + col < a.N) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(lds + row * CF_STRIDE + col * 4);
        f32x4* xp = reinterpret_cast<f32x4*>(a.x + (size_t)gm * a.ldx + n0 + col);
        f32x4 xv = *xp;
        if (a.gate) {
          const f32x4 g = *reinterpret_cast<const f32x4*>(
              a.gate + (size_t)(gm / a.rows_per_gate) * a.gate_stride + n0 + col);
          xv += v * g;
        } else {
          xv += v;
        }
        *xp = xv;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int m = wm * 64 * TM + 16 * i + fr, n = wn * 64 * TN + 16 * j + 4 * fq;
        f32x4 v = acc[i][j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] += bias[j][e];
          if constexpr (EPI == EPI_GELU) v[e] = gelu_tanh(v[e]);
        }
        *reinterpret_cast<uint2*>(lds + m * CB_STRIDE + n * 2) = pack4<F16>(v);
      }
    __syncthreads();
    // BM rows × BN·2 B: BN/8 threads per row (16 B each)
    constexpr int TPR = BN / 8, RPP = NT / TPR;
    char* obase = reinterpret_cast<char*>(a.out) + ((size_t)m0 * a.ldo + n0) * 2;
    const size_t ldo_b = (size_t)a.ldo * 2;
#pragma unroll 4
    for (int it = 0; it < BM / RPP; ++it) {
      const int row = it * RPP + tid / TPR, ch = tid % TPR;
      if (m0 + row < a.M && n0 + ch * 8 < a.N) {
        uint4 v = *reinterpret_cast<const uint4*>(lds + row * CB_STRIDE + ch * 16);
        if constexpr (EPI == EPI_ADD) {         // + the 16-bit addend (residual / shortcut)
          const uint4 rv = *reinterpret_cast<const uint4*>(
              a.r + (size_t)(m0 + row) * a.ldr + n0 + ch * 8);
          const uint32_t* pv = reinterpret_cast<const uint32_t*>(&v);
          const uint32_t* pr = reinterpret_cast<const uint32_t*>(&rv);
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x4 s4 = {h2f<F16>((uint16_t)(pv[e] & 0xffffu)) + h2f<F16>((uint16_t)(pr[e] & 0xffffu)),
                              h2f<F16>((uint16_t)(pv[e] >> 16)) + h2f<F16>((uint16_t)(pr[e] >> 16)),
                              0.f, 0.f};
            o[e] = pack4<F16>(s4).x;
          }
          v = make_uint4(o[0], o[1], o[2], o[3]);
        }
        *reinterpret_cast<uint4*>(obase + row * ldo_b + ch * 16) = v;
      }
    }
  }
}

// Split-K finalize: out = epi(ws + bias) (+ r), 8 columns per thread (N % 8 == 0).
template <int EPI, bool F16>
__global__ void __launch_bounds__(256) splitk_finalize(const Args a) {
  const long i8 = (long)blockIdx.x * 256 + threadIdx.x;   // 8-column group index
  const int groups = a.N >> 3;
  if (i8 >= (long)a.M * groups) return;
  const int m = (int)(i8 / groups), n = (int)(i8 - (long)m * groups) * 8;
  const f32x4* w = reinterpret_cast<const f32x4*>(a.ws + (size_t)m * a.N + n);
  f32x4 v0 = w[0], v1 = w[1];
  const size_t slice = (size_t)a.M * a.N / 4;      // in f32x4
  for (int sp = 1; sp < a.splits; ++sp) {          // fixed order: bitwise reproducible
    v0 += w[sp * slice];
    v1 += w[sp * slice + 1];
  }
  if (a.bias) {
    const uint4 bv = *reinterpret_cast<const uint4*>(a.bias + n);
    const uint32_t b32[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      v0[2 * e] += h2f<F16>((uint16_t)(b32[e] & 0xffffu));
      v0[2 * e + 1] += h2f<F16>((uint16_t)(b32[e] >> 16));
      v1[2 * e] += h2f<F16>((uint16_t)(b32[e + 2] & 0xffffu));
      v1[2 * e + 1] += h2f<F16>((uint16_t)(b32[e + 2] >> 16));
    }
  }
  if constexpr (EPI == EPI_RESID) {     // x += gate · (Y + bias), fp32 in place
    f32x4* xp = reinterpret_cast<f32x4*>(a.x + (size_t)m * a.ldx + n);
    f32x4 x0 = xp[0], x1 = xp[1];
    if (a.gate) {
      const f32x4* g = reinterpret_cast<const f32x4*>(
          a.gate + (size_t)(m / a.rows_per_gate) * a.gate_stride + n);
      x0 += v0 * g[0];
      x1 += v1 * g[1];
    } else {
      x0 += v0;
      x1 += v1;
    }
    xp[0] = x0;
    xp[1] = x1;
    return;
  }
  if constexpr (EPI == EPI_GELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] = gelu_tanh(v0[e]);
      v1[e] = gelu_tanh(v1[e]);
    }
  }
  uint2 p0 = pack4<F16>(v0), p1 = pack4<F16>(v1);
  if constexpr (EPI == EPI_ADD) {      // round like the fused path: Y to 16 bit, then + r
    const uint4 rv = *reinterpret_cast<const uint4*>(a.r + (size_t)m * a.ldr + n);
    const uint32_t pv[4] = {p0.x, p0.y, p1.x, p1.y}, pr[4] = {rv.x, rv.y, rv.z, rv.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f32x4 s4 = {h2f<F16>((uint16_t)(pv[e] & 0xffffu)) + h2f<F16>((uint16_t)(pr[e] & 0xffffu)),
                        h2f<F16>((uint16_t)(pv[e] >> 16)) + h2f<F16>((uint16_t)(pr[e] >> 16)), 0.f, 0.f};
      o[e] = pack4<F16>(s4).x;
    }
    p0 = make_uint2(o[0], o[1]);
    p1 = make_uint2(o[2], o[3]);
  }
  *reinterpret_cast<uint4*>(a.out + (size_t)m * a.ldo + n) = make_uint4(p0.x, p0.y, p1.x, p1.y);
}

}  // namespace

extern "C" {

// Shape contract: N % 8 == 0, K % 64 == 0, lda/ldb/ldo % 8 == 0, ldx % 4 == 0, 16-B aligned
// operand bases (bias 8-B aligned), gate_stride % 4 == 0; any M ≥ 1.  dtype 1 = bf16, 0 = fp16.
int amdk8s_gemm_epi_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && N % 8 == 0 && K % BK == 0;
}

// Launch plan of an M × N × K problem: block tile (index into kTiles: 256×128, 128×128, 128×64,
// 64×64) and split-K factor.  A 256×128 / 128×128 grid of >= 160 workgroups runs unsplit (the Wan
// o / ffn2 projections at 2 × 2560 rows run 240 256×128 tiles 20-30 % faster than 480 128×128
// ones — profiles/r03/e); otherwise the largest tile that reaches 192 workgroups with K split
// into parts of >= 8 K-tiles (the ring's pipeline depth), else 64×64 with as many such splits as
// K allows (at most 16).  Overrides for A/B sweeps:
// amdk8s_gemm_epi_set_tile(0..3) / AMDK8S_GEMM_EPI_TILE pin the tile, AMDK8S_GEMM_SPLITK=<n> pins
// the split factor (1 = never split); -1 / unset = the plan above.
// (Measured and dropped: 256×128 on 4 waves of 128×64 — a quarter less LDS traffic per MFMA but
// half the waves to hide latency: 20-25 % slower than tile 0 on the Wan shapes, profiles/r03/o.
// The kernel template keeps the (TM, TN) wave-tile parameters.)
static const int kTiles[4][2] = {{256, 128}, {128, 128}, {128, 64}, {64, 64}};
static int g_tile = -2;     // -2: not initialised from the environment yet
static int g_splits = -2;

void amdk8s_gemm_epi_set_tile(int tile) { g_tile = (tile >= 0 && tile <= 3) ? tile : -1; }
void amdk8s_gemm_epi_set_splits(int s) { g_splits = (s >= 1 && s <= 64) ? s : -1; }

static long tile_grid(int tile, int M, int N) {
  return (long)((M + kTiles[tile][0] - 1) / kTiles[tile][0]) * ((N + kTiles[tile][1] - 1) / kTiles[tile][1]);
}

void amdk8s_gemm_epi_plan(int M, int N, int K, int* tile_out, int* splits_out) {
  if (g_tile == -2) {
    const char* e = getenv("AMDK8S_GEMM_EPI_TILE");
    g_tile = (e && e[0] >= '0' && e[0] <= '3' && !e[1]) ? e[0] - '0' : -1;
  }
  if (g_splits == -2) {
    const char* e = getenv("AMDK8S_GEMM_SPLITK");
    const int v = e ? atoi(e) : 0;
    g_splits = (v >= 1 && v <= 64) ? v : -1;
  }
  const int T = K / BK;
  auto max_splits = [&](int want) { int s = want < T / 8 ? want : T / 8; s = s < 16 ? s : 16; return s > 1 ? s : 1; };
  int tile = 3, splits = 1;
  if (g_tile >= 0) {
    tile = g_tile;
    const long nwg = tile_grid(tile, M, N);
    splits = nwg >= 224 ? 1 : max_splits((int)((224 + nwg - 1) / nwg));
  } else if (M <= 1024 && N >= 2048 && N <= 8192 && K >= 2048 && K <= 4096) {
    // narrow projections at prompt-chunk M (the LLM prefill's q|k|v N = 4608 and o_proj N = 3584
    // at M = 128 .. 1024): 128x64 tiles, split over K up to ~384 workgroups.  Swept per M
    // (tools/llm_prefill_gemm_probe.py, profiles/r06/prefill_gemm_narrow_*.log): q|k|v 21.4 / 26.4
    // / 34.5 / 76.9 -> 17.8 / 22.0 / 31.7 / 62.5 us and o_proj 18.4 / 22.6 / 30.2 / 43.0 -> 16.3 /
    // 20.0 / 27.3 / 39.5 us at M = 128 / 256 / 512 / 1024 against the plan below
    tile = 2;
    const long nwg = tile_grid(2, M, N);
    splits = nwg >= 256 ? 1 : max_splits((int)std::min<long>(8, (384 + nwg - 1) / nwg));
  } else {
    bool done = false;
    // a 4- or 8-wave tile whose grid nearly fills the chip runs unsplit: the split's finalize
    // pass (S × M × N fp32 through L2 / HBM) costs more than the idle CUs (SD 64² convs: 128×128
    // × 192 tiles 35.6 µs vs 256×128 × 96 tiles × 3 splits 50.3 µs — profiles/r03/h/conv_probe.log)
    for (int i = 0; i < 2 && !done; ++i)
      if (tile_grid(i, M, N) >= 160) { tile = i; splits = 1; done = true; }
    for (int i = 0; i < 4 && !done; ++i) {
      const long nwg = tile_grid(i, M, N);
      const int need = (int)((192 + nwg - 1) / nwg);
      if (need <= 16 && T / need >= 8) { tile = i; splits = need; done = true; }
    }
    if (!done) {
      tile = 3;
      const long nwg = tile_grid(3, M, N);
      splits = max_splits((int)((192 + nwg - 1) / nwg));
    }
  }
  if (g_splits >= 1) splits = g_splits < T ? g_splits : (T > 0 ? T : 1);
  *tile_out = tile;
  *splits_out = splits;
}

int amdk8s_gemm_epi_tile(int M, int N) {     // the tile the plan picks for a deep K (reporting)
  int t, s;
  amdk8s_gemm_epi_plan(M, N, 1 << 20, &t, &s);
  return t;
}

int amdk8s_gemm_epi_splits(int M, int N, int K) {
  int t, s;
  amdk8s_gemm_epi_plan(M, N, K, &t, &s);
  return s;
}

}  // extern "C"

namespace {

template <int CONV>
int launch_epi(Args a, int epi, bool f16, hipStream_t stream) {
  int tile, splits;
  amdk8s_gemm_epi_plan(a.M, a.N, a.K, &tile, &splits);
  if (!a.ws) splits = 1;                             // no workspace: one pass over K
  const long nwg = tile_grid(tile, a.M, a.N);
  if (nwg * splits > 0x7fffffff) return (int)hipErrorInvalidValue;
  a.splits = splits;
  auto go = [&](auto wm, auto wn, auto tm) {
    constexpr int WM = decltype(wm)::value, WN = decltype(wn)::value, TM = decltype(tm)::value;
    constexpr int NT = Geo<WM, WN, TM>::NT;
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(nwg * splits), dim3(NT), 0, stream, a);
    };
    if (splits > 1) {                          // partial sums; epilogue in splitk_finalize
      if (f16) launch(gemm_epi_kernel<EPI_PARTIAL, true, WM, WN, CONV, TM>);
      else launch(gemm_epi_kernel<EPI_PARTIAL, false, WM, WN, CONV, TM>);
    } else if constexpr (CONV != CONV_NONE) {  // convolutions: fp16 (the SD1.5 UNet / VAE)
      if (epi == EPI_ADD) launch(gemm_epi_kernel<EPI_ADD, true, WM, WN, CONV, TM>);
      else launch(gemm_epi_kernel<EPI_STORE, true, WM, WN, CONV, TM>);
    } else if (f16) {
      if (epi == EPI_STORE) launch(gemm_epi_kernel<EPI_STORE, true, WM, WN, CONV, TM>);
      else if (epi == EPI_GELU) launch(gemm_epi_kernel<EPI_GELU, true, WM, WN, CONV, TM>);
      else if (epi == EPI_RESID) launch(gemm_epi_kernel<EPI_RESID, true, WM, WN, CONV, TM>);
      else launch(gemm_epi_kernel<EPI_ADD, true, WM, WN, CONV, TM>);
    } else {
      if (epi == EPI_STORE) launch(gemm_epi_kernel<EPI_STORE, false, WM, WN, CONV, TM>);
      else if (epi == EPI_GELU) launch(gemm_epi_kernel<EPI_GELU, false, WM, WN, CONV, TM>);
      else if (epi == EPI_RESID) launch(gemm_epi_kernel<EPI_RESID, false, WM, WN, CONV, TM>);
      else launch(gemm_epi_kernel<EPI_ADD, false, WM, WN, CONV, TM>);
    }
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  switch (tile) {
    case 0: go(I4{}, I2{}, I1{}); break;
    case 1: go(I2{}, I2{}, I1{}); break;
    case 2: go(I2{}, I1{}, I1{}); break;
    default: go(I1{}, I1{}, I1{}); break;
  }
  if (splits > 1) {
    const long groups = (long)a.M * (a.N / 8);
    const dim3 grid((unsigned)((groups + 255) / 256));
    auto fin = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, a); };
    if (f16) {
      if (epi == EPI_GELU) fin(splitk_finalize<EPI_GELU, true>);
      else if (epi == EPI_ADD) fin(splitk_finalize<EPI_ADD, true>);
      else if (epi == EPI_RESID) fin(splitk_finalize<EPI_RESID, true>);
      else fin(splitk_finalize<EPI_STORE, true>);
    } else {
      if (epi == EPI_GELU) fin(splitk_finalize<EPI_GELU, false>);
      else if (epi == EPI_ADD) fin(splitk_finalize<EPI_ADD, false>);
      else if (epi == EPI_RESID) fin(splitk_finalize<EPI_RESID, false>);
      else fin(splitk_finalize<EPI_STORE, false>);
    }
  }
  return (int)hipGetLastError();
}

int check_out(int epi, int N, const void* out, int ldo, const void* r, int ldr) {
  if (!out || ldo % 8 || ldo < N || ((uintptr_t)out & 15)) return (int)hipErrorInvalidValue;
  if (epi == EPI_ADD && (!r || ldr % 8 || ldr < N || ((uintptr_t)r & 15)))
    return (int)hipErrorInvalidValue;
  return 0;
}

}  // namespace

extern "C" {

// epi: 0 store, 1 GELU, 2 fp32 gated residual (x, gate), 3 add (out = Y + bias + r, 16-bit r).
// ws: optional fp32 workspace of amdk8s_gemm_epi_splits(M, N, K) × M × N floats; when given,
// problems that cannot fill the chip run split-K (each split stores its partial tile to its own
// slice) + a finalize pass that sums the slices in a fixed order and applies the epilogue.
int amdk8s_gemm_epi(int epi, int dtype, const void* A, const void* B, const void* bias, void* out,
                    float* x, const float* gate, const void* r, int M, int N, int K, int lda,
                    int ldb, int ldo, int ldx, int ldr, int rows_per_gate, int gate_stride,
                    float* ws, hipStream_t stream) {
  if (!amdk8s_gemm_epi_supported(M, N, K)) return (int)hipErrorInvalidValue;
  if (epi < EPI_STORE || epi > EPI_ADD) return (int)hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || lda < K || ldb < K) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B) & 15 || ((uintptr_t)bias & 7)) return (int)hipErrorInvalidValue;
  if (epi == EPI_RESID) {
    if (!x || ldx % 4 || ldx < N || ((uintptr_t)x & 15)) return (int)hipErrorInvalidValue;
    if (gate && (rows_per_gate <= 0 || gate_stride % 4 || ((uintptr_t)gate & 15)))
      return (int)hipErrorInvalidValue;
  } else if (int rc = check_out(epi, N, out, ldo, r, ldr)) {
    return rc;
  }
  Args a{};
  a.A = (const uint16_t*)A;
  a.B = (const uint16_t*)B;
  a.bias = (const uint16_t*)bias;
  a.out = (uint16_t*)out;
  a.x = x;
  a.gate = gate;
  a.r = (const uint16_t*)r;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldo = ldo;
  a.ldx = ldx;
  a.ldr = ldr;
  a.rows_per_gate = rows_per_gate > 0 ? rows_per_gate : M;
  a.gate_stride = gate_stride;
  a.splits = 1;
  a.ws = ((uintptr_t)ws & 15) ? nullptr : ws;
  return launch_epi<CONV_NONE>(a, epi, dtype == 0, stream);
}

// 3×3 convolution, padding 1, fp16 NHWC: x [batch][Hin][Win][Cin] (channels-last, contiguous),
// w [Cout][3][3][Cin] (the OIHW weight permuted once), out [batch·Hout·Wout][ldo] (NHWC when
// ldo == Cout).  mode 1: stride 1 (Hout = Hin); 2: stride 2 (Hout = ceil(Hin/2)); 3: nearest 2×
// upsample then stride 1 (Hout = 2·Hin).  epi 0: out = conv + bias; 3: out = conv + bias + r.
// Cin % 64 == 0, Cout % 8 == 0.
int amdk8s_conv3x3_epi(int epi, int mode, const void* X, const void* W, const void* bias,
                       void* out, const void* r, int batch, int Hin, int Win, int Cin, int Cout,
                       int ldo, int ldr, float* ws, hipStream_t stream) {
  if (epi != EPI_STORE && epi != EPI_ADD) return (int)hipErrorInvalidValue;
  if (mode < CONV_S1 || mode > CONV_UP2 || batch <= 0 || Hin <= 0 || Win <= 0) return (int)hipErrorInvalidValue;
  if (Cin % 64 || Cout % 8 || Cout <= 0) return (int)hipErrorInvalidValue;
  if (((uintptr_t)X | (uintptr_t)W) & 15 || ((uintptr_t)bias & 7)) return (int)hipErrorInvalidValue;
  if (int rc = check_out(epi, Cout, out, ldo, r, ldr)) return rc;
  const int Hout = mode == CONV_S1 ? Hin : mode == CONV_S2 ? (Hin + 1) / 2 : 2 * Hin;
  const int Wout = mode == CONV_S1 ? Win : mode == CONV_S2 ? (Win + 1) / 2 : 2 * Win;
  if (Hout >= 32768 || Wout >= 32768) return (int)hipErrorInvalidValue;   // packed (y, x)
  const long M = (long)batch * Hout * Wout;
  if (M > 0x7fffffff) return (int)hipErrorInvalidValue;
  Args a{};
  a.A = (const uint16_t*)X;
  a.B = (const uint16_t*)W;
  a.bias = (const uint16_t*)bias;
  a.out = (uint16_t*)out;
  a.r = (const uint16_t*)r;
  a.M = (int)M;
  a.N = Cout;
  a.K = 9 * Cin;
  a.lda = Cin;
  a.ldb = 9 * Cin;
  a.ldo = ldo;
  a.ldr = ldr;
  a.rows_per_gate = a.M;
  a.Hin = Hin;
  a.Win = Win;
  a.Hout = Hout;
  a.Wout = Wout;
  a.Cin = Cin;
  a.splits = 1;
  a.ws = ((uintptr_t)ws & 15) ? nullptr : ws;
  if (mode == CONV_S1) return launch_epi<CONV_S1>(a, epi, true, stream);
  if (mode == CONV_S2) return launch_epi<CONV_S2>(a, epi, true, stream);
  return launch_epi<CONV_UP2>(a, epi, true, stream);
}

}  // extern "C"
