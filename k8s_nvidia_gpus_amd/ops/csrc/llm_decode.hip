// Decode-path kernels of the in-tree Qwen2 LLM engine (k8s_nvidia_gpus_amd/models/llm), gfx950.
//
// The reference serves a Qwen2.5-7B Q4_K_M GGUF with llama.cpp (reference
// cluster-config/apps/llm/deployment.yaml:31-34,61,76-84); decoding one token is a chain of
// matrix-vector products over ~4.4 GB of 4/6-bit weights, i.e. HBM-bound.  These kernels are laid
// out for that regime on MI355X:
//
// * Activations are quantised once per matrix input to int8 per 32 values ("Q8 act": x8, a fp32
//   scale per 32, and a pre-multiplied fp32 sum per 16 for the K-quant min / offset terms), fused
//   into the RMSNorm (amdk8s_llm_rmsnorm_q8) or the attention combine.  The GEMV inner product is
//   then v_dot4_i32_i8 on nibbles masked straight out of the weight words: ~0.5 VALU op per
//   weight, so the streaming load, not the ALU, is the bound.
// * One wavefront walks one weight row: 8 lanes x 16 B cover a 256-weight super-block, so each
//   wave-wide 16-byte load reads 8 consecutive super-blocks (1 KiB of quants) fully coalesced; a
//   wave's rows run as one software pipeline (next stage's loads in flight during this stage's
//   maths).
//   Both formats are repacked at load time into planes (Q4_K: nibbles + the 6-bit scales/mins
//   decoded to bytes, one dword per lane pair, + d/dmin; Q6_K: ql / qh / lane-ordered scales / d)
//   so every load is aligned and the per-lane scale decode is a byte extract (the GGUF 6-bit
//   unpacking cost more VALU than the dot products).  Same information, 148 vs 144 bytes/block.
// * The activations of the (<= 4) tokens are staged once per workgroup in LDS (x8 padded 32 B per
//   256 so the 16-lane groups of a ds_read_b128 hit disjoint banks); every wave of the workgroup
//   then streams its rows against them.
// * Epilogues are fused: bias add (q/k/v), residual add in place (o_proj, ffn_down), and the SwiGLU
//   pair mode that runs ffn_gate and ffn_up rows in the same wave and writes silu(g)*u.
// * Decode attention is split over the context (flash-decoding): per (kv head, 64-position chunk,
//   token) one workgroup scores all q heads of the GQA group with every K/V load of the chunk in
//   flight at once, and the combine kernel merges the chunks and emits the Q8 activations of the
//   o_proj input directly.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

namespace {

constexpr int kWave = 64;
constexpr int kQ4KBytes = 144;
constexpr int kMaxTok = 8;          // tokens per decode step (MFMA GEMV: two quads of 4 per wave)
constexpr int kValuMaxTok = 4;      // tokens per VALU GEMV launch (activations staged in LDS)
constexpr int kAttnChunk = 64;      // context positions per decode-attention workgroup
constexpr int kHeadDim = 128;
constexpr int kMaxGroup = 8;        // q heads per kv head

enum { kQ4K = 0, kQ6K = 1 };
enum { kStore = 0, kResid = 1, kPair = 2 };

__device__ __forceinline__ float h2f(uint16_t h) {
  _Float16 v;
  __builtin_memcpy(&v, &h, 2);
  return (float)v;
}

__device__ __forceinline__ uint16_t f2h(float f) {
  _Float16 v = (_Float16)f;
  uint16_t h;
  __builtin_memcpy(&h, &v, 2);
  return h;
}

// NeoX RoPE of one pair with explicit roundings: every kernel that rotates (rope_kv, the fused
// attention kernels) produces the same bits.
__device__ __forceinline__ float rope_lo(float x0, float x1, float c, float sn) {
  return __fmaf_rn(x0, c, -__fmul_rn(x1, sn));
}
__device__ __forceinline__ float rope_hi(float x0, float x1, float c, float sn) {
  return __fmaf_rn(x0, sn, __fmul_rn(x1, c));
}

__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// a . b with a zero accumulator as the VOP3P form's inline constant (the builtin always selects
// v_dot4c with a v_mov of 0 into the accumulator first: 2 extra VALU per 8 dot products)
__device__ __forceinline__ int dot4z(uint32_t a, uint32_t b) {
  int r;
  asm("v_dot4_i32_i8 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// LDS offset of activation byte p of one token (32-byte pad per 256 bytes)
__device__ __forceinline__ int xoff(int p) { return (p >> 8) * 288 + (p & 255); }

struct QMat {            // one quantised weight matrix [N, K], repacked at load into aligned planes
  const uint8_t* q;      // Q4_K: nibbles [N][nb][128];  Q6_K: low bits [N][nb][128]
  const uint8_t* qh;     // Q6_K: high bits [N][nb][64]
  const int8_t* sc;      // Q4_K: decoded 6-bit scales/mins [N][nb][4] dwords, dword c =
                         //   sc[2c] | sc[2c+1] << 8 | m[2c] << 16 | m[2c+1] << 24;
                         // Q6_K: scales [N][nb][16] ordered so lane `sub` reads bytes 2sub, 2sub+1
  const uint16_t* d;     // Q4_K: [N][nb] dwords (d | dmin << 16);  Q6_K: [N][nb] f16
};

// Q6_K: stored scale position of GGUF scale index i (pairs (i, i+4) adjacent per lane).
__host__ __device__ constexpr int q6_scale_pos(int i) {
  return (i & 8) + 2 * (i & 3) + ((i >> 2) & 1);
}

struct GemvArgs {
  QMat w0, w1;           // w1: ffn_up in pair mode
  const int8_t* x8;      // Q8 input: [T][K]
  const float* dx;       //           [T][K/32]
  const float* sx;       //           [T][K/16]  (dx * sum of the 16 int8 values)
  const float* xf;       // fp32 input [T][ldx] (quantised in the prologue) — instead of x8/dx/sx
  const float* norm_w;   //   optional RMSNorm weight [K] applied first
  float eps;
  int ldx;
  const float* bias;     // [N] or null (store mode)
  float* out;            // [T][ldo]
  int ldo, N, K, T;
  int rows_per_wg;
  // pair mode: emit silu(g)·u quantised to Q8 (the ffn_down input) instead of fp32 — needs
  // rows_per_wg == 32 so a workgroup owns whole 32-value blocks
  int8_t* ox8;           // [T][N]
  float* odx;            // [T][N/32]
  float* osx;            // [T][N/16]
};

// Weights are streamed exactly once per step: non-temporal loads keep them from evicting the
// activations and KV cache from L2 / the Infinity Cache.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt(const void* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// One lane's share of a 256-weight super-block: Q4_K = the block header (d, dmin, 12 scale bytes)
// + 16 B of nibbles; Q6_K = 16 B of low bits + 16 B of high bits + the 16 scales + d.
template <int TYPE> struct Blk;
template <> struct Blk<kQ4K> { uint4 q; uint32_t sm, dd; };
template <> struct Blk<kQ6K> { uint4 l, hb; uint32_t s2, d; };

template <int TYPE>
__device__ __forceinline__ void load_blk(const QMat& w, long rowblk, int blk, int sub,
                                         Blk<TYPE>& r) {
  if constexpr (TYPE == kQ4K) {
    const long rb = rowblk + blk;
    r.q = ldnt(w.q + rb * 128 + sub * 16);
    r.sm = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(w.sc) + rb * 4 + (sub >> 1));
    r.dd = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(w.d) + rb);
  } else {
    const long rb = rowblk + blk;
    r.l = ldnt(w.q + rb * 128 + sub * 16);
    r.hb = ldnt(w.qh + rb * 64 + (sub >> 2) * 32 + (sub & 1) * 16);
    r.s2 = __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(w.sc) + rb * 8 + sub);
    r.d = __builtin_nontemporal_load(w.d + rb);
  }
}

struct XView {           // the workgroup's staged activations
  const int8_t* xs;
  const float* dxs;
  const float* sxs;
  int xstride, dstride, sstride;
};

// One lane's activations for one super-block and one token: 2 x 16 int8 + their scales / sums.
struct XReg {
  uint4 xl, xh;
  float dxl, dxh, sxl, sxh;
};

template <int TYPE>
__device__ __forceinline__ XReg load_x(const XView& x, int t, int blk, int sub) {
  XReg r;
  if constexpr (TYPE == kQ4K) {
    const int p_lo = blk * 256 + (sub >> 1) * 64 + (sub & 1) * 16;   // low run; high = +32
    const int g_lo = p_lo >> 4, d_lo = p_lo >> 5;
    r.xl = *reinterpret_cast<const uint4*>(x.xs + t * x.xstride + xoff(p_lo));
    r.xh = *reinterpret_cast<const uint4*>(x.xs + t * x.xstride + xoff(p_lo + 32));
    const float2 dxv = *reinterpret_cast<const float2*>(x.dxs + t * x.dstride + d_lo);
    r.dxl = dxv.x; r.dxh = dxv.y;
    r.sxl = x.sxs[t * x.sstride + g_lo]; r.sxh = x.sxs[t * x.sstride + g_lo + 2];
  } else {
    const int n = sub >> 2, h1 = sub & 1, klo = (sub & 3) >> 1;
    const int p_lo = blk * 256 + n * 128 + klo * 32 + h1 * 16;       // low run; high = +64
    const int g_lo = p_lo >> 4, d_lo = p_lo >> 5;
    r.xl = *reinterpret_cast<const uint4*>(x.xs + t * x.xstride + xoff(p_lo));
    r.xh = *reinterpret_cast<const uint4*>(x.xs + t * x.xstride + xoff(p_lo + 64));
    r.dxl = x.dxs[t * x.dstride + d_lo]; r.dxh = x.dxs[t * x.dstride + d_lo + 2];
    r.sxl = x.sxs[t * x.sstride + g_lo]; r.sxh = x.sxs[t * x.sstride + g_lo + 4];
  }
  return r;
}

// acc += (this lane's part of) w . x for one super-block, in two halves: prep_blk decodes the
// lane's weights (nibbles / 6-bit values, block scales) once, dot_apply runs the per-token part —
// so with T tokens the decode is not repeated T times.  Explicit roundings: the same instruction
// sequence for every T instantiation and activation source (LDS or registers), so a token's
// result does not depend on how many sequences share the step (batch-invariant decode).
template <int TYPE> struct Prep;
template <> struct Prep<kQ4K> { uint32_t ql[4], qh[4]; float dsc0, dsc1, dm0, dm1; };
template <> struct Prep<kQ6K> { uint32_t ql[4], qh[4]; float sc0, sc1; };

template <int TYPE>
__device__ __forceinline__ Prep<TYPE> prep_blk(const Blk<TYPE>& r, int sub) {
  Prep<TYPE> p;
  if constexpr (TYPE == kQ4K) {
    const float d = h2f(r.dd & 0xffffu), dmin = h2f(r.dd >> 16);
    // the lane's two scales and mins were decoded from the 6-bit packing at load time
    const uint32_t sc0 = r.sm & 0xffu, sc1 = (r.sm >> 8) & 0xffu;
    const uint32_t m0 = (r.sm >> 16) & 0xffu, m1 = r.sm >> 24;
    p.dsc0 = __fmul_rn(d, (float)sc0);
    p.dsc1 = __fmul_rn(d, (float)sc1);
    p.dm0 = __fmul_rn(dmin, (float)m0);
    p.dm1 = __fmul_rn(dmin, (float)m1);
    const uint32_t q[4] = {r.q.x, r.q.y, r.q.z, r.q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      p.ql[i] = q[i] & 0x0f0f0f0fu;
      p.qh[i] = (q[i] >> 4) & 0x0f0f0f0fu;
    }
  } else {
    const int klo = (sub & 3) >> 1;
    const float d = h2f(r.d & 0xffffu);
    // scales 8n + h1 + 2klo and that + 4, stored adjacent for this lane (q6_scale_pos)
    p.sc0 = __fmul_rn(d, (float)(int8_t)(r.s2 & 0xffu));
    p.sc1 = __fmul_rn(d, (float)(int8_t)((r.s2 >> 8) & 0xffu));
    const uint32_t l[4] = {r.l.x, r.l.y, r.l.z, r.l.w};
    const uint32_t hb[4] = {r.hb.x, r.hb.y, r.hb.z, r.hb.w};
    const int sh = 2 * klo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      p.ql[i] = (l[i] & 0x0f0f0f0fu) | (((hb[i] >> sh) & 0x03030303u) << 4);
      p.qh[i] = ((l[i] >> 4) & 0x0f0f0f0fu) | (((hb[i] >> (sh + 4)) & 0x03030303u) << 4);
    }
  }
  return p;
}

template <int TYPE>
__device__ __forceinline__ float dot_apply(const Prep<TYPE>& p, const XReg& x, float acc) {
  int il = dot4z(p.ql[0], x.xl.x), ih = dot4z(p.qh[0], x.xh.x);
  il = dot4(p.ql[1], x.xl.y, il);
  il = dot4(p.ql[2], x.xl.z, il); il = dot4(p.ql[3], x.xl.w, il);
  ih = dot4(p.qh[1], x.xh.y, ih);
  ih = dot4(p.qh[2], x.xh.z, ih); ih = dot4(p.qh[3], x.xh.w, ih);
  if constexpr (TYPE == kQ4K) {
    float a = __fmaf_rn(__fmul_rn(p.dsc0, x.dxl), (float)il, acc);
    a = __fmaf_rn(__fmul_rn(p.dsc1, x.dxh), (float)ih, a);
    a = __fmaf_rn(-p.dm0, x.sxl, a);
    return __fmaf_rn(-p.dm1, x.sxh, a);
  } else {
    const float u0 = __fmaf_rn(x.dxl, (float)il, __fmul_rn(-32.f, x.sxl));
    const float u1 = __fmaf_rn(x.dxh, (float)ih, __fmul_rn(-32.f, x.sxh));
    return __fmaf_rn(p.sc1, u1, __fmaf_rn(p.sc0, u0, acc));
  }
}

template <int TYPE>
__device__ __forceinline__ float dot_core(const Blk<TYPE>& r, int sub, const XReg& x, float acc) {
  return dot_apply<TYPE>(prep_blk<TYPE>(r, sub), x, acc);
}

template <int TYPE, int T>
__device__ __forceinline__ void dot_blk(const Blk<TYPE>& r, int blk, int sub, const XView& x,
                                        float* acc) {
  const Prep<TYPE> p = prep_blk<TYPE>(r, sub);
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = dot_apply<TYPE>(p, load_x<TYPE>(x, t, blk, sub), acc[t]);
}

// Blocks per lane per pipeline stage (one stage = 8*U super-blocks of a row).
template <int TYPE, int MODE>
constexpr int kBatch = TYPE == kQ4K ? (MODE == kPair ? 2 : 4) : (MODE == kPair ? 1 : 2);

template <int TYPE, int MODE, int U>
__device__ __forceinline__ void load_stage(const GemvArgs& a, int row, int b0, int nb, int sub,
                                           int bl, Blk<TYPE> (&c)[U], Blk<TYPE> (&c1)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int blk = min(b0 + 8 * u + bl, nb - 1);  // unconditional (see attention): clamped
    load_blk<TYPE>(a.w0, (long)row * nb, blk, sub, c[u]);
    if constexpr (MODE == kPair) load_blk<TYPE>(a.w1, (long)row * nb, blk, sub, c1[u]);
  }
}

template <int TYPE, int T, int MODE, int U>
__device__ __forceinline__ void compute_stage(int b0, int nb, int sub, int bl, const XView& xv,
                                              const Blk<TYPE> (&c)[U], const Blk<TYPE> (&c1)[U],
                                              float (&acc)[T], float (&acc1)[T]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int blk = b0 + 8 * u + bl;
    if (blk < nb) {
      dot_blk<TYPE, T>(c[u], blk, sub, xv, acc);
      if constexpr (MODE == kPair) dot_blk<TYPE, T>(c1[u], blk, sub, xv, acc1);
    }
  }
}

// Cross-lane sums without the LDS unit (gfx950): v_permlane32_swap / v_permlane16_swap exchange
// 32- / 16-lane halves between two registers, DPP row_mirror / row_half_mirror / quad_perm pair
// the remaining lanes.  Every step pairs lanes symmetrically (a + b in one lane, b + a in its
// partner: the same bits), so after a full reduction every lane of a group holds identical bits.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppMirror = 0x140, kDppHalfMirror = 0x141;

// lanes < 32: a[l] + a[l + 32];  lanes >= 32: b[l - 32] + b[l]
__device__ __forceinline__ float swap_sum32(float a, float b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false,
                                                   false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// within each 32-lane half: rows of 16 — row 0: a[l] + a[l + 16];  row 1: b[l - 16] + b[l]
__device__ __forceinline__ float swap_sum16(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false,
                                                   false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Sum NV values (1, 2, 4 or 8) over the wave in 6 steps: at each of the first log2(NV) steps a
// lane keeps half of its values and hands the other half to its partner (lane bit 5, 4, then 3
// decides which half), then one value finishes.  Every lane of group l / (64 / NV) ends with the
// full sum of value l / (64 / NV).  Each value is reduced over the same lane pairings in the same
// order for any NV (bit 5, bit 4, mirror, half mirror, xor 2, xor 1), so its bits do not depend on
// how many values share the reduction: decode stays batch-invariant.
template <int NV>
__device__ __forceinline__ float wave_sum_multi(float (&x)[NV], int lane) {
  static_assert(NV == 1 || NV == 2 || NV == 4 || NV == 8, "NV must be 1, 2, 4 or 8");
  if constexpr (NV >= 2) {
#pragma unroll
    for (int i = 0; i < NV / 2; ++i) x[i] = swap_sum32(x[i], x[NV / 2 + i]);
  } else {
    x[0] = swap_sum32(x[0], x[0]);
  }
  constexpr int C1 = NV >= 2 ? NV / 2 : 1;
  if constexpr (C1 >= 2) {
#pragma unroll
    for (int i = 0; i < C1 / 2; ++i) x[i] = swap_sum16(x[i], x[C1 / 2 + i]);
  } else {
    x[0] = swap_sum16(x[0], x[0]);
  }
  constexpr int C2 = C1 >= 2 ? C1 / 2 : 1;
  float v;
  if constexpr (C2 == 2) {
    const bool hi = (lane & 8) != 0;                 // the row_mirror partner has the other bit 3
    const float keep = hi ? x[1] : x[0], give = hi ? x[0] : x[1];
    v = keep + dppf<kDppMirror>(give);
  } else {
    v = x[0] + dppf<kDppMirror>(x[0]);
  }
  v = v + dppf<kDppHalfMirror>(v);
  v = v + dppf<kDppXor2>(v);
  return v + dppf<kDppXor1>(v);
}

// Single-value full-wave max / sum without the LDS unit (same pairings as wave_sum_multi<1>).
__device__ __forceinline__ float wave_max_fast(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  v = fmaxf(v, dppf<kDppMirror>(v));
  v = fmaxf(v, dppf<kDppHalfMirror>(v));
  v = fmaxf(v, dppf<kDppXor2>(v));
  return fmaxf(v, dppf<kDppXor1>(v));
}
__device__ __forceinline__ float wave_sum_fast(float v) {
  float x[1] = {v};
  return wave_sum_multi<1>(x, 0);
}

template <int T, int MODE>
__device__ __forceinline__ void finish_row(const GemvArgs& a, int row, int lane, float (&acc)[T],
                                           float (&acc1)[T], float* q8s = nullptr, int wrow0 = 0) {
  // values: token t's acc (and, in pair mode, acc1 right after it), padded to a power of two
  constexpr int NV0 = MODE == kPair ? 2 * T : T;
  constexpr int NV = NV0 <= 1 ? 1 : NV0 <= 2 ? 2 : NV0 <= 4 ? 4 : 8;
  constexpr int SP = 64 / NV;                        // lanes holding each value
  constexpr int PER = MODE == kPair ? 2 : 1;
  float x[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) x[i] = 0.f;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    x[PER * t] = acc[t];
    if constexpr (MODE == kPair) x[2 * t + 1] = acc1[t];
  }
  const float v = wave_sum_multi<NV>(x, lane);
  float v1 = 0.f;                                    // pair: acc1 of the same token (next group)
  if constexpr (MODE == kPair) {
    if constexpr (SP == 32) {
      v1 = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v),
                                                            false, false)[1]);
    } else if constexpr (SP == 16) {
      v1 = __uint_as_float(__builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v),
                                                            false, false)[1]);
    } else {
      v1 = dppf<kDppMirror>(v);                      // SP == 8: lane 15 of the row = the next group
    }
  }
  const int t = lane / (SP * PER);
  if (lane % (SP * PER) == 0 && t < T) {
    float* o = a.out + (long)t * a.ldo + row;
    if constexpr (MODE == kStore) *o = v + (a.bias ? a.bias[row] : 0.f);
    else if constexpr (MODE == kResid) *o += v;
    else {
      const float y = v / (1.f + __expf(-v)) * v1;
      if (q8s) q8s[t * 32 + (row - wrow0)] = y;      // quantised at the end of the workgroup
      else *o = y;
    }
  }
#pragma unroll
  for (int i = 0; i < T; ++i) acc[i] = acc1[i] = 0.f;
}

// Workgroup = W waves (blockDim/64) over rows_per_wg rows; wave w takes rows w, w+W, ...  Each
// wave walks its (row, stage) items as one flat software pipeline with two register sets: the
// loads of item i+1 are in flight while item i is computed, across row boundaries, so a wave
// always has a stage of weights on the way.  Item 0's loads are issued before the activations
// are staged, so the staging (L2 → LDS → barrier) overlaps the first HBM round trip.
template <int TYPE, int T, int MODE, int U>
__device__ __forceinline__ void compute_reg(int nb, int sub, int bl, const XReg (&xr)[U][T],
                                            const Blk<TYPE> (&c)[U], const Blk<TYPE> (&c1)[U],
                                            float (&acc)[T], float (&acc1)[T]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (8 * u + bl < nb) {
      const Prep<TYPE> p = prep_blk<TYPE>(c[u], sub);
#pragma unroll
      for (int t = 0; t < T; ++t) acc[t] = dot_apply<TYPE>(p, xr[u][t], acc[t]);
      if constexpr (MODE == kPair) {
        const Prep<TYPE> p1 = prep_blk<TYPE>(c1[u], sub);
#pragma unroll
        for (int t = 0; t < T; ++t) acc1[t] = dot_apply<TYPE>(p1, xr[u][t], acc1[t]);
      }
    }
  }
}


// Stage the T tokens' activations of one GEMV in LDS: x8 (padded 32 B per 256), dx and sx, then
// the [W][T] reduction scratch.  Q8 input is copied; fp32 input (+ RMSNorm) is normalised and
// quantised by the workgroup itself.  Ends with a barrier.
template <int T>
__device__ __forceinline__ XView stage_x(const GemvArgs& a, uint8_t* lds) {
  const int K = a.K, nb = K >> 8;
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int xstride = nb * 288;                      // padded bytes per token
  int8_t* xs = reinterpret_cast<int8_t*>(lds);
  float* dxs = reinterpret_cast<float*>(lds + T * xstride);
  float* sxs = dxs + T * (K >> 5);
  float* red = sxs + T * (K >> 4);                   // [W][T] block-reduction scratch
  if (a.xf == nullptr) {
    // Q8 input: copy into LDS.  x8 [T][K], dx [T][K/32] and sx [T][K/16] are read as flat arrays
    // (index i = one 16-byte x8 unit = one sx value; dx for i < T*K/32), four units per thread
    // per round with every load of the round issued before any LDS store (clamped indices, no
    // load under a branch): one L2 round trip per round instead of one per loop iteration.
    const int nx = T * (K >> 4), nd = T * (K >> 5);
    for (int i0 = threadIdx.x; i0 < nx; i0 += 4 * (int)blockDim.x) {
      uint4 xv[4];
      float dv[4], sv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = min(i0 + u * (int)blockDim.x, nx - 1);
        xv[u] = *reinterpret_cast<const uint4*>(a.x8 + (long)i * 16);
        sv[u] = a.sx[i];
        dv[u] = a.dx[min(i, nd - 1)];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * (int)blockDim.x;
        if (i < nx) {
          const int t = i / (K >> 4), p = (i - t * (K >> 4)) << 4;
          *reinterpret_cast<uint4*>(xs + t * xstride + xoff(p)) = xv[u];
          sxs[i] = sv[u];
          if (i < nd) dxs[i] = dv[u];
        }
      }
    }
  } else if constexpr (T <= kValuMaxTok) {
    // fp32 input (+ RMSNorm): every workgroup normalises and quantises the (L2-resident) rows
    // itself, which removes a launch and its boundary per matrix.  All T tokens are processed
    // together (their loads in flight at once); per token the thread mapping and reduction order
    // do not depend on T, so results are batch-invariant.
    // chunk c = 8 values; 4 consecutive chunks (one lane quad) = one 32-value block.  Whole
    // quads leave the loops together (K % 256 == 0).
    auto quantise = [&](int t, int c, float (&v)[8], float r, const float (&wv)[8]) {
      if (a.norm_w) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] *= r * wv[i];
      }
      float amax = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
      amax = fmaxf(amax, __shfl_xor(amax, 1, kWave));
      amax = fmaxf(amax, __shfl_xor(amax, 2, kWave));
      const float d = amax / 127.f;
      const float id = d > 0.f ? 1.f / d : 0.f;
      uint32_t pk0 = 0u, pk1 = 0u;
      int sq = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int q = (int)__builtin_rintf(v[i] * id);
        if (i < 4) pk0 |= ((uint32_t)(q & 0xff)) << (8 * i);
        else pk1 |= ((uint32_t)(q & 0xff)) << (8 * (i - 4));
        sq += q;
      }
      sq += __shfl_xor(sq, 1, kWave);
      *reinterpret_cast<uint2*>(xs + t * xstride + xoff(c * 8)) = make_uint2(pk0, pk1);
      if ((c & 3) == 0) dxs[t * (K >> 5) + (c >> 2)] = d;
      if ((c & 1) == 0) sxs[t * (K >> 4) + (c >> 1)] = d * (float)sq;
    };
    auto load8 = [&](const float* p, float (&v)[8]) {
      const float4 x0 = *reinterpret_cast<const float4*>(p);
      const float4 x1 = *reinterpret_cast<const float4*>(p + 4);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
      v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    };
    const int nch = K >> 3;
    if (a.norm_w && nch <= 2 * (int)blockDim.x) {
      // single pass: each thread keeps its (<= 2) chunks of every token in registers for the
      // sum of squares and the quantisation — one L2 round trip instead of two
      float v[T][2][8], wv[2][8];
      float ss[T];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = min((int)threadIdx.x + u * (int)blockDim.x, nch - 1);
        load8(a.norm_w + c * 8, wv[u]);
#pragma unroll
        for (int t = 0; t < T; ++t) load8(a.xf + (long)t * a.ldx + c * 8, v[t][u]);
      }
#pragma unroll
      for (int t = 0; t < T; ++t) {
        ss[t] = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if ((int)threadIdx.x + u * (int)blockDim.x < nch) {
#pragma unroll
            for (int i = 0; i < 8; ++i) ss[t] = __fmaf_rn(v[t][u][i], v[t][u][i], ss[t]);
          }
        ss[t] = wave_sum_fast(ss[t]);     // = rmsnorm_q8_kernel's sum bit for bit at 256 threads
        if (lane == 0) red[wave * T + t] = ss[t];
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < T; ++t) {
        float tot = 0.f;
        for (int w = 0; w < W; ++w) tot += red[w * T + t];
        const float r = rsqrtf(tot / (float)K + a.eps);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = (int)threadIdx.x + u * (int)blockDim.x;
          if (c < nch) quantise(t, c, v[t][u], r, wv[u]);
        }
      }
    } else {
      float rs[T];
#pragma unroll
      for (int t = 0; t < T; ++t) rs[t] = 1.f;
      if (a.norm_w) {
        float ss[T];
#pragma unroll
        for (int t = 0; t < T; ++t) ss[t] = 0.f;
        for (int i0 = threadIdx.x * 4; i0 < K; i0 += blockDim.x * 8) {
          float4 v[T][2];
#pragma unroll
          for (int t = 0; t < T; ++t)
#pragma unroll
            for (int u = 0; u < 2; ++u)
              v[t][u] = *reinterpret_cast<const float4*>(
                  a.xf + (long)t * a.ldx + min(i0 + u * (int)blockDim.x * 4, K - 4));
#pragma unroll
          for (int t = 0; t < T; ++t)
#pragma unroll
            for (int u = 0; u < 2; ++u)
              if (i0 + u * (int)blockDim.x * 4 < K)
                ss[t] += v[t][u].x * v[t][u].x + v[t][u].y * v[t][u].y +
                         v[t][u].z * v[t][u].z + v[t][u].w * v[t][u].w;
        }
#pragma unroll
        for (int t = 0; t < T; ++t) {
          ss[t] = wave_sum(ss[t]);
          if (lane == 0) red[wave * T + t] = ss[t];
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < T; ++t) {
          float tot = 0.f;
          for (int w = 0; w < W; ++w) tot += red[w * T + t];
          rs[t] = rsqrtf(tot / (float)K + a.eps);
        }
      }
      for (int c = threadIdx.x; c < nch; c += blockDim.x) {
        float v[T][8], wv[8];
        if (a.norm_w) load8(a.norm_w + c * 8, wv);
#pragma unroll
        for (int t = 0; t < T; ++t) load8(a.xf + (long)t * a.ldx + c * 8, v[t]);
#pragma unroll
        for (int t = 0; t < T; ++t) quantise(t, c, v[t], rs[t], wv);
      }
    }
  }
  __syncthreads();
  return XView{xs, dxs, sxs, xstride, K >> 5, K >> 4};
}

// Pair → Q8 epilogue: the workgroup's 32 silu(g)*u outputs per token (q8s [T][32], complete in LDS)
// quantised as one 32-value block per token — half a wave per token (lane & 31 = row).
template <int T>
__device__ __forceinline__ void emit_q8_block(const GemvArgs& a, const float* q8s, int wrow0) {
  const int t = threadIdx.x >> 5, i = threadIdx.x & 31;
  if (t < T) {
    const int row = wrow0 + i;
    const float v = row < a.N ? q8s[t * 32 + i] : 0.f;
    float amax = fabsf(v);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, kWave));
    const float d = amax / 127.f;
    const int qv = d > 0.f ? (int)__builtin_rintf(v / d) : 0;
    int s16 = qv;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s16 += __shfl_xor(s16, o, kWave);
    if (row < a.N) {
      a.ox8[(long)t * a.N + row] = (int8_t)qv;
      if (i == 0) a.odx[(long)t * (a.N >> 5) + (row >> 5)] = d;
      if ((i & 15) == 0) a.osx[(long)t * (a.N >> 4) + (row >> 4)] = d * (float)s16;
    }
  }
}

// REGX (a whole row is one stage, nb <= 8U): each lane touches the same <= U super-block columns
// in every row, so its activations are read from LDS once into registers and every row after
// that is pure weight streaming + VALU (no per-row LDS traffic).
// bid = the workgroup's index within this matrix's grid.
template <int TYPE, int T, int MODE, int U, bool REGX>
__device__ __forceinline__ void qgemv_body(const GemvArgs& a, const int bid) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int K = a.K, nb = K >> 8;
  const int W = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 7, bl = lane >> 3;
  const int nst = (nb + 8 * U - 1) / (8 * U);       // pipeline stages per row
  const int r0 = bid * a.rows_per_wg + wave;
  const int r1 = min(a.N, bid * a.rows_per_wg + a.rows_per_wg);
  const int nrows = r0 < r1 ? (r1 - r0 + W - 1) / W : 0;
  const int items = nrows * nst;

  Blk<TYPE> A[U], A1[U], B[U], B1[U];
  if (items > 0) load_stage<TYPE, MODE, U>(a, r0, 0, nb, sub, bl, A, A1);

  const XView xv = stage_x<T>(a, lds);
  float* red = const_cast<float*>(xv.sxs) + T * (K >> 4);   // [W][T] block-reduction scratch

  float acc[T], acc1[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = acc1[t] = 0.f;
  // pair → Q8: the workgroup's 32 outputs per token collect in LDS (after the [W][T] scratch)
  float* q8s = (MODE == kPair && a.ox8) ? red + W * T : nullptr;
  const int wrow0 = bid * a.rows_per_wg;
  if constexpr (REGX) {
    XReg xr[U][T];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < T; ++t) xr[u][t] = load_x<TYPE>(xv, t, min(8 * u + bl, nb - 1), sub);
    for (int it = 0; it < nrows; it += 2) {
      if (it + 1 < nrows) load_stage<TYPE, MODE, U>(a, r0 + (it + 1) * W, 0, nb, sub, bl, B, B1);
      compute_reg<TYPE, T, MODE, U>(nb, sub, bl, xr, A, A1, acc, acc1);
      finish_row<T, MODE>(a, r0 + it * W, lane, acc, acc1, q8s, wrow0);
      if (it + 1 >= nrows) break;
      if (it + 2 < nrows) load_stage<TYPE, MODE, U>(a, r0 + (it + 2) * W, 0, nb, sub, bl, A, A1);
      compute_reg<TYPE, T, MODE, U>(nb, sub, bl, xr, B, B1, acc, acc1);
      finish_row<T, MODE>(a, r0 + (it + 1) * W, lane, acc, acc1, q8s, wrow0);
    }
  } else {
  for (int it = 0; it < items; it += 2) {
    if (it + 1 < items) {
      const int j = it + 1;
      load_stage<TYPE, MODE, U>(a, r0 + (j / nst) * W, (j % nst) * 8 * U, nb, sub, bl, B, B1);
    }
    compute_stage<TYPE, T, MODE, U>((it % nst) * 8 * U, nb, sub, bl, xv, A, A1, acc, acc1);
    if (it % nst == nst - 1) finish_row<T, MODE>(a, r0 + (it / nst) * W, lane, acc, acc1, q8s, wrow0);
    if (it + 1 >= items) break;
    if (it + 2 < items) {
      const int j = it + 2;
      load_stage<TYPE, MODE, U>(a, r0 + (j / nst) * W, (j % nst) * 8 * U, nb, sub, bl, A, A1);
    }
    const int i1 = it + 1;
    compute_stage<TYPE, T, MODE, U>((i1 % nst) * 8 * U, nb, sub, bl, xv, B, B1, acc, acc1);
    if (i1 % nst == nst - 1) finish_row<T, MODE>(a, r0 + (i1 / nst) * W, lane, acc, acc1, q8s, wrow0);
  }
  }
  if constexpr (MODE == kPair) {
    if (q8s) {
      __syncthreads();
      emit_q8_block<T>(a, q8s, wrow0);
    }
  }
}

template <int TYPE, int T, int MODE, int U, bool REGX>
__global__ void __launch_bounds__(512) qgemv_kernel(GemvArgs a) {
  qgemv_body<TYPE, T, MODE, U, REGX>(a, blockIdx.x);
}

// Two matrices of different quantisation types that read the same input, in ONE launch (store
// mode): Q4_K_M keeps attn_q|attn_k in Q4_K and attn_v in Q6_K in about half the layers, which
// would otherwise cost the short v GEMV a launch of its own.  Workgroups [0, grid0) run a0.
template <int TYPE0, int TYPE1, int T, int U, bool REGX>
__global__ void __launch_bounds__(512) qgemv2_kernel(GemvArgs a0, GemvArgs a1, int grid0) {
  if ((int)blockIdx.x < grid0) qgemv_body<TYPE0, T, kStore, U, REGX>(a0, blockIdx.x);
  else qgemv_body<TYPE1, T, kStore, U, REGX>(a1, blockIdx.x - grid0);
}

// ---------------------------------------------------------------- MFMA GEMV (int8 matrix cores)
// The VALU GEMV above spends ~90 VALU per lane and super-block at T = 4 (eight v_dot4 plus the
// scale arithmetic per token on top of the weight decode), which makes steps of 2-4 tokens
// VALU-bound (profiles/r04/f: gate|up 30 µs at T = 4 vs 20 µs at T = 1).  Here the integer
// sub-block sums come from v_mfma_i32_16x16x64_i8 and only the per-sub-block scaling stays on the
// VALU, once per (row, token, sub-block) instead of once per weight byte.
//
// Geometry: one wave = 16 weight rows (the MFMA's N) × a range of super-blocks; lane l loads row
// l & 15, K-group g = l >> 4 (Q4_K: nibble bytes 16g.. of each 64-byte half of the super-block, so
// each load instruction reads 64 contiguous bytes per row).  M = 16 = (token t, slot s): A row
// (t, s) carries token t's activations in K-group s only (zeros in the other three), so output
// (t, s) of row r is the sum over K-group s alone, and every K-group's 16 values of one MFMA lie in
// one sub-block.  Four MFMAs per super-block leave lane l = (row l & 15, token l >> 4) with the
// sub-block sums of its own row and token (mfma_q4_block).  Each lane then scales its own
// (row, token) in a fixed order, so a token's bits never depend on how many tokens share the
// launch (batch-invariant).
// Super-blocks are split over KW waves (reduced in LDS in wave order); RG row groups per workgroup.
typedef int i32x4 __attribute__((ext_vector_type(4)));

// The MFMA kernel reads an MFMA-packed copy of the planes (amdk8s_llm_mfma_pack), laid out per
// (16-row group G, super-block b) so that each of a wave's loads per block reads whole contiguous
// lines instead of a 64/16/4-byte piece of 16 different rows:
//   Q4_K: q [2][16 rows][64 B] (bytes 64h.. of each row's nibbles), sc [16][4] dwords, d [16] dwords
//   Q6_K: ql as Q4_K's q, qh [2][16][32 B], sc [16][16] int8 in natural order, d [16] dwords (f16)
template <int TYPE> struct MBlk;
template <> struct MBlk<kQ4K> { uint4 q0, q1, sc; uint32_t dd; };
template <> struct MBlk<kQ6K> { uint4 q0, q1, h0, h1, sc; uint32_t dd; };

template <int TYPE>
__device__ __forceinline__ void mload(const QMat& w, long gb, int lane, MBlk<TYPE>& r) {
  const int row = lane & 15, g = lane >> 4;
  const uint8_t* q = w.q + gb * 2048 + row * 64 + g * 16;
  r.q0 = ldnt(q);
  r.q1 = ldnt(q + 1024);
  if constexpr (TYPE == kQ6K) {
    const uint8_t* h = w.qh + gb * 1024 + row * 32 + (g & 1) * 16;
    r.h0 = ldnt(h);
    r.h1 = ldnt(h + 512);
    r.sc = ldnt(reinterpret_cast<const uint8_t*>(w.sc) + gb * 256 + row * 16);
  } else {
    r.sc = ldnt(reinterpret_cast<const uint32_t*>(w.sc) + gb * 64 + row * 4);
  }
  r.dd = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(w.d) + gb * 16 + row);
}

__device__ __forceinline__ i32x4 nib_lo(const uint4& v) {
  const uint32_t m = 0x0f0f0f0fu;
  return i32x4{(int)(v.x & m), (int)(v.y & m), (int)(v.z & m), (int)(v.w & m)};
}
__device__ __forceinline__ i32x4 nib_hi(const uint4& v) {
  const uint32_t m = 0x0f0f0f0fu;
  return i32x4{(int)((v.x >> 4) & m), (int)((v.y >> 4) & m), (int)((v.z >> 4) & m),
               (int)((v.w >> 4) & m)};
}
// Q6_K: 6-bit values (0..63) of 4 bytes — low / high nibbles of q with the 2-bit fields at bit k /
// k + 4 of each qh byte as bits 4-5
__device__ __forceinline__ uint32_t q6lo(uint32_t q, uint32_t h, int k) {
  return (q & 0x0f0f0f0fu) | (((h >> k) << 4) & 0x30303030u);
}
__device__ __forceinline__ uint32_t q6hi(uint32_t q, uint32_t h, int k) {
  return ((q >> 4) & 0x0f0f0f0fu) | ((h >> k) & 0x30303030u);
}

// acc += this lane's (row, token) share of one super-block.
// Q4_K: K-group g holds bytes 16g.. of each 64-byte half (q0: chunks 0-1, q1: chunks 2-3), so in
//   MFMA m (0: q0 low nibbles, 1: q0 high, 2: q1 low, 3: q1 high) groups 2h and 2h + 1 carry the
//   two 16-value halves of sub-block 2(2(m >> 1) + h) + (m & 1): c[2h] + c[2h + 1] is that
//   sub-block.  acc += d * sum_j sc_j dx_j I_j - dmin * sum_j m_j sxp_j (aux = sxp, the dx-scaled
//   sums of x per 32).
// Q6_K: group g holds values 16g.. of each 64 (bytes 16g.. of the ql halves, qh fields of
//   "l" / "32 + l" by g >> 1), so c_m[s] is the 16-value sub-block 4m + s.  Integer per 32-value
//   pair: S = sc_j (I_j - 32 X_j) + sc_j+1 (I_j+1 - 32 X_j+1) (aux = X, the int sums of x per 16),
//   then acc += d * sum_i dx_i S_i.
template <int TYPE>
__device__ __forceinline__ float mfma_block(const MBlk<TYPE>& w, const i32x4 (&xa)[4],
                                            const float (&dxv)[8], const uint4 (&aux)[4], int g,
                                            float acc) {
  const i32x4 z = {0, 0, 0, 0};
  if constexpr (TYPE == kQ4K) {
    const i32x4 c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[0], nib_lo(w.q0), z, 0, 0, 0);
    const i32x4 c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[1], nib_hi(w.q0), z, 0, 0, 0);
    const i32x4 c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[2], nib_lo(w.q1), z, 0, 0, 0);
    const i32x4 c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[3], nib_hi(w.q1), z, 0, 0, 0);
    const int I[8] = {c0[0] + c0[1], c1[0] + c1[1], c0[2] + c0[3], c1[2] + c1[3],
                      c2[0] + c2[1], c3[0] + c3[1], c2[2] + c2[3], c3[2] + c3[3]};
    const float spv[8] = {__uint_as_float(aux[0].x), __uint_as_float(aux[0].y),
                          __uint_as_float(aux[0].z), __uint_as_float(aux[0].w),
                          __uint_as_float(aux[1].x), __uint_as_float(aux[1].y),
                          __uint_as_float(aux[1].z), __uint_as_float(aux[1].w)};
    const uint32_t scw[4] = {w.sc.x, w.sc.y, w.sc.z, w.sc.w};
    float sm = 0.f, mn = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float s0 = (float)(scw[i] & 0xffu), s1 = (float)((scw[i] >> 8) & 0xffu);
      const float m0 = (float)((scw[i] >> 16) & 0xffu), m1 = (float)(scw[i] >> 24);
      sm = __fmaf_rn((float)I[2 * i], __fmul_rn(s0, dxv[2 * i]), sm);
      sm = __fmaf_rn((float)I[2 * i + 1], __fmul_rn(s1, dxv[2 * i + 1]), sm);
      mn = __fmaf_rn(m0, spv[2 * i], mn);
      mn = __fmaf_rn(m1, spv[2 * i + 1], mn);
    }
    acc = __fmaf_rn(h2f(w.dd & 0xffffu), sm, acc);
    return __fmaf_rn(-h2f(w.dd >> 16), mn, acc);
  } else {
    const int k = 2 * (g >> 1);
    const uint4 q0 = w.q0, q1 = w.q1, h0 = w.h0, h1 = w.h1;
    const i32x4 b0 = {(int)q6lo(q0.x, h0.x, k), (int)q6lo(q0.y, h0.y, k), (int)q6lo(q0.z, h0.z, k),
                      (int)q6lo(q0.w, h0.w, k)};
    const i32x4 b1 = {(int)q6hi(q0.x, h0.x, k), (int)q6hi(q0.y, h0.y, k), (int)q6hi(q0.z, h0.z, k),
                      (int)q6hi(q0.w, h0.w, k)};
    const i32x4 b2 = {(int)q6lo(q1.x, h1.x, k), (int)q6lo(q1.y, h1.y, k), (int)q6lo(q1.z, h1.z, k),
                      (int)q6lo(q1.w, h1.w, k)};
    const i32x4 b3 = {(int)q6hi(q1.x, h1.x, k), (int)q6hi(q1.y, h1.y, k), (int)q6hi(q1.z, h1.z, k),
                      (int)q6hi(q1.w, h1.w, k)};
    const i32x4 c[4] = {__builtin_amdgcn_mfma_i32_16x16x64_i8(xa[0], b0, z, 0, 0, 0),
                        __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[1], b1, z, 0, 0, 0),
                        __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[2], b2, z, 0, 0, 0),
                        __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[3], b3, z, 0, 0, 0)};
    const uint32_t X[16] = {aux[0].x, aux[0].y, aux[0].z, aux[0].w, aux[1].x, aux[1].y,
                            aux[1].z, aux[1].w, aux[2].x, aux[2].y, aux[2].z, aux[2].w,
                            aux[3].x, aux[3].y, aux[3].z, aux[3].w};
    const uint32_t scw[4] = {w.sc.x, w.sc.y, w.sc.z, w.sc.w};
    float blk = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int j = 4 * m + 2 * pr;                 // sub-blocks j, j + 1: 32-group j / 2
        const int s0 = (int)(int8_t)((scw[j >> 2] >> (8 * (j & 3))) & 0xffu);
        const int s1 = (int)(int8_t)((scw[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 0xffu);
        const int i0 = c[m][2 * pr] - 32 * (int)X[j];
        const int i1 = c[m][2 * pr + 1] - 32 * (int)X[j + 1];
        blk = __fmaf_rn((float)(s0 * i0 + s1 * i1), dxv[j >> 1], blk);
      }
    }
    return __fmaf_rn(h2f(w.dd & 0xffffu), blk, acc);
  }
}

// LDS after stage_x's arrays: [W][T] prologue scratch (rounded to 16 B), the per-type activation
// sums (Q4_K sxp float [T][K/32], Q6_K X int [T][K/16]), 256 zero bytes (the A operand of
// inactive lanes), the K-split partials [waves][token quads][P][64], q8s [T][32].
struct MfmaLds { int aux, zero, kred, q8s, total; };
__host__ __device__ inline MfmaLds mfma_lds(int type, int T, int K, int waves, int P) {
  MfmaLds L;
  const int nb = K >> 8;
  const int base = T * (nb * 288 + (K >> 5) * 4 + (K >> 4) * 4);
  const int red = ((waves * T * 4) + 15) & ~15;
  L.aux = base + red;
  L.zero = L.aux + T * (type == kQ6K ? K >> 4 : K >> 5) * 4;
  L.kred = L.zero + 256;
  L.q8s = L.kred + waves * ((T + 3) / 4) * P * 64 * 4;
  L.total = L.q8s + T * 32 * 4;
  return L;
}

// gate|up (pair, <= 4 tokens): 592 4-wave workgroups need 3 waves per SIMD to be co-resident
// bid = the workgroup's index within this matrix's grid
template <int TYPE, int T, int MODE, int KW, int RG, int D>
__device__ __forceinline__ void qgemv_mfma_body(const GemvArgs& a, const int bid) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int P = MODE == kPair ? 2 : 1;
  constexpr int NA = TYPE == kQ6K ? 4 : 2;          // uint4 of activation sums per block
  constexpr int NQ = (T + 3) / 4;                   // token quads: MFMA M = 4 tokens x 4 K-groups
  const int K = a.K, nb = K >> 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rg = wave / KW, kw = wave % KW;
  const int kb0 = kw * nb / KW, n = (kw + 1) * nb / KW - kb0;    // host: nb >= KW, so n >= 1
  const int r = lane & 15, g = lane >> 4;
  const int wrow0 = bid * RG * 16;
  const long rb0 = (long)(min(wrow0 + rg * 16, a.N - 16) >> 4) * nb + kb0;   // host: N % 16 == 0
  // ring of D super-blocks: D - 1 in flight before the activations are staged
  MBlk<TYPE> w0[D], w1[D];
#pragma unroll
  for (int d = 0; d < D - 1; ++d) {
    const long rb = rb0 + min(d, n - 1);
    mload<TYPE>(a.w0, rb, lane, w0[d]);
    if constexpr (P == 2) mload<TYPE>(a.w1, rb, lane, w1[d]);
  }
  const XView xv = stage_x<T>(a, lds);
  const MfmaLds L = mfma_lds(TYPE, T, K, KW * RG, P);
  if constexpr (TYPE == kQ4K) {
    float* sxp = reinterpret_cast<float*>(lds + L.aux);
    for (int i = threadIdx.x; i < T * (K >> 5); i += blockDim.x)
      sxp[i] = xv.sxs[2 * i] + xv.sxs[2 * i + 1];
  } else {
    int* X = reinterpret_cast<int*>(lds + L.aux);
    for (int i = threadIdx.x; i < T * (K >> 4); i += blockDim.x) {
      const int t = i / (K >> 4), p = (i - t * (K >> 4)) << 4;
      const uint4 v = *reinterpret_cast<const uint4*>(xv.xs + t * xv.xstride + xoff(p));
      int sum = dot4z(v.x, 0x01010101u);
      sum = dot4(v.y, 0x01010101u, sum);
      sum = dot4(v.z, 0x01010101u, sum);
      X[i] = dot4(v.w, 0x01010101u, sum);
    }
  }
  if (threadIdx.x < 16) reinterpret_cast<uint4*>(lds + L.zero)[threadIdx.x] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  // A operand of quad q: lane l is row (t, s) = (4q + ((l & 15) >> 2), l & 3) of K-group g; live
  // only for s == g.  MFMA m's 16 activations: Q4_K +0 / +32 / +128 / +160 from
  // 64 (g >> 1) + 16 (g & 1); Q6_K +0 / +64 / +128 / +192 from 16 g (zero lanes: the zero bytes)
  const int xb = TYPE == kQ6K ? 16 * g : 64 * (g >> 1) + 16 * (g & 1);
  int xa0[NQ], xstep[NQ], xo1[NQ], xo2[NQ], xo3[NQ];
  const float* dxb[NQ];
  const uint4* axb[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int at = 4 * q + ((lane & 15) >> 2);
    const bool live = (lane & 3) == g && at < T;
    xa0[q] = live ? at * xv.xstride + xb : L.zero;
    xstep[q] = live ? 288 : 0;
    xo1[q] = live ? (TYPE == kQ6K ? 64 : 32) : 0;
    xo2[q] = live ? 128 : 0;
    xo3[q] = live ? (TYPE == kQ6K ? 192 : 160) : 0;
    const int tt = min(4 * q + g, T - 1);            // this lane's output token in quad q
    dxb[q] = xv.dxs + tt * (K >> 5);
    axb[q] = reinterpret_cast<const uint4*>(lds + L.aux) + tt * nb * NA;
  }
  float acc[NQ], acc1[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) acc[q] = acc1[q] = 0.f;
  auto compute = [&](const MBlk<TYPE>& q0, const MBlk<TYPE>& q1, int i) {
    const int kb = kb0 + i;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint8_t* xp = lds + xa0[q] + kb * xstep[q];
      i32x4 xa[4];
      xa[0] = *reinterpret_cast<const i32x4*>(xp);
      xa[1] = *reinterpret_cast<const i32x4*>(xp + xo1[q]);
      xa[2] = *reinterpret_cast<const i32x4*>(xp + xo2[q]);
      xa[3] = *reinterpret_cast<const i32x4*>(xp + xo3[q]);
      float dxv[8];
      const float4 d0 = *reinterpret_cast<const float4*>(dxb[q] + kb * 8);
      const float4 d1 = *reinterpret_cast<const float4*>(dxb[q] + kb * 8 + 4);
      dxv[0] = d0.x; dxv[1] = d0.y; dxv[2] = d0.z; dxv[3] = d0.w;
      dxv[4] = d1.x; dxv[5] = d1.y; dxv[6] = d1.z; dxv[7] = d1.w;
      uint4 aux[4];
#pragma unroll
      for (int u = 0; u < NA; ++u) aux[u] = axb[q][kb * NA + u];
      acc[q] = mfma_block<TYPE>(q0, xa, dxv, aux, g, acc[q]);
      if constexpr (P == 2) acc1[q] = mfma_block<TYPE>(q1, xa, dxv, aux, g, acc1[q]);
    }
  };
  // Whole groups of D steps: every step first refills the slot consumed one step ago with block
  // i + D - 1 (clamped: the last group re-reads the final block from L2), then computes slot d.
  // No load sits under a branch (that makes the compiler drain every outstanding load at the
  // join, which serialises the ring); the < D leftover blocks are computed after the loop from
  // slots already in flight.
  int i0 = 0;
  for (; i0 + D <= n; i0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int ps = (d + D - 1) % D;
      const long nxt = rb0 + min(i0 + d + D - 1, n - 1);
      mload<TYPE>(a.w0, nxt, lane, w0[ps]);
      if constexpr (P == 2) mload<TYPE>(a.w1, nxt, lane, w1[ps]);
      // keep the refill ahead of this step's maths and the steps in ring order: the scheduler
      // otherwise sinks the refills, and the next step's wait then drains them too
      __builtin_amdgcn_sched_barrier(0);
      compute(w0[d], w1[d], i0 + d);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < D - 1; ++d)
    if (i0 + d < n) compute(w0[d], w1[d], i0 + d);
  // K-split partials: wave kw = 0 of each row group adds its group's in wave order
  float v[NQ], v1[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) v[q] = acc[q], v1[q] = acc1[q];
  if constexpr (KW > 1) {
    float* kred = reinterpret_cast<float*>(lds + L.kred);      // [waves][NQ][P][64]
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      kred[((wave * NQ + q) * P) * 64 + lane] = acc[q];
      if constexpr (P == 2) kred[((wave * NQ + q) * P + 1) * 64 + lane] = acc1[q];
    }
    __syncthreads();
    if (kw == 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        v[q] = 0.f; v1[q] = 0.f;
#pragma unroll
        for (int k = 0; k < KW; ++k) {
          v[q] += kred[(((rg * KW + k) * NQ + q) * P) * 64 + lane];
          if constexpr (P == 2) v1[q] += kred[(((rg * KW + k) * NQ + q) * P + 1) * 64 + lane];
        }
      }
    }
  }
  float* q8s = (MODE == kPair && a.ox8) ? reinterpret_cast<float*>(lds + L.q8s) : nullptr;
  const int orow = wrow0 + rg * 16 + r;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int t = 4 * q + g;
    if (kw == 0 && t < T && orow < a.N) {
      float* o = a.out + (long)t * a.ldo + orow;
      if constexpr (MODE == kStore) *o = v[q] + (a.bias ? a.bias[orow] : 0.f);
      else if constexpr (MODE == kResid) *o += v[q];
      else {
        const float y = v[q] / (1.f + __expf(-v[q])) * v1[q];
        if (q8s) q8s[t * 32 + rg * 16 + r] = y;
        else *o = y;
      }
    }
  }
  if constexpr (MODE == kPair && RG == 2) {
    if (q8s) {
      __syncthreads();
      emit_q8_block<T>(a, q8s, wrow0);
    }
  }
}

template <int TYPE, int T, int MODE, int KW, int RG, int D>
__global__ void __launch_bounds__(KW * RG * 64)
__attribute__((amdgpu_waves_per_eu(MODE == kPair && T <= 4 ? 3 : 1, 8)))
qgemv_mfma_kernel(GemvArgs a) {
  qgemv_mfma_body<TYPE, T, MODE, KW, RG, D>(a, blockIdx.x);
}

// Two store-mode matrices of (possibly) different types over the same input in ONE launch (q|k
// and v of Q4_K_M): workgroups [0, grid0) run a0.  Each keeps the shape and the arithmetic it has
// alone, so a row's bits do not depend on which launch computed it.
template <int TYPE0, int TYPE1, int T, int KW, int RG, int D>
__global__ void __launch_bounds__(KW * RG * 64)
qgemv2_mfma_kernel(GemvArgs a0, GemvArgs a1, int grid0) {
  if ((int)blockIdx.x < grid0) qgemv_mfma_body<TYPE0, T, kStore, KW, RG, D>(a0, blockIdx.x);
  else qgemv_mfma_body<TYPE1, T, kStore, KW, RG, D>(a1, blockIdx.x - grid0);
}

// ---------------------------------------------------------------- RMSNorm + Q8 activation quant
// grid (ceil(K/2048), T), 256 threads; thread = 8 consecutive values, 4 threads = one 32-block.
// With a norm weight every workgroup first reduces the whole row's sum of squares (the row is
// L2-resident: 14-74 KB), then scales its slice.  x fp32 [T][K]; w fp32 [K] or null.
__global__ void __launch_bounds__(256) rmsnorm_q8_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ w, float eps,
                                                         int K, int8_t* __restrict__ x8,
                                                         float* __restrict__ dx,
                                                         float* __restrict__ sx) {
  __shared__ float red[4];
  const int t = blockIdx.y;
  const float* xr = x + (long)t * K;
  const int i0 = blockIdx.x * 2048 + threadIdx.x * 8;
  // unconditional (clamped) loads: in flight together with the sum-of-squares loads below
  const int ic = min(i0, K - 8);
  const float4 a = *reinterpret_cast<const float4*>(xr + ic);
  const float4 b = *reinterpret_cast<const float4*>(xr + ic + 4);
  const float* wp = w ? w : xr;              // the norm weight loads are issued up front too
  const float4 wa = *reinterpret_cast<const float4*>(wp + ic);
  const float4 wb = *reinterpret_cast<const float4*>(wp + ic + 4);
  float rs = 1.f;
  if (w) {
    // sum of squares in the order of the qgemv prologue at 256 threads (8-value chunks tid + 256u,
    // explicit fma, wave_sum_fast, waves in order), so a row normalised here and one normalised
    // in a 4-wave GEMV prologue quantise to the same bits (decode stays batch-invariant when
    // small steps normalise in the prologue and large ones here)
    const int nch = K >> 3;
    float ss = 0.f;
    for (int u0 = 0; u0 * 256 < nch; u0 += 4) {
      float4 v[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {          // 4 chunks in flight (clamped, masked below)
        const int c = min((int)threadIdx.x + 256 * (u0 + u), nch - 1);
        v[u][0] = *reinterpret_cast<const float4*>(xr + c * 8);
        v[u][1] = *reinterpret_cast<const float4*>(xr + c * 8 + 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if ((int)threadIdx.x + 256 * (u0 + u) < nch) {
          const float e[8] = {v[u][0].x, v[u][0].y, v[u][0].z, v[u][0].w,
                              v[u][1].x, v[u][1].y, v[u][1].z, v[u][1].w};
#pragma unroll
          for (int i = 0; i < 8; ++i) ss = __fmaf_rn(e[i], e[i], ss);
        }
    }
    ss = wave_sum_fast(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    ss = red[0] + red[1] + red[2] + red[3];
    rs = rsqrtf(ss / (float)K + eps);
  }
  if (i0 >= K) return;                       // K % 256 == 0: whole quads leave together
  float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  if (w) {
    const float ww[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= rs * ww[i];
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
  amax = fmaxf(amax, dppf<kDppXor1>(amax));
  amax = fmaxf(amax, dppf<kDppXor2>(amax));
  const float d = amax / 127.f;
  const float id = d > 0.f ? 1.f / d : 0.f;
  uint32_t pk[2] = {0u, 0u};
  int s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int q = (int)__builtin_rintf(v[i] * id);
    pk[i >> 2] |= ((uint32_t)(q & 0xff)) << (8 * (i & 3));
    s += q;
  }
  s += __float_as_int(dppf<kDppXor1>(__int_as_float(s)));   // 16-value sums: lanes (0,1), (2,3)
  *reinterpret_cast<uint2*>(x8 + (long)t * K + i0) = make_uint2(pk[0], pk[1]);
  const int q4 = threadIdx.x & 3;
  if (q4 == 0) dx[(long)t * (K >> 5) + (i0 >> 5)] = d;
  if ((q4 & 1) == 0) sx[(long)t * (K >> 4) + (i0 >> 4)] = d * (float)s;
}

// ---------------------------------------------------------------- RoPE (NeoX) + KV-cache write
// qkv fp32 [T][ldq] = [q (H*128) | k (Hkv*128) | v (Hkv*128)] (bias already added by the GEMV).
// q_out fp32 [T][H*128] rotated; K/V cache fp16 [slots][Hkv][max_ctx][128] of this layer.
__global__ void __launch_bounds__(256) rope_kv_kernel(const float* __restrict__ qkv, int ldq,
                                                      const int* __restrict__ pos,
                                                      const int* __restrict__ slot,
                                                      const float* __restrict__ cos_t,
                                                      const float* __restrict__ sin_t, int H,
                                                      int Hkv, int max_ctx,
                                                      float* __restrict__ q_out,
                                                      uint16_t* __restrict__ kc,
                                                      uint16_t* __restrict__ vc) {
  // grid (ceil(((H + Hkv) * 64 + Hkv * 64) / 256), T): one thread per rotated pair or V pair
  const int t = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int p = pos[t], s = slot[t];
  const float* row = qkv + (long)t * ldq;
  const int pairs = (H + Hkv) * (kHeadDim / 2);
  if (i < pairs) {
    const int h = i / (kHeadDim / 2), j = i % (kHeadDim / 2);
    const float x0 = row[h * kHeadDim + j], x1 = row[h * kHeadDim + j + kHeadDim / 2];
    const float c = cos_t[(long)p * (kHeadDim / 2) + j], sn = sin_t[(long)p * (kHeadDim / 2) + j];
    const float y0 = rope_lo(x0, x1, c, sn), y1 = rope_hi(x0, x1, c, sn);
    if (h < H) {
      q_out[(long)t * H * kHeadDim + h * kHeadDim + j] = y0;
      q_out[(long)t * H * kHeadDim + h * kHeadDim + j + kHeadDim / 2] = y1;
    } else {
      const long base = (((long)s * Hkv + (h - H)) * max_ctx + p) * kHeadDim;
      kc[base + j] = f2h(y0);
      kc[base + j + kHeadDim / 2] = f2h(y1);
    }
  } else if (i < pairs + Hkv * (kHeadDim / 2)) {
    const int e = (i - pairs) * 2;                 // V: two values per thread
    const int h = e / kHeadDim, j = e % kHeadDim;
    const float2 v = *reinterpret_cast<const float2*>(row + (H + Hkv) * kHeadDim + e);
    const uint32_t pk = f2h(v.x) | ((uint32_t)f2h(v.y) << 16);
    *reinterpret_cast<uint32_t*>(vc + (((long)s * Hkv + h) * max_ctx + p) * kHeadDim + j) = pk;
  }
}

// ---------------------------------------------------------------- split-context decode attention
// grid (Hkv, max_ctx/64, T); 256 threads.  One workgroup: the G = H/Hkv q heads of one kv head
// over the 64 positions [s*64, min(s*64+64, len)).  Scores: 4 lanes per position (32 dims each,
// all four 16-byte K loads in flight), softmax by one wave (lane = position), P.V: wave w takes
// 16 positions with all 16 V loads in flight, lane = 2 dims.  Writes the unnormalised partial
// output and (max, sum) per head.
// Fused form (qkv != null): the workgroup rotates its q heads from the raw q|k|v projection
// itself, and the one workgroup per (token, kv head) whose chunk holds the new position also
// rotates k, writes K/V to the cache and uses them from LDS — which replaces rope_kv_kernel and its
// launch.  Valid when every token of the step is in its own slot (decode); chunked prefill of one
// sequence through this path keeps the separate rope_kv_kernel.
struct AttnArgs {
  const float* q;        // rotated q [T][H*128] (unfused)
  const float* qkv;      // raw projection [T][ldq] (fused) or null
  int ldq;
  const float* cos_t;
  const float* sin_t;
  const int* pos;
  const int* slot;
  uint16_t* kc;
  uint16_t* vc;
  int H, Hkv, max_ctx, nsplit;
  float scale;
  float* po;
  float* pml;
};

// Merge the context chunks of head h of token t and quantise the attention output to Q8 (the o_proj
// input): thread dd = one output dim; a 32-dim block = half a wave (dd & 31 within a wave).  One
// pass over the chunks in groups of 8 with every partial of the group loaded before any maths
// (online max: one memory round trip per 8 chunks), explicit roundings.
template <int NH>
__device__ __forceinline__ void combine_heads(const float* __restrict__ po,
                                              const float* __restrict__ pml,
                                              const int* __restrict__ pos, int H, int nsplit,
                                              int chunk, int h0, int hstep, int hend, int t, int dd,
                                              float* __restrict__ out, int8_t* __restrict__ x8,
                                              float* __restrict__ dx, float* __restrict__ sx) {
  const int ns = min(nsplit, (pos[t] + chunk) / chunk);
  long hb[NH];
#pragma unroll
  for (int k = 0; k < NH; ++k) hb[k] = ((long)t * H + min(h0 + k * hstep, hend - 1)) * nsplit;
  float m[NH], den[NH], v[NH];
#pragma unroll
  for (int k = 0; k < NH; ++k) { m[k] = -INFINITY; den[k] = 0.f; v[k] = 0.f; }
  for (int s0 = 0; s0 < ns; s0 += 8) {
    float mx[NH][8], l[NH][8], ov[NH][8];
#pragma unroll
    for (int k = 0; k < NH; ++k)
#pragma unroll
      for (int u = 0; u < 8; ++u) {                  // indices clamped, extra terms masked below
        const long sidx = hb[k] + min(s0 + u, ns - 1);
        mx[k][u] = pml[sidx * 2];
        l[k][u] = pml[sidx * 2 + 1];
        ov[k][u] = po[sidx * kHeadDim + dd];
      }
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      float mn = m[k];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (s0 + u < ns) mn = fmaxf(mn, mx[k][u]);
      if (mn == -INFINITY) continue;                 // nothing attended yet
      // explicit roundings (no fp-contract choice left to the compiler): the same bits for any NH
      const float sc = m[k] == -INFINITY ? 0.f : __expf(__fsub_rn(m[k], mn));
      den[k] = __fmul_rn(den[k], sc);
      v[k] = __fmul_rn(v[k], sc);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float wgt =
            (s0 + u < ns && mx[k][u] != -INFINITY) ? __expf(__fsub_rn(mx[k][u], mn)) : 0.f;
        den[k] = __fmaf_rn(wgt, l[k][u], den[k]);
        v[k] = __fmaf_rn(wgt, ov[k][u], v[k]);
      }
      m[k] = mn;
    }
  }
  const int K = H * kHeadDim;
#pragma unroll
  for (int k = 0; k < NH; ++k) {
    const int h = h0 + k * hstep;
    if (h >= hend) break;                            // uniform per wave (hstep multiple of waves)
    const float y = den[k] > 0.f ? __fdiv_rn(v[k], den[k]) : 0.f;
    const int col = h * kHeadDim + dd;
    if (out) out[(long)t * K + col] = y;
    float amax = fabsf(y);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, kWave));
    const float d = amax / 127.f;
    const int qv = d > 0.f ? (int)__builtin_rintf(y / d) : 0;
    x8[(long)t * K + col] = (int8_t)qv;
    int s16 = qv;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s16 += __shfl_xor(s16, o, kWave);
    if ((dd & 31) == 0) dx[(long)t * (K >> 5) + (col >> 5)] = d;
    if ((dd & 15) == 0) sx[(long)t * (K >> 4) + (col >> 4)] = d * (float)s16;
  }
}

// grid (H, T), 128 threads.
__global__ void __launch_bounds__(128) attn_combine_q8_kernel(const float* __restrict__ po,
                                                              const float* __restrict__ pml,
                                                              const int* __restrict__ pos, int H,
                                                              int nsplit, int chunk,
                                                              float* __restrict__ out,
                                                              int8_t* __restrict__ x8,
                                                              float* __restrict__ dx,
                                                              float* __restrict__ sx) {
  combine_heads<1>(po, pml, pos, H, nsplit, chunk, blockIdx.x, 1, H, blockIdx.y, threadIdx.x, out,
                   x8, dx, sx);
}

template <int G>
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnArgs a) {
  const float* __restrict__ q = a.q;
  const int* __restrict__ pos = a.pos;
  const int* __restrict__ slot = a.slot;
  const uint16_t* __restrict__ kc = a.kc;
  const uint16_t* __restrict__ vc = a.vc;
  const int H = a.H, Hkv = a.Hkv, max_ctx = a.max_ctx, nsplit = a.nsplit;
  const float scale = a.scale;
  float* __restrict__ po = a.po;
  float* __restrict__ pml = a.pml;
  __shared__ float qs[G][kHeadDim];
  __shared__ __align__(16) uint16_t knew[kHeadDim];   // the new position's rotated K (fp16)
  __shared__ __align__(16) uint16_t vnew[kHeadDim];   // and its V
  __shared__ float ps[G][kAttnChunk];
  __shared__ float mls[G][2];
  __shared__ float opart[4][G][kHeadDim];
  const int kh = blockIdx.x, sp = blockIdx.y, t = blockIdx.z;
  const int len = pos[t] + 1;
  const int p0 = sp * kAttnChunk;
  const long pidx = ((long)t * H + kh * G) * nsplit + sp;   // + g * nsplit
  if (p0 >= len) {
    if (threadIdx.x < G) {
      float* dst = pml + (pidx + (long)threadIdx.x * nsplit) * 2;
      dst[0] = -INFINITY;
      dst[1] = 0.f;
    }
    return;
  }
  const int n = min(kAttnChunk, len - p0);
  const long cbase = ((long)slot[t] * Hkv + kh) * max_ctx * kHeadDim;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // K loads first (independent of q)
  const int pi = threadIdx.x >> 2, qd = threadIdx.x & 3;
  // every load is unconditional (positions clamped into the chunk): a load under a branch ends
  // its basic block and the join waits for it, which would serialise the HBM round trips
  uint4 kv[4];
  {
    const uint4* kr = reinterpret_cast<const uint4*>(kc + cbase + (long)(p0 + min(pi, n - 1))
                                                     * kHeadDim + qd * 32);
#pragma unroll
    for (int c = 0; c < 4; ++c) kv[c] = kr[c];
  }
  // V rows too (P.V: wave w → positions w*16 .. w*16+15, lane = 2 dims): independent of the
  // scores, so their HBM round trip overlaps the K one instead of following the softmax
  uint32_t vv[16];
  {
    const uint32_t* vr = reinterpret_cast<const uint32_t*>(vc + cbase) + lane;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int p = min(wave * 16 + j, n - 1);        // ps[.][p >= n] == 0
      vv[j] = vr[(long)(p0 + p) * (kHeadDim / 2)];
    }
  }
  const int pnew = len - 1;
  const bool own = a.qkv != nullptr && pnew >= p0 && pnew < p0 + kAttnChunk;
  if (a.qkv) {
    const float* row = a.qkv + (long)t * a.ldq;
    const float* ct = a.cos_t + (long)pnew * (kHeadDim / 2);
    const float* st = a.sin_t + (long)pnew * (kHeadDim / 2);
    // every load of the q rotation and of the new k / v row in flight at once (indices clamped,
    // no load under a branch), then the maths and the stores
    constexpr int QR = (G * (kHeadDim / 2) + 255) / 256;   // rotation pairs per thread
    float qx0[QR], qx1[QR], qc[QR], qsn[QR];
#pragma unroll
    for (int u = 0; u < QR; ++u) {
      const int i = min((int)threadIdx.x + 256 * u, G * (kHeadDim / 2) - 1);
      const int g = i / (kHeadDim / 2), j = i % (kHeadDim / 2);
      qx0[u] = row[(kh * G + g) * kHeadDim + j];
      qx1[u] = row[(kh * G + g) * kHeadDim + j + kHeadDim / 2];
      qc[u] = ct[j];
      qsn[u] = st[j];
    }
    const int jk = threadIdx.x & (kHeadDim / 2 - 1), ev = threadIdx.x & (kHeadDim - 1);
    const float k0 = row[(H + kh) * kHeadDim + jk], k1 = row[(H + kh) * kHeadDim + jk + kHeadDim / 2];
    const float vn = row[(H + Hkv + kh) * kHeadDim + ev];
#pragma unroll
    for (int u = 0; u < QR; ++u) {
      const int i = (int)threadIdx.x + 256 * u;
      if (i < G * (kHeadDim / 2)) {
        const int g = i / (kHeadDim / 2), j = i % (kHeadDim / 2);
        qs[g][j] = rope_lo(qx0[u], qx1[u], qc[u], qsn[u]) * scale;
        qs[g][j + kHeadDim / 2] = rope_hi(qx0[u], qx1[u], qc[u], qsn[u]) * scale;
      }
    }
    if (own) {
      const long cpos = cbase + (long)pnew * kHeadDim;
      if (threadIdx.x < kHeadDim / 2) {
        const float c = qc[0], sn = qsn[0];          // thread j < 64 loaded ct[j] / st[j] at u = 0
        const uint16_t h0 = f2h(rope_lo(k0, k1, c, sn)), h1 = f2h(rope_hi(k0, k1, c, sn));
        a.kc[cpos + jk] = h0;
        a.kc[cpos + jk + kHeadDim / 2] = h1;
        knew[jk] = h0;
        knew[jk + kHeadDim / 2] = h1;
      }
      if (threadIdx.x < kHeadDim) {
        const uint16_t hv = f2h(vn);
        a.vc[cpos + ev] = hv;
        vnew[ev] = hv;
      }
    }
  } else {
    for (int i = threadIdx.x; i < G * kHeadDim; i += blockDim.x)
      qs[i / kHeadDim][i % kHeadDim] = q[(long)t * H * kHeadDim + (kh * G) * kHeadDim + i] * scale;
  }
  __syncthreads();
  if (own && p0 + pi == pnew) {   // the new position: its K row was loaded before it was written
#pragma unroll
    for (int c = 0; c < 4; ++c) kv[c] = reinterpret_cast<const uint4*>(knew)[qd * 4 + c];
  }
  if (own) {                      // ... and so was its V row
    const int jn = pnew - p0 - wave * 16;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j == jn) vv[j] = reinterpret_cast<const uint32_t*>(vnew)[lane];
  }
  float sc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) sc[g] = 0.f;
  {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t kw[4] = {kv[c].x, kv[c].y, kv[c].z, kv[c].w};
      float kf[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        kf[2 * e] = h2f(kw[e] & 0xffffu);
        kf[2 * e + 1] = h2f(kw[e] >> 16);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int e = 0; e < 8; ++e) sc[g] += kf[e] * qs[g][qd * 32 + c * 8 + e];
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    sc[g] += __shfl_xor(sc[g], 1, kWave);
    sc[g] += __shfl_xor(sc[g], 2, kWave);
  }
  if (qd == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g)
      ps[g][pi] = pi < n ? sc[g] : -INFINITY;
  }
  __syncthreads();
  // softmax: head g on wave g % 4 (lane = position), LDS-free cross-lane max / sum
#pragma unroll
  for (int g0 = 0; g0 < G; g0 += 4) {
    const int g = g0 + wave;
    if (g < G) {
      const float s = ps[g][lane];
      const float m = wave_max_fast(s);
      const float p = lane < n ? __expf(s - m) : 0.f;
      ps[g][lane] = p;
      const float l = wave_sum_fast(p);
      if (lane == 0) { mls[g][0] = m; mls[g][1] = l; }
    }
  }
  __syncthreads();
  // P.V: wave w → positions w*16 .. w*16+15 (rows loaded at the top)
  float o[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) o[g][0] = o[g][1] = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float v0 = h2f(vv[j] & 0xffffu), v1 = h2f(vv[j] >> 16);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float pw = ps[g][wave * 16 + j];
      o[g][0] += pw * v0;
      o[g][1] += pw * v1;
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    opart[wave][g][2 * lane] = o[g][0];
    opart[wave][g][2 * lane + 1] = o[g][1];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * kHeadDim; i += blockDim.x) {
    const int g = i / kHeadDim, dd = i % kHeadDim;
    const float v = opart[0][g][dd] + opart[1][g][dd] + opart[2][g][dd] + opart[3][g][dd];
    po[(pidx + (long)g * nsplit) * kHeadDim + dd] = v;
  }
  if (threadIdx.x < G) {
    const int g = threadIdx.x;
    float* dst = pml + (pidx + (long)g * nsplit) * 2;
    dst[0] = mls[g][0];
    dst[1] = mls[g][1];
  }
}

// ---------------------------------------------------------------- greedy sampling
// out[t] = argmax of logits row t (the first index of the maximum, as torch.argmax): one 1024-thread
// workgroup per row, 16-byte loads, (value, index) reductions.  Captured into the decode step's HIP
// graph so a greedy step ends with one 4-byte-per-token copy instead of a separate argmax launch.
__global__ void __launch_bounds__(1024) argmax_rows_kernel(const float* __restrict__ x, int V,
                                                           long ld, int* __restrict__ out) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const float* row = x + blockIdx.x * ld;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  const int nv4 = V >> 2;
  // 8 loads in flight per thread per round (a 152k-entry row is 5 rounds, not 38 dependent trips);
  // indices increase per thread, so strict '>' keeps the first maximum
  constexpr int kU = 8;
  for (int i0 = threadIdx.x; i0 < nv4; i0 += kU * blockDim.x) {
    float4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      v[u] = reinterpret_cast<const float4*>(row)[min(i0 + u * (int)blockDim.x, nv4 - 1)];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * (int)blockDim.x;
      const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (i < nv4 && e[k] > best) { best = e[k]; bi = 4 * i + k; }
    }
  }
  for (int i = (nv4 << 2) + threadIdx.x; i < V; i += blockDim.x)
    if (row[i] > best) { best = row[i]; bi = i; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, kWave);
    const int oi = __shfl_xor(bi, o, kWave);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { sv[wave] = best; si[wave] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
      if (sv[w] > best || (sv[w] == best && si[w] < bi)) { best = sv[w]; bi = si[w]; }
    out[blockIdx.x] = bi == 0x7fffffff ? 0 : bi;
  }
}

// ---------------------------------------------------------------- dequantisation (rows → fp16/fp32)
// One thread per 32-weight run.  rows: optional row indices (embedding gather).
template <int TYPE, bool F32OUT>
__global__ void __launch_bounds__(256) dequant_kernel(QMat w, const int* __restrict__ rows,
                                                      int nrows, int K, void* __restrict__ out) {
  const int nb = K >> 8;
  const long runs = (long)nrows * (K >> 5);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < runs;
       i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / (K >> 5));
    const int run = (int)(i % (K >> 5));
    const int row = rows ? rows[r] : r;
    const int blk = run >> 3, j = run & 7;            // super-block, 32-run within it
    float v[32];
    if constexpr (TYPE == kQ4K) {
      const long rb = (long)row * nb + blk;
      const uint32_t dd = reinterpret_cast<const uint32_t*>(w.d)[rb];
      const float d = h2f(dd & 0xffffu), dmin = h2f(dd >> 16);
      const uint32_t smw = reinterpret_cast<const uint32_t*>(w.sc)[rb * 4 + (j >> 1)];
      const uint32_t sc = (smw >> (8 * (j & 1))) & 0xffu, m = (smw >> (16 + 8 * (j & 1))) & 0xffu;
      const uint8_t* qs = w.q + rb * 128 + (j >> 1) * 32;
#pragma unroll
      for (int l = 0; l < 32; ++l) {
        const uint32_t q = (j & 1) ? (qs[l] >> 4) : (qs[l] & 0xf);
        v[l] = d * (float)sc * (float)q - dmin * (float)m;
      }
    } else {
      const long rb = (long)row * nb + blk;
      const int n = j >> 2, k = j & 3;                // half, 32-run within the half
      const uint8_t* ql = w.q + rb * 128 + n * 64 + (k & 1) * 32;
      const uint8_t* qh = w.qh + rb * 64 + n * 32;
      const int8_t* sc = w.sc + rb * 16;
      const float d = h2f(w.d[rb]);
#pragma unroll
      for (int l = 0; l < 32; ++l) {
        const uint32_t lo = (k < 2) ? (ql[l] & 0xf) : (ql[l] >> 4);
        const int q = (int)(lo | (((qh[l] >> (2 * k)) & 3) << 4)) - 32;
        v[l] = d * (float)sc[q6_scale_pos(8 * n + 2 * k + (l >> 4))] * (float)q;
      }
    }
    if constexpr (F32OUT) {
      float* o = reinterpret_cast<float*>(out) + (long)r * K + run * 32;
#pragma unroll
      for (int l = 0; l < 32; l += 4) *reinterpret_cast<float4*>(o + l) = make_float4(v[l], v[l + 1], v[l + 2], v[l + 3]);
    } else {
      uint16_t* o = reinterpret_cast<uint16_t*>(out) + (long)r * K + run * 32;
#pragma unroll
      for (int l = 0; l < 32; l += 8) {
        uint4 pk;
        pk.x = f2h(v[l]) | ((uint32_t)f2h(v[l + 1]) << 16);
        pk.y = f2h(v[l + 2]) | ((uint32_t)f2h(v[l + 3]) << 16);
        pk.z = f2h(v[l + 4]) | ((uint32_t)f2h(v[l + 5]) << 16);
        pk.w = f2h(v[l + 6]) | ((uint32_t)f2h(v[l + 7]) << 16);
        *reinterpret_cast<uint4*>(o + l) = pk;
      }
    }
  }
}

// Q6_K GGUF blocks (210 B) → the four aligned planes the GEMV reads.
__global__ void q6k_repack_kernel(const uint8_t* __restrict__ src, long nblocks,
                                  uint8_t* __restrict__ ql, uint8_t* __restrict__ qh,
                                  int8_t* __restrict__ sc, uint16_t* __restrict__ d) {
  for (long b = blockIdx.x * (long)blockDim.x + threadIdx.x; b < nblocks;
       b += (long)gridDim.x * blockDim.x) {
    const uint8_t* s = src + b * 210;
    for (int i = 0; i < 128; ++i) ql[b * 128 + i] = s[i];
    for (int i = 0; i < 64; ++i) qh[b * 64 + i] = s[128 + i];
    for (int i = 0; i < 16; ++i) sc[b * 16 + q6_scale_pos(i)] = (int8_t)s[192 + i];
    d[b] = (uint16_t)(s[208] | (s[209] << 8));
  }
}

// Q4_K GGUF blocks (144 B) → nibbles [nb][128] + decoded scales/mins [nb][4 dwords] + d/dmin.
__global__ void q4k_repack_kernel(const uint8_t* __restrict__ src, long nblocks,
                                  uint8_t* __restrict__ qs, uint32_t* __restrict__ scm,
                                  uint32_t* __restrict__ dm) {
  for (long b = blockIdx.x * (long)blockDim.x + threadIdx.x; b < nblocks;
       b += (long)gridDim.x * blockDim.x) {
    const uint8_t* s = src + b * kQ4KBytes;
    dm[b] = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
    const uint8_t* q = s + 4;
    uint32_t sc[8], m[8];
    for (int j = 0; j < 8; ++j) {
      if (j < 4) { sc[j] = q[j] & 63; m[j] = q[j + 4] & 63; }
      else { sc[j] = (q[j + 4] & 0xf) | ((q[j - 4] >> 6) << 4); m[j] = (q[j + 4] >> 4) | ((q[j] >> 6) << 4); }
    }
    for (int c = 0; c < 4; ++c)
      scm[b * 4 + c] = sc[2 * c] | (sc[2 * c + 1] << 8) | (m[2 * c] << 16) | (m[2 * c + 1] << 24);
    for (int c = 0; c < 8; ++c)
      *reinterpret_cast<uint4*>(qs + b * 128 + c * 16) =
          *reinterpret_cast<const uint4*>(s + 16 + c * 16);
  }
}

// Repacked planes → the MFMA-packed copy (see mload): one thread per (row, super-block).
// Q4_K: q [N][nb*128], sc [N][nb*4] dwords, d [N][nb] dwords.  Q6_K: ql [N][nb*128],
// qh [N][nb*64], sc [N][nb*16] int8 (lane order, q6_scale_pos), d [N][nb] f16.
template <int TYPE>
__global__ void mfma_pack_kernel(QMat w, int N, int nb, uint8_t* __restrict__ mq,
                                 uint8_t* __restrict__ mqh, uint8_t* __restrict__ msc,
                                 uint32_t* __restrict__ md) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * nb) return;
  const int row = (int)(i / nb), b = (int)(i % nb);
  const long gb = (long)(row >> 4) * nb + b;
  const int r = row & 15;
  const uint4* src = reinterpret_cast<const uint4*>(w.q + i * 128);
  uint4* dst = reinterpret_cast<uint4*>(mq + gb * 2048 + r * 64);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[h * 64 + j] = src[h * 4 + j];
  if constexpr (TYPE == kQ4K) {
    reinterpret_cast<uint4*>(msc + gb * 256 + r * 16)[0] =
        reinterpret_cast<const uint4*>(w.sc + i * 16)[0];
    md[gb * 16 + r] = reinterpret_cast<const uint32_t*>(w.d)[i];
  } else {
    const uint4* hs = reinterpret_cast<const uint4*>(w.qh + i * 64);
    uint4* hd = reinterpret_cast<uint4*>(mqh + gb * 1024 + r * 32);
    hd[0] = hs[0]; hd[1] = hs[1];                   // half 0: qh bytes 0..31
    hd[32] = hs[2]; hd[33] = hs[3];                 // half 1: bytes 32..63, 512 B further
    uint8_t sc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) sc[j] = (uint8_t)w.sc[i * 16 + q6_scale_pos(j)];
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      wv[j] = sc[4 * j] | (sc[4 * j + 1] << 8) | (sc[4 * j + 2] << 16) | ((uint32_t)sc[4 * j + 3] << 24);
    reinterpret_cast<uint4*>(msc + gb * 256 + r * 16)[0] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    md[gb * 16 + r] = w.d[i];
  }
}

template <int TYPE, int T, int MODE, int U, bool REGX>
int launch_one(const GemvArgs& a, int waves, hipStream_t st) {
  const int nb = a.K >> 8;
  const size_t lds = (size_t)T * (nb * 288 + (a.K >> 5) * 4 + (a.K >> 4) * 4) + 16 * T * 4 +
                     (a.ox8 ? (size_t)T * 32 * 4 : 0);
  if (lds > 160 * 1024) return 3;
  const int grid = (a.N + a.rows_per_wg - 1) / a.rows_per_wg;
  hipLaunchKernelGGL((qgemv_kernel<TYPE, T, MODE, U, REGX>), dim3(grid), dim3(waves * 64), lds, st,
                     a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Stage width U (super-blocks per lane per stage): the smallest that covers a row in one stage
// (short rows), else the type/mode batch; register-resident activations when a row is one stage
// and T <= kRegxMaxT (VGPR budget; 4 measured slower, docs/experiments/llm_decode_rejected.md).
// Every variant runs the same dot_core, so the choice never changes a result bit.
constexpr int kRegxMaxT = 2;

// Long rows (ffn_down: 74 super-blocks) in two balanced stages (U = ceil(nb / 16)) instead of
// KB-wide ones: faster from T = 3 (T=3 / T=4 2.43 / 2.64 -> 2.39 / 2.60 ms, profiles/r03/ag); at
// T = 1 faster for Q4_K rows (14.5 -> 13.5 us) and slower for Q6_K ones (13.8 -> 17.1 us; step
// 1.740 -> 1.721 ms with Q4_K only, profiles/r03/ap), so Q4_K always, Q6_K from T = 3.  The stage
// width never changes a result bit.
static bool longrow_enabled(int type, int T) { return type == kQ4K || T >= 3; }

template <int TYPE, int T, int MODE>
int launch_gemv(const GemvArgs& a, int waves, hipStream_t st) {
  constexpr int KB = kBatch<TYPE, MODE>;
  const int nb = a.K >> 8;
  if (nb <= 8) return launch_one<TYPE, T, MODE, 1, true>(a, waves, st);
  if constexpr (KB >= 2) {
    if (nb <= 16) {
      if constexpr (T <= 2) return launch_one<TYPE, T, MODE, 2, true>(a, waves, st);
      else if (T <= kRegxMaxT) return launch_one<TYPE, T, MODE, 2, true>(a, waves, st);
      else return launch_one<TYPE, T, MODE, 2, false>(a, waves, st);
    }
  }
  if constexpr (MODE != kPair) {
    // long rows (ffn_down: 74 super-blocks): two stages per row with U = ceil(nb / 16) instead of
    // KB-wide stages whose last one is mostly clamped lanes (74 = 32 + 32 + 10 at U = 4)
    if (longrow_enabled(TYPE, T)) {
      const int u2 = (nb + 15) / 16;
      if (u2 == 5) return launch_one<TYPE, T, MODE, 5, false>(a, waves, st);
      if (u2 == 6) return launch_one<TYPE, T, MODE, 6, false>(a, waves, st);
    }
  }
  return launch_one<TYPE, T, MODE, KB, false>(a, waves, st);
}

template <int TYPE, int MODE>
int dispatch_t(const GemvArgs& a, int waves, hipStream_t st) {
  switch (a.T) {
    case 1: return launch_gemv<TYPE, 1, MODE>(a, waves, st);
    case 2: return launch_gemv<TYPE, 2, MODE>(a, waves, st);
    case 3: return launch_gemv<TYPE, 3, MODE>(a, waves, st);
    case 4: return launch_gemv<TYPE, 4, MODE>(a, waves, st);
    default: return 2;
  }
}

// Two matrices in one launch (qgemv2_kernel): rows of one pipeline stage only (nb <= 16, the
// q|k|v shapes), with the stage width each type takes alone; 4 = not supported here (the caller
// launches the two matrices separately).
template <int TYPE0, int TYPE1, int T>
int launch_gemv2(const GemvArgs& a0, const GemvArgs& a1, int waves, hipStream_t st) {
  const int nb = a0.K >> 8;
  const size_t lds = (size_t)T * (nb * 288 + (a0.K >> 5) * 4 + (a0.K >> 4) * 4) + 16 * T * 4;
  const int g0 = (a0.N + a0.rows_per_wg - 1) / a0.rows_per_wg;
  const int g1 = (a1.N + a1.rows_per_wg - 1) / a1.rows_per_wg;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(g0 + g1), dim3(waves * 64), lds, st, a0, a1, g0);
    return hipGetLastError() == hipSuccess ? 0 : 1;
  };
  if (nb <= 8) return go(qgemv2_kernel<TYPE0, TYPE1, T, 1, true>);
  if (nb <= 16) {
    if (T <= kRegxMaxT) return go(qgemv2_kernel<TYPE0, TYPE1, T, 2, true>);
    return go(qgemv2_kernel<TYPE0, TYPE1, T, 2, false>);
  }
  return 4;
}

template <int TYPE0, int TYPE1>
int dispatch2_t(const GemvArgs& a0, const GemvArgs& a1, int waves, hipStream_t st) {
  switch (a0.T) {
    case 1: return launch_gemv2<TYPE0, TYPE1, 1>(a0, a1, waves, st);
    case 2: return launch_gemv2<TYPE0, TYPE1, 2>(a0, a1, waves, st);
    case 3: return launch_gemv2<TYPE0, TYPE1, 3>(a0, a1, waves, st);
    case 4: return launch_gemv2<TYPE0, TYPE1, 4>(a0, a1, waves, st);
    default: return 2;
  }
}

// Default decomposition (measured on MI355X, tools/llm_bench.py --gemv, T = 1): 4-wave
// workgroups of 8 rows for the 3584/4608/18944-row matrices, 8 waves for the 18944-long rows of
// ffn_down, and 32 rows per workgroup for the 152064-row lm_head (longer per-wave pipelines).
// From T = 3 on, the 18944-long ffn_down rows run 16 per workgroup (2 per wave: the staged
// activations serve twice the weights; 20.8 / 24.2 vs 24.4 / 26.6 us for Q4_K / Q6_K at T = 4,
// profiles/r03/y — at T = 1 the 8-row grid is faster).
// Q4_K ffn_down rows (long-row stages at every T) take 16 rows per workgroup at T = 1 too:
// 13.6 -> 12.2 us (profiles/r03/aq); Q6_K ones stay at 8 (13.8 vs 17.2 us).
void gemv_shape(int type, int N, int K, int T, int& waves, int& rows) {
  if (waves <= 0) waves = K >= 8192 ? 8 : 4;
  if (rows <= 0)
    rows = N >= 65536 ? 32
           : (K >= 8192 && waves == 8 && (T >= 3 || (type == kQ4K && longrow_enabled(type, T))))
               ? 16 : 8;
}

// MFMA GEMV launch shapes (K-waves x row groups, swept with tools/llm_bench.py --gemv, profiles/r04/l):
// pair (gate|up) 2 x 2 (a whole 32-row Q8 block per workgroup); long rows (K >= 8192: ffn_down)
// 8 x 1; very tall matrices (lm_head) 2 x 2; the rest 4 x 1 (q|k|v, o_proj: 2 x 1 measured the same).  4 = shape not covered (N % 16, fewer super-blocks than K-waves, LDS): use qgemv_kernel.
template <int TYPE, int T, int MODE, int KW, int RG>
int launch_mfma_one(const GemvArgs& a, hipStream_t st) {
  // ring depth: pair 2 (two matrices per slot, 3 waves/SIMD), else 3 (6 for ffn_down's 8-wave
  // shape measured slower: Q6_K 13.9 -> 15.6 us, T = 1 1.629 -> 1.656 ms, profiles/r04/o)
  constexpr int D = MODE == kPair ? 2 : 3;
  if ((a.K >> 8) < KW) return 4;
  if (KW == 8 && T > 4) return 4;                   // register budget: tokens in two launches
  const MfmaLds L = mfma_lds(TYPE, T, a.K, KW * RG, MODE == kPair ? 2 : 1);
  if (L.total > 160 * 1024) return 4;
  const int grid = (a.N + 16 * RG - 1) / (16 * RG);
  hipLaunchKernelGGL((qgemv_mfma_kernel<TYPE, T, MODE, KW, RG, D>), dim3(grid), dim3(KW * RG * 64),
                     L.total, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Default shape: a function of the matrix only (never of T or of the input form), so each matrix
// sums its K-split partials in one order at every T (batch invariance), and 4 waves wherever the
// fp32-row prologue may run (stage_x reduces the RMSNorm over 4 waves in rmsnorm_q8's order;
// models with dim >= 8192 use the prologue at every T).
void mfma_shape(bool pair, int N, int K, int& kw, int& rg) {
  const int nb = K >> 8;
  if (pair) kw = nb >= 2 ? 2 : 1, rg = 2;
  else if (K >= 8192) kw = 8, rg = 1;
  else if (N >= 65536 && nb >= 2) kw = 2, rg = 2;    // lm_head: 75.0 / 80.2 us at T = 1 / 4
  else if (nb >= 4) kw = 4, rg = 1;
  else if (nb >= 2) kw = 2, rg = 2;
  else kw = 1, rg = 4;
}

template <int TYPE, int T, int MODE>
int launch_mfma(const GemvArgs& a, int kw, int rg, hipStream_t st) {
  if (a.N % 16) return 4;
  if (kw <= 0) mfma_shape(MODE == kPair, a.N, a.K, kw, rg);
  if (MODE == kPair && a.ox8 && rg != 2) return 2;   // a whole 32-row Q8 block per workgroup
  if (MODE == kPair && a.ox8 && kw * rg * 64 < 32 * T) return 2;   // emit_q8_block: 32 lanes/token
  switch (kw * 8 + rg) {
    case 1 * 8 + 2: return launch_mfma_one<TYPE, T, MODE, 1, 2>(a, st);
    case 1 * 8 + 4: return launch_mfma_one<TYPE, T, MODE, 1, 4>(a, st);
    case 2 * 8 + 1: return launch_mfma_one<TYPE, T, MODE, 2, 1>(a, st);
    case 2 * 8 + 2: return launch_mfma_one<TYPE, T, MODE, 2, 2>(a, st);
    case 4 * 8 + 1: return launch_mfma_one<TYPE, T, MODE, 4, 1>(a, st);
    case 4 * 8 + 2: return launch_mfma_one<TYPE, T, MODE, 4, 2>(a, st);
    case 8 * 8 + 1: return launch_mfma_one<TYPE, T, MODE, 8, 1>(a, st);
    default: return 2;
  }
}

// kw / rg: K-waves and 16-row groups per workgroup (0 = the default shape for the matrix)
template <int TYPE, int MODE>
int dispatch_mfma(const GemvArgs& a, int kw, int rg, hipStream_t st) {
  switch (a.T) {
    case 1: return launch_mfma<TYPE, 1, MODE>(a, kw, rg, st);
    case 2: return launch_mfma<TYPE, 2, MODE>(a, kw, rg, st);
    case 3: return launch_mfma<TYPE, 3, MODE>(a, kw, rg, st);
    case 4: return launch_mfma<TYPE, 4, MODE>(a, kw, rg, st);
    case 5: return launch_mfma<TYPE, 5, MODE>(a, kw, rg, st);
    case 6: return launch_mfma<TYPE, 6, MODE>(a, kw, rg, st);
    case 7: return launch_mfma<TYPE, 7, MODE>(a, kw, rg, st);
    case 8: return launch_mfma<TYPE, 8, MODE>(a, kw, rg, st);
    default: return 2;
  }
}

// More than 4 tokens whose activations do not fit the LDS with T (ffn_down's K = 18944 at T > 4):
// tokens [0, 4) and [4, T) as two launches.  Every token's arithmetic is the same in either form.
template <int TYPE, int MODE>
int dispatch_mfma_split(const GemvArgs& a, int kw, int rg, hipStream_t st) {
  const int rc = dispatch_mfma<TYPE, MODE>(a, kw, rg, st);
  if (rc != 4 || a.T <= 4) return rc;
  GemvArgs lo = a, hi = a;
  lo.T = 4;
  hi.T = a.T - 4;
  const long K = a.K;
  if (hi.x8) { hi.x8 += 4 * K; hi.dx += 4 * (K >> 5); hi.sx += 4 * (K >> 4); }
  if (hi.xf) hi.xf += 4L * a.ldx;
  hi.out += 4L * a.ldo;
  if (hi.ox8) { hi.ox8 += 4L * a.N; hi.odx += 4L * (a.N >> 5); hi.osx += 4L * (a.N >> 4); }
  const int r0 = dispatch_mfma<TYPE, MODE>(lo, kw, rg, st);
  if (r0) return r0;
  return dispatch_mfma<TYPE, MODE>(hi, kw, rg, st);
}


template <int TYPE0, int TYPE1, int T, int KW, int RG>
int launch_mfma2_one(const GemvArgs& a0, const GemvArgs& a1, hipStream_t st) {
  constexpr int D = 3;
  if ((a0.K >> 8) < KW) return 4;
  const int lds = max(mfma_lds(TYPE0, T, a0.K, KW * RG, 1).total,
                      mfma_lds(TYPE1, T, a0.K, KW * RG, 1).total);
  if (lds > 160 * 1024) return 4;
  const int g0 = (a0.N + 16 * RG - 1) / (16 * RG), g1 = (a1.N + 16 * RG - 1) / (16 * RG);
  hipLaunchKernelGGL((qgemv2_mfma_kernel<TYPE0, TYPE1, T, KW, RG, D>), dim3(g0 + g1),
                     dim3(KW * RG * 64), lds, st, a0, a1, g0);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

template <int TYPE0, int TYPE1, int T>
int launch_mfma2(const GemvArgs& a0, const GemvArgs& a1, hipStream_t st) {
  if (a0.N % 16 || a1.N % 16) return 4;
  int kw = 0, rg = 0;
  mfma_shape(false, a0.N + a1.N, a0.K, kw, rg);
  switch (kw * 8 + rg) {
    case 1 * 8 + 4: return launch_mfma2_one<TYPE0, TYPE1, T, 1, 4>(a0, a1, st);
    case 2 * 8 + 2: return launch_mfma2_one<TYPE0, TYPE1, T, 2, 2>(a0, a1, st);
    case 4 * 8 + 1: return launch_mfma2_one<TYPE0, TYPE1, T, 4, 1>(a0, a1, st);
    default: return 4;
  }
}

template <int TYPE0, int TYPE1>
int dispatch_mfma2(const GemvArgs& a0, const GemvArgs& a1, hipStream_t st) {
  switch (a0.T) {
    case 1: return launch_mfma2<TYPE0, TYPE1, 1>(a0, a1, st);
    case 2: return launch_mfma2<TYPE0, TYPE1, 2>(a0, a1, st);
    case 3: return launch_mfma2<TYPE0, TYPE1, 3>(a0, a1, st);
    case 4: return launch_mfma2<TYPE0, TYPE1, 4>(a0, a1, st);
    case 5: return launch_mfma2<TYPE0, TYPE1, 5>(a0, a1, st);
    case 6: return launch_mfma2<TYPE0, TYPE1, 6>(a0, a1, st);
    case 7: return launch_mfma2<TYPE0, TYPE1, 7>(a0, a1, st);
    case 8: return launch_mfma2<TYPE0, TYPE1, 8>(a0, a1, st);
    default: return 2;
  }
}

}  // namespace

extern "C" {

int amdk8s_llm_max_tokens() { return kMaxTok; }
int amdk8s_llm_attn_chunk() { return kAttnChunk; }

// Quantised GEMV: out[t][n] (mode 0: = W.x + bias; 1: += W.x; 2: = silu(W0.x) * (W1.x)).
// x: Q8 (x8/dx/sx) or fp32 rows xf [T][ldx] with an optional fused RMSNorm (norm_w, eps).
// type 0 = Q4_K (w0q: GGUF rows), 1 = Q6_K (w0q/w0qh/w0sc/w0d planes).
int amdk8s_llm_qgemv(int type, int mode, const void* w0q, const void* w0qh, const void* w0sc,
                     const void* w0d, const void* w1q, const void* w1qh, const void* w1sc,
                     const void* w1d, const void* x8, const void* dx, const void* sx,
                     const void* xf, int ldx, const void* norm_w, float eps,
                     const void* bias, void* out, int ldo, int N, int K, int T, int waves,
                     int rows_per_wg, void* ox8, void* odx, void* osx, void* stream) {
  if (T > kValuMaxTok) return 4;                // more tokens: the MFMA GEMV only
  if (K % 256 || N <= 0 || T < 1) return 2;
  if (mode == kPair && !w1q) return 2;
  if (ox8) {                                  // pair → Q8 output: whole 32-row blocks per workgroup
    if (mode != kPair || N % 32 || !odx || !osx) return 2;
    rows_per_wg = 32;                         // 4 waves share them (8 and 2 measured slower)
  }
  gemv_shape(type, N, K, T, waves, rows_per_wg);
  if (ox8 && waves * 64 < 32 * T) return 2;
  if (waves < 1 || waves > 8 || rows_per_wg < 1) return 2;
  GemvArgs a{};                               // every field not set below stays null / 0
  a.w0 = {static_cast<const uint8_t*>(w0q), static_cast<const uint8_t*>(w0qh),
          static_cast<const int8_t*>(w0sc), static_cast<const uint16_t*>(w0d)};
  a.w1 = {static_cast<const uint8_t*>(w1q), static_cast<const uint8_t*>(w1qh),
          static_cast<const int8_t*>(w1sc), static_cast<const uint16_t*>(w1d)};
  a.x8 = static_cast<const int8_t*>(x8);
  a.dx = static_cast<const float*>(dx);
  a.sx = static_cast<const float*>(sx);
  a.xf = static_cast<const float*>(xf);
  a.ldx = ldx;
  a.norm_w = static_cast<const float*>(norm_w);
  a.eps = eps;
  if (!xf && !(x8 && dx && sx)) return 2;
  if (xf && ldx % 4) return 2;
  a.bias = static_cast<const float*>(bias);
  a.out = static_cast<float*>(out);
  a.ldo = ldo; a.N = N; a.K = K; a.T = T; a.rows_per_wg = rows_per_wg;
  a.ox8 = static_cast<int8_t*>(ox8);
  a.odx = static_cast<float*>(odx);
  a.osx = static_cast<float*>(osx);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type == kQ4K) {
    if (mode == kStore) return dispatch_t<kQ4K, kStore>(a, waves, st);
    if (mode == kResid) return dispatch_t<kQ4K, kResid>(a, waves, st);
    if (mode == kPair) return dispatch_t<kQ4K, kPair>(a, waves, st);
  } else if (type == kQ6K) {
    if (mode == kStore) return dispatch_t<kQ6K, kStore>(a, waves, st);
    if (mode == kResid) return dispatch_t<kQ6K, kResid>(a, waves, st);
    if (mode == kPair) return dispatch_t<kQ6K, kPair>(a, waves, st);
  }
  return 2;
}

// Quantised GEMV on the int8 matrix cores (qgemv_mfma_kernel) over the MFMA-packed planes (w*q /
// w*qh / w*sc / w*d from amdk8s_llm_mfma_pack; qh: Q6_K only); arguments otherwise as
// amdk8s_llm_qgemv.  kw / rows_per_wg: K-waves and rows (16 x row groups) per workgroup, 0 = the
// default shape.  4 = shape not covered (N % 16, fewer super-blocks than K-waves, LDS): use
// amdk8s_llm_qgemv on the plain planes.
int amdk8s_llm_qgemv_mfma(int type, int mode, const void* w0q, const void* w0qh, const void* w0sc,
                          const void* w0d, const void* w1q, const void* w1qh, const void* w1sc,
                          const void* w1d, const void* x8, const void* dx, const void* sx,
                          const void* xf, int ldx, const void* norm_w, float eps,
                          const void* bias, void* out, int ldo, int N, int K, int T, int kw,
                          int rows_per_wg, void* ox8, void* odx, void* osx, void* stream) {
  if (K % 256 || N <= 0 || T < 1 || T > kMaxTok) return 2;
  if (type != kQ4K && type != kQ6K) return 2;
  if (mode == kPair && !w1q) return 2;
  if (!xf && !(x8 && dx && sx)) return 2;
  if (xf && (ldx % 4 || T > kValuMaxTok)) return 2;  // fp32-row prologue: steps of <= 4 tokens
  if (ox8 && (mode != kPair || N % 32 || !odx || !osx)) return 2;
  GemvArgs a{};
  a.w0 = {static_cast<const uint8_t*>(w0q), static_cast<const uint8_t*>(w0qh),
          static_cast<const int8_t*>(w0sc), static_cast<const uint16_t*>(w0d)};
  a.w1 = {static_cast<const uint8_t*>(w1q), static_cast<const uint8_t*>(w1qh),
          static_cast<const int8_t*>(w1sc), static_cast<const uint16_t*>(w1d)};
  a.x8 = static_cast<const int8_t*>(x8);
  a.dx = static_cast<const float*>(dx);
  a.sx = static_cast<const float*>(sx);
  a.xf = static_cast<const float*>(xf);
  a.ldx = ldx;
  a.norm_w = static_cast<const float*>(norm_w);
  a.eps = eps;
  a.bias = static_cast<const float*>(bias);
  a.out = static_cast<float*>(out);
  a.ldo = ldo; a.N = N; a.K = K; a.T = T; a.rows_per_wg = 0;
  a.ox8 = static_cast<int8_t*>(ox8);
  a.odx = static_cast<float*>(odx);
  a.osx = static_cast<float*>(osx);
  const int rg = ox8 ? 2 : (rows_per_wg > 0 && rows_per_wg % 16 == 0 ? rows_per_wg / 16 : 0);
  if (rg == 0) kw = 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type == kQ4K) {
    if (mode == kStore) return dispatch_mfma_split<kQ4K, kStore>(a, kw, rg, st);
    if (mode == kResid) return dispatch_mfma_split<kQ4K, kResid>(a, kw, rg, st);
    if (mode == kPair) return dispatch_mfma_split<kQ4K, kPair>(a, kw, rg, st);
  } else {
    if (mode == kStore) return dispatch_mfma_split<kQ6K, kStore>(a, kw, rg, st);
    if (mode == kResid) return dispatch_mfma_split<kQ6K, kResid>(a, kw, rg, st);
    if (mode == kPair) return dispatch_mfma_split<kQ6K, kPair>(a, kw, rg, st);
  }
  return 2;
}

// Repacked planes (amdk8s_llm_q4k_repack / q6k_repack layout) → the MFMA-packed copy: mq
// [N*nb*128] bytes, mqh [N*nb*64] bytes (Q6_K), msc [N*nb*16] bytes, md [N*nb] dwords.  N % 16 == 0.
int amdk8s_llm_mfma_pack(int type, const void* q, const void* qh, const void* sc, const void* d,
                         int N, int nb, void* mq, void* mqh, void* msc, void* md, void* stream) {
  if (N <= 0 || N % 16 || nb <= 0 || (type != kQ4K && type != kQ6K)) return 2;
  if (type == kQ6K && !(qh && mqh)) return 2;
  const QMat w = {static_cast<const uint8_t*>(q), static_cast<const uint8_t*>(qh),
                  static_cast<const int8_t*>(sc), static_cast<const uint16_t*>(d)};
  const long n = (long)N * nb;
  const dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type == kQ4K)
    hipLaunchKernelGGL(mfma_pack_kernel<kQ4K>, grid, dim3(256), 0, st, w, N, nb,
                       static_cast<uint8_t*>(mq), nullptr, static_cast<uint8_t*>(msc),
                       static_cast<uint32_t*>(md));
  else
    hipLaunchKernelGGL(mfma_pack_kernel<kQ6K>, grid, dim3(256), 0, st, w, N, nb,
                       static_cast<uint8_t*>(mq), static_cast<uint8_t*>(mqh),
                       static_cast<uint8_t*>(msc), static_cast<uint32_t*>(md));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// amdk8s_llm_qgemv2 on the int8 matrix cores over the MFMA-packed planes (q|k and v of different
// quantisation types in one launch, up to 8 tokens).  4 = not covered (same types, N % 16, LDS):
// launch the matrices with amdk8s_llm_qgemv_mfma.
int amdk8s_llm_qgemv2_mfma(int type0, const void* w0q, const void* w0qh, const void* w0sc,
                           const void* w0d, int N0, const void* bias0, void* out0, int type1,
                           const void* w1q, const void* w1qh, const void* w1sc, const void* w1d,
                           int N1, const void* bias1, void* out1, int ldo, const void* x8,
                           const void* dx, const void* sx, const void* xf, int ldx,
                           const void* norm_w, float eps, int K, int T, void* stream) {
  if (K % 256 || N0 <= 0 || N1 <= 0 || T < 1 || T > kMaxTok) return 2;
  if (!xf && !(x8 && dx && sx)) return 2;
  if (xf && (ldx % 4 || T > kValuMaxTok)) return 2;
  if (type0 == type1 || (type0 != kQ4K && type0 != kQ6K) || (type1 != kQ4K && type1 != kQ6K))
    return 4;
  GemvArgs a[2];
  const int N[2] = {N0, N1};
  const void* q[2][4] = {{w0q, w0qh, w0sc, w0d}, {w1q, w1qh, w1sc, w1d}};
  const void* bias[2] = {bias0, bias1};
  void* out[2] = {out0, out1};
  for (int i = 0; i < 2; ++i) {
    GemvArgs& g = a[i];
    g = GemvArgs{};
    g.w0 = {static_cast<const uint8_t*>(q[i][0]), static_cast<const uint8_t*>(q[i][1]),
            static_cast<const int8_t*>(q[i][2]), static_cast<const uint16_t*>(q[i][3])};
    g.x8 = static_cast<const int8_t*>(x8);
    g.dx = static_cast<const float*>(dx);
    g.sx = static_cast<const float*>(sx);
    g.xf = static_cast<const float*>(xf);
    g.ldx = ldx;
    g.norm_w = static_cast<const float*>(norm_w);
    g.eps = eps;
    g.bias = static_cast<const float*>(bias[i]);
    g.out = static_cast<float*>(out[i]);
    g.ldo = ldo; g.N = N[i]; g.K = K; g.T = T; g.rows_per_wg = 0;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type0 == kQ4K) return dispatch_mfma2<kQ4K, kQ6K>(a[0], a[1], st);
  return dispatch_mfma2<kQ6K, kQ4K>(a[0], a[1], st);
}

// Two store-mode GEMVs over the same input in one launch: out_i[t][n] = W_i.x + bias_i (the
// q|k and v projections when their quantisation types differ); Q8 input, or fp32 rows xf
// (+ RMSNorm norm_w) quantised in each workgroup's prologue.  Returns 4 when the shape is not
// covered (K > 4096): launch the two with amdk8s_llm_qgemv instead.
int amdk8s_llm_qgemv2(int type0, const void* w0q, const void* w0qh, const void* w0sc,
                      const void* w0d, int N0, const void* bias0, void* out0, int type1,
                      const void* w1q, const void* w1qh, const void* w1sc, const void* w1d, int N1,
                      const void* bias1, void* out1, int ldo, const void* x8, const void* dx,
                      const void* sx, const void* xf, int ldx, const void* norm_w, float eps,
                      int K, int T, int waves, int rows_per_wg, void* stream) {
  if (T > kValuMaxTok) return 4;
  if (K % 256 || N0 <= 0 || N1 <= 0 || T < 1) return 2;
  if (!xf && !(x8 && dx && sx)) return 2;
  if (xf && ldx % 4) return 2;
  if ((type0 != kQ4K && type0 != kQ6K) || (type1 != kQ4K && type1 != kQ6K)) return 2;
  int rows = rows_per_wg;
  gemv_shape(type0, N0 + N1, K, T, waves, rows);
  if (waves < 1 || waves > 8 || rows < 1) return 2;
  GemvArgs a[2];
  const int N[2] = {N0, N1};
  const void* q[2][4] = {{w0q, w0qh, w0sc, w0d}, {w1q, w1qh, w1sc, w1d}};
  const void* bias[2] = {bias0, bias1};
  void* out[2] = {out0, out1};
  for (int i = 0; i < 2; ++i) {
    GemvArgs& g = a[i];
    g = GemvArgs{};
    g.w0 = {static_cast<const uint8_t*>(q[i][0]), static_cast<const uint8_t*>(q[i][1]),
            static_cast<const int8_t*>(q[i][2]), static_cast<const uint16_t*>(q[i][3])};
    g.x8 = static_cast<const int8_t*>(x8);
    g.dx = static_cast<const float*>(dx);
    g.sx = static_cast<const float*>(sx);
    g.xf = static_cast<const float*>(xf);
    g.ldx = ldx;
    g.norm_w = static_cast<const float*>(norm_w);
    g.eps = eps;
    g.bias = static_cast<const float*>(bias[i]);
    g.out = static_cast<float*>(out[i]);
    g.ldo = ldo; g.N = N[i]; g.K = K; g.T = T; g.rows_per_wg = rows;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type0 == kQ4K && type1 == kQ6K) return dispatch2_t<kQ4K, kQ6K>(a[0], a[1], waves, st);
  if (type0 == kQ6K && type1 == kQ4K) return dispatch2_t<kQ6K, kQ4K>(a[0], a[1], waves, st);
  if (type0 == kQ4K) return dispatch2_t<kQ4K, kQ4K>(a[0], a[1], waves, st);
  return dispatch2_t<kQ6K, kQ6K>(a[0], a[1], waves, st);
}

int amdk8s_llm_argmax_rows(const void* x, int V, long ld, int T, void* out, void* stream) {
  if (V < 1 || T < 1 || ld < V || ((uintptr_t)x & 15) || (ld & 3)) return 2;
  hipLaunchKernelGGL(argmax_rows_kernel, dim3(T), dim3(1024), 0, static_cast<hipStream_t>(stream),
                     static_cast<const float*>(x), V, ld, static_cast<int*>(out));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int amdk8s_llm_rmsnorm_q8(const void* x, const void* w, float eps, int K, int T, void* x8,
                          void* dx, void* sx, void* stream) {
  if (K % 256 || T < 1) return 2;
  hipLaunchKernelGGL(rmsnorm_q8_kernel, dim3((K + 2047) / 2048, T), dim3(256), 0,
                     static_cast<hipStream_t>(stream),
                     static_cast<const float*>(x), static_cast<const float*>(w), eps, K,
                     static_cast<int8_t*>(x8), static_cast<float*>(dx), static_cast<float*>(sx));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int amdk8s_llm_rope_kv(const void* qkv, int ldq, const void* pos, const void* slot,
                       const void* cos_t, const void* sin_t, int H, int Hkv, int head_dim,
                       int max_ctx, void* q_out, void* kc, void* vc, int T, void* stream) {
  if (head_dim != kHeadDim || T < 1) return 2;
  const int threads = (H + 2 * Hkv) * (kHeadDim / 2);
  hipLaunchKernelGGL(rope_kv_kernel, dim3((threads + 255) / 256, T), dim3(256), 0,
                     static_cast<hipStream_t>(stream),
                     static_cast<const float*>(qkv), ldq, static_cast<const int*>(pos),
                     static_cast<const int*>(slot), static_cast<const float*>(cos_t),
                     static_cast<const float*>(sin_t), H, Hkv, max_ctx,
                     static_cast<float*>(q_out), static_cast<uint16_t*>(kc),
                     static_cast<uint16_t*>(vc));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Decode attention over the KV cache + combine + Q8 quantisation of the output.
// po/pml: workspace [T][H][nsplit][128] / [T][H][nsplit][2]; out (nullable) fp32 [T][H*128].
// span: positions covered by this launch (a multiple of 64, <= max_ctx, > every pos[t]); the
// caller buckets it so a captured graph does not launch empty chunks up to max_ctx.
// qkv (nullable): the raw q|k|v projection [T][ldq] — fused RoPE + KV write (distinct slots
// only, see attn_decode_kernel); q is then unused.
int amdk8s_llm_attn_decode(const void* q, const void* qkv, int ldq, const void* cos_t,
                           const void* sin_t, const void* pos, const void* slot, void* kc,
                           void* vc, int H, int Hkv, int head_dim, int max_ctx, int span,
                           float scale, void* po, void* pml, void* out, void* x8, void* dx,
                           void* sx, int T, void* stream) {
  if (span <= 0) span = max_ctx;
  if (head_dim != kHeadDim || H % Hkv || H / Hkv > kMaxGroup || max_ctx % kAttnChunk ||
      span % kAttnChunk || span > max_ctx || T < 1)
    return 2;
  if (!qkv && !q) return 2;
  if (qkv && (!cos_t || !sin_t)) return 2;
  if (!(x8 && dx && sx)) return 2;
  hipStream_t st = static_cast<hipStream_t>(stream);
  AttnArgs aa{};
  aa.q = static_cast<const float*>(q);
  aa.qkv = static_cast<const float*>(qkv);
  aa.ldq = ldq;
  aa.cos_t = static_cast<const float*>(cos_t);
  aa.sin_t = static_cast<const float*>(sin_t);
  aa.pos = static_cast<const int*>(pos);
  aa.slot = static_cast<const int*>(slot);
  aa.kc = static_cast<uint16_t*>(kc);
  aa.vc = static_cast<uint16_t*>(vc);
  aa.H = H; aa.Hkv = Hkv; aa.max_ctx = max_ctx; aa.scale = scale;
  aa.po = static_cast<float*>(po);
  aa.pml = static_cast<float*>(pml);
  // the GQA group size is a template parameter: fully unrolled head loops, no per-head branches
  auto by_group = [&](auto launch) -> int {
    switch (H / Hkv) {
      case 1: launch(std::integral_constant<int, 1>{}); break;
      case 2: launch(std::integral_constant<int, 2>{}); break;
      case 3: launch(std::integral_constant<int, 3>{}); break;
      case 4: launch(std::integral_constant<int, 4>{}); break;
      case 5: launch(std::integral_constant<int, 5>{}); break;
      case 6: launch(std::integral_constant<int, 6>{}); break;
      case 7: launch(std::integral_constant<int, 7>{}); break;
      case 8: launch(std::integral_constant<int, 8>{}); break;
      default: return 2;
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
  };
  aa.nsplit = span / kAttnChunk;
  const int rc = by_group([&](auto g) {
    hipLaunchKernelGGL(attn_decode_kernel<decltype(g)::value>, dim3(Hkv, aa.nsplit, T), dim3(256), 0,
                       st, aa);
  });
  if (rc) return rc;
  hipLaunchKernelGGL(attn_combine_q8_kernel, dim3(H, T), dim3(128), 0, st,
                     static_cast<const float*>(po), static_cast<const float*>(pml),
                     static_cast<const int*>(pos), H, aa.nsplit, kAttnChunk, static_cast<float*>(out),
                     static_cast<int8_t*>(x8), static_cast<float*>(dx), static_cast<float*>(sx));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Dequantise rows (all, or the listed ones) of a Q4_K / Q6_K matrix to fp16 (f32out=0) or fp32.
int amdk8s_llm_dequant(int type, const void* q, const void* qh, const void* sc, const void* d,
                       const void* rows, int nrows, int K, void* out, int f32out, void* stream) {
  if (K % 256 || nrows < 1) return 2;
  QMat w = {static_cast<const uint8_t*>(q), static_cast<const uint8_t*>(qh),
            static_cast<const int8_t*>(sc), static_cast<const uint16_t*>(d)};
  const long runs = (long)nrows * (K >> 5);
  const int grid = (int)((runs + 255) / 256 < 65536 ? (runs + 255) / 256 : 65536);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int* r = static_cast<const int*>(rows);
  if (type == kQ4K && f32out)
    hipLaunchKernelGGL((dequant_kernel<kQ4K, true>), dim3(grid), dim3(256), 0, st, w, r, nrows, K, out);
  else if (type == kQ4K)
    hipLaunchKernelGGL((dequant_kernel<kQ4K, false>), dim3(grid), dim3(256), 0, st, w, r, nrows, K, out);
  else if (type == kQ6K && f32out)
    hipLaunchKernelGGL((dequant_kernel<kQ6K, true>), dim3(grid), dim3(256), 0, st, w, r, nrows, K, out);
  else if (type == kQ6K)
    hipLaunchKernelGGL((dequant_kernel<kQ6K, false>), dim3(grid), dim3(256), 0, st, w, r, nrows, K, out);
  else
    return 2;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int amdk8s_llm_q4k_repack(const void* src, long nblocks, void* qs, void* scm, void* dm,
                          void* stream) {
  if (nblocks < 1) return 2;
  const int grid = (int)((nblocks + 255) / 256 < 65536 ? (nblocks + 255) / 256 : 65536);
  hipLaunchKernelGGL(q4k_repack_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(src), nblocks, static_cast<uint8_t*>(qs),
                     static_cast<uint32_t*>(scm), static_cast<uint32_t*>(dm));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int amdk8s_llm_q6k_repack(const void* src, long nblocks, void* ql, void* qh, void* sc, void* d,
                          void* stream) {
  if (nblocks < 1) return 2;
  const int grid = (int)((nblocks + 255) / 256 < 65536 ? (nblocks + 255) / 256 : 65536);
  hipLaunchKernelGGL(q6k_repack_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(src), nblocks, static_cast<uint8_t*>(ql),
                     static_cast<uint8_t*>(qh), static_cast<int8_t*>(sc),
                     static_cast<uint16_t*>(d));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}


}  // extern "C"
