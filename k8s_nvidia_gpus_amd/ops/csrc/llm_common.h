// Shared definitions of the LLM decode kernels (llm_decode.hip: VALU GEMVs, attention, norms;
// llm_gemv_mfma.hip: the int8-MFMA GEMVs): constants, weight-plane and argument structs, the
// cross-lane reductions and the activation staging / Q8 epilogue both GEMV families use.
#pragma once
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
  int temporal = 0;      // MFMA GEMV: default-policy weight loads (a second launch re-reads them)
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
  // split-K over workgroups (MFMA GEMV, Q8 input, store / resid modes): ksplit slices of the
  // super-blocks per row tile; each slice publishes its partials to kpart (write-through), the
  // last to arrive on kcnt[tile] sums them in slice order and writes the output
  int ksplit;
  float* kpart;          // [tiles][ksplit][row groups][token quads][64]
  unsigned* kcnt;        // [tiles], zero between launches (the last arriver resets its word)
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

}  // namespace
