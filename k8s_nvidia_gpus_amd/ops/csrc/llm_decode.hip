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
constexpr int kMaxTok = 4;          // tokens per GEMV launch (activations staged in LDS)
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
  } else {
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
  const XView xv = {xs, dxs, sxs, xstride, K >> 5, K >> 4};

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
    if (q8s) {       // quantise the 32-row block per token: half a wave per token (lane & 31 = row)
      __syncthreads();
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
  if (K % 256 || N <= 0 || T < 1 || T > kMaxTok) return 2;
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
  if (K % 256 || N0 <= 0 || N1 <= 0 || T < 1 || T > kMaxTok) return 2;
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
