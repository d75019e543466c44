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
//   wave-wide 16-byte load reads 8 consecutive super-blocks (1 KiB of quants) fully coalesced.
//   Q4_K rows keep the GGUF block layout (144 B, 16-byte aligned); Q6_K (210 B, unaligned) is
//   repacked at load time into four planes (ql / qh / scales / d) so every load is aligned.
// * The activations of the (<= 4) tokens are staged once per workgroup in LDS (x8 padded 32 B per
//   256 so the 16-lane groups of a ds_read_b128 hit disjoint banks); every wave of the workgroup
//   then streams its rows against them.
// * Epilogues are fused: bias add (q/k/v), residual add in place (o_proj, ffn_down), and the SwiGLU
//   pair mode that runs ffn_gate and ffn_up rows in the same wave and writes silu(g)*u.
// * Decode attention is split over the context (flash-decoding): per (kv head, 256-position chunk,
//   token) one workgroup scores all q heads of the GQA group, and the combine kernel merges the
//   chunks and emits the Q8 activations of the o_proj input directly.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kWave = 64;
constexpr int kQ4KBytes = 144;
constexpr int kMaxTok = 4;          // tokens per GEMV launch (activations staged in LDS)
constexpr int kAttnChunk = 256;     // context positions per decode-attention workgroup
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

__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
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

struct QMat {            // one quantised weight matrix [N, K]
  const uint8_t* q;      // Q4_K: rows of nb*144 B;  Q6_K: ql plane [N][nb][128]
  const uint8_t* qh;     // Q6_K: [N][nb][64]
  const int8_t* sc;      // Q6_K: [N][nb][16]
  const uint16_t* d;     // Q6_K: [N][nb]
};

struct GemvArgs {
  QMat w0, w1;           // w1: ffn_up in pair mode
  const int8_t* x8;      // [T][K]
  const float* dx;       // [T][K/32]
  const float* sx;       // [T][K/16]  (dx * sum of the 16 int8 values)
  const float* bias;     // [N] or null (store mode)
  float* out;            // [T][ldo]
  int ldo, N, K, T, rows_per_wg;
};

// Partial dot products of one lane for one 256-weight super-block of a Q4_K row.
template <int T>
__device__ __forceinline__ void q4k_block(const uint8_t* __restrict__ row, int blk, int sub,
                                          const int8_t* xs, const float* dxs, const float* sxs,
                                          int xstride, int dstride, int sstride, float* acc) {
  const uint8_t* b = row + (long)blk * kQ4KBytes;
  const uint4 hdr = *reinterpret_cast<const uint4*>(b);
  const uint4 qv = *reinterpret_cast<const uint4*>(b + 16 + sub * 16);
  const int c = sub >> 1;                 // 64-weight chunk: sub-blocks 2c (low) and 2c+1 (high)
  const float d = h2f(hdr.x & 0xffffu), dmin = h2f(hdr.x >> 16);
  const uint32_t s[3] = {hdr.y, hdr.z, hdr.w};
  auto sbyte = [&](int i) -> uint32_t { return (s[i >> 2] >> ((i & 3) * 8)) & 0xffu; };
  const int j0 = 2 * c, j1 = 2 * c + 1;
  uint32_t sc0, m0, sc1, m1;
  if (c < 2) {
    sc0 = sbyte(j0) & 63; m0 = sbyte(j0 + 4) & 63;
    sc1 = sbyte(j1) & 63; m1 = sbyte(j1 + 4) & 63;
  } else {
    sc0 = (sbyte(j0 + 4) & 0xf) | ((sbyte(j0 - 4) >> 6) << 4);
    m0 = (sbyte(j0 + 4) >> 4) | ((sbyte(j0) >> 6) << 4);
    sc1 = (sbyte(j1 + 4) & 0xf) | ((sbyte(j1 - 4) >> 6) << 4);
    m1 = (sbyte(j1 + 4) >> 4) | ((sbyte(j1) >> 6) << 4);
  }
  const uint32_t q[4] = {qv.x, qv.y, qv.z, qv.w};
  const int p_lo = blk * 256 + c * 64 + (sub & 1) * 16;    // weight index of this lane's low run
  const int g_lo = p_lo >> 4;                                // 16-group
  const int d_lo = p_lo >> 5;                                // 32-block
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const uint4 xl = *reinterpret_cast<const uint4*>(xs + t * xstride + xoff(p_lo));
    const uint4 xh = *reinterpret_cast<const uint4*>(xs + t * xstride + xoff(p_lo + 32));
    int il = 0, ih = 0;
    il = dot4(q[0] & 0x0f0f0f0fu, xl.x, il);
    il = dot4(q[1] & 0x0f0f0f0fu, xl.y, il);
    il = dot4(q[2] & 0x0f0f0f0fu, xl.z, il);
    il = dot4(q[3] & 0x0f0f0f0fu, xl.w, il);
    ih = dot4((q[0] >> 4) & 0x0f0f0f0fu, xh.x, ih);
    ih = dot4((q[1] >> 4) & 0x0f0f0f0fu, xh.y, ih);
    ih = dot4((q[2] >> 4) & 0x0f0f0f0fu, xh.z, ih);
    ih = dot4((q[3] >> 4) & 0x0f0f0f0fu, xh.w, ih);
    const float dxl = dxs[t * dstride + d_lo], dxh = dxs[t * dstride + d_lo + 1];
    const float sxl = sxs[t * sstride + g_lo], sxh = sxs[t * sstride + g_lo + 2];
    acc[t] += d * ((float)sc0 * dxl * (float)il + (float)sc1 * dxh * (float)ih)
              - dmin * ((float)m0 * sxl + (float)m1 * sxh);
  }
}

template <int T>
__device__ __forceinline__ void q6k_block(const QMat& w, long rowblk, int blk, int sub,
                                          const int8_t* xs, const float* dxs, const float* sxs,
                                          int xstride, int dstride, int sstride, float* acc) {
  const long rb = rowblk + blk;                       // (row * nb + blk)
  const int n = sub >> 2, h1 = sub & 1, klo = (sub & 3) >> 1;
  const uint4 ql = *reinterpret_cast<const uint4*>(w.q + rb * 128 + sub * 16);
  const uint4 qh = *reinterpret_cast<const uint4*>(w.qh + rb * 64 + n * 32 + h1 * 16);
  const uint4 scv = *reinterpret_cast<const uint4*>(w.sc + rb * 16);
  const float d = h2f(w.d[rb]);
  const uint32_t scw[4] = {scv.x, scv.y, scv.z, scv.w};
  const int i0 = 8 * n + h1 + 2 * klo, i1 = i0 + 4;
  const float sc0 = (float)(int8_t)((scw[i0 >> 2] >> ((i0 & 3) * 8)) & 0xffu);
  const float sc1 = (float)(int8_t)((scw[i1 >> 2] >> ((i1 & 3) * 8)) & 0xffu);
  const uint32_t l[4] = {ql.x, ql.y, ql.z, ql.w};
  const uint32_t hb[4] = {qh.x, qh.y, qh.z, qh.w};
  const int sh = 2 * klo;
  uint32_t qlo[4], qhi[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    qlo[i] = (l[i] & 0x0f0f0f0fu) | (((hb[i] >> sh) & 0x03030303u) << 4);
    qhi[i] = ((l[i] >> 4) & 0x0f0f0f0fu) | (((hb[i] >> (sh + 4)) & 0x03030303u) << 4);
  }
  const int p_lo = blk * 256 + n * 128 + klo * 32 + h1 * 16;
  const int g_lo = p_lo >> 4, d_lo = p_lo >> 5;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const uint4 xl = *reinterpret_cast<const uint4*>(xs + t * xstride + xoff(p_lo));
    const uint4 xh = *reinterpret_cast<const uint4*>(xs + t * xstride + xoff(p_lo + 64));
    int il = 0, ih = 0;
    il = dot4(qlo[0], xl.x, il); il = dot4(qlo[1], xl.y, il);
    il = dot4(qlo[2], xl.z, il); il = dot4(qlo[3], xl.w, il);
    ih = dot4(qhi[0], xh.x, ih); ih = dot4(qhi[1], xh.y, ih);
    ih = dot4(qhi[2], xh.z, ih); ih = dot4(qhi[3], xh.w, ih);
    const float dxl = dxs[t * dstride + d_lo], dxh = dxs[t * dstride + d_lo + 2];
    const float sxl = sxs[t * sstride + g_lo], sxh = sxs[t * sstride + g_lo + 4];
    acc[t] += d * (sc0 * (dxl * (float)il - 32.f * sxl) + sc1 * (dxh * (float)ih - 32.f * sxh));
  }
}

template <int TYPE, int T>
__device__ __forceinline__ void row_dot(const QMat& w, int row, int nb, int lane,
                                        const int8_t* xs, const float* dxs, const float* sxs,
                                        int xstride, int dstride, int sstride, float* acc) {
  const int sub = lane & 7;
  const int bl = lane >> 3;
  if constexpr (TYPE == kQ4K) {
    const uint8_t* r = w.q + (long)row * nb * kQ4KBytes;
#pragma unroll 2
    for (int b0 = 0; b0 < nb; b0 += 8) {
      const int blk = b0 + bl;
      if (blk < nb) q4k_block<T>(r, blk, sub, xs, dxs, sxs, xstride, dstride, sstride, acc);
    }
  } else {
    const long rowblk = (long)row * nb;
#pragma unroll 2
    for (int b0 = 0; b0 < nb; b0 += 8) {
      const int blk = b0 + bl;
      if (blk < nb) q6k_block<T>(w, rowblk, blk, sub, xs, dxs, sxs, xstride, dstride, sstride, acc);
    }
  }
}

template <int TYPE, int T, int MODE>
__global__ void __launch_bounds__(256) qgemv_kernel(GemvArgs a) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int K = a.K, nb = K >> 8;
  const int xstride = nb * 288;                      // padded bytes per token
  int8_t* xs = reinterpret_cast<int8_t*>(lds);
  float* dxs = reinterpret_cast<float*>(lds + T * xstride);
  float* sxs = dxs + T * (K >> 5);
  // ---- stage the T tokens' activations (16-byte vectors) ----
  for (int i = threadIdx.x; i < T * (K >> 4); i += blockDim.x) {
    const int t = i / (K >> 4), p = (i - t * (K >> 4)) << 4;
    *reinterpret_cast<uint4*>(xs + t * xstride + xoff(p)) =
        *reinterpret_cast<const uint4*>(a.x8 + (long)t * K + p);
  }
  for (int i = threadIdx.x; i < T * (K >> 5); i += blockDim.x) dxs[i] = a.dx[i];
  for (int i = threadIdx.x; i < T * (K >> 4); i += blockDim.x) sxs[i] = a.sx[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int r0 = blockIdx.x * a.rows_per_wg;
  const int r1 = min(a.N, r0 + a.rows_per_wg);
  for (int row = r0 + wave; row < r1; row += nw) {
    float acc[T], acc1[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = acc1[t] = 0.f;
    row_dot<TYPE, T>(a.w0, row, nb, lane, xs, dxs, sxs, xstride, K >> 5, K >> 4, acc);
    if constexpr (MODE == kPair)
      row_dot<TYPE, T>(a.w1, row, nb, lane, xs, dxs, sxs, xstride, K >> 5, K >> 4, acc1);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      acc[t] = wave_sum(acc[t]);
      if constexpr (MODE == kPair) acc1[t] = wave_sum(acc1[t]);
    }
    if (lane < T) {
      float v = 0.f, v1 = 0.f;
#pragma unroll
      for (int t = 0; t < T; ++t)
        if (t == lane) { v = acc[t]; v1 = acc1[t]; }
      float* o = a.out + (long)lane * a.ldo + row;
      if constexpr (MODE == kStore) *o = v + (a.bias ? a.bias[row] : 0.f);
      else if constexpr (MODE == kResid) *o += v;
      else *o = v / (1.f + __expf(-v)) * v1;
    }
  }
}

// ---------------------------------------------------------------- RMSNorm + Q8 activation quant
// One workgroup per token.  x fp32 [T][K]; w fp32 [K] or null (quantise only).
__global__ void __launch_bounds__(256) rmsnorm_q8_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ w, float eps,
                                                         int K, int8_t* __restrict__ x8,
                                                         float* __restrict__ dx,
                                                         float* __restrict__ sx) {
  __shared__ float red[4];
  const int t = blockIdx.x;
  const float* xr = x + (long)t * K;
  float rs = 1.f;
  if (w) {
    float ss = 0.f;
    for (int i = threadIdx.x * 4; i < K; i += blockDim.x * 4) {
      const float4 v = *reinterpret_cast<const float4*>(xr + i);
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    ss = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) ss += red[i];
    rs = rsqrtf(ss / (float)K + eps);
  }
  for (int blk = threadIdx.x; blk < (K >> 5); blk += blockDim.x) {
    float v[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 a = *reinterpret_cast<const float4*>(xr + blk * 32 + i * 4);
      v[4 * i] = a.x; v[4 * i + 1] = a.y; v[4 * i + 2] = a.z; v[4 * i + 3] = a.w;
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      v[i] *= rs * (w ? w[blk * 32 + i] : 1.f);
      amax = fmaxf(amax, fabsf(v[i]));
    }
    const float d = amax / 127.f;
    const float id = d > 0.f ? 1.f / d : 0.f;
    uint32_t pk[8];
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = (int)__builtin_rintf(v[4 * i + j] * id);
        word |= ((uint32_t)(q & 0xff)) << (8 * j);
        if (i < 4) s0 += q; else s1 += q;
      }
      pk[i] = word;
    }
    int8_t* o = x8 + (long)t * K + blk * 32;
    reinterpret_cast<uint4*>(o)[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    reinterpret_cast<uint4*>(o)[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
    dx[(long)t * (K >> 5) + blk] = d;
    sx[(long)t * (K >> 4) + 2 * blk] = d * (float)s0;
    sx[(long)t * (K >> 4) + 2 * blk + 1] = d * (float)s1;
  }
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
  const int t = blockIdx.x;
  const int p = pos[t], s = slot[t];
  const float* row = qkv + (long)t * ldq;
  const float* ct = cos_t + (long)p * (kHeadDim / 2);
  const float* st = sin_t + (long)p * (kHeadDim / 2);
  const int pairs = (H + Hkv) * (kHeadDim / 2);
  for (int i = threadIdx.x; i < pairs; i += blockDim.x) {
    const int h = i / (kHeadDim / 2), j = i % (kHeadDim / 2);
    const float x0 = row[h * kHeadDim + j], x1 = row[h * kHeadDim + j + kHeadDim / 2];
    const float c = ct[j], sn = st[j];
    const float y0 = x0 * c - x1 * sn, y1 = x0 * sn + x1 * c;
    if (h < H) {
      q_out[(long)t * H * kHeadDim + h * kHeadDim + j] = y0;
      q_out[(long)t * H * kHeadDim + h * kHeadDim + j + kHeadDim / 2] = y1;
    } else {
      const long base = (((long)s * Hkv + (h - H)) * max_ctx + p) * kHeadDim;
      kc[base + j] = f2h(y0);
      kc[base + j + kHeadDim / 2] = f2h(y1);
    }
  }
  const float* vrow = row + (H + Hkv) * kHeadDim;
  for (int i = threadIdx.x; i < Hkv * kHeadDim; i += blockDim.x) {
    const int h = i / kHeadDim, j = i % kHeadDim;
    vc[(((long)s * Hkv + h) * max_ctx + p) * kHeadDim + j] = f2h(vrow[i]);
  }
}

// ---------------------------------------------------------------- split-context decode attention
// grid (Hkv, nsplit, T); 256 threads.  Each workgroup: the G = H/Hkv q heads of one kv head over
// positions [s*256, min(s*256+256, len)).  Writes unnormalised partial outputs + (max, sum).
__global__ void __launch_bounds__(256) attn_decode_kernel(const float* __restrict__ q,
                                                          const int* __restrict__ pos,
                                                          const int* __restrict__ slot,
                                                          const uint16_t* __restrict__ kc,
                                                          const uint16_t* __restrict__ vc,
                                                          int H, int Hkv, int max_ctx, int nsplit,
                                                          float scale, float* __restrict__ po,
                                                          float* __restrict__ pml) {
  __shared__ float qs[kMaxGroup][kHeadDim];
  __shared__ float ps[kMaxGroup][kAttnChunk];
  __shared__ float red[kMaxGroup][4];
  __shared__ float opart[4][kMaxGroup][kHeadDim];
  const int kh = blockIdx.x, sp = blockIdx.y, t = blockIdx.z;
  const int G = H / Hkv;
  const int len = pos[t] + 1;
  const int p0 = sp * kAttnChunk;
  const long pidx = ((long)t * H + kh * G) * nsplit + sp;   // + g * nsplit
  if (p0 >= len) {
    if (threadIdx.x < G) {
      pml[(pidx + (long)threadIdx.x * nsplit) * 2] = -INFINITY;
      pml[(pidx + (long)threadIdx.x * nsplit) * 2 + 1] = 0.f;
    }
    return;
  }
  const int n = min(kAttnChunk, len - p0);
  for (int i = threadIdx.x; i < G * kHeadDim; i += blockDim.x)
    qs[i / kHeadDim][i % kHeadDim] = q[(long)t * H * kHeadDim + (kh * G) * kHeadDim + i] * scale;
  __syncthreads();
  const long cbase = ((long)slot[t] * Hkv + kh) * max_ctx * kHeadDim;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // scores: one position per thread
  float sc[kMaxGroup];
  const int pi = threadIdx.x;
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) sc[g] = -INFINITY;
  if (pi < n) {
#pragma unroll
    for (int g = 0; g < kMaxGroup; ++g) sc[g] = 0.f;
    const uint4* kr = reinterpret_cast<const uint4*>(kc + cbase + (long)(p0 + pi) * kHeadDim);
#pragma unroll 4
    for (int c = 0; c < kHeadDim / 8; ++c) {
      const uint4 kv = kr[c];
      const uint32_t kw[4] = {kv.x, kv.y, kv.z, kv.w};
      float kf[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        kf[2 * e] = h2f(kw[e] & 0xffffu);
        kf[2 * e + 1] = h2f(kw[e] >> 16);
      }
#pragma unroll
      for (int g = 0; g < kMaxGroup; ++g) {
        if (g < G) {
#pragma unroll
          for (int e = 0; e < 8; ++e) sc[g] += kf[e] * qs[g][c * 8 + e];
        }
      }
    }
  }
  // row max / sum over the chunk, per head
  float mx[kMaxGroup];
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) {
    const float m = wave_max(sc[g]);
    if (lane == 0) red[g][wave] = m;
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g)
    mx[g] = fmaxf(fmaxf(red[g][0], red[g][1]), fmaxf(red[g][2], red[g][3]));
  __syncthreads();
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) {
    const float p = (pi < n && g < G) ? __expf(sc[g] - mx[g]) : 0.f;
    ps[g][pi] = p;
    const float s = wave_sum(p);
    if (lane == 0) red[g][wave] = s;
  }
  __syncthreads();
  // P.V: wave w takes positions w, w+4, ...; lane owns dims 2*lane, 2*lane+1
  float o[kMaxGroup][2];
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) o[g][0] = o[g][1] = 0.f;
  const uint32_t* vr = reinterpret_cast<const uint32_t*>(vc + cbase) + lane;
  for (int p = wave; p < n; p += 4) {
    const uint32_t vv = vr[(long)(p0 + p) * (kHeadDim / 2)];
    const float v0 = h2f(vv & 0xffffu), v1 = h2f(vv >> 16);
#pragma unroll
    for (int g = 0; g < kMaxGroup; ++g) {
      const float pw = ps[g][p];
      o[g][0] += pw * v0;
      o[g][1] += pw * v1;
    }
  }
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) {
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
    pml[(pidx + (long)g * nsplit) * 2] = mx[g];
    pml[(pidx + (long)g * nsplit) * 2 + 1] = red[g][0] + red[g][1] + red[g][2] + red[g][3];
  }
}

// Merge the chunks of every head and quantise the attention output to Q8 (the o_proj input).
// grid T; thread i < H*4 owns one 32-value block (head i/4, dims (i%4)*32..+32).
__global__ void __launch_bounds__(256) attn_combine_q8_kernel(const float* __restrict__ po,
                                                              const float* __restrict__ pml,
                                                              const int* __restrict__ pos, int H,
                                                              int nsplit, float* __restrict__ out,
                                                              int8_t* __restrict__ x8,
                                                              float* __restrict__ dx,
                                                              float* __restrict__ sx) {
  const int t = blockIdx.x;
  const int ns = min(nsplit, (pos[t] + kAttnChunk) / kAttnChunk);
  const int K = H * kHeadDim;
  for (int blk = threadIdx.x; blk < H * (kHeadDim / 32); blk += blockDim.x) {
    const int h = blk / (kHeadDim / 32), d0 = (blk % (kHeadDim / 32)) * 32;
    const long hb = ((long)t * H + h) * nsplit;
    float m = -INFINITY;
    for (int s = 0; s < ns; ++s) m = fmaxf(m, pml[(hb + s) * 2]);
    float den = 0.f;
    float v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = 0.f;
    for (int s = 0; s < ns; ++s) {
      const float ms = pml[(hb + s) * 2];
      if (ms == -INFINITY) continue;
      const float wgt = __expf(ms - m);
      den += wgt * pml[(hb + s) * 2 + 1];
      const float4* src = reinterpret_cast<const float4*>(po + (hb + s) * kHeadDim + d0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 a = src[i];
        v[4 * i] += wgt * a.x; v[4 * i + 1] += wgt * a.y;
        v[4 * i + 2] += wgt * a.z; v[4 * i + 3] += wgt * a.w;
      }
    }
    const float inv = den > 0.f ? 1.f / den : 0.f;
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      v[i] *= inv;
      amax = fmaxf(amax, fabsf(v[i]));
    }
    if (out) {
      float4* dst = reinterpret_cast<float4*>(out + (long)t * K + h * kHeadDim + d0);
#pragma unroll
      for (int i = 0; i < 8; ++i) dst[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
    }
    const float d = amax / 127.f;
    const float id = d > 0.f ? 1.f / d : 0.f;
    uint32_t pk[8];
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = (int)__builtin_rintf(v[4 * i + j] * id);
        word |= ((uint32_t)(q & 0xff)) << (8 * j);
        if (i < 4) s0 += q; else s1 += q;
      }
      pk[i] = word;
    }
    const int gb = h * (kHeadDim / 32) + d0 / 32;      // 32-block index within the row
    int8_t* o = x8 + (long)t * K + gb * 32;
    reinterpret_cast<uint4*>(o)[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    reinterpret_cast<uint4*>(o)[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
    dx[(long)t * (K >> 5) + gb] = d;
    sx[(long)t * (K >> 4) + 2 * gb] = d * (float)s0;
    sx[(long)t * (K >> 4) + 2 * gb + 1] = d * (float)s1;
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
      const uint8_t* b = w.q + ((long)row * nb + blk) * kQ4KBytes;
      const float d = h2f(*reinterpret_cast<const uint16_t*>(b));
      const float dmin = h2f(*reinterpret_cast<const uint16_t*>(b + 2));
      const uint8_t* s = b + 4;
      uint32_t sc, m;
      if (j < 4) { sc = s[j] & 63; m = s[j + 4] & 63; }
      else { sc = (s[j + 4] & 0xf) | ((s[j - 4] >> 6) << 4); m = (s[j + 4] >> 4) | ((s[j] >> 6) << 4); }
      const uint8_t* qs = b + 16 + (j >> 1) * 32;
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
      const int8_t* sc = w.sc + rb * 16 + n * 8 + 2 * k;
      const float d = h2f(w.d[rb]);
#pragma unroll
      for (int l = 0; l < 32; ++l) {
        const uint32_t lo = (k < 2) ? (ql[l] & 0xf) : (ql[l] >> 4);
        const int q = (int)(lo | (((qh[l] >> (2 * k)) & 3) << 4)) - 32;
        v[l] = d * (float)sc[l >> 4] * (float)q;
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
    for (int i = 0; i < 16; ++i) sc[b * 16 + i] = (int8_t)s[192 + i];
    d[b] = (uint16_t)(s[208] | (s[209] << 8));
  }
}

template <int TYPE, int T, int MODE>
int launch_gemv(const GemvArgs& a, hipStream_t st) {
  const int nb = a.K >> 8;
  const size_t lds = (size_t)T * (nb * 288 + (a.K >> 5) * 4 + (a.K >> 4) * 4);
  if (lds > 160 * 1024) return 3;
  const int grid = (a.N + a.rows_per_wg - 1) / a.rows_per_wg;
  hipLaunchKernelGGL((qgemv_kernel<TYPE, T, MODE>), dim3(grid), dim3(256), lds, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

template <int TYPE, int MODE>
int dispatch_t(const GemvArgs& a, hipStream_t st) {
  switch (a.T) {
    case 1: return launch_gemv<TYPE, 1, MODE>(a, st);
    case 2: return launch_gemv<TYPE, 2, MODE>(a, st);
    case 3: return launch_gemv<TYPE, 3, MODE>(a, st);
    case 4: return launch_gemv<TYPE, 4, MODE>(a, st);
    default: return 2;
  }
}

}  // namespace

extern "C" {

int amdk8s_llm_max_tokens() { return kMaxTok; }
int amdk8s_llm_attn_chunk() { return kAttnChunk; }

// Quantised GEMV: out[t][n] (mode 0: = W.x + bias; 1: += W.x; 2: = silu(W0.x) * (W1.x)).
// type 0 = Q4_K (w0q: GGUF rows), 1 = Q6_K (w0q/w0qh/w0sc/w0d planes).
int amdk8s_llm_qgemv(int type, int mode, const void* w0q, const void* w0qh, const void* w0sc,
                     const void* w0d, const void* w1q, const void* w1qh, const void* w1sc,
                     const void* w1d, const void* x8, const void* dx, const void* sx,
                     const void* bias, void* out, int ldo, int N, int K, int T, int rows_per_wg,
                     void* stream) {
  if (K % 256 || N <= 0 || T < 1 || T > kMaxTok || rows_per_wg < 1) return 2;
  if (mode == kPair && !w1q) return 2;
  GemvArgs a;
  a.w0 = {static_cast<const uint8_t*>(w0q), static_cast<const uint8_t*>(w0qh),
          static_cast<const int8_t*>(w0sc), static_cast<const uint16_t*>(w0d)};
  a.w1 = {static_cast<const uint8_t*>(w1q), static_cast<const uint8_t*>(w1qh),
          static_cast<const int8_t*>(w1sc), static_cast<const uint16_t*>(w1d)};
  a.x8 = static_cast<const int8_t*>(x8);
  a.dx = static_cast<const float*>(dx);
  a.sx = static_cast<const float*>(sx);
  a.bias = static_cast<const float*>(bias);
  a.out = static_cast<float*>(out);
  a.ldo = ldo; a.N = N; a.K = K; a.T = T; a.rows_per_wg = rows_per_wg;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type == kQ4K) {
    if (mode == kStore) return dispatch_t<kQ4K, kStore>(a, st);
    if (mode == kResid) return dispatch_t<kQ4K, kResid>(a, st);
    if (mode == kPair) return dispatch_t<kQ4K, kPair>(a, st);
  } else if (type == kQ6K) {
    if (mode == kStore) return dispatch_t<kQ6K, kStore>(a, st);
    if (mode == kResid) return dispatch_t<kQ6K, kResid>(a, st);
    if (mode == kPair) return dispatch_t<kQ6K, kPair>(a, st);
  }
  return 2;
}

int amdk8s_llm_rmsnorm_q8(const void* x, const void* w, float eps, int K, int T, void* x8,
                          void* dx, void* sx, void* stream) {
  if (K % 256 || T < 1) return 2;
  hipLaunchKernelGGL(rmsnorm_q8_kernel, dim3(T), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const float*>(x), static_cast<const float*>(w), eps, K,
                     static_cast<int8_t*>(x8), static_cast<float*>(dx), static_cast<float*>(sx));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int amdk8s_llm_rope_kv(const void* qkv, int ldq, const void* pos, const void* slot,
                       const void* cos_t, const void* sin_t, int H, int Hkv, int head_dim,
                       int max_ctx, void* q_out, void* kc, void* vc, int T, void* stream) {
  if (head_dim != kHeadDim || T < 1) return 2;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(T), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const float*>(qkv), ldq, static_cast<const int*>(pos),
                     static_cast<const int*>(slot), static_cast<const float*>(cos_t),
                     static_cast<const float*>(sin_t), H, Hkv, max_ctx,
                     static_cast<float*>(q_out), static_cast<uint16_t*>(kc),
                     static_cast<uint16_t*>(vc));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Decode attention over the KV cache + combine + Q8 quantisation of the output.
// po/pml: workspace [T][H][nsplit][128] / [T][H][nsplit][2]; out (nullable) fp32 [T][H*128].
int amdk8s_llm_attn_decode(const void* q, const void* pos, const void* slot, const void* kc,
                           const void* vc, int H, int Hkv, int head_dim, int max_ctx, float scale,
                           void* po, void* pml, void* out, void* x8, void* dx, void* sx, int T,
                           void* stream) {
  if (head_dim != kHeadDim || H % Hkv || H / Hkv > kMaxGroup || max_ctx % kAttnChunk || T < 1)
    return 2;
  const int nsplit = max_ctx / kAttnChunk;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(attn_decode_kernel, dim3(Hkv, nsplit, T), dim3(256), 0, st,
                     static_cast<const float*>(q), static_cast<const int*>(pos),
                     static_cast<const int*>(slot), static_cast<const uint16_t*>(kc),
                     static_cast<const uint16_t*>(vc), H, Hkv, max_ctx, nsplit, scale,
                     static_cast<float*>(po), static_cast<float*>(pml));
  if (hipGetLastError() != hipSuccess) return 1;
  hipLaunchKernelGGL(attn_combine_q8_kernel, dim3(T), dim3(256), 0, st,
                     static_cast<const float*>(po), static_cast<const float*>(pml),
                     static_cast<const int*>(pos), H, nsplit, static_cast<float*>(out),
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
