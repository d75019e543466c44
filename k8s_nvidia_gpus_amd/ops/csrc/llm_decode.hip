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
// * Decode attention (split over the context, flash-decoding) and its chunk merge, which emits the
//   Q8 activations of the o_proj input directly: llm_attn.hip.
//
// Since round 4 the default GEMV runs on the int8 matrix cores (llm_gemv_mfma.hip); the VALU
// GEMV below serves gemv_impl(VALU) and shapes that kernel does not cover.  Definitions shared by
// both files: llm_common.h.
#include "llm_common.h"

namespace {

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
