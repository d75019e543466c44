// Split-context decode attention of the in-tree Qwen2 LLM engine (k8s_nvidia_gpus_amd/models/llm),
// gfx950: flash-decoding over the fp16 KV cache, fused RoPE + KV write, and the chunk merge that
// emits the Q8 activations of the o_proj input (llm_decode.hip has the rest of the decode path).
#include "llm_common.h"

namespace {

// ---------------------------------------------------------------- split-context decode attention
// grid (Hkv, attn_parts_max(span), T); 64 x kAttnWaves threads.  One workgroup: the G = H/Hkv q heads of one
// kv head over cpw consecutive 64-position chunks (one partial); writes the unnormalised partial
// output and (max, sum) per head (attn_decode_kernel).
//
// Chunks per workgroup (cpw) follow the token's own length only: 1 up to 4096 positions, then 2,
// 4, 8 — at most kAttnParts = 64 partials per head up to 32768 positions.  At 32k positions one
// chunk per workgroup meant 2000 workgroups per layer and a 10.7 us merge of 500 partials per head
// (profiles/r05/llm_decode_32k_vs_512_kernels_r05f).  Swept at 32000 positions (session r05n,
// T = 1 / 4 / 8 tok/s): 128 partials 475 / 1119 / 1321, 64 partials 482 / 1181 / 1397; a third
// chunk buffer per wave (kAttnRing 3) lost at both (212 VGPRs).
// The split depends on nothing but the token, so its bits do not depend on its batch.
#ifndef AMDK8S_ATTN_RING
#define AMDK8S_ATTN_RING 2
#endif
constexpr int kAttnRing = AMDK8S_ATTN_RING;           // chunk buffers per wave (attn_decode_kernel)
#ifndef AMDK8S_ATTN_PARTS
#define AMDK8S_ATTN_PARTS 64
#endif
constexpr int kAttnParts = AMDK8S_ATTN_PARTS;
constexpr int kAttnMaxCpw = 8;
__host__ __device__ __forceinline__ int attn_cpw(int len) {
  int c = 1;
  while (c < kAttnMaxCpw && len > kAttnChunk * kAttnParts * c) c <<= 1;
  return c;
}
__host__ __device__ __forceinline__ int attn_parts(int len) {
  const int w = kAttnChunk * attn_cpw(len);
  return (len + w - 1) / w;
}
// the most partials of any length <= span (within one cpw band the count grows with the length,
// and each band ends at kAttnParts)
inline int attn_parts_max(int span) {
  int m = attn_parts(span);
  for (int e = kAttnChunk * kAttnParts; e < span; e <<= 1) m = m > attn_parts(e) ? m : attn_parts(e);
  return m;
}

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

// Output dim dd of head h, token t: fp32 (optional) and Q8 with its 32-block scale and 16-block
// scaled sums (the o_proj GEMV input); a 32-dim block = half a wave.
__device__ __forceinline__ void attn_out_q8(float y, int h, int t, int dd, int H,
                                            float* __restrict__ out, int8_t* __restrict__ x8,
                                            float* __restrict__ dx, float* __restrict__ sx) {
  const int K = H * kHeadDim;
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

// Merge the context chunks of head h of token t and quantise the attention output to Q8 (the o_proj
// input): thread dd = one output dim; a 32-dim block = half a wave (dd & 31 within a wave).  One
// pass over the chunks in groups of 8 with every partial of the group loaded before any maths
// (online max: one memory round trip per 8 chunks), explicit roundings.
template <int NH>
__device__ __forceinline__ void combine_heads(const float* __restrict__ po,
                                              const float* __restrict__ pml,
                                              const int* __restrict__ pos, int H, int nsplit,
                                              int h0, int hstep, int hend, int t, int dd,
                                              float* __restrict__ out, int8_t* __restrict__ x8,
                                              float* __restrict__ dx, float* __restrict__ sx) {
  const int ns = min(nsplit, attn_parts(pos[t] + 1));
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
#pragma unroll
  for (int k = 0; k < NH; ++k) {
    const int h = h0 + k * hstep;
    if (h >= hend) break;                            // uniform per wave (hstep multiple of waves)
    attn_out_q8(den[k] > 0.f ? __fdiv_rn(v[k], den[k]) : 0.f, h, t, dd, H, out, x8, dx, sx);
  }
}

// grid (H, T), 128 threads.
__global__ void __launch_bounds__(128) attn_combine_q8_kernel(const float* __restrict__ po,
                                                              const float* __restrict__ pml,
                                                              const int* __restrict__ pos, int H,
                                                              int nsplit,
                                                              float* __restrict__ out,
                                                              int8_t* __restrict__ x8,
                                                              float* __restrict__ dx,
                                                              float* __restrict__ sx) {
  combine_heads<1>(po, pml, pos, H, nsplit, blockIdx.x, 1, H, blockIdx.y, threadIdx.x, out,
                   x8, dx, sx);
}

// Two-pass merge of the chunks of head h of token t, with 128·G threads (G row groups of 128 dims):
// every chunk's (max, sum) loads at once (PER per thread, up to kCombMaxSplit chunks); the max and
// the denominator are workgroup reductions (the chunk weights go to LDS); then each of ng row groups
// sums a contiguous range of the partial rows with their weights, kCombBatch row loads in flight at
// a time, and the group sums add up in group order.  ng = min(G, ceil(ns / kCombBatch)) depends only
// on this token's own chunk count, and G only on the engine's max_ctx (the launcher), so a token's
// bits never depend on the batch it runs in.  At 32k positions with one chunk per
// partial (512 per head) the 128-thread form took 16 dependent row batches per head (~1 ms per
// 28-layer step at T = 1, profiles/r05); with streamed chunks (<= 64 partials up to 32768
// positions) two groups take one batch each.
constexpr int kCombBatch = 32;
constexpr int kCombMaxSplit = 1024;                 // max_ctx <= 524288 (8 chunks per partial)

template <int G>
__global__ void __launch_bounds__(128 * G) attn_combine2_q8_kernel(const float* __restrict__ po,
                                                                   const float* __restrict__ pml,
                                                                   const int* __restrict__ pos,
                                                                   int H, int nsplit,
                                                                   float* __restrict__ out,
                                                                   int8_t* __restrict__ x8,
                                                                   float* __restrict__ dx,
                                                                   float* __restrict__ sx) {
  constexpr int NT = 128 * G, NW = NT / kWave, PER = kCombMaxSplit / NT;
  __shared__ float wts[kCombMaxSplit];
  __shared__ float red[2][NW];
  __shared__ float part[G][kHeadDim];
  const int h = blockIdx.x, t = blockIdx.y, tid = threadIdx.x, wave = tid >> 6;
  const int dd = tid & (kHeadDim - 1), grp = tid >> 7;
  const int ns = min(nsplit, attn_parts(pos[t] + 1));
  const long hb = ((long)t * H + h) * nsplit;
  const int ng = min(G, (ns + kCombBatch - 1) / kCombBatch);
  const int gl = grp < ng ? grp * ns / ng : 0, gh = grp < ng ? (grp + 1) * ns / ng : 0;
  // this group's first row batch, in flight with the (max, sum) loads (indices clamped into the
  // written rows: rows of other groups or past ns are read but weighted 0)
  float ov[kCombBatch];
#pragma unroll
  for (int u = 0; u < kCombBatch; ++u) ov[u] = po[(hb + min(gl + u, ns - 1)) * kHeadDim + dd];
  float mx[PER], l[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const long sidx = hb + min(tid + NT * k, ns - 1);
    mx[k] = pml[sidx * 2];
    l[k] = pml[sidx * 2 + 1];
  }
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (tid + NT * k >= ns) mx[k] = -INFINITY;
    m = fmaxf(m, mx[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, kWave));
  if ((tid & 63) == 0) red[0][wave] = m;
  __syncthreads();
  float M = red[0][0];
#pragma unroll
  for (int w = 1; w < NW; ++w) M = fmaxf(M, red[0][w]);
  float dp = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const float w = (M == -INFINITY || mx[k] == -INFINITY) ? 0.f : __expf(__fsub_rn(mx[k], M));
    wts[tid + NT * k] = w;
    dp = __fmaf_rn(w, l[k], dp);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dp = __fadd_rn(dp, __shfl_xor(dp, o, kWave));
  if ((tid & 63) == 0) red[1][wave] = dp;
  __syncthreads();
  float den = red[1][0];
#pragma unroll
  for (int w = 1; w < NW; ++w) den = __fadd_rn(den, red[1][w]);
  float v = 0.f;
  for (int s0 = gl; s0 < gh; s0 += kCombBatch) {
    if (s0 != gl) {
#pragma unroll
      for (int u = 0; u < kCombBatch; ++u) ov[u] = po[(hb + min(s0 + u, ns - 1)) * kHeadDim + dd];
    }
#pragma unroll
    for (int u = 0; u < kCombBatch; ++u)
      v = __fmaf_rn(s0 + u < gh ? wts[min(s0 + u, kCombMaxSplit - 1)] : 0.f, ov[u], v);
  }
  if (G > 1) {
    part[grp][dd] = v;
    __syncthreads();
    if (grp != 0) return;
    v = part[0][dd];
#pragma unroll
    for (int g = 1; g < G; ++g)
      if (g < ng) v = __fadd_rn(v, part[g][dd]);
  }
  attn_out_q8(den > 0.f ? __fdiv_rn(v, den) : 0.f, h, t, dd, H, out, x8, dx, sx);
}

// Row groups of the merge for an engine whose KV cache holds max_ctx positions: one row batch
// per group at the engine's longest partial count (64 partials, every max_ctx >= 4096: 2 groups).
inline int comb_groups(int max_ctx) {
  const int parts = attn_parts_max(max_ctx);
  return parts <= kCombBatch ? 1 : parts <= 2 * kCombBatch ? 2 : parts <= 4 * kCombBatch ? 4 : 8;
}

// cpw chunks of 64 positions per workgroup (attn_cpw).  Each wave streams its own 16 positions of
// every chunk with its own online softmax, so the chunk loop has no barrier; the four waves'
// (max, sum, output) merge once at the end.  Both products run on the matrix cores:
// * scores S^T = K q^T (v_mfma_f32_16x16x32_f16): A = the K rows straight from memory (16
//   contiguous bytes per lane), B = the q heads as fp16, held in registers for every chunk; lane l
//   gets head l & 15 at positions 4 (l >> 4) .. + 3, so each lane keeps the online max / sum of
//   one head;
// * O += P V (v_mfma_f32_16x16x16_f16): A = those P values as they lie (fp16), B = the V rows,
//   loaded as whole 1 KiB row groups, written to a per-wave LDS image and read back transposed
//   with ds_read_b64_tr_b16 (cdna_hip_programming.md T10; the XOR-swizzled 256-byte-row image of
//   its "(b)" layout).
// q and P are rounded to fp16 for the MFMA (llama.cpp's flash-attention kernels do the same);
// scores, softmax and the output accumulate in fp32.  History (profiles/r05/README.md): one
// chunk per workgroup on the VALU took 20.1 + 10.7 us (attention + merge) per 32k layer; VALU
// scores read every q value from LDS once per position (LDS-bound, 22.7 us streamed); MFMA
// scores with a v_readlane VALU P.V 19.6 + 6.0 us; both products on MFMA with 64 partials per
// head 17.2 + 5.3 us; q fragments straight from memory (no LDS staging, no barrier) 16.6 + 5.2.
// Measured and rejected (session r05n / r05t): a third chunk buffer per wave, 8 waves per
// workgroup (two chunk parities), 128 or 256 partials per head, a 168-VGPR cap (3 waves/SIMD).
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

// x of lane l ^ 16 / l ^ 32 on the VALU (v_permlane16/32_swap: a half-row exchange; with both
// operands x, the swapped-in copy is the partner's value): no LDS round trip, unlike __shfl_xor
__device__ __forceinline__ float lane_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float lane_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}

// byte offset of 16-byte chunk ch (0..15) of row `row` in a [16][128 x fp16] V image
__device__ __forceinline__ int vimg_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

#ifndef AMDK8S_ATTN_WAVES
#define AMDK8S_ATTN_WAVES 4
#endif
constexpr int kAttnWaves = AMDK8S_ATTN_WAVES;         // 4 or 8 waves per workgroup
#ifndef AMDK8S_ATTN_FAST1
#define AMDK8S_ATTN_FAST1 1
#endif
#ifndef AMDK8S_ATTN_WPE
#define AMDK8S_ATTN_WPE 1
#endif
template <int G>
__global__ void __launch_bounds__(64 * kAttnWaves) __attribute__((amdgpu_waves_per_eu(AMDK8S_ATTN_WPE)))
attn_decode_kernel(AttnArgs a) {
  const float* __restrict__ q = a.q;
  const int* __restrict__ pos = a.pos;
  const int* __restrict__ slot = a.slot;
  const uint16_t* __restrict__ kc = a.kc;
  const uint16_t* __restrict__ vc = a.vc;
  const int H = a.H, Hkv = a.Hkv, max_ctx = a.max_ctx, nsplit = a.nsplit;
  const float scale = a.scale;
  float* __restrict__ po = a.po;
  float* __restrict__ pml = a.pml;
  __shared__ __align__(16) uint16_t knew[kHeadDim];   // the new position's rotated K (fp16)
  __shared__ __align__(16) uint16_t vnew[kHeadDim];   // and its V
  constexpr int NW = kAttnWaves, NT = 64 * NW, NPAR = NW / 4;
  __shared__ __align__(16) uint8_t vimg[NW][16 * 256];  // per wave: the chunk's V rows
  __shared__ float wml[NW][16][2];                    // per wave: running max, sum per head
  __shared__ float wo[NW][G][kHeadDim];               // per wave: unnormalised output
  const int kh = blockIdx.x, sp = blockIdx.y, t = blockIdx.z;
  const int len = pos[t] + 1;
  const int cpw = attn_cpw(len);
  const int w0 = sp * kAttnChunk * cpw;                 // this workgroup's first position
  if (w0 >= len) return;                                // past the token's partials: never merged
  const int nc = min(cpw, (len - w0 + kAttnChunk - 1) / kAttnChunk);   // chunks streamed here
  const long pidx = ((long)t * H + kh * G) * nsplit + sp;   // + g * nsplit
  const long cbase = ((long)slot[t] * Hkv + kh) * max_ctx * kHeadDim;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pr = lane & 15, kg = lane >> 4;
  // wave = (chunk parity wpar, 16-position slot wsub): it streams chunks wpar, wpar + NPAR, ...
  const int wsub = wave & 3, wpar = wave >> 2;
  const int ncw = nc > wpar ? (nc - wpar + NPAR - 1) / NPAR : 0;   // this wave's chunks
  // this wave's 16 positions of chunk c.  K: lane = (position pr, dims 32 s + 8 kg .. + 7 for
  // s = 0..3), positions clamped into the token.  V: lane = (row 4 r + kg, dims 8 pr .. + 7 for
  // r = 0..3): 1 KiB contiguous per instruction; rows past the token are inside the cache
  // (max_ctx % 64 == 0) and zeroed before use.  Every load unconditional.
  auto load_rows = [&](int c, uint4 (&kr)[4], uint4 (&vr)[4]) __attribute__((always_inline)) {
    const int pb = w0 + (c * NPAR + wpar) * kAttnChunk + wsub * 16;
    const uint4* kp = reinterpret_cast<const uint4*>(kc + cbase + (long)min(pb + pr, len - 1)
                                                     * kHeadDim) + kg;
#pragma unroll
    for (int s = 0; s < 4; ++s) kr[s] = kp[4 * s];
    const uint4* vp = reinterpret_cast<const uint4*>(                  // an idle wave's rows may
        vc + cbase + (long)(min(pb, max_ctx - 16) + kg) * kHeadDim) + pr;  // pass max_ctx: clamped
#pragma unroll
    for (int r = 0; r < 4; ++r) vr[r] = vp[r * 4 * (kHeadDim / 8)];
  };
  // ring of R chunk buffers (R - 1 chunks in flight during a chunk's maths), constant indices
  uint4 kr[kAttnRing][4];
  uint4 vr[kAttnRing][4];
#pragma unroll
  for (int r = 0; r < kAttnRing - 1; ++r)               // in flight during the q work
    load_rows(min(r, max(ncw - 1, 0)), kr[r], vr[r]);
  const int pnew = len - 1;
  const bool own = a.qkv != nullptr && pnew >= w0 && pnew < w0 + kAttnChunk * cpw;
  // B fragments of the scores, straight from memory: q head pr (zero rows past G), dims
  // 32 s + 8 kg .. + 7, fp16.  With the fused RoPE the lane's dims pair up with their rotation
  // partners (d, d + 64: s and s + 2) in its own registers, so no LDS round trip or barrier.
  h8 qa[4];
  {
    const int hq = kh * G + min(pr, G - 1);
    float qv[4][8];
    if (a.qkv) {
      const float* row = a.qkv + (long)t * a.ldq + hq * kHeadDim;
      const float* ct = a.cos_t + (long)pnew * (kHeadDim / 2);
      const float* st = a.sin_t + (long)pnew * (kHeadDim / 2);
      float x[4][8], cs[2][8], sn[2][8];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float4 u0 = *reinterpret_cast<const float4*>(row + 32 * s + 8 * kg);
        const float4 u1 = *reinterpret_cast<const float4*>(row + 32 * s + 8 * kg + 4);
        x[s][0] = u0.x; x[s][1] = u0.y; x[s][2] = u0.z; x[s][3] = u0.w;
        x[s][4] = u1.x; x[s][5] = u1.y; x[s][6] = u1.z; x[s][7] = u1.w;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float4 c0 = *reinterpret_cast<const float4*>(ct + 32 * s + 8 * kg);
        const float4 c1 = *reinterpret_cast<const float4*>(ct + 32 * s + 8 * kg + 4);
        const float4 s0 = *reinterpret_cast<const float4*>(st + 32 * s + 8 * kg);
        const float4 s1 = *reinterpret_cast<const float4*>(st + 32 * s + 8 * kg + 4);
        cs[s][0] = c0.x; cs[s][1] = c0.y; cs[s][2] = c0.z; cs[s][3] = c0.w;
        cs[s][4] = c1.x; cs[s][5] = c1.y; cs[s][6] = c1.z; cs[s][7] = c1.w;
        sn[s][0] = s0.x; sn[s][1] = s0.y; sn[s][2] = s0.z; sn[s][3] = s0.w;
        sn[s][4] = s1.x; sn[s][5] = s1.y; sn[s][6] = s1.z; sn[s][7] = s1.w;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          qv[s][jj] = rope_lo(x[s][jj], x[s + 2][jj], cs[s][jj], sn[s][jj]) * scale;
          qv[s + 2][jj] = rope_hi(x[s][jj], x[s + 2][jj], cs[s][jj], sn[s][jj]) * scale;
        }
    } else {
      const float* row = q + (long)t * H * kHeadDim + hq * kHeadDim;
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) qv[s][jj] = row[32 * s + 8 * kg + jj] * scale;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) qa[s][jj] = (_Float16)(pr < G ? qv[s][jj] : 0.f);
  }
  // the one workgroup per (token, kv head) whose range holds the new position rotates its k,
  // writes K / V to the cache and keeps them in LDS for the chunk that reads them (uniform)
  if (own) {
    const float* row = a.qkv + (long)t * a.ldq;
    const long cpos = cbase + (long)pnew * kHeadDim;
    const int jk = threadIdx.x & (kHeadDim / 2 - 1), ev = threadIdx.x & (kHeadDim - 1);
    if (threadIdx.x < kHeadDim / 2) {
      const float c = a.cos_t[(long)pnew * (kHeadDim / 2) + jk];
      const float sn = a.sin_t[(long)pnew * (kHeadDim / 2) + jk];
      const float k0 = row[(H + kh) * kHeadDim + jk], k1 = row[(H + kh) * kHeadDim + jk + kHeadDim / 2];
      const uint16_t h0 = f2h(rope_lo(k0, k1, c, sn)), h1 = f2h(rope_hi(k0, k1, c, sn));
      a.kc[cpos + jk] = h0;
      a.kc[cpos + jk + kHeadDim / 2] = h1;
      knew[jk] = h0;
      knew[jk + kHeadDim / 2] = h1;
    }
    if (threadIdx.x < kHeadDim) {
      const uint16_t hv = f2h(row[(H + Hkv + kh) * kHeadDim + ev]);
      a.vc[cpos + ev] = hv;
      vnew[ev] = hv;
    }
    __syncthreads();
  }
  float mrun = -INFINITY, lrun = 0.f;                   // head pr
  f4 o[8];                                              // O[head 4 kg + i][dim 16 n + pr]
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f4{0.f, 0.f, 0.f, 0.f};
  uint8_t* img = vimg[wave];
  // transposed-read address of n-tile 0 (lane 4 q + p of its 16-lane group: row 4 kg + q,
  // columns 4 p .. 4 p + 3 of the tile); tile n adds 2 chunks, which the XOR keeps inside the
  // same 64-byte half-row pair only up to the swizzle: recomputed per tile (constants fold)
  const int tq = pr >> 2, tp = pr & 3;
  auto chunk = [&](int c, uint4 (&kb)[4], uint4 (&vb)[4]) __attribute__((always_inline)) {
    const int pb = w0 + (c * NPAR + wpar) * kAttnChunk + wsub * 16;
    const int jn = pnew - pb;                           // the new position among these 16?
    if (own && jn >= 0 && jn < 16) {                    // its rows were loaded before they were written
      uint4 kq[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) kq[s] = reinterpret_cast<const uint4*>(knew)[4 * s + kg];
      const uint4 vq = reinterpret_cast<const uint4*>(vnew)[pr];
      const bool nw = pr == jn;
#pragma unroll
      for (int s = 0; s < 4; ++s) {                     // per component (a uint4 select is a
        kb[s].x = nw ? kq[s].x : kb[s].x;               // pointer select: scratch)
        kb[s].y = nw ? kq[s].y : kb[s].y;
        kb[s].z = nw ? kq[s].z : kb[s].z;
        kb[s].w = nw ? kq[s].w : kb[s].w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool vw = 4 * r + kg == jn;
        vb[r].x = vw ? vq.x : vb[r].x;
        vb[r].y = vw ? vq.y : vb[r].y;
        vb[r].z = vw ? vq.z : vb[r].z;
        vb[r].w = vw ? vq.w : vb[r].w;
      }
    }
    const int nv = len - pb;                            // rows of these 16 inside the token
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool in = 4 * r + kg < nv;
      const uint4 z = in ? vb[r] : make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(img + vimg_off(4 * r + kg, pr)) = z;
    }
    // scores: acc[i] = S[position 4 kg + i][head pr]
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      h8 ka;
      __builtin_memcpy(&ka, &kb[s], sizeof(ka));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ka, qa[s], acc, 0, 0, 0);
    }
    float sc[4];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sc[i] = 4 * kg + i < nv ? acc[i] : -INFINITY;
      mx = fmaxf(mx, sc[i]);
    }
    mx = fmaxf(mx, lane_xor16(mx));
    mx = fmaxf(mx, lane_xor32(mx));
    const float mn = fmaxf(mrun, mx);
    const float mref = mn == -INFINITY ? 0.f : mn;      // nothing attended yet: every term is 0
    const float al = __expf(mrun - mref);
    h4 pa;
    float ls = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = __expf(sc[i] - mref);
      pa[i] = (_Float16)p;
      ls += p;
    }
    ls += lane_xor16(ls);
    ls += lane_xor32(ls);
    lrun = lrun * al + ls;
    mrun = mn;
    // rescale: output row 4 kg + i takes the alpha of head 4 kg + i (lane 4 kg + i); rows past
    // G (kg >= 2 when G <= 8) are padding
    f4 a4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float lo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(al), i));
      const float hi = G > 4 ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(al), 4 + i)) : lo;
      a4[i] = kg == 0 ? lo : hi;
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) o[n] *= a4;
    // P.V: B = V[position 4 kg + j][dim 16 n + pr] from the image, transposed
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int off = vimg_off(4 * kg + tq, 2 * n + (tp >> 1)) + 8 * (tp & 1);
      const s4 braw = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + off));
      h4 bv;
      __builtin_memcpy(&bv, &braw, sizeof(bv));
      o[n] = __builtin_amdgcn_mfma_f32_16x16x16f16(pa, bv, o[n], 0, 0, 0);
    }
  };
  // the ring: before each chunk's maths, the load of the chunk R - 1 ahead goes into the slot
  // consumed one step ago.  A copy between buffers would wait for the loads it copies (every chunk
  // a full HBM round trip), and a load under a branch leaves the wait counter unknown at the join,
  // where the compiler then waits for it too — so the loads past the last chunk are issued
  // anyway, clamped to it (an L2 re-read).
  if (AMDK8S_ATTN_FAST1 && ncw == 1) {                  // one chunk (every token <= 4096): no ring
    chunk(0, kr[0], vr[0]);
  } else if (ncw > 1) {
#pragma unroll 1
    for (int c = 0; c < ncw; c += kAttnRing) {
#pragma unroll
      for (int r = 0; r < kAttnRing; ++r) {
        const int nx = (r + kAttnRing - 1) % kAttnRing;
        load_rows(min(c + r + kAttnRing - 1, ncw - 1), kr[nx], vr[nx]);
        if (r == 0 || c + r < ncw) chunk(c + r, kr[r], vr[r]);
      }
    }
  }
  // merge the waves (an idle wave: max -inf, sum 0, output 0 — weight 0)
  if (kg == 0) { wml[wave][pr][0] = mrun; wml[wave][pr][1] = lrun; }
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (4 * kg + i < G) wo[wave][min(4 * kg + i, G - 1)][16 * n + pr] = o[n][i];
  __syncthreads();
  for (int i = threadIdx.x; i < G * kHeadDim; i += blockDim.x) {
    const int g = i / kHeadDim, dd = i % kHeadDim;
    float m = wml[0][g][0];
#pragma unroll
    for (int w = 1; w < NW; ++w) m = fmaxf(m, wml[w][g][0]);
    float v = 0.f, l = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float e = wml[w][g][0] == -INFINITY ? 0.f : __expf(wml[w][g][0] - m);
      v += e * wo[w][g][dd];
      l += e * wml[w][g][1];
    }
    po[(pidx + (long)g * nsplit) * kHeadDim + dd] = v;
    if (dd == 0) {
      float* dst = pml + (pidx + (long)g * nsplit) * 2;
      dst[0] = m;
      dst[1] = l;
    }
  }
}

}  // namespace

extern "C" {

int amdk8s_llm_attn_chunk() { return kAttnChunk; }

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
  aa.nsplit = span / kAttnChunk;                         // partial-row stride of po / pml
  const int rc = by_group([&](auto g) {
    hipLaunchKernelGGL(attn_decode_kernel<decltype(g)::value>, dim3(Hkv, attn_parts_max(span), T),
                       dim3(64 * kAttnWaves), 0, st, aa);
  });
  if (rc) return rc;
  // the merge kernel and its row groups follow max_ctx (fixed per engine), never this launch's
  // span: a token's bits must not depend on the longest sequence it is batched with
  const float* po_c = static_cast<const float*>(po);
  const float* pml_c = static_cast<const float*>(pml);
  const int* pos_c = static_cast<const int*>(pos);
  float* out_f = static_cast<float*>(out);
  int8_t* x8_c = static_cast<int8_t*>(x8);
  float* dx_f = static_cast<float*>(dx);
  float* sx_f = static_cast<float*>(sx);
  if (attn_parts_max(max_ctx) > kCombMaxSplit) {
    hipLaunchKernelGGL(attn_combine_q8_kernel, dim3(H, T), dim3(128), 0, st, po_c, pml_c, pos_c, H,
                       aa.nsplit, out_f, x8_c, dx_f, sx_f);
  } else {
    switch (comb_groups(max_ctx)) {
      case 1:
        hipLaunchKernelGGL(attn_combine2_q8_kernel<1>, dim3(H, T), dim3(128), 0, st, po_c, pml_c,
                           pos_c, H, aa.nsplit, out_f, x8_c, dx_f, sx_f);
        break;
      case 2:
        hipLaunchKernelGGL(attn_combine2_q8_kernel<2>, dim3(H, T), dim3(256), 0, st, po_c, pml_c,
                           pos_c, H, aa.nsplit, out_f, x8_c, dx_f, sx_f);
        break;
      case 4:
        hipLaunchKernelGGL(attn_combine2_q8_kernel<4>, dim3(H, T), dim3(512), 0, st, po_c, pml_c,
                           pos_c, H, aa.nsplit, out_f, x8_c, dx_f, sx_f);
        break;
      default:
        hipLaunchKernelGGL(attn_combine2_q8_kernel<8>, dim3(H, T), dim3(1024), 0, st, po_c, pml_c,
                           pos_c, H, aa.nsplit, out_f, x8_c, dx_f, sx_f);
        break;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
