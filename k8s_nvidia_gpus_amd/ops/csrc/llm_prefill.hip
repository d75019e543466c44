// Prompt-prefill glue kernels of the in-tree Qwen2 engine (models/llm/engine.py, dense fp16 path),
// gfx950.
//
// A 512-token prefill of the Qwen2.5-7B layout ran ~48 kernels per layer, ~1300 per prompt, most
// of them PyTorch elementwise launches around the hand-written GEMMs: the RMSNorms (pow, mean,
// add, rsqrt, mul, mul, cast), bias adds and fp16 <-> fp32 casts, RoPE as slices / products / cat,
// the KV-cache writes and SwiGLU — 7 of 17.8 ms (profiles/r03/ac/llm_prefill_kernels.txt).  Each of
// those launches costs at least ~4.5 us on MI355X whatever it does, so these three kernels replace
// them (one launch each per layer and use):
//   rmsnorm_f16   x fp32 [P][K] -> y fp16 = x * rsqrt(mean(x^2) + eps) * w   (one workgroup per row)
//   rope_kv_f16   q|k|v fp16 [P][ldq] (bias already added by the GEMM epilogue) -> rotated q fp16
//                 [H][P][128] for SDPA (any head / position strides: the engine stores it as
//                 [P][H][128], so SDPA's output comes back in token-major order) and rotated k / v
//                 written to the fp16 KV cache at positions start .. start + P - 1
//   swiglu_f16    gate|up fp16 [P][2F] -> silu(gate) * up fp16 [P][F] (halves or 128-blocks)
// The arithmetic is fp32 in registers; the RoPE uses the same explicit roundings as the decode
// kernels (llm_decode.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kWave = 64;
constexpr int kHeadDim = 128;

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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// grid P, 256 threads; thread = 8-value chunks tid + 256 u (K % 8 == 0, K <= 8192)
constexpr int kNormCh = 4;
__global__ void __launch_bounds__(256) rmsnorm_f16_kernel(const float* __restrict__ x, int ldx,
                                                          const float* __restrict__ w, float eps,
                                                          int K, uint16_t* __restrict__ y,
                                                          int ldy) {
  __shared__ float red[4];
  const float* xr = x + (long)blockIdx.x * ldx;
  const int nch = K >> 3, tid = threadIdx.x;
  float4 v[kNormCh][2];
#pragma unroll
  for (int u = 0; u < kNormCh; ++u) {          // every load in flight (clamped, masked below)
    const int c = min(tid + 256 * u, nch - 1);
    v[u][0] = *reinterpret_cast<const float4*>(xr + c * 8);
    v[u][1] = *reinterpret_cast<const float4*>(xr + c * 8 + 4);
  }
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < kNormCh; ++u)
    if (tid + 256 * u < nch) {
      const float e[8] = {v[u][0].x, v[u][0].y, v[u][0].z, v[u][0].w,
                          v[u][1].x, v[u][1].y, v[u][1].z, v[u][1].w};
#pragma unroll
      for (int i = 0; i < 8; ++i) ss = __fmaf_rn(e[i], e[i], ss);
    }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float r = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)K + eps);
  uint16_t* yr = y + (long)blockIdx.x * ldy;
#pragma unroll
  for (int u = 0; u < kNormCh; ++u) {
    const int c = tid + 256 * u;
    if (c >= nch) break;
    const float4 wa = *reinterpret_cast<const float4*>(w + c * 8);
    const float4 wb = *reinterpret_cast<const float4*>(w + c * 8 + 4);
    const float e[8] = {v[u][0].x, v[u][0].y, v[u][0].z, v[u][0].w,
                        v[u][1].x, v[u][1].y, v[u][1].z, v[u][1].w};
    const float ww[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
    uint32_t pk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      pk[i] = (uint32_t)f2h(e[2 * i] * r * ww[2 * i]) |
              ((uint32_t)f2h(e[2 * i + 1] * r * ww[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(yr + c * 8) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }
}

__device__ __forceinline__ float rope_lo(float x0, float x1, float c, float sn) {
  return __fmaf_rn(x0, c, -__fmul_rn(x1, sn));
}
__device__ __forceinline__ float rope_hi(float x0, float x1, float c, float sn) {
  return __fmaf_rn(x0, sn, __fmul_rn(x1, c));
}

// grid (ceil((H + 2 Hkv) * 64 / 256), P), 256 threads: one thread per rotated pair (q, k) or per
// two v values.  kc / vc: this layer's cache slab of one sequence slot, fp16 [Hkv][max_ctx][128].
__global__ void __launch_bounds__(256) rope_kv_f16_kernel(const uint16_t* __restrict__ qkv,
                                                          int ldq, const float* __restrict__ cos_t,
                                                          const float* __restrict__ sin_t,
                                                          int start, int P, int H, int Hkv,
                                                          int max_ctx, long qsh, long qsp,
                                                          uint16_t* __restrict__ q_out,
                                                          uint16_t* __restrict__ kc,
                                                          uint16_t* __restrict__ vc) {
  const int p = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int pos = start + p;
  const uint16_t* row = qkv + (long)p * ldq;
  const int pairs = (H + Hkv) * (kHeadDim / 2);
  if (i < pairs) {
    const int h = i / (kHeadDim / 2), j = i % (kHeadDim / 2);
    const float x0 = h2f(row[h * kHeadDim + j]), x1 = h2f(row[h * kHeadDim + j + kHeadDim / 2]);
    const float c = cos_t[(long)pos * (kHeadDim / 2) + j];
    const float sn = sin_t[(long)pos * (kHeadDim / 2) + j];
    const uint16_t y0 = f2h(rope_lo(x0, x1, c, sn)), y1 = f2h(rope_hi(x0, x1, c, sn));
    uint16_t* dst = h < H ? q_out + (long)h * qsh + (long)p * qsp
                          : kc + ((long)(h - H) * max_ctx + pos) * kHeadDim;
    dst[j] = y0;
    dst[j + kHeadDim / 2] = y1;
  } else if (i < pairs + Hkv * (kHeadDim / 2)) {
    const int e = (i - pairs) * 2;
    const int h = e / kHeadDim, j = e % kHeadDim;
    const uint32_t v = *reinterpret_cast<const uint32_t*>(row + (H + Hkv) * kHeadDim + e);
    *reinterpret_cast<uint32_t*>(vc + ((long)h * max_ctx + pos) * kHeadDim + j) = v;
  }
}

// grid-stride over P * F / 8; thread = 8 outputs
// blk 0: gate|up rows [gate F | up F]; blk > 0: interleaved in blocks of blk (gate columns
// [2 blk j, 2 blk j + blk), then the same blk up columns) — the layout the fused-SwiGLU GEMM
// epilogue reads (gemm_bf16_gfx950_w4a.hip, kEpiSwiGLU)
__global__ void __launch_bounds__(256) swiglu_f16_kernel(const uint16_t* __restrict__ gu, int P,
                                                         int F, int blk, uint16_t* __restrict__ t) {
  const long n8 = (long)P * (F >> 3);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    const long p = i / (F >> 3), c = (i - p * (F >> 3)) * 8;
    const long gc = blk ? (c / blk) * 2 * blk + c % blk : c, uo = blk ? blk : F;
    const uint4 g = *reinterpret_cast<const uint4*>(gu + p * 2 * F + gc);
    const uint4 u = *reinterpret_cast<const uint4*>(gu + p * 2 * F + gc + uo);
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, uw[4] = {u.x, u.y, u.z, u.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float g0 = h2f(gw[k] & 0xffffu), g1 = h2f(gw[k] >> 16);
      const float u0 = h2f(uw[k] & 0xffffu), u1 = h2f(uw[k] >> 16);
      const float y0 = g0 / (1.f + __expf(-g0)) * u0, y1 = g1 / (1.f + __expf(-g1)) * u1;
      o[k] = (uint32_t)f2h(y0) | ((uint32_t)f2h(y1) << 16);
    }
    *reinterpret_cast<uint4*>(t + p * F + c) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace

extern "C" {

int amdk8s_llm_rmsnorm_f16(const void* x, int ldx, const void* w, float eps, int P, int K, void* y,
                           int ldy, void* stream) {
  if (K % 8 || K > kNormCh * 256 * 8 || P < 1 || ldx % 4 || ldy % 8) return 2;
  hipLaunchKernelGGL(rmsnorm_f16_kernel, dim3(P), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const float*>(x), ldx, static_cast<const float*>(w), eps, K,
                     static_cast<uint16_t*>(y), ldy);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int amdk8s_llm_rope_kv_f16(const void* qkv, int ldq, const void* cos_t, const void* sin_t,
                           int start, int P, int H, int Hkv, int head_dim, int max_ctx,
                           long qsh, long qsp, void* q_out, void* kc, void* vc, void* stream) {
  if (head_dim != kHeadDim || P < 1 || start < 0 || start + P > max_ctx || ldq % 2) return 2;
  if (qsh < kHeadDim || qsp < kHeadDim) return 2;
  const int threads = (H + 2 * Hkv) * (kHeadDim / 2);
  hipLaunchKernelGGL(rope_kv_f16_kernel, dim3((threads + 255) / 256, P), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint16_t*>(qkv), ldq,
                     static_cast<const float*>(cos_t), static_cast<const float*>(sin_t), start, P,
                     H, Hkv, max_ctx, qsh, qsp, static_cast<uint16_t*>(q_out),
                     static_cast<uint16_t*>(kc),
                     static_cast<uint16_t*>(vc));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int amdk8s_llm_swiglu_f16(const void* gu, int P, int F, int blk, void* t, void* stream) {
  if (F % 8 || P < 1 || blk < 0 || blk % 8 || (blk && F % blk)) return 2;
  const long n8 = (long)P * (F / 8);
  const int grid = (int)((n8 + 255) / 256 < 4096 ? (n8 + 255) / 256 : 4096);
  hipLaunchKernelGGL(swiglu_f16_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint16_t*>(gu), P, F, blk, static_cast<uint16_t*>(t));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
