// Row-fused glue kernels of the Wan2.1 DiT (k8s_nvidia_gpus_amd/models/wan): gfx950, wave64,
// bf16 storage, fp32 maths.  Both kernels are HBM-bound row passes; one wave owns one token row
// of width C (C % 512 == 0, C <= 5120: 1.3B C=1536, 14B C=5120), each lane holding C/512 vectors
// of 8 consecutive columns in registers for the whole row (no LDS, no second read of the row).
//
// amdk8s_wan_add_ln — the residual update fused with the LayerNorm that follows it:
//     x[r, :] += y[r, :] * gate[b, :]            (fp32 residual stream, in place; y optional)
//     out[r, :] = LN(x[r, :]) * mul[b, :] + add[b, :]     (bf16, feeds the next GEMM)
//   b = r / L.  mul/add are AdaLN rows (1 + scale, shift) with batch stride C, or an affine
//   LayerNorm's weight/bias with batch stride 0.  Two-pass mean/variance over the registers.
//
// amdk8s_wan_rmsnorm_rope — in place on 1 or 2 column sections of a strided row (the q and k
// slices of the fused q|k|v projection):  t = t * rsqrt(mean(t²) + eps) * w, then (optional) the
// rotary embedding of each head's adjacent pairs, angle table cos/sin[pos, hd/2] with pos = r % L
// (Wan's 3-D frame/row/column split lives in the table).  A lane's 8 columns are 4 pairs of one
// head, so its table slice is one 16-byte load of each of cos and sin.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return 0x7fc0u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf16_to_f32(w[i] & 0xffffu);
    f[2 * i + 1] = bf16_to_f32(w[i] >> 16);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = f32_to_bf16(f[0]) | (f32_to_bf16(f[1]) << 16);
  r.y = f32_to_bf16(f[2]) | (f32_to_bf16(f[3]) << 16);
  r.z = f32_to_bf16(f[4]) | (f32_to_bf16(f[5]) << 16);
  r.w = f32_to_bf16(f[6]) | (f32_to_bf16(f[7]) << 16);
  return r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void load8f(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

__device__ __forceinline__ void store8f(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}

constexpr int kRowsPerBlock = 4;   // 4 waves, one row each

template <int VPL, bool HAS_Y, bool HAS_GATE>
__global__ __launch_bounds__(256) void add_ln_kernel(float* __restrict__ x,
                                                     const uint16_t* __restrict__ y, long sy,
                                                     const float* __restrict__ gate, long sg,
                                                     const float* __restrict__ mul, long sm,
                                                     const float* __restrict__ add, long sa,
                                                     uint16_t* __restrict__ out, long rows, int L,
                                                     float eps) {
  constexpr int C = VPL * 512;
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (r >= rows) return;                       // whole wave exits together
  const long b = r / L;
  float* xr = x + r * C;
  float v[VPL][8];
  uint4 yv[VPL];
  if constexpr (HAS_Y) {
#pragma unroll
    for (int j = 0; j < VPL; ++j)
    {
      const u32x4 t = __builtin_nontemporal_load(
          reinterpret_cast<const u32x4*>(y + r * sy + (j * 64 + lane) * 8));
      yv[j] = make_uint4(t.x, t.y, t.z, t.w);
    }
  }
#pragma unroll
  for (int j = 0; j < VPL; ++j) load8f(xr + (j * 64 + lane) * 8, v[j]);
  if constexpr (HAS_Y) {
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = (j * 64 + lane) * 8;
      float yf[8], g[8];
      unpack8(yv[j], yf);
      if constexpr (HAS_GATE) {
        load8f(gate + b * sg + c, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[j][e] = fmaf(yf[e], g[e], v[j][e]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[j][e] += yf[e];
      }
      store8f(xr + c, v[j]);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[j][e];
  const float mean = wave_sum(s) * (1.0f / C);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[j][e] - mean;
      q = fmaf(d, d, q);
    }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / C) + eps);
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = (j * 64 + lane) * 8;
    float m[8], a[8], o[8];
    load8f(mul + b * sm + c, m);
    load8f(add + b * sa + c, a);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = fmaf((v[j][e] - mean) * rstd, m[e], a[e]);
    *reinterpret_cast<uint4*>(out + r * C + c) = pack8(o);
  }
}

template <int VPL, bool ROPE>
__global__ __launch_bounds__(256) void rmsnorm_rope_kernel(uint16_t* __restrict__ t, long st,
                                                           const float* __restrict__ w,
                                                           const float* __restrict__ cs,
                                                           const float* __restrict__ sn, long rows,
                                                           int L, int hd, float eps) {
  constexpr int C = VPL * 512;
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int sec = blockIdx.y;                  // 0: q slice, 1: k slice (column offset sec*C)
  uint16_t* tr = t + r * st + (long)sec * C;
  const float* ws = w + (long)sec * C;
  float v[VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j) unpack8(*reinterpret_cast<const uint4*>(tr + (j * 64 + lane) * 8), v[j]);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) q = fmaf(v[j][e], v[j][e], q);
  const float rs = rsqrtf(wave_sum(q) * (1.0f / C) + eps);
  const int pos = (int)(r % L);
  const int half = hd >> 1;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = (j * 64 + lane) * 8;
    float g[8];
    load8f(ws + c, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[j][e] = v[j][e] * rs * g[e];
    if constexpr (ROPE) {
      const int p = (c % hd) >> 1;             // first of this lane's 4 pairs
      const float4 cv = *reinterpret_cast<const float4*>(cs + (long)pos * half + p);
      const float4 sv = *reinterpret_cast<const float4*>(sn + (long)pos * half + p);
      const float cc[4] = {cv.x, cv.y, cv.z, cv.w}, ss[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float a = v[j][2 * k], bb = v[j][2 * k + 1];
        v[j][2 * k] = a * cc[k] - bb * ss[k];
        v[j][2 * k + 1] = a * ss[k] + bb * cc[k];
      }
    }
    *reinterpret_cast<uint4*>(tr + c) = pack8(v[j]);
  }
}

template <int VPL>
int launch_add_ln(float* x, const uint16_t* y, long sy, const float* gate, long sg, const float* mul,
                  long sm, const float* add, long sa, uint16_t* out, long rows, int L, float eps,
                  hipStream_t s) {
  const dim3 grid((unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock));
  if (y && gate)
    add_ln_kernel<VPL, true, true><<<grid, 256, 0, s>>>(x, y, sy, gate, sg, mul, sm, add, sa, out, rows, L, eps);
  else if (y)
    add_ln_kernel<VPL, true, false><<<grid, 256, 0, s>>>(x, y, sy, gate, sg, mul, sm, add, sa, out, rows, L, eps);
  else
    add_ln_kernel<VPL, false, false><<<grid, 256, 0, s>>>(x, y, sy, gate, sg, mul, sm, add, sa, out, rows, L, eps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int VPL>
int launch_rms(uint16_t* t, long st, const float* w, const float* cs, const float* sn, long rows,
               int L, int hd, int nsec, float eps, hipStream_t s) {
  const dim3 grid((unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock), (unsigned)nsec);
  if (cs)
    rmsnorm_rope_kernel<VPL, true><<<grid, 256, 0, s>>>(t, st, w, cs, sn, rows, L, hd, eps);
  else
    rmsnorm_rope_kernel<VPL, false><<<grid, 256, 0, s>>>(t, st, w, cs, sn, rows, L, hd, eps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// amdk8s_wan_vae_rms_silu_stack — the Wan VAE's "RMS_norm → SiLU → causal 3×3×3 conv input" glue
// in one pass over channels-last frames x [B·T, H·W, C] (C = 96 / 192 / 384):
//     y = silu(x / max(‖x‖₂, 1e-12) · √C · γ)                       (per pixel, over channels)
// written either plainly (kt = 1) or straight into the temporal-tap-stacked input of the next
// causal convolution (kt = 3): out[t][p][j·C : (j+1)·C] = y[t − 2 + j] (zero before frame 0 of
// each sample), so the convolution runs as ONE 2-D conv over 3·C input channels with no
// separate normalise / activation / concatenate passes (each a full-resolution HBM round trip).
// 4 lanes per pixel, each holding CPL 16-byte chunks; 16 pixels per wave, 64 per workgroup.
template <int CPL, int KT>
__global__ __launch_bounds__(256) void vae_rms_silu_stack_kernel(const uint16_t* __restrict__ x,
                                                                 const float* __restrict__ gamma,
                                                                 uint16_t* __restrict__ out,
                                                                 long pixels, int hw, int T) {
  constexpr int C = CPL * 32;
  const int lane = threadIdx.x & 63, sub = lane & 3;
  const long px = ((long)blockIdx.x * 256 + threadIdx.x) >> 2;     // global pixel row
  if (px >= pixels) return;                                        // 4-lane groups exit together
  const uint16_t* xr = x + px * C;
  float v[CPL][8];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    unpack8(*reinterpret_cast<const uint4*>(xr + (j * 4 + sub) * 8), v[j]);
#pragma unroll
    for (int e = 0; e < 8; ++e) ss = fmaf(v[j][e], v[j][e], ss);
  }
  ss += __shfl_xor(ss, 1, 64);
  ss += __shfl_xor(ss, 2, 64);
  const float sc = sqrtf((float)C) / fmaxf(sqrtf(ss), 1e-12f);
  uint4 y[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    float g[8], o[8];
    load8f(gamma + (j * 4 + sub) * 8, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = v[j][e] * sc * g[e];
      o[e] = t / (1.f + __expf(-t));
    }
    y[j] = pack8(o);
  }
  if constexpr (KT == 1) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) *reinterpret_cast<uint4*>(out + px * C + (j * 4 + sub) * 8) = y[j];
  } else {
    const long n = px / hw, p = px - n * hw;       // frame index (b·T + t) and pixel in frame
    const int t = (int)(n % T);
    // y[t] feeds out[t + j'] at slot 2 − j'  (j' = 0, 1, 2 while t + j' < T)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      if (t + jj < T) {
        uint16_t* dst = out + ((n + jj) * hw + p) * (3 * C) + (2 - jj) * C;
#pragma unroll
        for (int j = 0; j < CPL; ++j) *reinterpret_cast<uint4*>(dst + (j * 4 + sub) * 8) = y[j];
      }
    }
    // slots of this frame that reach before frame 0 are zero
    if (t < 2) {
      uint16_t* dst = out + (n * hw + p) * (3 * C);
      const uint4 z = make_uint4(0, 0, 0, 0);
      for (int slot = 0; slot < 2 - t; ++slot)
#pragma unroll
        for (int j = 0; j < CPL; ++j) *reinterpret_cast<uint4*>(dst + slot * C + (j * 4 + sub) * 8) = z;
    }
  }
}

template <int CPL>
int launch_vae(const uint16_t* x, const float* g, uint16_t* out, long pixels, int hw, int T, int kt,
               hipStream_t s) {
  const unsigned blocks = (unsigned)((pixels * 4 + 255) / 256);
  if (kt == 3)
    vae_rms_silu_stack_kernel<CPL, 3><<<blocks, 256, 0, s>>>(x, g, out, pixels, hw, T);
  else
    vae_rms_silu_stack_kernel<CPL, 1><<<blocks, 256, 0, s>>>(x, g, out, pixels, hw, T);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace

extern "C" {

int amdk8s_wan_row_supported(int C) {
  if (C % 512 != 0) return 0;
  const int v = C / 512;   // instantiated row widths: 512..2048, 3072, 4096, 5120
  return (v >= 1 && v <= 4) || v == 6 || v == 8 || v == 10 ? 1 : 0;
}

// x fp32 [rows, C] contiguous (updated in place when y != null); y bf16 rows (stride sy elements,
// may be null); gate/mul/add fp32 with batch strides (elements; 0 = shared row); out bf16 [rows, C].
int amdk8s_wan_add_ln(float* x, const void* y, long sy, const float* gate, long sg, const float* mul,
                      long sm, const float* add, long sa, void* out, long rows, int L, int C,
                      float eps, hipStream_t s) {
  if (!amdk8s_wan_row_supported(C) || rows <= 0 || L <= 0) return -1;
  if (y && sy % 8) return -3;
  const uint16_t* yp = static_cast<const uint16_t*>(y);
  uint16_t* op = static_cast<uint16_t*>(out);
  switch (C / 512) {
    case 1: return launch_add_ln<1>(x, yp, sy, gate, sg, mul, sm, add, sa, op, rows, L, eps, s);
    case 2: return launch_add_ln<2>(x, yp, sy, gate, sg, mul, sm, add, sa, op, rows, L, eps, s);
    case 3: return launch_add_ln<3>(x, yp, sy, gate, sg, mul, sm, add, sa, op, rows, L, eps, s);
    case 4: return launch_add_ln<4>(x, yp, sy, gate, sg, mul, sm, add, sa, op, rows, L, eps, s);
    case 6: return launch_add_ln<6>(x, yp, sy, gate, sg, mul, sm, add, sa, op, rows, L, eps, s);
    case 8: return launch_add_ln<8>(x, yp, sy, gate, sg, mul, sm, add, sa, op, rows, L, eps, s);
    case 10: return launch_add_ln<10>(x, yp, sy, gate, sg, mul, sm, add, sa, op, rows, L, eps, s);
    default: return -1;
  }
}

int amdk8s_wan_rms_supported(int C, int hd) {
  return (amdk8s_wan_row_supported(C) && hd % 8 == 0 && C % hd == 0) ? 1 : 0;
}

// t bf16: section s of row r starts at t + r*st + s*C (nsec 1 or 2); w fp32 [nsec*C];
// cs/sn fp32 [L, hd/2] or null (no rotary).
int amdk8s_wan_rmsnorm_rope(void* t, long st, const float* w, const float* cs, const float* sn,
                            long rows, int L, int C, int hd, int nsec, float eps, hipStream_t s) {
  if (!amdk8s_wan_rms_supported(C, hd) || rows <= 0 || L <= 0 || nsec < 1 || nsec > 2) return -1;
  if (st % 8) return -3;
  uint16_t* tp = static_cast<uint16_t*>(t);
  switch (C / 512) {
    case 1: return launch_rms<1>(tp, st, w, cs, sn, rows, L, hd, nsec, eps, s);
    case 2: return launch_rms<2>(tp, st, w, cs, sn, rows, L, hd, nsec, eps, s);
    case 3: return launch_rms<3>(tp, st, w, cs, sn, rows, L, hd, nsec, eps, s);
    case 4: return launch_rms<4>(tp, st, w, cs, sn, rows, L, hd, nsec, eps, s);
    case 6: return launch_rms<6>(tp, st, w, cs, sn, rows, L, hd, nsec, eps, s);
    case 8: return launch_rms<8>(tp, st, w, cs, sn, rows, L, hd, nsec, eps, s);
    case 10: return launch_rms<10>(tp, st, w, cs, sn, rows, L, hd, nsec, eps, s);
    default: return -1;
  }
}

int amdk8s_wan_vae_supported(int C) { return (C == 96 || C == 192 || C == 384) ? 1 : 0; }

// x bf16 [pixels = B·T·hw, C] contiguous; gamma fp32 [C]; out bf16 [pixels, C] (kt 1) or
// [pixels, 3C] (kt 3, every element written).
int amdk8s_wan_vae_rms_silu_stack(const void* x, const float* gamma, void* out, long pixels, int hw,
                                  int T, int C, int kt, hipStream_t s) {
  if (!amdk8s_wan_vae_supported(C) || pixels <= 0 || hw <= 0 || T <= 0 || (kt != 1 && kt != 3) ||
      pixels % ((long)hw * T) != 0)
    return -1;
  const uint16_t* xp = static_cast<const uint16_t*>(x);
  uint16_t* op = static_cast<uint16_t*>(out);
  switch (C) {
    case 96: return launch_vae<3>(xp, gamma, op, pixels, hw, T, kt, s);
    case 192: return launch_vae<6>(xp, gamma, op, pixels, hw, T, kt, s);
    default: return launch_vae<12>(xp, gamma, op, pixels, hw, T, kt, s);
  }
}

}  // extern "C"
