// GroupNorm (+ fused SiLU) over channels-last activations, and GEGLU, for the SD1.5 model family
// (k8s_nvidia_gpus_amd/models/sd15).  gfx950, wave64, fp16 / bf16 storage, fp32 maths.
//
// GroupNorm on NHWC memory ([N, HW, C] rows): a group is Cg = C/G adjacent channels of every pixel,
// so a 16-byte vector of 8 channels touches at most two groups (Cg >= 4 is required; SD1.5 has
// Cg = 4..80).  Each thread owns ONE fixed 8-channel vector column (vc) and walks rows, so rows are
// read fully coalesced (C*2 bytes contiguous per pixel) and the per-thread group split is a compile-
// free constant.  Two launches:
//   1. gn_partial: blocks = N x (<= 16 chunks).  Per (n, chunk, group): count / mean / M2 in fp32
//      (per-thread sums over a few rows, then a tree reduction over the block's row slots).
//   2. gn_apply: every block first merges its image's chunk partials (LDS, Chan's parallel-variance
//      formula) into (mean, rstd) per group — no block publishes stats to another, so there is no
//      inter-block fence (on MI355X an agent-scope fence writes back L2 across the 8 XCDs) and
//      nothing to reset between calls — then y = x * a_c + b_c (a_c = rstd*w_c, b_c = bias_c -
//      mean*a_c, per thread in registers), optional SiLU, 16-byte stores.
// Deterministic: no atomics anywhere.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace {

constexpr int kMaxThreads = 1024;
constexpr int kMaxChunks = 16;  // stats-pass chunks per image (merged by every apply block)

// AMDK8S_GN_CHUNKS overrides kMaxChunks (A/B: more, shorter stats blocks vs a longer merge).
int max_chunks() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("AMDK8S_GN_CHUNKS");
    const int c = e ? atoi(e) : 0;
    v = (c >= 1 && c <= 256) ? c : kMaxChunks;
  }
  return v;
}

__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return 0x7fc0u;  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

template <bool BF16>
__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (BF16) {
      f[2 * i] = bf16_to_f32(w[i] & 0xffffu);
      f[2 * i + 1] = bf16_to_f32(w[i] >> 16);
    } else {
      _Float16 lo, hi;
      uint16_t l = w[i] & 0xffffu, h = w[i] >> 16;
      __builtin_memcpy(&lo, &l, 2);
      __builtin_memcpy(&hi, &h, 2);
      f[2 * i] = (float)lo;
      f[2 * i + 1] = (float)hi;
    }
  }
}

template <bool BF16>
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (BF16) {
      w[i] = f32_to_bf16(f[2 * i]) | (f32_to_bf16(f[2 * i + 1]) << 16);
    } else {
      _Float16 lo = (_Float16)f[2 * i], hi = (_Float16)f[2 * i + 1];
      uint16_t l, h;
      __builtin_memcpy(&l, &lo, 2);
      __builtin_memcpy(&h, &hi, 2);
      w[i] = (uint32_t)l | ((uint32_t)h << 16);
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <bool BF16>
__device__ __forceinline__ float load_scalar(const uint16_t* p, int i) {
  uint32_t h = p[i];
  if constexpr (BF16) {
    return bf16_to_f32(h);
  } else {
    _Float16 x;
    uint16_t b = (uint16_t)h;
    __builtin_memcpy(&x, &b, 2);
    return (float)x;
  }
}

struct GnShape {
  int N, HW, C, G, Cg, VC, R;  // VC = C/8 vector columns, R = rows in flight per block (per pass)
  int chunks1, rows1;          // stats pass: chunks per image, rows per chunk
  int chunks2, rows2;          // apply pass
};

// Partial layout: part[((n * chunks1 + chunk) * G + g) * 3 + {count, mean, M2}]
template <bool BF16>
__global__ void gn_partial(const uint16_t* __restrict__ x, const uint16_t* __restrict__ add,
                           long add_stride, float* __restrict__ part, GnShape s) {
  const int tid = threadIdx.x;
  const int chunk = blockIdx.x, n = blockIdx.y;
  const int vc = tid % s.VC, r = tid / s.VC;
  const int c0 = vc * 8;
  const int g_lo = c0 / s.Cg;
  const int split = min(8, (g_lo + 1) * s.Cg - c0);  // elements [0, split) are in g_lo
  const int row0 = chunk * s.rows1, row1 = min(s.HW, row0 + s.rows1);
  float s_lo = 0.f, q_lo = 0.f, s_hi = 0.f, q_hi = 0.f;
  float ad[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (add) unpack8<BF16>(*reinterpret_cast<const uint4*>(add + n * add_stride + c0), ad);
  const uint16_t* base = x + ((size_t)n * s.HW) * s.C + c0;
#pragma unroll 8
  for (int row = row0 + r; row < row1; row += s.R) {
    const uint4 v = *reinterpret_cast<const uint4*>(base + (size_t)row * s.C);
    float f[8];
    unpack8<BF16>(v, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f[i] += ad[i];
      if (i < split) {
        s_lo += f[i];
        q_lo += f[i] * f[i];
      } else {
        s_hi += f[i];
        q_hi += f[i] * f[i];
      }
    }
  }
  // in-block reduction, deterministic: [R][VC][4] in LDS, row 0 sums over r, then one thread per group
  extern __shared__ float lds[];
  float* red = lds;  // R * VC * 4
  red[(r * s.VC + vc) * 4 + 0] = s_lo;
  red[(r * s.VC + vc) * 4 + 1] = q_lo;
  red[(r * s.VC + vc) * 4 + 2] = s_hi;
  red[(r * s.VC + vc) * 4 + 3] = q_hi;
  __syncthreads();
  // tree over the R row-slots (log2 R dependent steps instead of R)
  int span = 1;
  while (span < s.R) span <<= 1;
  for (int st = span >> 1; st > 0; st >>= 1) {
    if (r < st && r + st < s.R) {
#pragma unroll
      for (int k = 0; k < 4; ++k) red[(r * s.VC + vc) * 4 + k] += red[((r + st) * s.VC + vc) * 4 + k];
    }
    __syncthreads();
  }
  const int rows_in_chunk = max(0, row1 - row0);
  for (int g = tid; g < s.G; g += blockDim.x) {
    const int cbeg = g * s.Cg, cend = cbeg + s.Cg;  // [cbeg, cend)
    float sum = 0.f, sq = 0.f;
    for (int v = cbeg / 8; v <= (cend - 1) / 8; ++v) {
      const int vlo = v * 8 / s.Cg;  // group of the vector's first element
      if (vlo == g) {
        sum += red[v * 4 + 0];
        sq += red[v * 4 + 1];
      } else {
        sum += red[v * 4 + 2];
        sq += red[v * 4 + 3];
      }
    }
    const float cnt = (float)rows_in_chunk * (float)s.Cg;
    const float mean = cnt > 0.f ? sum / cnt : 0.f;
    const float m2 = cnt > 0.f ? fmaxf(sq - sum * mean, 0.f) : 0.f;
    float* p = part + (((size_t)n * s.chunks1 + chunk) * s.G + g) * 3;
    p[0] = cnt;
    p[1] = mean;
    p[2] = m2;
  }
}

template <bool BF16, bool SILU>
__global__ void gn_apply(const uint16_t* __restrict__ x, const uint16_t* __restrict__ add,
                         long add_stride, uint16_t* __restrict__ y,
                         const uint16_t* __restrict__ w, const uint16_t* __restrict__ b,
                         const float* __restrict__ part, int chunks1, float eps, GnShape s) {
  const int tid = threadIdx.x;
  // prologue: this image's chunk partials → LDS (coalesced), then per-group Chan merge.  Every
  // block redoes this small merge (chunks1 * G * 3 floats, L2-resident) instead of any block
  // publishing stats to the others: no inter-block fences (cross-XCD L2 writeback) and no tickets.
  extern __shared__ float lds[];
  float* pl = lds;                           // [chunks1][G][3]
  float2* st = reinterpret_cast<float2*>(lds + ((chunks1 * s.G * 3 + 1) & ~1));  // [G]
  const float* pn = part + (size_t)blockIdx.y * chunks1 * s.G * 3;
  for (int i = tid; i < chunks1 * s.G * 3; i += blockDim.x) pl[i] = pn[i];
  __syncthreads();
  // (group, sub) threads each merge a strided subset of the chunks, then one thread per group
  // merges the nsub results: two short serial chains instead of one chunks1-long one
  const int nsub = max(1, min((int)blockDim.x / s.G, chunks1));
  float* mg = lds + ((chunks1 * s.G * 3 + 1) & ~1) + 2 * s.G;  // [nsub][G][3]
  if (tid < nsub * s.G) {
    const int g = tid % s.G, sub = tid / s.G;
    float cnt = 0.f, mean = 0.f, m2 = 0.f;
    for (int k = sub; k < chunks1; k += nsub) {
      const float cb = pl[(k * s.G + g) * 3 + 0];
      const float tot = cnt + cb;
      const float f = cb > 0.f ? cb / tot : 0.f;
      const float d = pl[(k * s.G + g) * 3 + 1] - mean;
      mean += d * f;
      m2 += pl[(k * s.G + g) * 3 + 2] + d * d * cnt * f;
      cnt = tot;
    }
    mg[(sub * s.G + g) * 3 + 0] = cnt;
    mg[(sub * s.G + g) * 3 + 1] = mean;
    mg[(sub * s.G + g) * 3 + 2] = m2;
  }
  __syncthreads();
  for (int g = tid; g < s.G; g += blockDim.x) {
    float cnt = 0.f, mean = 0.f, m2 = 0.f;
    for (int k = 0; k < nsub; ++k) {
      const float cb = mg[(k * s.G + g) * 3 + 0];
      const float tot = cnt + cb;
      const float f = cb > 0.f ? cb / tot : 0.f;
      const float d = mg[(k * s.G + g) * 3 + 1] - mean;
      mean += d * f;
      m2 += mg[(k * s.G + g) * 3 + 2] + d * d * cnt * f;
      cnt = tot;
    }
    st[g] = make_float2(mean, rsqrtf((cnt > 0.f ? m2 / cnt : 0.f) + eps));
  }
  __syncthreads();
  const int chunk = blockIdx.x, n = blockIdx.y;
  const int vc = tid % s.VC, r = tid / s.VC;
  const int c0 = vc * 8;
  float a[8], sh[8], wv[8], bv[8], av[8];
  unpack8<BF16>(*reinterpret_cast<const uint4*>(w + c0), wv);
  unpack8<BF16>(*reinterpret_cast<const uint4*>(b + c0), bv);
  if (add)
    unpack8<BF16>(*reinterpret_cast<const uint4*>(add + n * add_stride + c0), av);
  const int g_lo = c0 / s.Cg, g_hi = (c0 + 7) / s.Cg;  // at most two groups per vector
  const float2 st_lo = st[g_lo];
  const float2 st_hi = st[g_hi];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool lo = (c0 + i) / s.Cg == g_lo;
    const float mean = lo ? st_lo.x : st_hi.x, rstd = lo ? st_lo.y : st_hi.y;
    a[i] = rstd * wv[i];
    // (x + add) * a + b - mean * a: the per-(n, c) addend folds into the shift
    sh[i] = bv[i] - mean * a[i] + (add ? av[i] * a[i] : 0.f);
  }
  const int row0 = chunk * s.rows2, row1 = min(s.HW, row0 + s.rows2);
  const size_t off = ((size_t)n * s.HW) * s.C + c0;
#pragma unroll 8
  for (int row = row0 + r; row < row1; row += s.R) {
    const size_t o = off + (size_t)row * s.C;
    const uint4 v = *reinterpret_cast<const uint4*>(x + o);
    float f[8];
    unpack8<BF16>(v, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float t = f[i] * a[i] + sh[i];
      if constexpr (SILU) t = t / (1.f + __expf(-t));
      f[i] = t;
    }
    *reinterpret_cast<uint4*>(y + o) = pack8<BF16>(f);
  }
}

// GEGLU: x [M, 2D] -> out [M, D], out = h * gelu_erf(g), x = [h | g]
template <bool BF16>
__global__ void geglu_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ out, long M,
                             int D) {
  const int DV = D / 8;
  const long total = M * DV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long m = i / DV;
    const int j = (int)(i - m * DV) * 8;
    const uint16_t* row = x + m * 2L * D;
    float h[8], g[8];
    unpack8<BF16>(*reinterpret_cast<const uint4*>(row + j), h);
    unpack8<BF16>(*reinterpret_cast<const uint4*>(row + D + j), g);
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] *= 0.5f * g[k] * (1.f + erff(g[k] * 0.70710678118654752f));
    *reinterpret_cast<uint4*>(out + m * (long)D + j) = pack8<BF16>(h);
  }
}

// out[m, c] = a[m, c] + b[m, c] (+ bias[c]) over [M, C] rows (C % 8 == 0): the ResNet block's
// residual add with the convolution bias folded in (one pass instead of bias kernel + add kernel)
template <bool BF16>
__global__ void add3_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                            const uint16_t* __restrict__ bias, uint16_t* __restrict__ out, long M,
                            int C) {
  const int CV = C / 8;
  const long total = M * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % CV) * 8;
    float fa[8], fb[8];
    unpack8<BF16>(reinterpret_cast<const uint4*>(a)[i], fa);
    unpack8<BF16>(reinterpret_cast<const uint4*>(b)[i], fb);
    if (bias) {
      float fc[8];
      unpack8<BF16>(*reinterpret_cast<const uint4*>(bias + c0), fc);
#pragma unroll
      for (int k = 0; k < 8; ++k) fa[k] += fc[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) fa[k] += fb[k];
    reinterpret_cast<uint4*>(out)[i] = pack8<BF16>(fa);
  }
}

// LayerNorm over rows of C channels (C % 8 == 0, C <= 64*8*kLnVec), one wave per row, values held
// in registers between the mean and the variance pass (exact two-pass variance).  With `delta`
// it is the transformer block's residual add fused in front: xs = x + delta is written out (the
// next residual) and y = LN(xs).
constexpr int kLnVec = 4;  // 16-byte vectors per lane: C <= 2048

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <bool BF16, bool DELTA>
__global__ __launch_bounds__(256) void add_layernorm_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ delta, uint16_t* __restrict__ xs,
    uint16_t* __restrict__ y, const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ beta,
    long M, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;  // whole waves only: the row is wave-uniform
  const int CV = C / 8;
  const size_t base = (size_t)row * C;
  float v[kLnVec][8];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < kLnVec; ++k) {
    const int vi = lane + 64 * k;
    if (vi < CV) {
      unpack8<BF16>(*reinterpret_cast<const uint4*>(x + base + vi * 8), v[k]);
      if constexpr (DELTA) {
        float dl[8];
        unpack8<BF16>(*reinterpret_cast<const uint4*>(delta + base + vi * 8), dl);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[k][e] += dl[e];
        *reinterpret_cast<uint4*>(xs + base + vi * 8) = pack8<BF16>(v[k]);
        unpack8<BF16>(pack8<BF16>(v[k]), v[k]);  // normalise exactly what the residual stores
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += v[k][e];
    }
  }
  const float mean = wave_sum(sum) / C;
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < kLnVec; ++k) {
    if (lane + 64 * k < CV) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dd = v[k][e] - mean;
        sq += dd * dd;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / C + eps);
#pragma unroll
  for (int k = 0; k < kLnVec; ++k) {
    const int vi = lane + 64 * k;
    if (vi < CV) {
      float gm[8], bt[8], o[8];
      unpack8<BF16>(*reinterpret_cast<const uint4*>(gamma + vi * 8), gm);
      unpack8<BF16>(*reinterpret_cast<const uint4*>(beta + vi * 8), bt);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[k][e] - mean) * rstd * gm[e] + bt[e];
      *reinterpret_cast<uint4*>(y + base + vi * 8) = pack8<BF16>(o);
    }
  }
}

// ---- single-launch GroupNorm for small images --------------------------------------------------
// Every launch of this stack costs ~4.5 us of device time whatever it does (profiles/r03/z), so
// the two-launch form above spends most of its ~17 us on two floors at the UNet's sizes.  Here a
// block owns a GROUP SET — lcm(Cg, 8) channels, i.e. whole groups AND whole 16-byte vectors — of one
// image, so no block needs another's statistics: it walks the set's rows once for the sums (same
// per-thread vector-column scheme and in-block tree as gn_partial), turns them into (mean, rstd)
// per group in LDS, and walks the rows again for the apply (L1 / L2-warm).  Used when a set's rows
// are small (gn_fused_ok); the VAE's 512² activations keep the two-launch form.
struct GnSet {
  int N, HW, C, G, Cg, VS, GS, R;   // VS vectors / GS groups per set, R row slots per block
};

template <bool BF16, bool SILU>
__global__ void gn_fused(const uint16_t* __restrict__ x, const uint16_t* __restrict__ add,
                         long add_stride, uint16_t* __restrict__ y, const uint16_t* __restrict__ w,
                         const uint16_t* __restrict__ b, float eps, GnSet s) {
  const int set = blockIdx.x, n = blockIdx.y, tid = threadIdx.x;
  const int vs = tid % s.VS, r = tid / s.VS;
  const int c0 = (set * s.VS + vs) * 8;
  const int g_lo = c0 / s.Cg, g_hi = (c0 + 7) / s.Cg;
  const int split = min(8, (g_lo + 1) * s.Cg - c0);  // elements [0, split) are in g_lo
  float ad[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (add) unpack8<BF16>(*reinterpret_cast<const uint4*>(add + n * add_stride + c0), ad);
  const size_t off = ((size_t)n * s.HW) * s.C + c0;
  float s_lo = 0.f, q_lo = 0.f, s_hi = 0.f, q_hi = 0.f;
  if (r < s.R) {
#pragma unroll 8
    for (int row = r; row < s.HW; row += s.R) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + off + (size_t)row * s.C);
      float f[8];
      unpack8<BF16>(v, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f[i] += ad[i];
        if (i < split) {
          s_lo += f[i];
          q_lo += f[i] * f[i];
        } else {
          s_hi += f[i];
          q_hi += f[i] * f[i];
        }
      }
    }
  }
  // per thread (count, mean, M2) for its lo / hi group part, then Chan merges over the row slots
  // and the set's vectors: no sum-of-squares cancellation at large means (a group's sum of squares
  // over a whole 64x64 image would lose the variance in fp32)
  extern __shared__ float lds[];
  float* red = lds;                                    // [R][VS][6]: lo (n, mean, m2), hi (...)
  float2* st = reinterpret_cast<float2*>(lds + ((s.R * s.VS * 6 + 1) & ~1));   // [GS]
  {
    const int rows_t = r < s.R ? (s.HW - r + s.R - 1) / s.R : 0;
    const float n_lo = (float)(rows_t * split), n_hi = (float)(rows_t * (8 - split));
    const float m_lo = n_lo > 0.f ? s_lo / n_lo : 0.f, m_hi = n_hi > 0.f ? s_hi / n_hi : 0.f;
    float* e = red + (r * s.VS + vs) * 6;
    e[0] = n_lo; e[1] = m_lo; e[2] = fmaxf(q_lo - s_lo * m_lo, 0.f);
    e[3] = n_hi; e[4] = m_hi; e[5] = fmaxf(q_hi - s_hi * m_hi, 0.f);
  }
  __syncthreads();
  auto chan = [](float* a, const float* b) {           // a <- merge(a, b) for (n, mean, m2)
    const float n = a[0] + b[0];
    if (b[0] > 0.f) {
      const float d = b[1] - a[1], f = b[0] / n;
      a[1] += d * f;
      a[2] += b[2] + d * d * a[0] * f;
      a[0] = n;
    }
  };
  int span = 1;
  while (span < s.R) span <<= 1;
  for (int stp = span >> 1; stp > 0; stp >>= 1) {     // tree over the row slots
    if (r < stp && r + stp < s.R) {
      float* e = red + (r * s.VS + vs) * 6;
      const float* o = red + ((r + stp) * s.VS + vs) * 6;
      chan(e, o);
      chan(e + 3, o + 3);
    }
    __syncthreads();
  }
  for (int gg = tid; gg < s.GS; gg += blockDim.x) {
    const int g = set * s.GS + gg;
    const int cbeg = g * s.Cg, cend = cbeg + s.Cg;
    float acc[3] = {0.f, 0.f, 0.f};
    for (int v = cbeg / 8; v <= (cend - 1) / 8; ++v) {
      const int lv = v - set * s.VS;
      chan(acc, red + lv * 6 + (v * 8 / s.Cg == g ? 0 : 3));
    }
    st[gg] = make_float2(acc[1], rsqrtf((acc[0] > 0.f ? acc[2] / acc[0] : 0.f) + eps));
  }
  __syncthreads();
  if (r >= s.R) return;
  float a[8], sh[8], wv[8], bv[8];
  unpack8<BF16>(*reinterpret_cast<const uint4*>(w + c0), wv);
  unpack8<BF16>(*reinterpret_cast<const uint4*>(b + c0), bv);
  const float2 st_lo = st[g_lo - set * s.GS];
  const float2 st_hi = st[g_hi - set * s.GS];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool lo = (c0 + i) / s.Cg == g_lo;
    const float mean = lo ? st_lo.x : st_hi.x, rstd = lo ? st_lo.y : st_hi.y;
    a[i] = rstd * wv[i];
    sh[i] = bv[i] - mean * a[i] + (add ? ad[i] * a[i] : 0.f);
  }
#pragma unroll 8
  for (int row = r; row < s.HW; row += s.R) {
    const size_t o = off + (size_t)row * s.C;
    const uint4 v = *reinterpret_cast<const uint4*>(x + o);
    float f[8];
    unpack8<BF16>(v, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float t = f[i] * a[i] + sh[i];
      if constexpr (SILU) t = t / (1.f + __expf(-t));
      f[i] = t;
    }
    *reinterpret_cast<uint4*>(y + o) = pack8<BF16>(f);
  }
}

int gcd_int(int a, int b) { return b == 0 ? a : gcd_int(b, a % b); }

GnSet gn_set_shape(int N, int HW, int C, int G) {
  GnSet s{};
  s.N = N; s.HW = HW; s.C = C; s.G = G; s.Cg = C / G;
  const int set = s.Cg / gcd_int(s.Cg, 8) * 8;       // lcm(Cg, 8) channels
  s.VS = set / 8;
  s.GS = set / s.Cg;
  s.R = 1024 / s.VS;
  if (s.R > HW) s.R = HW;
  return s;
}

// AMDK8S_GN_FUSED=0 keeps the two-launch form everywhere (A/B); otherwise a set's rows up to
// AMDK8S_GN_FUSED_KB (default 128 KB: the UNet levels up to 32², 6.58 -> 6.55 ms against 64 KB,
// profiles/r03/am) and at least 8 blocks use
// gn_fused.  At 384 KB (every UNet GroupNorm at 512²) the 64² ones ran on 16 blocks and the pass
// got slower (6.74 -> 6.94 ms, profiles/r03/ak): one CU cannot stream a set's rows fast enough.
int g_gn_fused_force = -1;                  // amdk8s_groupnorm_set_fused (tests / A/B)

bool gn_fused_ok(int N, int HW, int C, int G) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("AMDK8S_GN_FUSED");
    v = e ? atoi(e) : 1;
  }
  if (!(g_gn_fused_force >= 0 ? g_gn_fused_force : v)) return false;
  static long kb = -1;
  if (kb < 0) {
    const char* e = getenv("AMDK8S_GN_FUSED_KB");
    kb = e ? atol(e) : 128;
  }
  const GnSet s = gn_set_shape(N, HW, C, G);
  if (C % (s.VS * 8) || s.VS > 64) return false;
  if (g_gn_fused_force == 2) return true;            // every supported shape (tests)
  return (long)HW * s.VS * 16 <= kb * 1024 && N * (C / (s.VS * 8)) >= 8;
}

// pass = 1: stats pass shape; pass = 2: apply pass shape
GnShape gn_shape(int N, int HW, int C, int G, int pass) {
  GnShape s{};
  s.N = N;
  s.HW = HW;
  s.C = C;
  s.G = G;
  s.Cg = C / G;
  s.VC = C / 8;
  if (pass == 1) {
    // stats: ~1024-thread blocks, <= kMaxChunks chunks per image (every apply block merges them)
    s.R = s.VC >= 1024 ? 1 : 1024 / s.VC;
    if (s.R > HW) s.R = HW;
    int chunks = (HW + s.R - 1) / s.R;
    if (chunks > max_chunks()) chunks = max_chunks();
    s.rows1 = (HW + chunks - 1) / chunks;
    s.chunks1 = (HW + s.rows1 - 1) / s.rows1;
  } else {
    // apply: ~256-thread blocks, 8 rows per thread (unrolled loads)
    s.R = s.VC >= 256 ? 1 : 256 / s.VC;
    if (s.R > HW) s.R = HW;
    s.rows2 = s.R * 8;
    s.chunks2 = (HW + s.rows2 - 1) / s.rows2;
  }
  return s;
}

// Every 16-byte vector of 8 channels must touch at most two groups (the per-thread split).
bool gn_supported(int C, int G) {
  if (C <= 0 || G <= 0 || G > 128 || C % 8 != 0 || C % G != 0 || C / 8 > kMaxThreads) return false;
  const int Cg = C / G;
  for (int c0 = 0; c0 < C; c0 += 8)
    if ((c0 + 7) / Cg - c0 / Cg > 1) return false;
  return true;
}

}  // namespace

extern "C" {

int amdk8s_groupnorm_supported(int C, int G) { return gn_supported(C, G) ? 1 : 0; }

// 1 / 0: single-launch GroupNorm where it applies / never; 2: wherever the shape allows (tests);
// -1: AMDK8S_GN_FUSED (default on).
void amdk8s_groupnorm_set_fused(int v) { g_gn_fused_force = v; }

// Workspace floats needed by amdk8s_groupnorm_nhwc (the stats pass's chunk partials).
long amdk8s_groupnorm_workspace(int N, int HW, int C, int G) {
  GnShape s = gn_shape(N, HW, C, G, 1);
  return (long)N * s.chunks1 * G * 3;
}

// y = GroupNorm(x) * w + b (optionally SiLU), x/y [N, HW, C] (channels-last), w/b [C].
// dtype: 0 = fp16, 1 = bf16.
// add (nullable): per-(n, c) addend [N, C] with row stride add_stride: y = GroupNorm(x + add[n, c])
int amdk8s_groupnorm_nhwc(const void* x, const void* add, long add_stride, void* y, const void* w,
                          const void* b, float* workspace, int N, int HW, int C, int G, float eps,
                          int silu, int dtype, hipStream_t stream) {
  if (N <= 0 || HW <= 0 || !gn_supported(C, G)) return -1;
  if (gn_fused_ok(N, HW, C, G)) {
    const GnSet fs = gn_set_shape(N, HW, C, G);
    const dim3 grid(C / (fs.VS * 8), N), block(fs.VS * fs.R);
    const size_t lds = ((size_t)((fs.R * fs.VS * 6 + 1) & ~1) + 2 * fs.GS) * sizeof(float);
    const auto* xi = static_cast<const uint16_t*>(x);
    const auto* ai = static_cast<const uint16_t*>(add);
    auto* yo = static_cast<uint16_t*>(y);
    const auto* wi = static_cast<const uint16_t*>(w);
    const auto* bi = static_cast<const uint16_t*>(b);
    if (dtype == 1 && silu)
      hipLaunchKernelGGL((gn_fused<true, true>), grid, block, lds, stream, xi, ai, add_stride, yo, wi, bi, eps, fs);
    else if (dtype == 1)
      hipLaunchKernelGGL((gn_fused<true, false>), grid, block, lds, stream, xi, ai, add_stride, yo, wi, bi, eps, fs);
    else if (silu)
      hipLaunchKernelGGL((gn_fused<false, true>), grid, block, lds, stream, xi, ai, add_stride, yo, wi, bi, eps, fs);
    else
      hipLaunchKernelGGL((gn_fused<false, false>), grid, block, lds, stream, xi, ai, add_stride, yo, wi, bi, eps, fs);
    return hipGetLastError() == hipSuccess ? 0 : -2;
  }
  GnShape s = gn_shape(N, HW, C, G, 1);
  GnShape s2 = gn_shape(N, HW, C, G, 2);
  const int threads = s.VC * s.R, threads2 = s2.VC * s2.R;
  const size_t lds1 = (size_t)s.R * s.VC * 4 * sizeof(float);
  const int nsub2 = threads2 / G > 0 ? (threads2 / G < s.chunks1 ? threads2 / G : s.chunks1) : 1;
  const size_t lds2 =
      ((size_t)((s.chunks1 * G * 3 + 1) & ~1) + 2 * G + (size_t)nsub2 * G * 3) * sizeof(float);
  const auto* xi = static_cast<const uint16_t*>(x);
  const auto* ai = static_cast<const uint16_t*>(add);
  auto* yo = static_cast<uint16_t*>(y);
  const auto* wi = static_cast<const uint16_t*>(w);
  const auto* bi = static_cast<const uint16_t*>(b);
  dim3 g1(s.chunks1, N), g2(s2.chunks2, N);
  const int c1 = s.chunks1;
  if (dtype == 1) {
    hipLaunchKernelGGL(gn_partial<true>, g1, dim3(threads), lds1, stream, xi, ai, add_stride, workspace, s);
    if (silu)
      hipLaunchKernelGGL((gn_apply<true, true>), g2, dim3(threads2), lds2, stream, xi, ai, add_stride, yo, wi, bi, workspace, c1, eps, s2);
    else
      hipLaunchKernelGGL((gn_apply<true, false>), g2, dim3(threads2), lds2, stream, xi, ai, add_stride, yo, wi, bi, workspace, c1, eps, s2);
  } else {
    hipLaunchKernelGGL(gn_partial<false>, g1, dim3(threads), lds1, stream, xi, ai, add_stride, workspace, s);
    if (silu)
      hipLaunchKernelGGL((gn_apply<false, true>), g2, dim3(threads2), lds2, stream, xi, ai, add_stride, yo, wi, bi, workspace, c1, eps, s2);
    else
      hipLaunchKernelGGL((gn_apply<false, false>), g2, dim3(threads2), lds2, stream, xi, ai, add_stride, yo, wi, bi, workspace, c1, eps, s2);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int amdk8s_geglu(const void* x, void* out, long M, int D, int dtype, hipStream_t stream) {
  if (M <= 0 || D % 8 != 0) return -1;
  const long vecs = M * (D / 8);
  long blocks = (vecs + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  const auto* xi = static_cast<const uint16_t*>(x);
  auto* o = static_cast<uint16_t*>(out);
  if (dtype == 1)
    hipLaunchKernelGGL(geglu_kernel<true>, dim3(blocks), dim3(256), 0, stream, xi, o, M, D);
  else
    hipLaunchKernelGGL(geglu_kernel<false>, dim3(blocks), dim3(256), 0, stream, xi, o, M, D);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// y = LayerNorm(x (+ delta)) over [M, C] rows; with delta, xs = x + delta is stored too.
int amdk8s_add_layernorm(const void* x, const void* delta, void* xs, void* y, const void* gamma,
                         const void* beta, long M, int C, float eps, int dtype, hipStream_t stream) {
  if (M <= 0 || C % 8 != 0 || C / 8 > 64 * kLnVec) return -1;
  const dim3 grid((unsigned)((M + 3) / 4)), block(256);
  const auto* xi = static_cast<const uint16_t*>(x);
  const auto* di = static_cast<const uint16_t*>(delta);
  auto* so = static_cast<uint16_t*>(xs);
  auto* yo = static_cast<uint16_t*>(y);
  const auto* gi = static_cast<const uint16_t*>(gamma);
  const auto* bi = static_cast<const uint16_t*>(beta);
  if (dtype == 1) {
    if (delta)
      hipLaunchKernelGGL((add_layernorm_kernel<true, true>), grid, block, 0, stream, xi, di, so, yo, gi, bi, M, C, eps);
    else
      hipLaunchKernelGGL((add_layernorm_kernel<true, false>), grid, block, 0, stream, xi, di, so, yo, gi, bi, M, C, eps);
  } else {
    if (delta)
      hipLaunchKernelGGL((add_layernorm_kernel<false, true>), grid, block, 0, stream, xi, di, so, yo, gi, bi, M, C, eps);
    else
      hipLaunchKernelGGL((add_layernorm_kernel<false, false>), grid, block, 0, stream, xi, di, so, yo, gi, bi, M, C, eps);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int amdk8s_add3(const void* a, const void* b, const void* bias, void* out, long M, int C, int dtype,
                hipStream_t stream) {
  if (M <= 0 || C % 8 != 0) return -1;
  long blocks = (M * (C / 8) + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  const auto* ai = static_cast<const uint16_t*>(a);
  const auto* bi = static_cast<const uint16_t*>(b);
  const auto* ci = static_cast<const uint16_t*>(bias);
  auto* o = static_cast<uint16_t*>(out);
  if (dtype == 1)
    hipLaunchKernelGGL(add3_kernel<true>, dim3(blocks), dim3(256), 0, stream, ai, bi, ci, o, M, C);
  else
    hipLaunchKernelGGL(add3_kernel<false>, dim3(blocks), dim3(256), 0, stream, ai, bi, ci, o, M, C);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
