// Load generators for the non-tensor pipes of an MI355X: HBM3E bandwidth (read / write / copy),
// fp32 vector FMA and fp64 MFMA throughput.
//
// These replace the remaining dcgmproftester targets of NVIDIA's operator stack (SURVEY.md §2.2 X5:
// "profiling load generator"; the tensor-pipe target is the bf16/fp8 MFMA GEMM of
// gemm_bf16_gfx950_w4a.hip / gemm_fp8_gfx950_f8a.hip).  dcgmproftester's DRAM-active, FP32-active
// and FP64-active loads become the three kernel families below; its PCIe and NVLink loads are host
// copies and peer copies in native/src/amd_proftester.hip (the peer copy can also run the copy
// kernel below over xGMI, with the source buffer on another GPU).
//
// Design for CDNA4 (gfx950):
//  * streaming kernels: one wave-instruction moves 1 KiB contiguous (16 B per lane), every lane
//    keeps UNROLL independent 16-B accesses in flight (blocks_per_cu × 4 waves × UNROLL KiB per
//    CU); the cache policy (non-temporal or not), the in-flight depth and the index layout are
//    template knobs, and amdk8s_hbm_stream runs the combination measured best per mode on
//    MI355X (see its comment).  Buffers must exceed ~512 MiB for the number to be HBM's and not
//    the 256 MiB Infinity Cache's.
//  * fp32: v_pk_fma_f32 (2 FMAs per lane per instruction, the instruction that reaches the
//    157 TF vector peak), 8 independent chains per lane so the ~4-cycle FMA latency is covered.
//  * fp64: v_mfma_f64_16x16x4_f64 with 4 independent AGPR/VGPR accumulators per wave.
//  * never zero data: the FMA chains start from per-lane hashed values and converge to a bounded
//    fixed point (|a| < 1), so the datapath toggles like real work (zero operands raise clocks:
//    cdna_hip_programming.md §5.4 rule 25).
// Each kernel keeps its result alive with a store that executes only for an impossible value, so
// the compiler cannot delete the work and nothing is written in practice.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(4))) double f64x4_t;

namespace {
constexpr int kThreads = 256;   // 4 wave64s per workgroup
constexpr uint32_t kNever = 0x7FC00001u;  // a quiet-NaN payload no XOR of the test data reaches

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  return x ^ (x >> 16);
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// HBM streaming kernels.  n16 = number of 16-byte words.  Template knobs (swept on MI355X with
// amdk8s_hbm_stream_variant, tools/hbm_sweep.py): non-temporal loads / stores and the number of
// independent 16-B accesses in flight per lane.
// ---------------------------------------------------------------------------------------------
template <bool NTL>
__device__ __forceinline__ u32x4_t ld16(const u32x4_t* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NTS>
__device__ __forceinline__ void st16(u32x4_t v, u32x4_t* p) {
  if constexpr (NTS) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Index space of one lane.  GRID (CHUNK = false): lane t of the whole grid touches t, t + S, …
// (S = grid threads), its U accesses per step S apart, so the chip sweeps one contiguous window.
// CHUNK: each workgroup owns one contiguous slice and walks it in steps of U KiB per wave.
template <bool CHUNK, int U>
struct Lanes {
  long i, end, step, ustride;
  __device__ __forceinline__ explicit Lanes(long n16) {
    if constexpr (CHUNK) {
      const long per = (long)kThreads * U;
      long chunk = (n16 + gridDim.x - 1) / gridDim.x;
      chunk = (chunk + per - 1) / per * per;
      i = (long)blockIdx.x * chunk + threadIdx.x;
      end = min(n16, (long)(blockIdx.x + 1) * chunk);
      step = per;
      ustride = kThreads;
    } else {
      ustride = (long)gridDim.x * kThreads;
      i = (long)blockIdx.x * kThreads + threadIdx.x;
      end = n16;
      step = U * ustride;
    }
  }
};

template <bool NTL, bool CHUNK, int U>
__global__ void __launch_bounds__(kThreads)
amdk8s_hbm_read_kernel(const u32x4_t* __restrict__ src, long n16, uint32_t* __restrict__ sink) {
  Lanes<CHUNK, U> l(n16);
  long i = l.i;
  u32x4_t acc = {0u, 0u, 0u, 0u};
  for (; i + (U - 1) * l.ustride < l.end; i += l.step) {
    u32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16<NTL>(&src[i + u * l.ustride]);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  for (; i < l.end; i += l.ustride) acc ^= ld16<NTL>(&src[i]);
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == kNever) sink[0] = x;
}

template <bool NTS, bool CHUNK, int U>
__global__ void __launch_bounds__(kThreads)
amdk8s_hbm_write_kernel(u32x4_t* __restrict__ dst, long n16, uint32_t seed) {
  Lanes<CHUNK, U> l(n16);
  long i = l.i;
  const uint32_t h = hash32(seed ^ (uint32_t)i);
  const u32x4_t v = {h, h ^ 0x55555555u, h ^ 0xAAAAAAAAu, ~h};  // non-zero, toggling pattern
  for (; i + (U - 1) * l.ustride < l.end; i += l.step) {
#pragma unroll
    for (int u = 0; u < U; ++u) st16<NTS>(v, &dst[i + u * l.ustride]);
  }
  for (; i < l.end; i += l.ustride) st16<NTS>(v, &dst[i]);
}

template <bool NTL, bool NTS, bool CHUNK, int U>
__global__ void __launch_bounds__(kThreads)
amdk8s_hbm_copy_kernel(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst, long n16) {
  Lanes<CHUNK, U> l(n16);
  long i = l.i;
  for (; i + (U - 1) * l.ustride < l.end; i += l.step) {
    u32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16<NTL>(&src[i + u * l.ustride]);
#pragma unroll
    for (int u = 0; u < U; ++u) st16<NTS>(v[u], &dst[i + u * l.ustride]);
  }
  for (; i < l.end; i += l.ustride) st16<NTS>(ld16<NTL>(&src[i]), &dst[i]);
}

namespace {
template <bool NTL, bool NTS, bool CHUNK, int U>
void launch_stream(int mode, const void* src, void* dst, long n16, int blocks, uint32_t* sink,
                   hipStream_t stream) {
  if (mode == 0)
    hipLaunchKernelGGL((amdk8s_hbm_read_kernel<NTL, CHUNK, U>), dim3(blocks), dim3(kThreads), 0,
                       stream, (const u32x4_t*)src, n16, sink);
  else if (mode == 1)
    hipLaunchKernelGGL((amdk8s_hbm_write_kernel<NTS, CHUNK, U>), dim3(blocks), dim3(kThreads), 0,
                       stream, (u32x4_t*)dst, n16, 0x1234567u);
  else
    hipLaunchKernelGGL((amdk8s_hbm_copy_kernel<NTL, NTS, CHUNK, U>), dim3(blocks), dim3(kThreads), 0,
                       stream, (const u32x4_t*)src, (u32x4_t*)dst, n16);
}

template <bool NTL, bool NTS, bool CHUNK>
bool dispatch_unroll(int unroll, int mode, const void* src, void* dst, long n16, int blocks,
                     uint32_t* sink, hipStream_t stream) {
  switch (unroll) {
    case 1: launch_stream<NTL, NTS, CHUNK, 1>(mode, src, dst, n16, blocks, sink, stream); return true;
    case 2: launch_stream<NTL, NTS, CHUNK, 2>(mode, src, dst, n16, blocks, sink, stream); return true;
    case 4: launch_stream<NTL, NTS, CHUNK, 4>(mode, src, dst, n16, blocks, sink, stream); return true;
    case 8: launch_stream<NTL, NTS, CHUNK, 8>(mode, src, dst, n16, blocks, sink, stream); return true;
    default: return false;
  }
}

template <bool NTL, bool NTS>
bool dispatch_layout(int chunked, int unroll, int mode, const void* src, void* dst, long n16,
                     int blocks, uint32_t* sink, hipStream_t stream) {
  return chunked ? dispatch_unroll<NTL, NTS, true>(unroll, mode, src, dst, n16, blocks, sink, stream)
                 : dispatch_unroll<NTL, NTS, false>(unroll, mode, src, dst, n16, blocks, sink, stream);
}
}  // namespace

// Sweep entry: mode 0 = read, 1 = write, 2 = copy; nt_load / nt_store select the cache policy,
// unroll ∈ {1, 2, 4, 8} the independent accesses per lane, blocks_per_cu the grid (× CUs), and
// chunked the index space (0 = grid-stride window, 1 = one contiguous slice per workgroup).
extern "C" int amdk8s_hbm_stream_variant(int mode, const void* src, void* dst, long bytes,
                                         int num_cus, int blocks_per_cu, int nt_load, int nt_store,
                                         int unroll, int chunked, uint32_t* sink,
                                         hipStream_t stream) {
  if (bytes <= 0 || (bytes & 15) || mode < 0 || mode > 2) return (int)hipErrorInvalidValue;
  if (((uintptr_t)src | (uintptr_t)dst) & 15) return (int)hipErrorInvalidValue;
  if ((mode != 1 && !src) || (mode != 0 && !dst) || (mode == 0 && !sink)) return (int)hipErrorInvalidValue;
  const long n16 = bytes / 16;
  const long per_block = (long)kThreads * (unroll > 0 ? unroll : 1);
  long blocks = (n16 + per_block - 1) / per_block;
  const long cap = (long)(num_cus > 0 ? num_cus : 256) * (blocks_per_cu > 0 ? blocks_per_cu : 8);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  bool ok;
  const int b = (int)blocks;
  if (nt_load && nt_store) ok = dispatch_layout<true, true>(chunked, unroll, mode, src, dst, n16, b, sink, stream);
  else if (nt_load) ok = dispatch_layout<true, false>(chunked, unroll, mode, src, dst, n16, b, sink, stream);
  else if (nt_store) ok = dispatch_layout<false, true>(chunked, unroll, mode, src, dst, n16, b, sink, stream);
  else ok = dispatch_layout<false, false>(chunked, unroll, mode, src, dst, n16, b, sink, stream);
  if (!ok) return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// Production entry (mode as above): per mode, the policy measured best on MI355X in
// tools/hbm_sweep.py (profiles/r02_session1/hbm_sweep*.txt; 2 GiB buffers, interleaved rounds):
//   read  nt loads, 1 access in flight per lane, 8 WG/CU, grid-stride window  ≈ 7.05-7.13 TB/s
//   write default-policy stores, 2 per lane, 8 WG/CU, contiguous slice per WG ≈ 5.87 TB/s
//   copy  nt loads + nt stores, 4 per lane, 8 WG/CU, contiguous slice per WG   ≈ 5.51 TB/s
// (of 8 TB/s peak).  blocks_per_cu > 0 overrides the grid of the chosen policy.
extern "C" int amdk8s_hbm_stream(int mode, const void* src, void* dst, long bytes, int num_cus,
                                 int blocks_per_cu, uint32_t* sink, hipStream_t stream) {
  struct Policy { int ntl, nts, unroll, bpc, chunked; };
  static const Policy kPolicy[3] = {{1, 0, 1, 8, 0}, {0, 0, 2, 8, 1}, {1, 1, 4, 8, 1}};
  if (mode < 0 || mode > 2) return (int)hipErrorInvalidValue;
  const Policy& p = kPolicy[mode];
  return amdk8s_hbm_stream_variant(mode, src, dst, bytes, num_cus,
                                   blocks_per_cu > 0 ? blocks_per_cu : p.bpc, p.ntl, p.nts, p.unroll,
                                   p.chunked, sink, stream);
}

// ---------------------------------------------------------------------------------------------
// fp32 vector FMA: 8 chains × v_pk_fma_f32 per lane per inner step = 32 FLOP per lane per
// instruction group of 8 (each v_pk_fma_f32 is 2 FMAs = 4 FLOP per lane).
// ---------------------------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(kThreads)
amdk8s_fp32_fma_kernel(int iters, float* __restrict__ sink) {
  const uint32_t tid = blockIdx.x * kThreads + threadIdx.x;
  // a in (0.5, 1): contraction → chains converge to b / (1 - a), bounded and non-zero
  const float a0 = 0.5f + (hash32(tid) >> 9) * (0.49f / 8388608.0f);
  const f32x2_t a = {a0, 0.999f - a0 * 0.25f};
  const f32x2_t b = {1e-3f, -2e-3f};
  f32x2_t c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t h = hash32(tid * 8u + j);
    c[j] = f32x2_t{(float)(h & 0xFFFF) * 1e-5f, (float)(h >> 16) * -1e-5f};
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        asm volatile("v_pk_fma_f32 %0, %1, %0, %2" : "+v"(c[j]) : "v"(a), "v"(b));
    }
  }
  f32x2_t s = c[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) s += c[j];
  if (__float_as_uint(s.x + s.y) == kNever) sink[0] = s.x;
}

// FLOP executed by one launch of amdk8s_fp32_fma (for the caller's TFLOPS arithmetic).
extern "C" double amdk8s_fp32_fma_flop(int blocks, int iters) {
  return (double)blocks * kThreads * iters * 4 /*r*/ * 8 /*chains*/ * 4 /*flop per pk_fma lane*/;
}

extern "C" int amdk8s_fp32_fma(int blocks, int iters, float* sink, hipStream_t stream) {
  if (blocks <= 0 || iters <= 0 || !sink) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(amdk8s_fp32_fma_kernel, dim3(blocks), dim3(kThreads), 0, stream, iters, sink);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// fp64 matrix: v_mfma_f64_16x16x4_f64 (2 048 FLOP per wave-instruction), 4 independent
// accumulators per wave, 4 MFMAs per accumulator per iteration.
// ---------------------------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(kThreads)
amdk8s_fp64_mfma_kernel(int iters, double* __restrict__ sink) {
  const uint32_t tid = blockIdx.x * kThreads + threadIdx.x;
  // |a·b| summed over K = 4 stays < 1 per step: the accumulators stay bounded
  const double a = 0.25 * (0.5 + (hash32(tid) >> 8) * (0.5 / 16777216.0));
  const double b = -0.25 * (0.5 + (hash32(tid ^ 0x9E3779B9u) >> 8) * (0.5 / 16777216.0));
  f64x4_t c[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double v = (double)(hash32(tid * 4u + j) & 0xFFFF) * 1e-6;
    c[j] = f64x4_t{v, -v, 0.5 * v, 1e-3};
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
    }
  }
  f64x4_t s = c[0] + c[1] + c[2] + c[3];
  const double t = s.x + s.y + s.z + s.w;
  if (t == 12345.678) sink[0] = t;
}

extern "C" double amdk8s_fp64_mfma_flop(int blocks, int iters) {
  // per wave: iters × 16 MFMAs × 16·16·4·2 FLOP; 4 waves per block
  return (double)blocks * (kThreads / 64) * iters * 16.0 * (16 * 16 * 4 * 2);
}

extern "C" int amdk8s_fp64_mfma(int blocks, int iters, double* sink, hipStream_t stream) {
  if (blocks <= 0 || iters <= 0 || !sink) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(amdk8s_fp64_mfma_kernel, dim3(blocks), dim3(kThreads), 0, stream, iters, sink);
  return (int)hipGetLastError();
}
