// Device-side synthetic data fill (counter-based hash → uniform [lo, hi) → bf16).
//
// Benchmarks must run on random data, not zeros: on gfx950 zero-filled MFMA operands let the chip
// hold a higher clock and inflate GEMM TFLOPS by ~15-20 % (cdna_hip_programming.md §5.4 rule 25).
// Filling on the device keeps multi-GiB operand setup out of host memory and PCIe.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
}  // namespace

extern "C" __global__ void __launch_bounds__(256)
amdk8s_fill_uniform_bf16_kernel(uint16_t* __restrict__ dst, long n, uint64_t seed, float lo,
                                float scale) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t h = splitmix64(seed ^ (uint64_t)i * 0xD1B54A32D192ED03ull);
    const float u = (float)(h >> 40) * (1.0f / 16777216.0f);  // [0, 1)
    const float v = lo + u * scale;
    // round-to-nearest-even to bf16 (v is finite by construction)
    const uint32_t bits = __float_as_uint(v);
    dst[i] = (uint16_t)((bits + 0x7FFFu + ((bits >> 16) & 1u)) >> 16);
  }
}

extern "C" int amdk8s_fill_uniform_bf16(void* dst, long n, unsigned long long seed, float lo,
                                        float hi, hipStream_t stream) {
  if (n <= 0) return (int)hipErrorInvalidValue;
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(amdk8s_fill_uniform_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     (uint16_t*)dst, n, (uint64_t)seed, lo, hi - lo);
  return (int)hipGetLastError();
}

// Same stream of uniform values, rounded to OCP fp8 e4m3 by gfx950's v_cvt_pk_fp8_f32 (round to
// nearest even, saturating): four values per thread-iteration, one 32-bit store.
extern "C" __global__ void __launch_bounds__(256)
amdk8s_fill_uniform_fp8_kernel(uint32_t* __restrict__ dst, long n4, uint64_t seed, float lo,
                               float scale) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t h = splitmix64(seed ^ (uint64_t)(4 * i + j) * 0xD1B54A32D192ED03ull);
      v[j] = lo + (float)(h >> 40) * (1.0f / 16777216.0f) * scale;
    }
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w, true);
    dst[i] = (uint32_t)w;
  }
}

extern "C" int amdk8s_fill_uniform_fp8(void* dst, long n, unsigned long long seed, float lo,
                                       float hi, hipStream_t stream) {
  if (n <= 0 || n % 4) return (int)hipErrorInvalidValue;
  const long n4 = n / 4;
  long blocks = (n4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(amdk8s_fill_uniform_fp8_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     (uint32_t*)dst, n4, (uint64_t)seed, lo, hi - lo);
  return (int)hipGetLastError();
}
