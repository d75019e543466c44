// HIP vectorAdd for MI355X — the validator's first GPU check.
//
// Behavioural parity target: the reference validates the cluster with NVIDIA's cuda-sample
// vectorAdd (reference README.md:264-299): 50 000 fp32 elements, ⌈50000/256⌉ = 196 blocks of
// 256 threads, host-side verification, "Test PASSED" / "Done".  The functional kernel below keeps
// that exact launch shape (256 threads = 4 wave64s per block) so log checks carry over.
//
// A second, bandwidth-shaped kernel (16 B per lane, grid-stride, ~8 blocks per CU) is used by the
// validator to report achieved HBM bandwidth on the same op — the exact-shape kernel is a
// functional probe, not a bandwidth test.
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __global__ void __launch_bounds__(256)
amdk8s_vector_add_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                             float* __restrict__ c, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = a[i] + b[i];
}

typedef __attribute__((ext_vector_type(4))) float f32x4_t;

extern "C" __global__ void __launch_bounds__(256)
amdk8s_vector_add_f32x4_kernel(const f32x4_t* __restrict__ a, const f32x4_t* __restrict__ b,
                               f32x4_t* __restrict__ c, long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4_t x = __builtin_nontemporal_load(&a[i]);
    const f32x4_t y = __builtin_nontemporal_load(&b[i]);
    __builtin_nontemporal_store(x + y, &c[i]);
  }
}

// Same launch shape as the reference sample: 256 threads per block, ceil(n / 256) blocks.
extern "C" int amdk8s_vector_add_f32(const float* a, const float* b, float* c, int n,
                                     hipStream_t stream) {
  if (n <= 0) return (int)hipErrorInvalidValue;
  const int threads = 256;
  const int blocks = (n + threads - 1) / threads;
  hipLaunchKernelGGL(amdk8s_vector_add_f32_kernel, dim3(blocks), dim3(threads), 0, stream, a, b, c, n);
  return (int)hipGetLastError();
}

// Bandwidth form; n must be a multiple of 4 and the pointers 16-B aligned.
extern "C" int amdk8s_vector_add_f32_bw(const float* a, const float* b, float* c, long n,
                                        int num_cus, hipStream_t stream) {
  if (n <= 0 || (n & 3)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15) return (int)hipErrorInvalidValue;
  const long n4 = n / 4;
  const int threads = 256;
  long blocks = (n4 + threads - 1) / threads;
  const long cap = (long)(num_cus > 0 ? num_cus : 256) * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(amdk8s_vector_add_f32x4_kernel, dim3((unsigned)blocks), dim3(threads), 0,
                     stream, (const f32x4_t*)a, (const f32x4_t*)b, (f32x4_t*)c, n4);
  return (int)hipGetLastError();
}

// Launch-shape helper for the validator protocol line.
extern "C" int amdk8s_vector_add_blocks(int n) { return (n + 255) / 256; }
