// Can a consumer kernel start before its producer finishes on MI355X, and does that hide the
// ~4.5 us per-kernel floor of the LLM decode chain (docs/llm_decode.md)?
//
//   A  two streams: consumer (256 workgroups, bounded spin on a flag) launched first on s2, producer
//      (1 workgroup, 50 us delay, then flag = 1) on s1.  All consumers see the flag <=> the two
//      queues run concurrently.
//   B  the same inside one captured HIP graph (fork s1 -> s2, join back).
//   C  a chain of 64 dependent pairs (producer: 256 workgroups write + count arrivals; consumer:
//      256 workgroups read): serial launches in one stream vs the consumer of each pair forked on a
//      second stream and waiting on the arrival counter — both captured in a graph, us per pair.
//
// Every spin gives up after 2 ms of s_memrealtime (100 MHz) and records the failure, so a runtime
// that serialises the branches ends with "gave up", never a hang.  Flags use agent-scope atomic
// loads / stores on the vector path.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/debug/overlap_probe tools/debug/overlap_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr unsigned long kGiveUpTicks = 200000;  // 2 ms at 100 MHz

__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

// returns spins (>= 0) or -1 after the give-up time
__device__ int wait_ge(const unsigned* p, unsigned target) {
  const unsigned long t0 = __builtin_amdgcn_s_memrealtime();
  int spins = 0;
  while (ld_flag(p) < target) {
    __builtin_amdgcn_s_sleep(2);
    ++spins;
    if (__builtin_amdgcn_s_memrealtime() - t0 > kGiveUpTicks) return -1;
  }
  return spins;
}

__global__ void producer_delay(unsigned* flag, unsigned ticks) {
  if (threadIdx.x == 0) {
    const unsigned long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void consumer_wait(const unsigned* flag, unsigned target, int* res) {
  if (threadIdx.x == 0) res[blockIdx.x] = wait_ge(flag, target);
}

// chain: producer writes data[blk] and arrives; consumer waits for all arrivals (when counter is
// non-null), then reads every producer's value.
__global__ void chain_producer(float* data, unsigned* counter, int step) {
  if (threadIdx.x == 0) {
    data[blockIdx.x] = (float)(step + blockIdx.x);
    if (counter) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void chain_consumer(const float* data, const unsigned* counter, unsigned target,
                               float* sink, int* fail) {
  __shared__ int ok;
  if (threadIdx.x == 0) ok = counter ? wait_ge(counter, target) >= 0 : 1;
  __syncthreads();
  if (!ok) {
    if (threadIdx.x == 0) fail[0] = 1;
    return;
  }
  float s = 0.f;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s += data[i];
  if (threadIdx.x == 0) sink[blockIdx.x] = s;
}

int main() {
  unsigned *flag, *counter;
  int *res, *fail;
  float *data, *sink;
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&counter, 4));
  CK(hipMalloc(&res, 256 * 4));
  CK(hipMalloc(&fail, 4));
  CK(hipMalloc(&data, 256 * 4));
  CK(hipMalloc(&sink, 256 * 4));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  int h[256];

  // A: two streams, consumer first
  CK(hipMemset(flag, 0, 4));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(consumer_wait, dim3(256), dim3(64), 0, s2, flag, 1u, res);
  hipLaunchKernelGGL(producer_delay, dim3(1), dim3(64), 0, s1, flag, 5000u);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h, res, sizeof h, hipMemcpyDeviceToHost));
  int seen = 0, mx = 0;
  for (int i = 0; i < 256; ++i) seen += h[i] >= 0, mx = h[i] > mx ? h[i] : mx;
  printf("A streams: %d/256 consumers saw the flag (max spins %d)\n", seen, mx);

  // B: one graph, forked branch
  hipEvent_t ef, ej;
  CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
  CK(hipMemsetAsync(flag, 0, 4, s1));
  CK(hipEventRecord(ef, s1));
  CK(hipStreamWaitEvent(s2, ef, 0));
  hipLaunchKernelGGL(consumer_wait, dim3(256), dim3(64), 0, s2, flag, 1u, res);
  hipLaunchKernelGGL(producer_delay, dim3(1), dim3(64), 0, s1, flag, 5000u);
  CK(hipEventRecord(ej, s2));
  CK(hipStreamWaitEvent(s1, ej, 0));
  CK(hipStreamEndCapture(s1, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < 3; ++r) {
    CK(hipGraphLaunch(ge, s1));
    CK(hipStreamSynchronize(s1));
    CK(hipMemcpy(h, res, sizeof h, hipMemcpyDeviceToHost));
    seen = 0;
    for (int i = 0; i < 256; ++i) seen += h[i] >= 0;
    printf("B graph run %d: %d/256 consumers saw the flag\n", r, seen);
  }

  // C: 64 dependent pairs, serial vs forked consumers
  constexpr int kPairs = 64;
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  hipEvent_t fk[kPairs], jn[kPairs];
  for (int i = 0; i < kPairs; ++i) {
    CK(hipEventCreateWithFlags(&fk[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&jn[i], hipEventDisableTiming));
  }
  for (int mode = 0; mode < 2; ++mode) {
    hipGraph_t gc;
    hipGraphExec_t gce;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    CK(hipMemsetAsync(counter, 0, 4, s1));
    CK(hipMemsetAsync(fail, 0, 4, s1));
    for (int i = 0; i < kPairs; ++i) {
      if (mode == 0) {
        hipLaunchKernelGGL(chain_producer, dim3(256), dim3(64), 0, s1, data, (unsigned*)nullptr, i);
        hipLaunchKernelGGL(chain_consumer, dim3(256), dim3(64), 0, s1, data,
                           (const unsigned*)nullptr, 0u, sink, fail);
      } else {
        // the consumer of pair i forks off before its producer and joins before pair i + 1
        CK(hipEventRecord(fk[i], s1));
        CK(hipStreamWaitEvent(s2, fk[i], 0));
        hipLaunchKernelGGL(chain_consumer, dim3(256), dim3(64), 0, s2, data, counter,
                           256u * (i + 1), sink, fail);
        hipLaunchKernelGGL(chain_producer, dim3(256), dim3(64), 0, s1, data, counter, i);
        CK(hipEventRecord(jn[i], s2));
        CK(hipStreamWaitEvent(s1, jn[i], 0));
      }
    }
    CK(hipStreamEndCapture(s1, &gc));
    CK(hipGraphInstantiate(&gce, gc, nullptr, nullptr, 0));
    CK(hipGraphLaunch(gce, s1));
    CK(hipStreamSynchronize(s1));
    const int reps = 20;
    CK(hipEventRecord(t0, s1));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(gce, s1));
    CK(hipEventRecord(t1, s1));
    CK(hipEventSynchronize(t1));
    float ms;
    CK(hipEventElapsedTime(&ms, t0, t1));
    int hf;
    CK(hipMemcpy(&hf, fail, 4, hipMemcpyDeviceToHost));
    printf("C %s: %.2f us per producer/consumer pair%s\n",
           mode ? "forked consumers" : "serial launches", ms * 1e3 / reps / kPairs,
           hf ? " (a consumer gave up)" : "");
    CK(hipGraphExecDestroy(gce));
    CK(hipGraphDestroy(gc));
  }
  CK(hipDeviceSynchronize());
  return 0;
}
