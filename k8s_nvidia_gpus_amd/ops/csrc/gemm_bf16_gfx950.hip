// Hand-written bf16 MFMA GEMM for MI355X (gfx950, CDNA4).
//
//   C[M,N] (bf16) = A[M,K] (bf16, row-major) · B[N,K]ᵀ (bf16, row-major, i.e. "weight" layout)
//   fp32 accumulation in the MFMA accumulator file.
//
// This is the validator / benchmark GEMM that replaces the reference's dcgmproftester-style
// tensor-core load (BASELINE.json config 3).  The reference itself ships no
// kernels (its GPU code comes from pulled images, reference README.md:264-299), so everything here
// is designed for CDNA4 from first principles:
//
//   * 256×256×64 block tile, 512 threads = 8 waves arranged 2 (M) × 4 (N); each wave owns a
//     128×64 output sub-tile = 4 quadrants of 64×32, computed with v_mfma_f32_16x16x32_bf16
//     (16 MFMAs per quadrant per 64-deep K-tile).
//   * Operands are staged HBM→LDS with LDS-DMA (global_load_lds_dwordx4, 16 B per lane): no VGPR
//     round trip, no ds_write pass.  Each K-tile is split in four 16 KiB half-tiles (A rows 0-127,
//     A rows 128-255, B rows 0-127, B rows 128-255), double-buffered → 128 KiB of the 160 KiB LDS.
//   * The LDS image is XOR-swizzled so the ds_read_b128 fragment reads are bank-conflict free:
//     physical 16-B chunk = logical chunk ^ ((row >> 1) & 7) inside 128-B rows.  LDS-DMA writes
//     lane-linearly, so the permutation is applied to the per-lane GLOBAL source address and the
//     same involution on the read address.
//   * Phase schedule: 4 phases per K-tile, one per C quadrant.  Every phase is
//       LOAD segment (ds_read fragments + one half-tile of LDS-DMA prefetch) | s_barrier |
//       MFMA segment (16 MFMAs)                                            | s_barrier
//     and the two wave groups (waves 0-3 / 4-7, one of each per SIMD) run one segment apart
//     (a "stagger"), so on every SIMD one wave feeds the matrix pipe while its partner loads.
//   * Prefetch depth: a half-tile is refilled two phases after its last reader (the stagger needs
//     one extra phase of WAR distance) and is consumed 5-6 phases after issue.  One counted
//     `s_waitcnt vmcnt(8)` per phase (4 half-tiles × 2 DMA instructions left in flight) retires
//     exactly the half-tile the next phase reads; the loop never drains vmcnt to 0 except in the
//     last two K-tiles.
//   * XCD-aware block remap: blocks b and b+8 share an XCD (private 4 MiB L2), so each XCD gets a
//     contiguous chunk of a grouped (GROUP_M = 8) tile order and neighbouring tiles share A/B
//     panels in that XCD's L2.
//   * Epilogue: accumulators → bf16 → padded LDS image (528-B rows) → 16-B coalesced stores.
//
// Shape contract (checked on the host in amdk8s_gemm_bf16_nt): M % 256 == 0, N % 256 == 0,
// K % 64 == 0, leading dimensions multiples of 8 elements, 16-B aligned base pointers.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 64;
constexpr int NTHREADS = 512;
constexpr int HALF_BYTES = 128 * BK * 2;          // one half-tile: 128 rows × 128 B = 16 KiB
constexpr int TILE_BYTES = 4 * HALF_BYTES;        // A0 A1 B0 B1 = 64 KiB per buffer parity
constexpr int SLOT_A0 = 0 * HALF_BYTES;
constexpr int SLOT_A1 = 1 * HALF_BYTES;
constexpr int SLOT_B0 = 2 * HALF_BYTES;
constexpr int SLOT_B1 = 3 * HALF_BYTES;
constexpr int C_STRIDE = BN * 2 + 16;             // padded epilogue row (528 B)
constexpr int LDS_BYTES = BM * C_STRIDE;          // 135168 B ≥ 2 × TILE_BYTES (131072 B)
static_assert(LDS_BYTES >= 2 * TILE_BYTES, "LDS image too small");
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void barrier_raw() {
  // Raw s_barrier: no implicit vmcnt(0) (a __syncthreads() would drain the in-flight LDS-DMA
  // prefetch every phase).  sched_barrier(0) pins the segment structure for the scheduler.
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Issue one half-tile (128 rows × 64 k) of LDS-DMA: 2 instructions per thread, 1 KiB per wave each.
// `src` already points at this thread's swizzled source chunk of row (tid >> 3) of the half-tile.
__device__ __forceinline__ void stage_half(const char* src, size_t row64_bytes, char* lds_half,
                                           int wave) {
  __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds_half + wave * 1024), 16, 0, 0);
  __builtin_amdgcn_global_load_lds((const void*)(src + row64_bytes),
                                   (lds_void*)(lds_half + 8192 + wave * 1024), 16, 0, 0);
}

__device__ __forceinline__ bf16x8 lds_read16(const char* p) {
  return *reinterpret_cast<const bf16x8*>(__builtin_assume_aligned(p, 16));
}

}  // namespace

extern "C" __global__ void __launch_bounds__(NTHREADS)
amdk8s_gemm_bf16_nt_256x256(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                            uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                            int ldc) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2;  // 0..1  (M) — also the stagger group
  const int wc = wave & 3;   // 0..3  (N)

  // ---- block → tile (bijective XCD remap, then grouped order) ----
  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  int wgid;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int group = wgid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * GROUP_M * tiles_n;
  const int tm = first_m + in_group % gsz;
  const int tn = in_group / gsz;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  // ---- per-thread LDS-DMA source addresses (swizzle on the source side) ----
  const size_t lda_b = (size_t)lda * 2, ldb_b = (size_t)ldb * 2;
  const int srow = tid >> 3;                               // 0..63 (and +64 for the 2nd DMA)
  const int schunk = (tid & 7) ^ ((tid >> 4) & 7);         // logical chunk for physical tid&7
  const char* a_src = reinterpret_cast<const char*>(A) + (size_t)(m0 + srow) * lda_b + schunk * 16;
  const char* b_src = reinterpret_cast<const char*>(B) + (size_t)(n0 + srow) * ldb_b + schunk * 16;
  const size_t a_half1 = 128 * lda_b, b_half1 = 128 * ldb_b;
  const size_t a_r64 = 64 * lda_b, b_r64 = 64 * ldb_b;

  // ---- per-lane fragment read offsets (same swizzle on the read side) ----
  const int frow = lane & 15;
  const int fq = lane >> 4;
  const int foff0 = frow * 128 + (((0 + fq) ^ (frow >> 1)) << 4);
  const int foff1 = frow * 128 + (((4 + fq) ^ (frow >> 1)) << 4);
  const int a_wave_off = wr * 64 * 128;   // this wave's 64 rows inside an A half-tile
  const int b_wave_off = wc * 32 * 128;   // this wave's 32 rows inside a B half-tile

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < 2; ++l) acc[i][j][k][l] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2];
  bf16x8 bfr[2][2][2];

  const int T = K / BK;

  auto stage = [&](int slot, int t) {
    char* dst = lds + (t & 1) * TILE_BYTES + slot;
    const size_t kb = (size_t)t * BK * 2;
    if (slot == SLOT_A0) stage_half(a_src + kb, a_r64, dst, wave);
    else if (slot == SLOT_A1) stage_half(a_src + a_half1 + kb, a_r64, dst, wave);
    else if (slot == SLOT_B0) stage_half(b_src + kb, b_r64, dst, wave);
    else stage_half(b_src + b_half1 + kb, b_r64, dst, wave);
  };

  // ---- prologue: tile 0 complete + the first two half-tiles of tile 1 ----
  stage(SLOT_A0, 0);
  stage(SLOT_B0, 0);
  stage(SLOT_B1, 0);
  stage(SLOT_A1, 0);
  if (T > 1) {
    stage(SLOT_A0, 1);
    stage(SLOT_B0, 1);
    wait_vmcnt<8>();
  } else {
    wait_vmcnt<0>();
  }
  barrier_raw();
  if (wr == 1) barrier_raw();  // stagger: group 1 runs one segment behind group 0

#define AMDK8S_MFMA_QUAD(MQ, NQ)                                                              \
  _Pragma("unroll") for (int mt = 0; mt < 4; ++mt) {                                          \
    _Pragma("unroll") for (int nt = 0; nt < 2; ++nt) {                                        \
      acc[MQ][NQ][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                          \
          bfr[NQ][nt][0], af[mt][0], acc[MQ][NQ][mt][nt], 0, 0, 0);                           \
      acc[MQ][NQ][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                          \
          bfr[NQ][nt][1], af[mt][1], acc[MQ][NQ][mt][nt], 0, 0, 0);                           \
    }                                                                                         \
  }

  for (int t = 0; t < T; ++t) {
    const char* tb = lds + (t & 1) * TILE_BYTES;
    const bool steady = (t + 2 < T);

    // ---------------- phase 0: quadrant (m0, n0) ----------------
    {
      const char* pa = tb + SLOT_A0 + a_wave_off;
      const char* pb = tb + SLOT_B0 + b_wave_off;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        af[mt][0] = lds_read16(pa + mt * 2048 + foff0);
        af[mt][1] = lds_read16(pa + mt * 2048 + foff1);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        bfr[0][nt][0] = lds_read16(pb + nt * 2048 + foff0);
        bfr[0][nt][1] = lds_read16(pb + nt * 2048 + foff1);
      }
      if (t + 1 < T) stage(SLOT_B1, t + 1);
      if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();
      barrier_raw();
      __builtin_amdgcn_s_setprio(1);
      AMDK8S_MFMA_QUAD(0, 0)
      __builtin_amdgcn_s_setprio(0);
      barrier_raw();
    }
    // ---------------- phase 1: quadrant (m0, n1) ----------------
    {
      const char* pb = tb + SLOT_B1 + b_wave_off;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        bfr[1][nt][0] = lds_read16(pb + nt * 2048 + foff0);
        bfr[1][nt][1] = lds_read16(pb + nt * 2048 + foff1);
      }
      if (t + 1 < T) stage(SLOT_A1, t + 1);
      if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();
      barrier_raw();
      __builtin_amdgcn_s_setprio(1);
      AMDK8S_MFMA_QUAD(0, 1)
      __builtin_amdgcn_s_setprio(0);
      barrier_raw();
    }
    // ---------------- phase 2: quadrant (m1, n1) ----------------
    {
      const char* pa = tb + SLOT_A1 + a_wave_off;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        af[mt][0] = lds_read16(pa + mt * 2048 + foff0);
        af[mt][1] = lds_read16(pa + mt * 2048 + foff1);
      }
      if (t + 2 < T) stage(SLOT_A0, t + 2);
      if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();
      barrier_raw();
      __builtin_amdgcn_s_setprio(1);
      AMDK8S_MFMA_QUAD(1, 1)
      __builtin_amdgcn_s_setprio(0);
      barrier_raw();
    }
    // ---------------- phase 3: quadrant (m1, n0) — registers only ----------------
    {
      if (t + 2 < T) stage(SLOT_B0, t + 2);
      if (steady) wait_vmcnt<8>(); else wait_vmcnt<0>();
      barrier_raw();
      __builtin_amdgcn_s_setprio(1);
      AMDK8S_MFMA_QUAD(1, 0)
      __builtin_amdgcn_s_setprio(0);
      barrier_raw();
    }
  }
#undef AMDK8S_MFMA_QUAD
  if (wr == 0) barrier_raw();  // close the stagger: every wave has passed the same barrier count

  // ---- epilogue: acc → bf16 → LDS (padded rows) → coalesced 16-B global stores ----
  // Swapped-operand MFMA: lane holds C[m = .. + (lane & 15)][n = .. + 4*(lane >> 4) + i], i = 0..3.
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int m = mq * 128 + wr * 64 + mt * 16 + frow;
          const int n = nq * 128 + wc * 32 + nt * 16 + fq * 4;
          bf16x4 o = __builtin_convertvector(acc[mq][nq][mt][nt], bf16x4);
          *reinterpret_cast<bf16x4*>(lds + m * C_STRIDE + n * 2) = o;
        }
  __syncthreads();
  char* cbase = reinterpret_cast<char*>(C) + ((size_t)m0 * ldc + n0) * 2;
  const size_t ldc_b = (size_t)ldc * 2;
#pragma unroll 4
  for (int it = 0; it < BM * BN * 2 / (NTHREADS * 16); ++it) {
    const int row = it * 16 + (tid >> 5);
    const int ch = tid & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(lds + row * C_STRIDE + ch * 16);
    *reinterpret_cast<uint4*>(cbase + row * ldc_b + ch * 16) = v;
  }
}

// ------------------------------------------------------------------------------------------
// Sampled fp32 reference check (used by the standalone validator, which has no torch):
// out[s] = Σ_k A[m_s,k]·B[n_s,k] in fp32 for a list of sample coordinates.
extern "C" __global__ void amdk8s_gemm_bf16_nt_sample_ref(const uint16_t* __restrict__ A,
                                                          const uint16_t* __restrict__ B,
                                                          const int* __restrict__ coords,
                                                          float* __restrict__ out, int nsamples,
                                                          int K, int lda, int ldb) {
  const int s = blockIdx.x;
  if (s >= nsamples) return;
  const int m = coords[2 * s], n = coords[2 * s + 1];
  float sum = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float a = __uint_as_float((uint32_t)A[(size_t)m * lda + k] << 16);
    const float b = __uint_as_float((uint32_t)B[(size_t)n * ldb + k] << 16);
    sum = fmaf(a, b, sum);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_down(sum, off, 64);
  __shared__ float part[16];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < (int)(blockDim.x + 63) / 64; ++w) tot += part[w];
    out[s] = tot;
  }
}

// ------------------------------------------------------------------------------------------
// Host launch API (C ABI, called from Python through ctypes and from the native validator).
extern "C" int amdk8s_gemm_bf16_nt(const void* A, const void* B, void* C, int M, int N, int K,
                                   int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  if (lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return (int)hipErrorInvalidValue;
  const int nwg = (M / BM) * (N / BN);
  hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_256x256, dim3(nwg), dim3(NTHREADS), 0, stream,
                     (const uint16_t*)A, (const uint16_t*)B, (uint16_t*)C, M, N, K, lda, ldb, ldc);
  return (int)hipGetLastError();
}

extern "C" int amdk8s_gemm_bf16_nt_sample_check(const void* A, const void* B, const int* coords,
                                                float* out, int nsamples, int K, int lda, int ldb,
                                                hipStream_t stream) {
  if (nsamples <= 0) return 0;
  hipLaunchKernelGGL(amdk8s_gemm_bf16_nt_sample_ref, dim3(nsamples), dim3(256), 0, stream,
                     (const uint16_t*)A, (const uint16_t*)B, coords, out, nsamples, K, lda, ldb);
  return (int)hipGetLastError();
}
