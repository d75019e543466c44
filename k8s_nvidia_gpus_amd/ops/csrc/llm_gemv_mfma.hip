// Quantised GEMVs of the LLM decode step on the int8 matrix cores (gfx950): the MFMA-packed weight
// planes, qgemv_mfma_kernel / qgemv2_mfma_kernel and their launchers.  Shared definitions:
// llm_common.h; the VALU GEMV, attention and norm kernels: llm_decode.hip; measurements:
// docs/llm_decode.md ("Round 4: the GEMVs on the int8 matrix cores").
#include "llm_common.h"

namespace {

// ---------------------------------------------------------------- MFMA GEMV (int8 matrix cores)
// The VALU GEMV (llm_decode.hip) spends ~90 VALU per lane and super-block at T = 4 (eight v_dot4 plus the
// scale arithmetic per token on top of the weight decode), which makes steps of 2-4 tokens
// VALU-bound (profiles/r04/f: gate|up 30 µs at T = 4 vs 20 µs at T = 1).  Here the integer
// sub-block sums come from v_mfma_i32_16x16x64_i8 and only the per-sub-block scaling stays on the
// VALU, once per (row, token, sub-block) instead of once per weight byte.
//
// Geometry: one wave = 16 weight rows (the MFMA's N) × a range of super-blocks; lane l loads row
// l & 15, K-group g = l >> 4 (Q4_K: nibble bytes 16g.. of each 64-byte half of the super-block, so
// each load instruction reads 64 contiguous bytes per row).  M = 16 = (token t, slot s): A row
// (t, s) carries token t's activations in K-group s only (zeros in the other three), so output
// (t, s) of row r is the sum over K-group s alone, and every K-group's 16 values of one MFMA lie in
// one sub-block.  Four MFMAs per super-block leave lane l = (row l & 15, token l >> 4) with the
// sub-block sums of its own row and token (mfma_block).  Each lane then scales its own
// (row, token) in a fixed order, so a token's bits never depend on how many tokens share the
// launch (batch-invariant).  Steps of 5-8 tokens run a second token quad against the same weight
// registers.  Super-blocks are split over KW waves (reduced in LDS in wave order); RG row groups
// per workgroup; the shape is a function of the matrix only (mfma_shape).
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// split-K default for K >= 8192 (ffn_down): K-waves per workgroup and slices per row tile.
// Measured and left off (SK 1): at T = 1 every split lost to the unsplit 8-wave shape — Q4_K
// ffn_down 10.8 us unsplit vs 12.1 (4 waves x 2 slices) .. 22.5 us (8 x 4), Q6_K 14.3 vs 15.8 ..
// 27.7 us, and the whole step 1.62 -> 1.79 ms with 4 x 4 (profiles/r05/gemv_split_k.log): the
// write-through partials, the ticket and the last slice's sc1 re-read cost more than the idle
// CUs of the 224-tile grid.  The combine stays for A/B sweeps (ksplit > 1).
#ifndef AMDK8S_SPLIT_KW
#define AMDK8S_SPLIT_KW 8
#endif
#ifndef AMDK8S_SPLIT_SK
#define AMDK8S_SPLIT_SK 1
#endif
constexpr int kSplitKW = AMDK8S_SPLIT_KW, kSplitSK = AMDK8S_SPLIT_SK;
// Wave partials are summed in groups of this many waves (then the group sums in order): the
// unsplit 8-wave ffn_down of 1-4 tokens and its 2-slice x 4-wave form for 5-8 tokens (one pass
// over the weights; their activations do not fit one workgroup's LDS) then add the same numbers
// in the same order — decode stays batch-invariant.
constexpr int kRedGroup = 4;

// The MFMA kernel reads an MFMA-packed copy of the planes (amdk8s_llm_mfma_pack), laid out per
// (16-row group G, super-block b) so that each of a wave's loads per block reads whole contiguous
// lines instead of a 64/16/4-byte piece of 16 different rows:
//   Q4_K: q [2][16 rows][64 B] (bytes 64h.. of each row's nibbles), sc [16][4] dwords, d [16] dwords
//   Q6_K: ql as Q4_K's q, qh [2][16][32 B], sc [16][16] int8 in natural order, d [16] dwords (f16)
template <int TYPE> struct MBlk;
template <> struct MBlk<kQ4K> { uint4 q0, q1, sc; uint32_t dd; };
template <> struct MBlk<kQ6K> { uint4 q0, q1, h0, h1, sc; uint32_t dd; };

// POL 0: non-temporal loads (a weight read once per step); 1: default policy, so the bytes stay
// in the Infinity Cache for a second launch that reads the same weights right after (the 5-8
// token ffn_down's second token quad)
template <int POL>
__device__ __forceinline__ uint4 wld(const void* p) {
  if constexpr (POL == 0) return ldnt(p);
  else return *reinterpret_cast<const uint4*>(p);
}

template <int TYPE, int POL = 0>
__device__ __forceinline__ void mload(const QMat& w, long gb, int lane, MBlk<TYPE>& r) {
  const int row = lane & 15, g = lane >> 4;
  const uint8_t* q = w.q + gb * 2048 + row * 64 + g * 16;
  r.q0 = wld<POL>(q);
  r.q1 = wld<POL>(q + 1024);
  if constexpr (TYPE == kQ6K) {
    const uint8_t* h = w.qh + gb * 1024 + row * 32 + (g & 1) * 16;
    r.h0 = wld<POL>(h);
    r.h1 = wld<POL>(h + 512);
    r.sc = wld<POL>(reinterpret_cast<const uint8_t*>(w.sc) + gb * 256 + row * 16);
  } else {
    r.sc = wld<POL>(reinterpret_cast<const uint32_t*>(w.sc) + gb * 64 + row * 4);
  }
  const uint32_t* dp = reinterpret_cast<const uint32_t*>(w.d) + gb * 16 + row;
  if constexpr (POL == 0) r.dd = __builtin_nontemporal_load(dp);
  else r.dd = *dp;
}

__device__ __forceinline__ i32x4 nib_lo(const uint4& v) {
  const uint32_t m = 0x0f0f0f0fu;
  return i32x4{(int)(v.x & m), (int)(v.y & m), (int)(v.z & m), (int)(v.w & m)};
}
__device__ __forceinline__ i32x4 nib_hi(const uint4& v) {
  const uint32_t m = 0x0f0f0f0fu;
  return i32x4{(int)((v.x >> 4) & m), (int)((v.y >> 4) & m), (int)((v.z >> 4) & m),
               (int)((v.w >> 4) & m)};
}
// Q6_K: 6-bit values (0..63) of 4 bytes — low / high nibbles of q with the 2-bit fields at bit k /
// k + 4 of each qh byte as bits 4-5
__device__ __forceinline__ uint32_t q6lo(uint32_t q, uint32_t h, int k) {
  return (q & 0x0f0f0f0fu) | (((h >> k) << 4) & 0x30303030u);
}
__device__ __forceinline__ uint32_t q6hi(uint32_t q, uint32_t h, int k) {
  return ((q >> 4) & 0x0f0f0f0fu) | ((h >> k) & 0x30303030u);
}

// acc += this lane's (row, token) share of one super-block.
// Q4_K: K-group g holds bytes 16g.. of each 64-byte half (q0: chunks 0-1, q1: chunks 2-3), so in
//   MFMA m (0: q0 low nibbles, 1: q0 high, 2: q1 low, 3: q1 high) groups 2h and 2h + 1 carry the
//   two 16-value halves of sub-block 2(2(m >> 1) + h) + (m & 1): c[2h] + c[2h + 1] is that
//   sub-block.  acc += d * sum_j sc_j dx_j I_j - dmin * sum_j m_j sxp_j (aux = sxp, the dx-scaled
//   sums of x per 32).
// Q6_K: group g holds values 16g.. of each 64 (bytes 16g.. of the ql halves, qh fields of
//   "l" / "32 + l" by g >> 1), so c_m[s] is the 16-value sub-block 4m + s.  Integer per 32-value
//   pair: S = sc_j (I_j - 32 X_j) + sc_j+1 (I_j+1 - 32 X_j+1) (aux = X, the int sums of x per 16),
//   then acc += d * sum_i dx_i S_i.
template <int TYPE>
__device__ __forceinline__ float mfma_block(const MBlk<TYPE>& w, const i32x4 (&xa)[4],
                                            const float (&dxv)[8], const uint4 (&aux)[4], int g,
                                            float acc) {
  const i32x4 z = {0, 0, 0, 0};
  if constexpr (TYPE == kQ4K) {
    const i32x4 c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[0], nib_lo(w.q0), z, 0, 0, 0);
    const i32x4 c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[1], nib_hi(w.q0), z, 0, 0, 0);
    const i32x4 c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[2], nib_lo(w.q1), z, 0, 0, 0);
    const i32x4 c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[3], nib_hi(w.q1), z, 0, 0, 0);
    const int I[8] = {c0[0] + c0[1], c1[0] + c1[1], c0[2] + c0[3], c1[2] + c1[3],
                      c2[0] + c2[1], c3[0] + c3[1], c2[2] + c2[3], c3[2] + c3[3]};
    const float spv[8] = {__uint_as_float(aux[0].x), __uint_as_float(aux[0].y),
                          __uint_as_float(aux[0].z), __uint_as_float(aux[0].w),
                          __uint_as_float(aux[1].x), __uint_as_float(aux[1].y),
                          __uint_as_float(aux[1].z), __uint_as_float(aux[1].w)};
    const uint32_t scw[4] = {w.sc.x, w.sc.y, w.sc.z, w.sc.w};
    // even / odd sub-blocks in the two halves of packed-fp32 registers (v_pk_mul_f32 /
    // v_pk_fma_f32: half the scaling instructions), added at the end in a fixed order
    f32x2 sm = {0.f, 0.f}, mn = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x2 sc2 = {(float)(scw[i] & 0xffu), (float)((scw[i] >> 8) & 0xffu)};
      const f32x2 m2 = {(float)((scw[i] >> 16) & 0xffu), (float)(scw[i] >> 24)};
      const f32x2 i2 = {(float)I[2 * i], (float)I[2 * i + 1]};
      const f32x2 dx2 = {dxv[2 * i], dxv[2 * i + 1]};
      const f32x2 sp2 = {spv[2 * i], spv[2 * i + 1]};
      sm = __builtin_elementwise_fma(i2, sc2 * dx2, sm);
      mn = __builtin_elementwise_fma(m2, sp2, mn);
    }
    acc = __fmaf_rn(h2f(w.dd & 0xffffu), __fadd_rn(sm.x, sm.y), acc);
    return __fmaf_rn(-h2f(w.dd >> 16), __fadd_rn(mn.x, mn.y), acc);
  } else {
    const int k = 2 * (g >> 1);
    const uint4 q0 = w.q0, q1 = w.q1, h0 = w.h0, h1 = w.h1;
    const i32x4 b0 = {(int)q6lo(q0.x, h0.x, k), (int)q6lo(q0.y, h0.y, k), (int)q6lo(q0.z, h0.z, k),
                      (int)q6lo(q0.w, h0.w, k)};
    const i32x4 b1 = {(int)q6hi(q0.x, h0.x, k), (int)q6hi(q0.y, h0.y, k), (int)q6hi(q0.z, h0.z, k),
                      (int)q6hi(q0.w, h0.w, k)};
    const i32x4 b2 = {(int)q6lo(q1.x, h1.x, k), (int)q6lo(q1.y, h1.y, k), (int)q6lo(q1.z, h1.z, k),
                      (int)q6lo(q1.w, h1.w, k)};
    const i32x4 b3 = {(int)q6hi(q1.x, h1.x, k), (int)q6hi(q1.y, h1.y, k), (int)q6hi(q1.z, h1.z, k),
                      (int)q6hi(q1.w, h1.w, k)};
    const i32x4 c[4] = {__builtin_amdgcn_mfma_i32_16x16x64_i8(xa[0], b0, z, 0, 0, 0),
                        __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[1], b1, z, 0, 0, 0),
                        __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[2], b2, z, 0, 0, 0),
                        __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[3], b3, z, 0, 0, 0)};
    const uint32_t X[16] = {aux[0].x, aux[0].y, aux[0].z, aux[0].w, aux[1].x, aux[1].y,
                            aux[1].z, aux[1].w, aux[2].x, aux[2].y, aux[2].z, aux[2].w,
                            aux[3].x, aux[3].y, aux[3].z, aux[3].w};
    const uint32_t scw[4] = {w.sc.x, w.sc.y, w.sc.z, w.sc.w};
    float blk = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int j = 4 * m + 2 * pr;                 // sub-blocks j, j + 1: 32-group j / 2
        const int s0 = (int)(int8_t)((scw[j >> 2] >> (8 * (j & 3))) & 0xffu);
        const int s1 = (int)(int8_t)((scw[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 0xffu);
        const int i0 = c[m][2 * pr] - 32 * (int)X[j];
        const int i1 = c[m][2 * pr + 1] - 32 * (int)X[j + 1];
        blk = __fmaf_rn((float)(s0 * i0 + s1 * i1), dxv[j >> 1], blk);
      }
    }
    return __fmaf_rn(h2f(w.dd & 0xffffu), blk, acc);
  }
}

// LDS after stage_x's arrays: [W][T] prologue scratch (rounded to 16 B), the per-type activation
// sums (Q4_K sxp float [T][K/32], Q6_K X int [T][K/16]), 256 zero bytes (the A operand of
// inactive lanes), the K-split partials [waves][token quads][P][64], q8s [T][32].
// K here is the staged window's (the whole row, or one split-K slice's super-blocks); flag: the
// split-K ticket a workgroup draws, broadcast through LDS (one __shared__ array for everything).
struct MfmaLds { int aux, zero, kred, q8s, flag, total; };
__host__ __device__ inline MfmaLds mfma_lds(int type, int T, int K, int waves, int P) {
  MfmaLds L;
  const int nb = K >> 8;
  const int base = T * (nb * 288 + (K >> 5) * 4 + (K >> 4) * 4);
  const int red = ((waves * T * 4) + 15) & ~15;
  L.aux = base + red;
  L.zero = L.aux + T * (type == kQ6K ? K >> 4 : K >> 5) * 4;
  L.kred = L.zero + 256;
  L.q8s = L.kred + waves * ((T + 3) / 4) * P * 64 * 4;
  L.flag = L.q8s + T * 32 * 4;
  L.total = L.flag + 16;
  return L;
}

// SX layout: [waves][2 slots][T x (288 + 32 + na x 16) + 256 zero bytes] activation rings, then
// as mfma_lds from the (unused) zero bytes on (aux unused)
__host__ __device__ inline MfmaLds mfma_lds_sx(int T, int na, int waves, int P) {
  MfmaLds L;
  L.aux = 0;
  L.zero = waves * 2 * (T * (320 + na * 16) + 256);
  L.kred = L.zero + 256;
  L.q8s = L.kred + waves * ((T + 3) / 4) * P * 64 * 4;
  L.flag = L.q8s + T * 32 * 4;
  L.total = L.flag + 16;
  return L;
}

// Q8 activations of super-blocks [kb_lo, kb_lo + nbw) staged as stage_x stages a whole row, with
// local block indices (the window of one split-K workgroup): 16-byte units, four per thread per
// round, every load of a round issued before its LDS stores.  Ends with a barrier.
template <int T>
__device__ __forceinline__ XView stage_x8_window(const GemvArgs& a, uint8_t* lds, int kb_lo,
                                                 int nbw) {
  const int K = a.K, Kw = nbw << 8, upt = Kw >> 4;
  const int xstride = nbw * 288;
  int8_t* xs = reinterpret_cast<int8_t*>(lds);
  float* dxs = reinterpret_cast<float*>(lds + T * xstride);
  float* sxs = dxs + T * (Kw >> 5);
  const int nx = T * upt;
  for (int i0 = threadIdx.x; i0 < nx; i0 += 4 * (int)blockDim.x) {
    uint4 xv[4];
    float dv[4], sv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(i0 + u * (int)blockDim.x, nx - 1);
      const int t = i / upt, j = i - t * upt;
      const long gi = (long)t * (K >> 4) + kb_lo * 16 + j;
      xv[u] = *reinterpret_cast<const uint4*>(a.x8 + gi * 16);
      sv[u] = a.sx[gi];
      dv[u] = a.dx[(long)t * (K >> 5) + kb_lo * 8 + (j >> 1)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * (int)blockDim.x;
      if (i < nx) {
        const int t = i / upt, j = i - t * upt;
        *reinterpret_cast<uint4*>(xs + t * xstride + xoff(j << 4)) = xv[u];
        sxs[t * upt + j] = sv[u];
        if ((j & 1) == 0) dxs[t * (Kw >> 5) + (j >> 1)] = dv[u];
      }
    }
  }
  __syncthreads();
  return XView{xs, dxs, sxs, xstride, Kw >> 5, Kw >> 4};
}

// gate|up (pair, <= 4 tokens): 592 4-wave workgroups need 3 waves per SIMD to be co-resident
// bid = the workgroup's index within this matrix's grid
// SX 1 (5-8 tokens, Q8 input, unsplit): no whole-row staging — each wave streams its own
// super-blocks' activations (x, dx and the per-type sums of every token) through a private
// two-slot LDS ring, one block ahead of its maths: ffn_down's 8 x 18944 activations do not fit
// the LDS at once, and this keeps the 8-wave shape (and so the T <= 4 bits) in one pass over the
// weights
template <int TYPE, int T, int MODE, int KW, int RG, int D, int POL = 0, int SX = 0>
__device__ __forceinline__ void qgemv_mfma_body(const GemvArgs& a, const int bid) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int P = MODE == kPair ? 2 : 1;
  constexpr int NA = TYPE == kQ6K ? 4 : 2;          // uint4 of activation sums per block
  constexpr int NQ = (T + 3) / 4;                   // token quads: MFMA M = 4 tokens x 4 K-groups
  const int K = a.K, nb = K >> 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rg = wave / KW, kw = wave % KW;
  // split-K over workgroups: this one takes super-blocks [kb_lo, kb_lo + nbw) of row tile `tile`
  const int SKr = a.ksplit > 1 ? a.ksplit : 1;
  const int tile = bid / SKr, slice = bid - tile * SKr;
  const int kb_lo = slice * nb / SKr, nbw = (slice + 1) * nb / SKr - kb_lo;
  const int Kl = nbw << 8;                                       // the staged window's K
  // this wave's super-blocks: part gw of the row cut into SKr x KW parts (inside this slice's
  // window), so an unsplit KW-wave launch and a split one of the same SKr x KW give every wave
  // the same blocks
  const int gw = slice * KW + kw, tw = SKr * KW;
  const int kb0 = gw * nb / tw, n = (gw + 1) * nb / tw - kb0;    // host: >= 1
  const int r = lane & 15, g = lane >> 4;
  const int wrow0 = tile * RG * 16;
  const long rb0 = (long)(min(wrow0 + rg * 16, a.N - 16) >> 4) * nb + kb0;   // host: N % 16 == 0
  // ring of D super-blocks: D - 1 in flight before the activations are staged
  MBlk<TYPE> w0[D], w1[D];
#pragma unroll
  for (int d = 0; d < D - 1; ++d) {
    const long rb = rb0 + min(d, n - 1);
    mload<TYPE, POL>(a.w0, rb, lane, w0[d]);
    if constexpr (P == 2) mload<TYPE, POL>(a.w1, rb, lane, w1[d]);
  }
  // SX ring slot: x [T][288] (the staged row's block layout), dx [T][8], sums [T][NA x 4 dwords],
  // 256 zero bytes (the A operand of this slot's inactive lanes: every fragment read is then one
  // base register plus constant offsets)
  constexpr int SXZ = T * (320 + NA * 16), SXS = SXZ + 256;
  const int sxbase = wave * 2 * SXS;
  // staging through registers (a direct-to-LDS load in flight would make every use of a weight
  // load wait for it); buffer loads: one 32-bit offset register per stream instead of a pointer
  uint4 sr_x0, sr_x1;                // two 16-byte x units per lane and block (80-128 for 5-8 tokens)
  float4 sr_d, sr_s;
  const __amdgpu_buffer_rsrc_t rs_x =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.x8), (short)0, T * K, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_d =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dx), (short)0, T * (K >> 3), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_s =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.sx), (short)0, T * (K >> 2), 0x00020000);
  uint32_t vo_x0 = 0, vo_x1 = 0, vo_d = 0, vo_s = 0;
  if constexpr (SX) {
    const int c1 = min(lane + 64, T * 16 - 1), cd = min(lane, 2 * T - 1), cs = min(lane, 4 * T - 1);
    vo_x0 = (uint32_t)((lane >> 4) * K + (lane & 15) * 16);
    vo_x1 = (uint32_t)((c1 >> 4) * K + (c1 & 15) * 16);
    vo_d = (uint32_t)(((cd >> 1) * (K >> 5) + (cd & 1) * 4) * 4);
    vo_s = (uint32_t)(((cs >> 2) * (K >> 4) + (cs & 3) * 4) * 4);
  }
  // one super-block (global index kb) of every token into the staging registers
  auto sx_load = [&](int kb) {
    const uint32_t ox = (uint32_t)kb * 256u, od = (uint32_t)kb * 32u;
    sr_x0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_x, vo_x0 + ox, 0, 0));
    sr_x1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_x, vo_x1 + ox, 0, 0));
    sr_d = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs_d, vo_d + od, 0, 0));
    if constexpr (TYPE == kQ4K)
      sr_s = __builtin_bit_cast(float4,
                                __builtin_amdgcn_raw_buffer_load_b128(rs_s, vo_s + 2 * od, 0, 0));
  };
  // the staging registers → ring slot s, with the sums the staged path computes (same arithmetic)
  auto sx_store = [&](int s) {
    uint8_t* base = lds + sxbase + s * SXS;
    auto put = [&](int c, const uint4& v) {
      *reinterpret_cast<uint4*>(base + (c >> 4) * 288 + (c & 15) * 16) = v;
      if constexpr (TYPE == kQ6K) {
        int sum = dot4z(v.x, 0x01010101u);
        sum = dot4(v.y, 0x01010101u, sum);
        sum = dot4(v.z, 0x01010101u, sum);
        reinterpret_cast<int*>(base + T * 320)[c] = dot4(v.w, 0x01010101u, sum);
      }
    };
    put(lane, sr_x0);
    if (lane + 64 < T * 16) put(lane + 64, sr_x1);
    if (lane < 2 * T) *reinterpret_cast<float4*>(base + T * 288 + lane * 16) = sr_d;
    if constexpr (TYPE == kQ4K) {
      if (lane < 4 * T)
        *reinterpret_cast<float2*>(base + T * 320 + lane * 8) =
            make_float2(sr_s.x + sr_s.y, sr_s.z + sr_s.w);
    }
  };
  // step i: block i + 1 (loaded one step ago) into its slot, then block i + 2's loads — issued
  // before the step's weight refill, so waiting for them never waits for that refill
  auto sx_step = [&](int i) {
    if constexpr (SX) {
      sx_store((i + 1) & 1);
      sx_load(kb0 + min(i + 2, n - 1));
    }
  };
  XView xv{};
  MfmaLds L;
  if constexpr (SX) {
    static_assert(T > 4, "the activation ring stages 80-128 x units per block");
    L = mfma_lds_sx(T, NA, KW * RG, P);
    if (lane < 32) {                     // both slots' zero bytes (this wave only reads them)
      uint4* z = reinterpret_cast<uint4*>(lds + sxbase + (lane >> 4) * SXS + SXZ);
      z[lane & 15] = make_uint4(0, 0, 0, 0);
    }
    sx_load(kb0);
    sx_store(0);
    sx_load(kb0 + min(1, n - 1));
  } else {
    xv = SKr > 1 ? stage_x8_window<T>(a, lds, kb_lo, nbw) : stage_x<T>(a, lds);
    L = mfma_lds(TYPE, T, Kl, KW * RG, P);
    if constexpr (TYPE == kQ4K) {
      float* sxp = reinterpret_cast<float*>(lds + L.aux);
      for (int i = threadIdx.x; i < T * (Kl >> 5); i += blockDim.x)
        sxp[i] = xv.sxs[2 * i] + xv.sxs[2 * i + 1];
    } else {
      int* X = reinterpret_cast<int*>(lds + L.aux);
      for (int i = threadIdx.x; i < T * (Kl >> 4); i += blockDim.x) {
        const int t = i / (Kl >> 4), p = (i - t * (Kl >> 4)) << 4;
        const uint4 v = *reinterpret_cast<const uint4*>(xv.xs + t * xv.xstride + xoff(p));
        int sum = dot4z(v.x, 0x01010101u);
        sum = dot4(v.y, 0x01010101u, sum);
        sum = dot4(v.z, 0x01010101u, sum);
        X[i] = dot4(v.w, 0x01010101u, sum);
      }
    }
  }
  if constexpr (!SX) {
    if (threadIdx.x < 16) reinterpret_cast<uint4*>(lds + L.zero)[threadIdx.x] = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }
  // A operand of quad q: lane l is row (t, s) = (4q + ((l & 15) >> 2), l & 3) of K-group g; live
  // only for s == g.  MFMA m's 16 activations: Q4_K +0 / +32 / +128 / +160 from
  // 64 (g >> 1) + 16 (g & 1); Q6_K +0 / +64 / +128 / +192 from 16 g (zero lanes: the zero bytes)
  const int xb = TYPE == kQ6K ? 16 * g : 64 * (g >> 1) + 16 * (g & 1);
  int xa0[NQ], xstep[NQ], xo1[NQ], xo2[NQ], xo3[NQ];
  const float* dxb[NQ];
  const uint4* axb[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int at = 4 * q + ((lane & 15) >> 2);
    const bool live = (lane & 3) == g && at < T;
    if constexpr (SX) {                 // dead lanes: the slot's zero bytes, same offsets
      xa0[q] = sxbase + (live ? at * 288 + xb : SXZ);
      xstep[q] = SXS;
      xo1[q] = TYPE == kQ6K ? 64 : 32;
      xo2[q] = 128;
      xo3[q] = TYPE == kQ6K ? 192 : 160;
    } else {
      xa0[q] = live ? at * xv.xstride + xb : L.zero;
      xstep[q] = live ? 288 : 0;
      xo1[q] = live ? (TYPE == kQ6K ? 64 : 32) : 0;
      xo2[q] = live ? 128 : 0;
      xo3[q] = live ? (TYPE == kQ6K ? 192 : 160) : 0;
    }
    const int tt = min(4 * q + g, T - 1);            // this lane's output token in quad q
    if constexpr (SX) {
      dxb[q] = reinterpret_cast<const float*>(lds + sxbase + T * 288) + tt * 8;
      axb[q] = reinterpret_cast<const uint4*>(lds + sxbase + T * 320) + tt * NA;
    } else {
      dxb[q] = xv.dxs + tt * (Kl >> 5);
      axb[q] = reinterpret_cast<const uint4*>(lds + L.aux) + tt * nbw * NA;
    }
  }
  // per-block strides: the staged row's next block, or the ring's other slot
  constexpr int DSTEP = SX ? SXS / 4 : 8, ASTEP = SX ? SXS / 16 : NA;
  float acc[NQ], acc1[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) acc[q] = acc1[q] = 0.f;
  auto compute = [&](const MBlk<TYPE>& q0, const MBlk<TYPE>& q1, int i) {
    const int kb = SX ? (i & 1) : kb0 - kb_lo + i;    // window-local block index / ring slot
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint8_t* xp = lds + xa0[q] + kb * xstep[q];
      i32x4 xa[4];
      xa[0] = *reinterpret_cast<const i32x4*>(xp);
      xa[1] = *reinterpret_cast<const i32x4*>(xp + xo1[q]);
      xa[2] = *reinterpret_cast<const i32x4*>(xp + xo2[q]);
      xa[3] = *reinterpret_cast<const i32x4*>(xp + xo3[q]);
      float dxv[8];
      const float4 d0 = *reinterpret_cast<const float4*>(dxb[q] + kb * DSTEP);
      const float4 d1 = *reinterpret_cast<const float4*>(dxb[q] + kb * DSTEP + 4);
      dxv[0] = d0.x; dxv[1] = d0.y; dxv[2] = d0.z; dxv[3] = d0.w;
      dxv[4] = d1.x; dxv[5] = d1.y; dxv[6] = d1.z; dxv[7] = d1.w;
      uint4 aux[4];
#pragma unroll
      for (int u = 0; u < NA; ++u) aux[u] = axb[q][kb * ASTEP + u];
      acc[q] = mfma_block<TYPE>(q0, xa, dxv, aux, g, acc[q]);
      if constexpr (P == 2) acc1[q] = mfma_block<TYPE>(q1, xa, dxv, aux, g, acc1[q]);
      // SX: one quad's fragments live at a time (both at once spill at 2 waves/SIMD)
      if constexpr (SX) __builtin_amdgcn_sched_barrier(0);
    }
  };
  // Whole groups of D steps: every step first refills the slot consumed one step ago with block
  // i + D - 1 (clamped: the last group re-reads the final block from L2), then computes slot d.
  // No load sits under a branch (that makes the compiler drain every outstanding load at the
  // join, which serialises the ring); the < D leftover blocks are computed after the loop from
  // slots already in flight.
  int i0 = 0;
  for (; i0 + D <= n; i0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int ps = (d + D - 1) % D;
      const long nxt = rb0 + min(i0 + d + D - 1, n - 1);
      sx_step(i0 + d);
      mload<TYPE, POL>(a.w0, nxt, lane, w0[ps]);
      if constexpr (P == 2) mload<TYPE, POL>(a.w1, nxt, lane, w1[ps]);
      // keep the refill ahead of this step's maths and the steps in ring order: the scheduler
      // otherwise sinks the refills, and the next step's wait then drains them too
      __builtin_amdgcn_sched_barrier(0);
      compute(w0[d], w1[d], i0 + d);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < D - 1; ++d)
    if (i0 + d < n) {
      sx_step(i0 + d);
      compute(w0[d], w1[d], i0 + d);
    }
  // K-split partials: wave kw = 0 of each row group adds its group's in wave order
  float v[NQ], v1[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) v[q] = acc[q], v1[q] = acc1[q];
  if constexpr (KW > 1) {
    float* kred = reinterpret_cast<float*>(lds + L.kred);      // [waves][NQ][P][64]
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      kred[((wave * NQ + q) * P) * 64 + lane] = acc[q];
      if constexpr (P == 2) kred[((wave * NQ + q) * P + 1) * 64 + lane] = acc1[q];
    }
    __syncthreads();
    if (kw == 0) {
      // in groups of kRedGroup waves, then the group sums in order: an 8-wave launch adds
      // (w0+..+w3) + (w4+..+w7), exactly what a 2-slice x 4-wave split-K launch of the same row
      // computes (each slice one group, the combine adds the slices in order)
      constexpr int GRP = KW < kRedGroup ? KW : kRedGroup;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        v[q] = 0.f; v1[q] = 0.f;
#pragma unroll
        for (int k0 = 0; k0 < KW; k0 += GRP) {
          float gs = 0.f, gs1 = 0.f;
#pragma unroll
          for (int k = k0; k < k0 + GRP; ++k) {
            gs += kred[(((rg * KW + k) * NQ + q) * P) * 64 + lane];
            if constexpr (P == 2) gs1 += kred[(((rg * KW + k) * NQ + q) * P + 1) * 64 + lane];
          }
          v[q] += gs;
          if constexpr (P == 2) v1[q] += gs1;
        }
      }
    }
  }
  if constexpr (MODE != kPair) {
    if (SKr > 1) {
      // split-K combine (cdna_hip_programming.md §5 "In-launch split-K reduction", sc1 form):
      // every slice stores its partials write-through, drains, and draws a ticket; the slice
      // that draws SKr - 1 reads all slabs with sc1 loads and sums them in slice order, so the
      // bits never depend on which slice arrived last
      float* slabs = a.kpart + (long)tile * SKr * (RG * NQ * 64);
      if (kw == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          __hip_atomic_store(slabs + ((long)slice * RG * NQ + rg * NQ + q) * 64 + lane, v[q],
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      unsigned* flag = reinterpret_cast<unsigned*>(lds + L.flag);
      if (threadIdx.x == 0)
        flag[0] = __hip_atomic_fetch_add(a.kcnt + tile, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if (flag[0] != (unsigned)(SKr - 1)) return;
      if (kw == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          float tot = 0.f;
          for (int s2 = 0; s2 < SKr; ++s2)
            tot += __hip_atomic_load(slabs + ((long)s2 * RG * NQ + rg * NQ + q) * 64 + lane,
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v[q] = tot;
        }
      }
      if (threadIdx.x == 0)      // every slice has drawn its ticket: ready for the next call
        __hip_atomic_store(a.kcnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  float* q8s = (MODE == kPair && a.ox8) ? reinterpret_cast<float*>(lds + L.q8s) : nullptr;
  const int orow = wrow0 + rg * 16 + r;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int t = 4 * q + g;
    if (kw == 0 && t < T && orow < a.N) {
      float* o = a.out + (long)t * a.ldo + orow;
      if constexpr (MODE == kStore) *o = v[q] + (a.bias ? a.bias[orow] : 0.f);
      else if constexpr (MODE == kResid) *o += v[q];
      else {
        const float y = v[q] / (1.f + __expf(-v[q])) * v1[q];
        if (q8s) q8s[t * 32 + rg * 16 + r] = y;
        else *o = y;
      }
    }
  }
  if constexpr (MODE == kPair && RG == 2) {
    if (q8s) {
      __syncthreads();
      emit_q8_block<T>(a, q8s, wrow0);
    }
  }
}

// A/B knobs (build-time): the pair kernel's ring depth and its waves-per-SIMD floor.  D = 3 needs
// 2 waves/SIMD (214 VGPRs; at 3 it spills): T = 1 1.680 -> 1.739 ms, T = 4 2.046 -> 2.065 ms
// (gate|up's 592 workgroups no longer co-resident; session r05g)
#ifndef AMDK8S_PAIR_D
#define AMDK8S_PAIR_D 2
#endif
#ifndef AMDK8S_PAIR_WPE
#define AMDK8S_PAIR_WPE 3
#endif
// Q6_K pairs (5 planes per slot) spill 336-428 bytes per lane at 3 waves/SIMD: 2 at every T.
// Steps of 5-8 tokens (two token quads per wave): without a floor the pair kernel took 209 VGPRs
// + 64 AGPRs, one wave per SIMD, so gate|up's 592 workgroups ran in 2.3 rounds (32.1 us at T = 8);
// at 2 waves/SIMD (252 VGPRs, no spill) 24.4 us, T = 8 step 3.02 -> 2.82 ms (session r05ac).
#ifndef AMDK8S_PAIR_WPE8
#define AMDK8S_PAIR_WPE8 2
#endif
// Q4_K store / resid GEMVs at 5-8 tokens: 170-176 VGPRs left them at 2 waves/SIMD; 3 fit
// without a spill (Q6_K would spill 172-232 B/lane, so it keeps the compiler's choice)
#ifndef AMDK8S_NP_WPE8
#define AMDK8S_NP_WPE8 3
#endif
constexpr int kPairD = AMDK8S_PAIR_D;

template <int TYPE, int T, int MODE, int KW, int RG, int D, int POL = 0, int SX = 0>
__global__ void __launch_bounds__(KW * RG * 64)
__attribute__((amdgpu_waves_per_eu(
    MODE == kPair ? (T <= 4 && TYPE == kQ4K ? AMDK8S_PAIR_WPE : AMDK8S_PAIR_WPE8)
                  : (SX ? 2 : (T > 4 && TYPE == kQ4K ? AMDK8S_NP_WPE8 : 1)), 8)))
qgemv_mfma_kernel(GemvArgs a) {
  qgemv_mfma_body<TYPE, T, MODE, KW, RG, D, POL, SX>(a, blockIdx.x);
}

// Two store-mode matrices of (possibly) different types over the same input in ONE launch (q|k
// and v of Q4_K_M): workgroups [0, grid0) run a0.  Each keeps the shape and the arithmetic it has
// alone, so a row's bits do not depend on which launch computed it.
template <int TYPE0, int TYPE1, int T, int KW, int RG, int D>
__global__ void __launch_bounds__(KW * RG * 64)
qgemv2_mfma_kernel(GemvArgs a0, GemvArgs a1, int grid0) {
  if ((int)blockIdx.x < grid0) qgemv_mfma_body<TYPE0, T, kStore, KW, RG, D>(a0, blockIdx.x);
  else qgemv_mfma_body<TYPE1, T, kStore, KW, RG, D>(a1, blockIdx.x - grid0);
}

// Repacked planes → the MFMA-packed copy (see mload): one thread per (row, super-block).
// Q4_K: q [N][nb*128], sc [N][nb*4] dwords, d [N][nb] dwords.  Q6_K: ql [N][nb*128],
// qh [N][nb*64], sc [N][nb*16] int8 (lane order, q6_scale_pos), d [N][nb] f16.
template <int TYPE>
__global__ void mfma_pack_kernel(QMat w, int N, int nb, uint8_t* __restrict__ mq,
                                 uint8_t* __restrict__ mqh, uint8_t* __restrict__ msc,
                                 uint32_t* __restrict__ md) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * nb) return;
  const int row = (int)(i / nb), b = (int)(i % nb);
  const long gb = (long)(row >> 4) * nb + b;
  const int r = row & 15;
  const uint4* src = reinterpret_cast<const uint4*>(w.q + i * 128);
  uint4* dst = reinterpret_cast<uint4*>(mq + gb * 2048 + r * 64);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[h * 64 + j] = src[h * 4 + j];
  if constexpr (TYPE == kQ4K) {
    reinterpret_cast<uint4*>(msc + gb * 256 + r * 16)[0] =
        reinterpret_cast<const uint4*>(w.sc + i * 16)[0];
    md[gb * 16 + r] = reinterpret_cast<const uint32_t*>(w.d)[i];
  } else {
    const uint4* hs = reinterpret_cast<const uint4*>(w.qh + i * 64);
    uint4* hd = reinterpret_cast<uint4*>(mqh + gb * 1024 + r * 32);
    hd[0] = hs[0]; hd[1] = hs[1];                   // half 0: qh bytes 0..31
    hd[32] = hs[2]; hd[33] = hs[3];                 // half 1: bytes 32..63, 512 B further
    uint8_t sc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) sc[j] = (uint8_t)w.sc[i * 16 + q6_scale_pos(j)];
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      wv[j] = sc[4 * j] | (sc[4 * j + 1] << 8) | (sc[4 * j + 2] << 16) | ((uint32_t)sc[4 * j + 3] << 24);
    reinterpret_cast<uint4*>(msc + gb * 256 + r * 16)[0] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    md[gb * 16 + r] = w.d[i];
  }
}

// MFMA GEMV launch shapes (K-waves x row groups, swept with tools/llm_bench.py --gemv, profiles/r04/l):
// pair (gate|up) 2 x 2 (a whole 32-row Q8 block per workgroup); long rows (K >= 8192: ffn_down)
// 8 x 1; very tall matrices (lm_head) 2 x 2; the rest 4 x 1 (q|k|v, o_proj: 2 x 1 measured the same).  4 = shape not covered (N % 16, fewer super-blocks than K-waves, LDS): use qgemv_kernel.
template <int TYPE, int T, int MODE, int KW, int RG>
int launch_mfma_one(const GemvArgs& a, hipStream_t st) {
  // ring depth: pair 2 (two matrices per slot, 3 waves/SIMD), else 3 (6 for ffn_down's 8-wave
  // shape measured slower: Q6_K 13.9 -> 15.6 us, T = 1 1.629 -> 1.656 ms, profiles/r04/o)
  constexpr int D = MODE == kPair ? kPairD : 3;
  const int nb = a.K >> 8, sk = a.ksplit > 1 ? a.ksplit : 1;
  if (nb / sk < KW) return 4;                      // every wave of every slice gets a block
  if (sk > 1 && (MODE == kPair || a.xf || !a.kpart || !a.kcnt)) return 2;
  const int nbw = (nb + sk - 1) / sk;              // the largest slice's window
  const MfmaLds L = mfma_lds(TYPE, T, nbw << 8, KW * RG, MODE == kPair ? 2 : 1);
  if (L.total > 160 * 1024) return 4;
  const int tiles = (a.N + 16 * RG - 1) / (16 * RG);
  if constexpr (MODE == kResid && KW == 8 && T <= 4) {
    if (a.w0.temporal) {          // the two-launch 5-8 token ffn_down (dispatch_mfma_split)
      hipLaunchKernelGGL((qgemv_mfma_kernel<TYPE, T, MODE, KW, RG, D, 1>), dim3(tiles * sk),
                         dim3(KW * RG * 64), L.total, st, a);
      return hipGetLastError() == hipSuccess ? 0 : 1;
    }
  }
  hipLaunchKernelGGL((qgemv_mfma_kernel<TYPE, T, MODE, KW, RG, D>), dim3(tiles * sk),
                     dim3(KW * RG * 64), L.total, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// 5-8 tokens on the 8-wave long-row shape (ffn_down): the activation-ring form (SX), one pass
// over the weights with the T <= 4 launch's parts and reduction order.  AMDK8S_DOWN_SX=0: the
// two-launch form instead (A/B runs).
static bool sx_enabled() {
  static const bool on = [] {
    const char* e = getenv("AMDK8S_DOWN_SX");
    return !e || e[0] != '0';
  }();
  return on;
}

template <int TYPE, int T, int MODE>
int launch_mfma_sx(const GemvArgs& a, hipStream_t st) {
  // ring depth: Q6_K 2 (its 3-deep weight ring spills 17-31 VGPRs next to two token quads and the
  // staging registers at 2 waves/SIMD), Q4_K 3 (230 VGPRs)
  constexpr int KW = 8, RG = 1, D = TYPE == kQ6K ? 2 : 3, NA = TYPE == kQ6K ? 4 : 2;
  if ((a.K >> 8) < KW || a.xf || a.ksplit > 1 || !sx_enabled()) return 4;
  if ((reinterpret_cast<uintptr_t>(a.x8) | reinterpret_cast<uintptr_t>(a.dx) |
       reinterpret_cast<uintptr_t>(a.sx)) & 15) return 4;       // 16-byte staging loads
  const MfmaLds L = mfma_lds_sx(T, NA, KW * RG, 1);
  if (L.total > 160 * 1024) return 4;
  hipLaunchKernelGGL((qgemv_mfma_kernel<TYPE, T, MODE, KW, RG, D, 0, 1>), dim3(a.N / 16),
                     dim3(KW * RG * 64), L.total, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Default shape: a function of the matrix only (never of T or of the input form), so each matrix
// sums its K-split partials in one order at every T (batch invariance), and 4 waves wherever the
// fp32-row prologue may run (stage_x reduces the RMSNorm over 4 waves in rmsnorm_q8's order;
// models with dim >= 8192 use the prologue at every T).
void mfma_shape(bool pair, int N, int K, int& kw, int& rg) {
  const int nb = K >> 8;
  (void)N;
  // pair: 2 x 2.  1 x 2 (2 waves, whole K per wave) is faster alone (17.8 / 19.0 vs 18.5 / 20.4 us
  // at T = 1 / 4) but, with its 2-wave RMSNorm prologue, slower in the step (T = 1 1.625 -> 1.664 ms,
  // T = 8 2.94 -> 3.10 ms; profiles/r04/w)
  if (pair) kw = nb >= 2 ? 2 : 1, rg = 2;
  else if (K >= 8192) kw = 8, rg = 1;
  else if (N >= 65536 && nb >= 2) kw = 2, rg = 2;    // lm_head: 75.0 / 80.2 us at T = 1 / 4
  else if (nb >= 4) kw = 4, rg = 1;
  else if (nb >= 2) kw = 2, rg = 2;
  else kw = 1, rg = 4;
}

// Split-K over workgroups for the long-row matrices fed Q8 (ffn_down, K = 18944): 224 row tiles
// of 8 waves left 32 of the 256 CUs idle and every wave a 9-block dependent chain; slices of the
// super-blocks on separate workgroups fill the chip.  A function of the matrix only (and of the
// input form, which is fixed per matrix in the engine), like the shape.
void mfma_ksplit_shape(int N, int K, int T, int& kw, int& rg, int& sk) {
  (void)N;
  if (K < 8192) return;
  kw = kSplitKW, rg = 1, sk = kSplitSK;
  // 5-8 tokens: their activations of the whole row do not fit one workgroup's LDS, so the
  // default is two launches (tokens 0-3 and 4..T-1: the weights streamed twice).  The one-pass
  // form runs each row tile as 2 slices of 4 waves (the same 8 parts of the row as the 8-wave
  // launch, so the bits are the same), but its 8-token window takes 135 KB of LDS: one 4-wave
  // workgroup per CU, 448 of them in 1.75 rounds.  Measured per step (profiles/r06/
  // llm_bench_down_{onepass,twopass}_T5-8.log): T = 5 2.640 vs 2.700 ms, T = 6 2.882 vs 2.787,
  // T = 7 3.001 vs 2.842, T = 8 3.036 vs 2.881 — one pass for T = 5 only.  Both lost to the
  // activation-ring form (launch_mfma_sx: the unsplit 8-wave shape, one pass, activations streamed
  // per wave): T = 5 / 6 / 7 / 8 2.298 / 2.358 / 2.412 / 2.446 ms vs two launches 2.633 / 2.770 /
  // 2.850 / 2.882 (profiles/r06/llm_bench_down_sx_T1-8.log, _sx_off_T5-8.log), so with it on the
  // split form is never the default.  AMDK8S_DOWN_ONEPASS=<max T> forces it for A/B runs.
  static const int onepass_max = [] {
    const char* e = getenv("AMDK8S_DOWN_ONEPASS");
    return e ? atoi(e) : (sx_enabled() ? 0 : 5);
  }();
  if (T > 4 && T <= onepass_max && kSplitKW == 8 && kSplitSK == 1) kw = 4, sk = 2;
}

template <int TYPE, int T, int MODE>
int launch_mfma(const GemvArgs& a, int kw, int rg, hipStream_t st) {
  if (a.N % 16) return 4;
  if (kw <= 0) mfma_shape(MODE == kPair, a.N, a.K, kw, rg);
  if (MODE == kPair && a.ox8 && rg != 2) return 2;   // a whole 32-row Q8 block per workgroup
  if (MODE == kPair && a.ox8 && kw * rg * 64 < 32 * T) return 2;   // emit_q8_block: 32 lanes/token
  // only the shapes mfma_shape picks are instantiated (build time)
  if constexpr (MODE == kPair) {
    if (kw == 2 && rg == 2) return launch_mfma_one<TYPE, T, MODE, 2, 2>(a, st);
    if (kw == 1 && rg == 2) return launch_mfma_one<TYPE, T, MODE, 1, 2>(a, st);
    return 2;
  } else {
    switch (kw * 8 + rg) {
      case 1 * 8 + 4: return launch_mfma_one<TYPE, T, MODE, 1, 4>(a, st);
      case 2 * 8 + 1: return launch_mfma_one<TYPE, T, MODE, 2, 1>(a, st);
      case 2 * 8 + 2: return launch_mfma_one<TYPE, T, MODE, 2, 2>(a, st);
      case 4 * 8 + 1: return launch_mfma_one<TYPE, T, MODE, 4, 1>(a, st);
      case 8 * 8 + 1:
        if constexpr (T <= 4) return launch_mfma_one<TYPE, T, MODE, 8, 1>(a, st);
        else return launch_mfma_sx<TYPE, T, MODE>(a, st);   // 4: tokens in two launches
      default: return 2;
    }
  }
}

// kw / rg: K-waves and 16-row groups per workgroup (0 = the default shape for the matrix)
template <int TYPE, int MODE>
int dispatch_mfma(const GemvArgs& a, int kw, int rg, hipStream_t st) {
  switch (a.T) {
    case 1: return launch_mfma<TYPE, 1, MODE>(a, kw, rg, st);
    case 2: return launch_mfma<TYPE, 2, MODE>(a, kw, rg, st);
    case 3: return launch_mfma<TYPE, 3, MODE>(a, kw, rg, st);
    case 4: return launch_mfma<TYPE, 4, MODE>(a, kw, rg, st);
    case 5: return launch_mfma<TYPE, 5, MODE>(a, kw, rg, st);
    case 6: return launch_mfma<TYPE, 6, MODE>(a, kw, rg, st);
    case 7: return launch_mfma<TYPE, 7, MODE>(a, kw, rg, st);
    case 8: return launch_mfma<TYPE, 8, MODE>(a, kw, rg, st);
    default: return 2;
  }
}

// More than 4 tokens whose activations do not fit the LDS with T (ffn_down's K = 18944 at T > 4):
// tokens [0, 4) and [4, T) as two launches.  Every token's arithmetic is the same in either form.
template <int TYPE, int MODE>
int dispatch_mfma_split(const GemvArgs& a, int kw, int rg, hipStream_t st) {
  const int rc = dispatch_mfma<TYPE, MODE>(a, kw, rg, st);
  if (rc != 4 || a.T <= 4) return rc;
  GemvArgs lo = a, hi = a;
  lo.T = 4;
  hi.T = a.T - 4;
  // The second launch re-reads the first one's weights.  Default-policy loads in both (to keep
  // them in the 256 MB Infinity Cache in between) measured SLOWER than non-temporal ones: T = 6
  // 2.856 vs 2.771 ms, T = 8 2.963 vs 2.879 (profiles/r06/llm_bench_down_temporal.log); kept as
  // an A/B knob, AMDK8S_SPLIT_TEMPORAL=1.
  static const bool temporal = [] {
    const char* e = getenv("AMDK8S_SPLIT_TEMPORAL");
    return e && e[0] == '1';
  }();
  lo.w0.temporal = hi.w0.temporal = temporal ? 1 : 0;
  const long K = a.K;
  if (hi.x8) { hi.x8 += 4 * K; hi.dx += 4 * (K >> 5); hi.sx += 4 * (K >> 4); }
  if (hi.xf) hi.xf += 4L * a.ldx;
  hi.out += 4L * a.ldo;
  if (hi.ox8) { hi.ox8 += 4L * a.N; hi.odx += 4L * (a.N >> 5); hi.osx += 4L * (a.N >> 4); }
  const int r0 = dispatch_mfma<TYPE, MODE>(lo, kw, rg, st);
  if (r0) return r0;
  return dispatch_mfma<TYPE, MODE>(hi, kw, rg, st);
}


template <int TYPE0, int TYPE1, int T, int KW, int RG>
int launch_mfma2_one(const GemvArgs& a0, const GemvArgs& a1, hipStream_t st) {
  constexpr int D = 3;
  if ((a0.K >> 8) < KW) return 4;
  const int lds = max(mfma_lds(TYPE0, T, a0.K, KW * RG, 1).total,
                      mfma_lds(TYPE1, T, a0.K, KW * RG, 1).total);
  if (lds > 160 * 1024) return 4;
  const int g0 = (a0.N + 16 * RG - 1) / (16 * RG), g1 = (a1.N + 16 * RG - 1) / (16 * RG);
  hipLaunchKernelGGL((qgemv2_mfma_kernel<TYPE0, TYPE1, T, KW, RG, D>), dim3(g0 + g1),
                     dim3(KW * RG * 64), lds, st, a0, a1, g0);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

template <int TYPE0, int TYPE1, int T>
int launch_mfma2(const GemvArgs& a0, const GemvArgs& a1, hipStream_t st) {
  if (a0.N % 16 || a1.N % 16) return 4;
  int kw = 0, rg = 0;
  mfma_shape(false, a0.N + a1.N, a0.K, kw, rg);
  switch (kw * 8 + rg) {
    case 1 * 8 + 4: return launch_mfma2_one<TYPE0, TYPE1, T, 1, 4>(a0, a1, st);
    case 2 * 8 + 2: return launch_mfma2_one<TYPE0, TYPE1, T, 2, 2>(a0, a1, st);
    case 4 * 8 + 1: return launch_mfma2_one<TYPE0, TYPE1, T, 4, 1>(a0, a1, st);
    default: return 4;
  }
}

template <int TYPE0, int TYPE1>
int dispatch_mfma2(const GemvArgs& a0, const GemvArgs& a1, hipStream_t st) {
  switch (a0.T) {
    case 1: return launch_mfma2<TYPE0, TYPE1, 1>(a0, a1, st);
    case 2: return launch_mfma2<TYPE0, TYPE1, 2>(a0, a1, st);
    case 3: return launch_mfma2<TYPE0, TYPE1, 3>(a0, a1, st);
    case 4: return launch_mfma2<TYPE0, TYPE1, 4>(a0, a1, st);
    case 5: return launch_mfma2<TYPE0, TYPE1, 5>(a0, a1, st);
    case 6: return launch_mfma2<TYPE0, TYPE1, 6>(a0, a1, st);
    case 7: return launch_mfma2<TYPE0, TYPE1, 7>(a0, a1, st);
    case 8: return launch_mfma2<TYPE0, TYPE1, 8>(a0, a1, st);
    default: return 2;
  }
}

}  // namespace

extern "C" {

// Quantised GEMV on the int8 matrix cores (qgemv_mfma_kernel) over the MFMA-packed planes (w*q /
// w*qh / w*sc / w*d from amdk8s_llm_mfma_pack; qh: Q6_K only); arguments otherwise as
// amdk8s_llm_qgemv.  kw / rows_per_wg: K-waves and rows (16 x row groups) per workgroup, 0 = the
// default shape.  4 = shape not covered (N % 16, fewer super-blocks than K-waves, LDS): use
// amdk8s_llm_qgemv on the plain planes.
// ksplit: split-K slices over workgroups (store / resid modes, Q8 input); -1 = the default for the
// matrix (mfma_ksplit_shape) when scratch is given, 0 / 1 = none.  kpart [kpart_floats] and kcnt
// [kcnt_words] (zeroed once at allocation; every launch leaves them zero) must hold
// tiles x ksplit x row groups x 2 x 64 floats and one word per tile, else rc 2.
int amdk8s_llm_qgemv_mfma(int type, int mode, const void* w0q, const void* w0qh, const void* w0sc,
                          const void* w0d, const void* w1q, const void* w1qh, const void* w1sc,
                          const void* w1d, const void* x8, const void* dx, const void* sx,
                          const void* xf, int ldx, const void* norm_w, float eps,
                          const void* bias, void* out, int ldo, int N, int K, int T, int kw,
                          int rows_per_wg, void* ox8, void* odx, void* osx, int ksplit,
                          void* kpart, long kpart_floats, void* kcnt, int kcnt_words,
                          void* stream) {
  if (K % 256 || N <= 0 || T < 1 || T > kMaxTok) return 2;
  if (type != kQ4K && type != kQ6K) return 2;
  if (mode == kPair && !w1q) return 2;
  if (!xf && !(x8 && dx && sx)) return 2;
  if (xf && (ldx % 4 || T > kValuMaxTok)) return 2;  // fp32-row prologue: steps of <= 4 tokens
  if (ox8 && (mode != kPair || N % 32 || !odx || !osx)) return 2;
  GemvArgs a{};
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
  a.bias = static_cast<const float*>(bias);
  a.out = static_cast<float*>(out);
  a.ldo = ldo; a.N = N; a.K = K; a.T = T; a.rows_per_wg = 0;
  a.ox8 = static_cast<int8_t*>(ox8);
  a.odx = static_cast<float*>(odx);
  a.osx = static_cast<float*>(osx);
  int rg = ox8 ? 2 : (rows_per_wg > 0 && rows_per_wg % 16 == 0 ? rows_per_wg / 16 : 0);
  if (rg == 0) kw = 0;
  a.ksplit = 1;
  if (mode != kPair && !xf && kpart && kcnt) {
    int sk = ksplit;
    if (ksplit < 0) {
      sk = 1;
      if (kw <= 0) mfma_ksplit_shape(N, K, T, kw, rg, sk);
    }
    if (sk > 1) {
      if (kw <= 0) mfma_shape(false, N, K, kw, rg);
      const long tiles = (N + 16 * rg - 1) / (16 * rg);
      if (tiles > kcnt_words || tiles * sk * rg * 2 * 64 > kpart_floats || sk > 64) return 2;
      a.ksplit = sk;
      a.kpart = static_cast<float*>(kpart);
      a.kcnt = static_cast<unsigned*>(kcnt);
    }
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type == kQ4K) {
    if (mode == kStore) return dispatch_mfma_split<kQ4K, kStore>(a, kw, rg, st);
    if (mode == kResid) return dispatch_mfma_split<kQ4K, kResid>(a, kw, rg, st);
    if (mode == kPair) return dispatch_mfma_split<kQ4K, kPair>(a, kw, rg, st);
  } else {
    if (mode == kStore) return dispatch_mfma_split<kQ6K, kStore>(a, kw, rg, st);
    if (mode == kResid) return dispatch_mfma_split<kQ6K, kResid>(a, kw, rg, st);
    if (mode == kPair) return dispatch_mfma_split<kQ6K, kPair>(a, kw, rg, st);
  }
  return 2;
}

// Repacked planes (amdk8s_llm_q4k_repack / q6k_repack layout) → the MFMA-packed copy: mq
// [N*nb*128] bytes, mqh [N*nb*64] bytes (Q6_K), msc [N*nb*16] bytes, md [N*nb] dwords.  N % 16 == 0.
int amdk8s_llm_mfma_pack(int type, const void* q, const void* qh, const void* sc, const void* d,
                         int N, int nb, void* mq, void* mqh, void* msc, void* md, void* stream) {
  if (N <= 0 || N % 16 || nb <= 0 || (type != kQ4K && type != kQ6K)) return 2;
  if (type == kQ6K && !(qh && mqh)) return 2;
  const QMat w = {static_cast<const uint8_t*>(q), static_cast<const uint8_t*>(qh),
                  static_cast<const int8_t*>(sc), static_cast<const uint16_t*>(d)};
  const long n = (long)N * nb;
  const dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type == kQ4K)
    hipLaunchKernelGGL(mfma_pack_kernel<kQ4K>, grid, dim3(256), 0, st, w, N, nb,
                       static_cast<uint8_t*>(mq), nullptr, static_cast<uint8_t*>(msc),
                       static_cast<uint32_t*>(md));
  else
    hipLaunchKernelGGL(mfma_pack_kernel<kQ6K>, grid, dim3(256), 0, st, w, N, nb,
                       static_cast<uint8_t*>(mq), static_cast<uint8_t*>(mqh),
                       static_cast<uint8_t*>(msc), static_cast<uint32_t*>(md));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// amdk8s_llm_qgemv2 on the int8 matrix cores over the MFMA-packed planes (q|k and v of different
// quantisation types in one launch, up to 8 tokens).  4 = not covered (same types, N % 16, LDS):
// launch the matrices with amdk8s_llm_qgemv_mfma.
int amdk8s_llm_qgemv2_mfma(int type0, const void* w0q, const void* w0qh, const void* w0sc,
                           const void* w0d, int N0, const void* bias0, void* out0, int type1,
                           const void* w1q, const void* w1qh, const void* w1sc, const void* w1d,
                           int N1, const void* bias1, void* out1, int ldo, const void* x8,
                           const void* dx, const void* sx, const void* xf, int ldx,
                           const void* norm_w, float eps, int K, int T, void* stream) {
  if (K % 256 || N0 <= 0 || N1 <= 0 || T < 1 || T > kMaxTok) return 2;
  if (!xf && !(x8 && dx && sx)) return 2;
  if (xf && (ldx % 4 || T > kValuMaxTok)) return 2;
  if (type0 == type1 || (type0 != kQ4K && type0 != kQ6K) || (type1 != kQ4K && type1 != kQ6K))
    return 4;
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
    g.ldo = ldo; g.N = N[i]; g.K = K; g.T = T; g.rows_per_wg = 0;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (type0 == kQ4K) return dispatch_mfma2<kQ4K, kQ6K>(a[0], a[1], st);
  return dispatch_mfma2<kQ6K, kQ4K>(a[0], a[1], st);
}

}  // extern "C"
