// Causal GQA prompt attention straight from the KV-cache slab (LLM prefill), gfx950, head dim 128.
//
//   O[p, h] = softmax_j≤start+p( q[p, h] · K[g(h), j] · scale ) V[g(h), j]     g(h) = h / group
//
// The prompt path of the in-tree Qwen2 engine (models/llm/engine.py) — the counterpart of the
// flash-attention llama-server runs over a prompt batch (reference cluster-config/apps/llm/
// deployment.yaml:61,78-84).  A chunk of P prompt tokens sits at positions start .. start+P-1 of one
// sequence slot; its keys are every cached position 0 .. start+P-1 (causal, aligned bottom-right).
//
// Layout of the work:
// * GQA: the query rows of one KV head are flattened token-major, row = p * group + (h % group), so
//   one workgroup of NW waves × 32 rows covers every head of the group for ~NW·32/group tokens and
//   each 64-key K/V tile is staged through LDS ONCE for all of them (7 q heads per KV head on
//   Qwen2.5-7B) — and the causal boundary of a 32-row wave spans only ~5 positions.
// * Causal: a workgroup loops over the key tiles up to its last token; a wave skips the tiles past
//   its own last token (wave-uniform branch, it still helps stage tiles) and masks per lane only
//   on the tiles that straddle its diagonal.
// * K/V are read in place: kc / vc point at the slot's [Hkv][max_ctx][128] fp16 slabs; q and the
//   output are token-major [P][H][128] views (any token / head stride).
// * Split over keys: a long context with few query rows (a 512-token chunk at position 31 488 has
//   4 KV heads × 28 row blocks) would leave most of the 256 CUs idle, so the key tiles are cut into
//   `nsplit` ranges; each workgroup writes unnormalised fp32 partials + (max, sum) and a combine
//   launch merges them.  nsplit = 1 writes the normalised output directly.
// The inner loop is the one of attn_d128.hip: Sᵀ = K·Qᵀ and Oᵀ += Vᵀ·Pᵀ on v_mfma_f32_32x32x16 with
// Qᵀ in registers, softmax in registers (a lane owns one query row), deferred max rescaling,
// XOR-swizzled LDS images, transposed V reads (ds_read_b64_tr_b16), double-buffered tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kD = 128;
constexpr int kKeys = 64;                 // keys per tile
constexpr int kRB = 256;                  // LDS row bytes (128 fp16)
constexpr int kCR = kD / 8;               // 16-byte chunks per row
constexpr int kTile = kKeys * kRB;        // 16 KiB per operand tile
constexpr int kBuf = 2 * kTile;           // K + V
constexpr int kLds = 2 * kBuf;            // double buffered: 64 KiB
constexpr int kKsteps = kD / 16;
constexpr int kDblk = kD / 32;
// A/B knobs (build-time): the tile loop unrolled by two (constant buffer parity, so every LDS
// read is a hoisted register + an immediate), and the first score MFMA with a zero C operand
// instead of zeroed accumulators.  Measured with tools/debug/attn_ab.sh (profiles/r06/attn_ab/):
// the unroll costs 4-6 % (8192 @ 0 728 vs 689-697 us, 512 @ 31488 316 vs 297-300 us: it cuts
// ~50 VALU per tile, but the loop is not issue-bound — PMC: MFMA busy 29 %, 7.6 VALU per MFMA,
// profiles/r06/prefill_attn_pmc_8192.txt), the zero C is neutral; the hoisted offsets alone
// (default) are within 1 % of the round-6 loop.
// -1 = per shape: the 8-wave one-slot kernel (write-after-barrier staging, prefetch schedule)
// unrolls by two — 32000 @ 0 9.42-9.46 -> 8.89-8.93 ms, 8192 @ 0 642-643 -> 609-610 us,
// 4096 @ 28000 1.75 -> 1.69 ms, 512 @ 31488 249 -> 242 us (profiles/r06/attn_ab_8w/)
#ifndef AMDK8S_PA_UNROLL2
#define AMDK8S_PA_UNROLL2 -1
#endif
#ifndef AMDK8S_PA_ZEROC
#define AMDK8S_PA_ZEROC 0
#endif
// WAB: write the next tile into LDS after the barrier (with the tile after it in flight) instead
// of before it.  SCHED: the score MFMAs' two 32-key chains interleaved, each K fragment read SCHED
// steps ahead (a sched_group_barrier pattern), instead of the compiler's order, which runs one
// chain's 8 reads and MFMAs back to back, each MFMA waiting on its own LDS round trip.
// -1 = per shape, from tools/debug/attn_ab.sh (profiles/r06/attn_ab_long/): with 8 waves WAB and
// SCHED 2 together take 32000 @ 0 10.02-10.09 -> 9.55-9.65 ms, 4096 @ 28000 1.844 -> 1.787-1.794,
// 512 @ 31488 260 -> 254 us; with key slots SCHED 2 takes 512 @ 0 13.2 -> 12.9-13.0 us (WAB
// 13.5); the 4-wave one-slot kernel keeps neither (8192 @ 0 within 1 %, profiles/r06/
// attn_ab_sched/)
#ifndef AMDK8S_PA_WAB
#define AMDK8S_PA_WAB -1
#endif
#ifndef AMDK8S_PA_SCHED
#define AMDK8S_PA_SCHED -1
#endif
constexpr float kNoMax = -1e30f;          // finite "no score yet" (a fully masked row stays NaN-free)

__device__ __forceinline__ int kswz(int row, int ch) { return ch ^ (row & 15); }
__device__ __forceinline__ int vswz(int row, int ch) { return ch ^ ((row & 3) << 2); }

template <bool BF16>
__device__ __forceinline__ f32x16 mfma32(const s16x8 a, const s16x8 b, const f32x16 c) {
  if constexpr (BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

template <bool BF16>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  if constexpr (BF16) {
    const bf16x2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
  } else {
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(lo, hi));
  }
}

struct Args {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* o;
  float* opart;      // [nsplit][P*H][128] (nsplit > 1)
  float* ml;         // [nsplit][P*H][2]   (max, sum)
  long sq_tok, sq_head, so_tok, so_head, skv_head;   // element strides (key row stride = 128)
  int P, start, H, Hkv, group, nrb, nsplit, tps;
  float c;           // scale * log2(e)
};

// KS key slots: the NW waves are NW / KS row waves x KS key slots.  Each step stages KS
// consecutive key tiles and slot j's waves take tile j of them, so a row block's chain of tiles is
// KS times shorter; the slots' (max, sum, O) merge through LDS at the end.  For grids that leave
// the chip idle (a short prompt from position 0: 112 four-wave workgroups for 512 tokens).
template <bool BF16, int NW, int KS>
__global__ __launch_bounds__(NW * 64, KS == 1 ? 2 : 1) void prefill_attn_kernel(const Args a) {
  constexpr int NT = NW * 64;
  constexpr int RW = NW / KS;                // row waves: the workgroup's rows are RW x 32
  constexpr int NCH = kKeys * kCR;
  constexpr int CH = KS * NCH / NT;          // 16-byte chunks per thread and step (KS tiles)
  static_assert(NCH % NT == 0 && NW % KS == 0, "tile chunks per thread");
  __shared__ __attribute__((aligned(16))) char lds[KS * kLds];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int rw = KS == 1 ? wave : wave % RW, ksl = KS == 1 ? 0 : wave / RW;
  constexpr bool WAB = AMDK8S_PA_WAB < 0 ? NW == 8 : AMDK8S_PA_WAB != 0;
  constexpr bool UNROLL2 = AMDK8S_PA_UNROLL2 < 0 ? NW == 8 && KS == 1 : AMDK8S_PA_UNROLL2 != 0;
  constexpr int SCHED = AMDK8S_PA_SCHED < 0 ? (NW == 8 || KS == 2 ? 2 : 0) : AMDK8S_PA_SCHED;

  // XCD-major block -> work item (consecutive work items share an XCD and so its L2); work order:
  // row block fastest (heaviest first, below), then KV head, then split
  int work;
  {
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, idx = bid >> 3;
    const int qn = nwg >> 3, rem = nwg & 7;
    work = (xcd < rem ? xcd * (qn + 1) : rem * (qn + 1) + (xcd - rem) * qn) + idx;
  }
  const int rbi = work % a.nrb;
  const int rest = work / a.nrb;
  const int g = rest % a.Hkv;
  const int split = rest / a.Hkv;
  // heaviest first (a causal row block's work grows with its position).  Measured and rejected:
  // a zigzag order (heaviest, lightest, 2nd heaviest, ...) meant to give every XCD's run of work
  // items the same mix — 8192 @ 0 681 -> 730 us, 2048 @ 0 62.7 -> 69.9 us
  // (profiles/r06/prefill_attn_sweep_zigzag.log)
  const int rb = a.nrb - 1 - rbi;

  const int rows = a.P * a.group;            // query rows of this KV head
  const long rowsH = (long)a.P * a.H;        // query rows of the whole chunk (partials' index)
  const int R0 = rb * (RW * 32);
  const int p_hi_wg = min(a.P - 1, (R0 + RW * 32 - 1) / a.group);
  const int kend = a.start + p_hi_wg + 1;    // keys [0, kend) reach this workgroup
  const int nt_wg = (kend + kKeys - 1) / kKeys;
  const int t0 = split * a.tps, t1 = min(nt_wg, t0 + a.tps);

  // this lane's query row
  const int row = R0 + rw * 32 + r;
  const bool valid = row < rows;
  const int p = valid ? row / a.group : a.P - 1;
  const int head = g * a.group + (valid ? row - p * a.group : 0);
  const int qpos = a.start + p;
  const long grow = (long)p * a.H + head;

  if (t0 >= t1) {                            // nothing of this split reaches the workgroup
    if (valid && h == 0)
      *reinterpret_cast<float2*>(a.ml + 2 * ((long)split * rowsH + grow)) = make_float2(kNoMax, 0.f);
    return;
  }

  // this wave's token range (wave-uniform)
  const int wrow0 = R0 + rw * 32;
  const bool wave_valid = wrow0 < rows;
  const int pw_lo = wrow0 / a.group;
  const int pw_hi = min(a.P - 1, (wrow0 + 31) / a.group);

  const uint16_t* kb = a.k + (long)g * a.skv_head;
  const uint16_t* vb = a.v + (long)g * a.skv_head;

  s16x8 qf[kKsteps];
  {
    const uint16_t* qr = a.q + (long)p * a.sq_tok + (long)head * a.sq_head;
#pragma unroll
    for (int s = 0; s < kKsteps; ++s) qf[s] = *reinterpret_cast<const s16x8*>(qr + 16 * s + 8 * h);
  }

  f32x16 o[kDblk];
#pragma unroll
  for (int t = 0; t < kDblk; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[t][i] = 0.f;
  float m = kNoMax, l = 0.f;

  uint4 kr[CH], vr[CH];
  auto load_tile = [&](int kbase) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = tid + j * NT, ti = c / NCH, cc = c - ti * NCH, krow = cc / kCR;
      const int ch = cc - krow * kCR, key = kbase + ti * kKeys + krow;
      if (key < kend) {
        kr[j] = *reinterpret_cast<const uint4*>(kb + (long)key * kD + ch * 8);
        vr[j] = *reinterpret_cast<const uint4*>(vb + (long)key * kD + ch * 8);
      } else {                               // past the last query: zeros (never NaN * 0)
        kr[j] = make_uint4(0, 0, 0, 0);
        vr[j] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = tid + j * NT, ti = c / NCH, cc = c - ti * NCH, krow = cc / kCR;
      const int ch = cc - krow * kCR;
      char* kl = lds + (buf * KS + ti) * kBuf;
      char* vl = kl + kTile;
      *reinterpret_cast<uint4*>(kl + krow * kRB + (kswz(krow, ch) << 4)) = kr[j];
      *reinterpret_cast<uint4*>(vl + krow * kRB + (vswz(krow, ch) << 4)) = vr[j];
    }
  };

  const int g16 = lane >> 4, qq = (lane & 15) >> 2, pl = lane & 3;
  const int vcol_chunk = 2 * (g16 & 1) + (pl >> 1);
  const int vsub = 8 * (pl & 1);
  const int vrow = 4 * h + qq;
  const float thr = 8.f / a.c;
  // per-lane LDS offsets, hoisted out of the tile loop (the XOR swizzles do not distribute over
  // the per-step offsets, so the compiler recomputed them every tile): K row r, chunk 2 st + h;
  // V rows 16 ks + vrow (+ 8), whose swizzle (row & 3) does not depend on ks, column block db.
  // The buffer parity, b, ks and the + 8 rows are then immediate offsets of the ds_reads.
  int koff[kKsteps], voff[kDblk];
#pragma unroll
  for (int st = 0; st < kKsteps; ++st) koff[st] = r * kRB + (kswz(r, 2 * st + h) << 4);
#pragma unroll
  for (int db = 0; db < kDblk; ++db)
    voff[db] = vrow * kRB + vsub + ((4 * (db ^ (vrow & 3)) + vcol_chunk) << 4);

  // one step: key tiles kt .. kt + KS - 1 in LDS buffer BUF, this wave's slot takes kt + ksl
  // (BUF a compile-time parity when the loop below is unrolled by two)
  auto tile = [&](const int kt, const int buf) {
    const int kstep = kt * kKeys;
    const int kbase = kstep + ksl * kKeys;
    const char* kl = lds + (buf * KS + ksl) * kBuf;
    const char* vl = kl + kTile;
    if constexpr (WAB) {
      // write-after-barrier staging: step kt + KS (in registers since the previous step) into the
      // buffer every wave finished reading before the barrier that ended the previous step, then
      // step kt + 2 KS's loads — their latency spans this step's maths
      if (kt + KS < t1) store_tile(buf ^ 1);
      if (kt + 2 * KS < t1) load_tile(kstep + 2 * KS * kKeys);
    } else {
      if (kt + KS < t1) load_tile(kstep + KS * kKeys);
    }

    if (wave_valid && kt + ksl < t1 && kbase <= a.start + pw_hi) {
      f32x16 s[2];
      if constexpr (SCHED > 0) {
        // the two 32-key chains interleaved, each K fragment read SCHED steps ahead of its MFMA
        // (the order is the sched_group_barrier pattern below)
        constexpr int DP = SCHED;
        s16x8 kf[2][kKsteps];
#pragma unroll
        for (int st = 0; st < kKsteps; ++st) {
          kf[0][st] = *reinterpret_cast<const s16x8*>(kl + koff[st]);
          kf[1][st] = *reinterpret_cast<const s16x8*>(kl + 32 * kRB + koff[st]);
        }
        const f32x16 z = {};
#pragma unroll
        for (int st = 0; st < kKsteps; ++st) {
          s[0] = mfma32<BF16>(kf[0][st], qf[st], st ? s[0] : z);
          s[1] = mfma32<BF16>(kf[1][st], qf[st], st ? s[1] : z);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * DP, 0);         // DS reads
#pragma unroll
        for (int st = 0; st < kKsteps; ++st) {
          if (st + DP < kKsteps) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);            // MFMA
        }
      } else {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#if AMDK8S_PA_ZEROC
        const f32x16 z = {};
        s[b] = mfma32<BF16>(*reinterpret_cast<const s16x8*>(kl + b * 32 * kRB + koff[0]), qf[0], z);
        constexpr int st0 = 1;
#else
#pragma unroll
        for (int i = 0; i < 16; ++i) s[b][i] = 0.f;
        constexpr int st0 = 0;
#endif
#pragma unroll
        for (int st = st0; st < kKsteps; ++st) {
          const s16x8 kf = *reinterpret_cast<const s16x8*>(kl + b * 32 * kRB + koff[st]);
          s[b] = mfma32<BF16>(kf, qf[st], s[b]);
        }
      }
      }
      if (kbase + kKeys - 1 > a.start + pw_lo) {     // the tile straddles this wave's diagonal
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (kbase + 32 * b + 8 * (i >> 2) + 4 * h + (i & 3) > qpos) s[b][i] = -INFINITY;
      }

      float lmax = s[0][0];
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) lmax = fmaxf(lmax, s[b][i]);
      if (__builtin_amdgcn_ballot_w64(lmax > m + thr) != 0) {
        const float tmax = fmaxf(lmax, __shfl_xor(lmax, 32, 64));
        const float mnew = fmaxf(m, tmax);
        const float alpha = __builtin_amdgcn_exp2f((m - mnew) * a.c);
        m = mnew;
        l *= alpha;
#pragma unroll
        for (int t = 0; t < kDblk; ++t) o[t] *= alpha;
      }
      const float mc = m * a.c;
      s16x8 pf[4];
      float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int b = ks >> 1, base = 8 * (ks & 1);
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = __builtin_amdgcn_exp2f(fmaf(s[b][base + j], a.c, -mc));
        rs0 += (e[0] + e[1]) + (e[2] + e[3]);
        rs1 += (e[4] + e[5]) + (e[6] + e[7]);
        pf[ks] = __builtin_bit_cast(
            s16x8, make_uint4(pack2<BF16>(e[0], e[1]), pack2<BF16>(e[2], e[3]),
                              pack2<BF16>(e[4], e[5]), pack2<BF16>(e[6], e[7])));
      }
      l += rs0 + rs1;

#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
        for (int db = 0; db < kDblk; ++db) {
          const char* v0 = vl + 16 * ks * kRB + voff[db];
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)v0);
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(v0 + 8 * kRB));
          const s16x8 vf = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o[db] = mfma32<BF16>(vf, pf[ks], o[db]);
        }
      }
    }

    if constexpr (!WAB) {
      if (kt + KS < t1) store_tile(buf ^ 1);
    }
    __syncthreads();
  };

  load_tile(t0 * kKeys);
  store_tile(0);
  if constexpr (WAB) {
    if (t0 + KS < t1) load_tile((t0 + KS) * kKeys);
  }
  __syncthreads();
  if constexpr (UNROLL2) {
    for (int kt = t0; kt < t1; kt += 2 * KS) {  // the buffer parity a constant in each half
      tile(kt, 0);
      if (kt + KS < t1) tile(kt + KS, 1);
    }
  } else {
    for (int kt = t0; kt < t1; kt += KS) tile(kt, ((kt - t0) / KS) & 1);
  }

  if constexpr (KS > 1) {
    // merge the key slots (the last step ended with a barrier, so the tile buffers are free):
    // slots 1.. write (O, m, l) per lane, slot 0 rescales both to the larger max and adds.  An
    // empty slot has m = kNoMax, l = 0, O = 0 and weight 0.
    float4* mo = reinterpret_cast<float4*>(lds);
    float* mls = reinterpret_cast<float*>(lds + (KS - 1) * RW * kDblk * 4 * 64 * 16);
    if (ksl > 0) {
      float4* dst = mo + ((ksl - 1) * RW + rw) * kDblk * 4 * 64 + lane;
#pragma unroll
      for (int db = 0; db < kDblk; ++db)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          dst[(db * 4 + gq) * 64] = make_float4(o[db][4 * gq], o[db][4 * gq + 1], o[db][4 * gq + 2],
                                                o[db][4 * gq + 3]);
      mls[((ksl - 1) * RW + rw) * 128 + lane] = m;
      mls[((ksl - 1) * RW + rw) * 128 + 64 + lane] = l;
    }
    __syncthreads();
    if (ksl > 0) return;
#pragma unroll
    for (int s = 1; s < KS; ++s) {
      const float m2 = mls[((s - 1) * RW + rw) * 128 + lane];
      const float l2 = mls[((s - 1) * RW + rw) * 128 + 64 + lane];
      const float M = fmaxf(m, m2);
      const float w1 = __builtin_amdgcn_exp2f((m - M) * a.c), w2 = __builtin_amdgcn_exp2f((m2 - M) * a.c);
      const float4* src = mo + ((s - 1) * RW + rw) * kDblk * 4 * 64 + lane;
#pragma unroll
      for (int db = 0; db < kDblk; ++db)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const float4 v = src[(db * 4 + gq) * 64];
          o[db][4 * gq] = fmaf(o[db][4 * gq], w1, v.x * w2);
          o[db][4 * gq + 1] = fmaf(o[db][4 * gq + 1], w1, v.y * w2);
          o[db][4 * gq + 2] = fmaf(o[db][4 * gq + 2], w1, v.z * w2);
          o[db][4 * gq + 3] = fmaf(o[db][4 * gq + 3], w1, v.w * w2);
        }
      l = fmaf(l, w1, l2 * w2);
      m = M;
    }
  }

  // epilogue: lane holds O[row][32db + 8(i>>2) + 4h + (i&3)] (unnormalised), its half of the sum
  const float lt = l + __shfl_xor(l, 32, 64);
  if (!valid) return;
  if (a.nsplit == 1) {
    const float inv = 1.f / lt;
    uint16_t* orow = a.o + (long)p * a.so_tok + (long)head * a.so_head;
#pragma unroll
    for (int db = 0; db < kDblk; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        uint2 w;
        w.x = pack2<BF16>(o[db][4 * gq] * inv, o[db][4 * gq + 1] * inv);
        w.y = pack2<BF16>(o[db][4 * gq + 2] * inv, o[db][4 * gq + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * db + 8 * gq + 4 * h) = w;
      }
    return;
  }
  const long prow = (long)split * rowsH + grow;
  float* op = a.opart + prow * kD;
#pragma unroll
  for (int db = 0; db < kDblk; ++db)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq)
      *reinterpret_cast<float4*>(op + 32 * db + 8 * gq + 4 * h) =
          make_float4(o[db][4 * gq], o[db][4 * gq + 1], o[db][4 * gq + 2], o[db][4 * gq + 3]);
  if (h == 0) *reinterpret_cast<float2*>(a.ml + 2 * prow) = make_float2(m, lt);
}

// one wave per query row (p, h): merge the nsplit partials -> normalised output
template <bool BF16>
__global__ __launch_bounds__(256) void prefill_attn_combine(const Args a) {
  const long rowsH = (long)a.P * a.H;
  const long grow = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (grow >= rowsH) return;
  float M = kNoMax;
  for (int s = 0; s < a.nsplit; ++s) {
    const float2 ml = *reinterpret_cast<const float2*>(a.ml + 2 * ((long)s * rowsH + grow));
    if (ml.y > 0.f) M = fmaxf(M, ml.x);
  }
  float L = 0.f, x0 = 0.f, x1 = 0.f;
  for (int s = 0; s < a.nsplit; ++s) {
    const long prow = (long)s * rowsH + grow;
    const float2 ml = *reinterpret_cast<const float2*>(a.ml + 2 * prow);
    if (!(ml.y > 0.f)) continue;               // empty split: its partial O was never written
    const float w = __builtin_amdgcn_exp2f((ml.x - M) * a.c);
    const float2 v = *reinterpret_cast<const float2*>(a.opart + prow * kD + 2 * lane);
    L = fmaf(ml.y, w, L);
    x0 = fmaf(v.x, w, x0);
    x1 = fmaf(v.y, w, x1);
  }
  const float inv = 1.f / L;
  const int p = (int)(grow / a.H), head = (int)(grow - (long)p * a.H);
  *reinterpret_cast<uint32_t*>(a.o + (long)p * a.so_tok + (long)head * a.so_head + 2 * lane) =
      pack2<BF16>(x0 * inv, x1 * inv);
}

struct Plan {
  int nw, ks, nrb, nsplit, tps;
};

Plan make_plan(int P, int start, int H, int Hkv, int nsplit_req, int nw_req, int ks_req) {
  // Measured on MI355X (tools/debug/prefill_attn_sweep.py, profiles/r06/prefill_attn_sweep.log):
  // * a prompt from position 0, or enough 4-wave row blocks to fill the chip: 4 waves, no split
  //   (512 @ 0: 17.6 us vs 22.5 with 8 waves; 8192 @ 0: 681 vs 725; any split only adds work);
  // * a chunk with many rows after a long prefix: 8 waves (each K/V tile feeds 256 rows) and the
  //   keys split until the grid is ONE round of 8-wave workgroups (<= 256; 512 @ 31488: 4 splits
  //   268 us, 5 splits 353, 8 splits 288; 512 @ 3072: 4 splits 51.1 us);
  // * few rows (a short chunk, a single token) after a long prefix: 4-wave row blocks, splits up
  //   to 256 workgroups (64 @ 8192: 12-16 splits 36.8-37.3 us vs 8 waves 43-49); since the key
  //   slots, the same row blocks as 8 waves x 2 slots (below).
  Plan pl;
  const int group = H / Hkv;
  const long rows = (long)P * group;
  const int ntiles = (start + P + kKeys - 1) / kKeys;
  const long base4 = (rows + 127) / 128 * Hkv, base8 = (rows + 255) / 256 * Hkv;
  int nw = 4, ns = 1, ks = 1;
  if (start > 0 && base4 < 256) {
    const int ns8 = (int)std::min<long>(256 / base8, ntiles / 12);
    if (rows >= 1024 && ns8 >= 2) {
      nw = 8;
      ns = ns8;
    } else if (ntiles >= 128) {
      // few rows after 8k+ positions: 8 waves as 4 row waves x 2 key slots (the 4-wave row block,
      // each step's two tiles to different waves), about half the splits (profiles/r06/
      // prefill_attn_plan_ab.log, same process: 64 @ 8192 34.6-37.2 vs 36.2-37.2 us, 128 @ 16000
      // 52.1-53.1 vs 55.9-57.9, one token at 31000 44.5-44.9 vs 48.0-49.1; after shorter
      // prefixes the split count gets too small: 7 @ 3000 29.7 vs 18.9, 200 @ 1000 26.1 vs 23.5)
      nw = 8;
      ks = 2;
      ns = (int)std::max<long>(1, std::min<long>(std::min<long>(256 / base4, ntiles / 16), 32));
    } else {
      ns = (int)std::max<long>(1, std::min<long>(std::min<long>(256 / base4, ntiles / 8), 32));
    }
  }
  // a grid of a round or more with long key runs: 8 waves, each staged K/V tile feeding 256 rows
  // (profiles/r06/prefill_attn_sweep_long.log: 32000 @ 0 10.07 vs 10.73 ms, 16384 @ 0 2.54 vs
  // 2.72, 12288 @ 0 1.52 vs 1.61, 4096 @ 28000 1.85 vs 2.12, 16384 @ 16384 6.67 vs 7.21; with
  // its write-after-barrier staging, profiles/r06/prefill_attn_sweep_8w_wab.log: 8192 @ 0 639 vs
  // 672 us, 4096 @ 0 182 vs 205, 3584 @ 0 145 vs 160; unrolled by two, profiles/r06/
  // prefill_attn_sweep_8w_u2.log: 2048 @ 0 60.9 vs 63.7 us, 2560 @ 0 89.4 vs 95.5; 1536 @ 0 a tie)
  static const bool long8 = [] {                // AMDK8S_PA_LONG8=0: 4 waves (A/B runs)
    const char* e = getenv("AMDK8S_PA_LONG8");
    return !e || e[0] != '0';
  }();
  if (long8 && base4 >= 256 && start + P >= 2048) nw = 8;
  // key slots, for a prompt from position 0 whose 4-wave grid is under one round (profiles/r06/
  // prefill_attn_sweep_key_slots.log): up to half a round, 4 waves as 2 row waves x 2 slots
  // (512 @ 0: 14.1 vs 17.1 us; 256 @ 0: 10.4 vs 11.0), else 8 waves as 4 x 2 (1024 @ 0: 25.4 vs
  // 28.2); a full round or more keeps one slot (2048 @ 0: 62.4 vs 68.7 with 8 x 2)
  if (start == 0 && ns == 1 && base4 <= 256) {
    ks = 2;
    if (base4 * 2 > 256) nw = 8;
  }
  if (nw_req == 4 || nw_req == 8) nw = nw_req;
  if (nsplit_req > 0) ns = nsplit_req;
  if (ks_req == 1 || ks_req == 2) ks = ks_req;
  pl.nw = nw;
  pl.ks = ks;
  const int rbr = nw / ks * 32;                // rows per row block
  pl.nrb = (int)((rows + rbr - 1) / rbr);
  ns = std::max(1, std::min(ns, ntiles));
  pl.tps = (ntiles + ns - 1) / ns;
  pl.nsplit = (ntiles + pl.tps - 1) / pl.tps;
  return pl;
}

template <bool BF16, int NW, int KS>
int launch(Args a, const Plan& pl, hipStream_t stream) {
  const long nwg = (long)pl.nrb * a.Hkv * pl.nsplit;
  if (nwg <= 0 || nwg > 0x7fffffff) return -1;
  hipLaunchKernelGGL((prefill_attn_kernel<BF16, NW, KS>), dim3((unsigned)nwg), dim3(NW * 64), 0,
                     stream, a);
  if (hipGetLastError() != hipSuccess) return -2;
  if (pl.nsplit > 1) {
    const long rowsH = (long)a.P * a.H;
    hipLaunchKernelGGL((prefill_attn_combine<BF16>), dim3((unsigned)((rowsH + 3) / 4)), dim3(256), 0,
                       stream, a);
    if (hipGetLastError() != hipSuccess) return -2;
  }
  return 0;
}

}  // namespace

extern "C" {

// fp32 workspace bytes the call with these arguments needs (0 when it does not split)
long amdk8s_llm_prefill_attn_workspace(int P, int start, int H, int Hkv, int nsplit, int nw,
                                       int ks) {
  if (P <= 0 || H <= 0 || Hkv <= 0 || H % Hkv != 0 || start < 0) return -1;
  const Plan pl = make_plan(P, start, H, Hkv, nsplit, nw, ks);
  if (pl.nsplit == 1) return 0;
  return (long)pl.nsplit * P * H * (kD + 2) * 4;
}

// Plan of the call: out[0] = waves per workgroup, out[1] = key splits, out[2] = tiles per split,
// out[3] = key slots per workgroup.
int amdk8s_llm_prefill_attn_plan(int P, int start, int H, int Hkv, int nsplit, int nw, int ks,
                                 int* out) {
  if (P <= 0 || H <= 0 || Hkv <= 0 || H % Hkv != 0 || start < 0) return -1;
  const Plan pl = make_plan(P, start, H, Hkv, nsplit, nw, ks);
  out[0] = pl.nw;
  out[1] = pl.nsplit;
  out[2] = pl.tps;
  out[3] = pl.ks;
  return 0;
}

// q: [P] x [H] rows of 128 (strides sq_tok / sq_head elements); kc / vc: one slot's [Hkv][.][128]
// slabs (stride skv_head), positions 0 .. start+P-1 valid; o: [P] x [H] rows (so_tok / so_head).
// dtype 0 = fp16, 1 = bf16.  work: >= amdk8s_llm_prefill_attn_workspace(...) bytes.
int amdk8s_llm_prefill_attn(const void* q, long sq_tok, long sq_head, const void* kc,
                            const void* vc, long skv_head, void* o, long so_tok, long so_head, int P,
                            int start, int H, int Hkv, float scale, void* work, long work_bytes,
                            int nsplit, int nw, int ks, int dtype, hipStream_t stream) {
  if (P <= 0 || H <= 0 || Hkv <= 0 || H % Hkv != 0 || start < 0) return -1;
  if ((sq_tok | sq_head | so_tok | so_head | skv_head) % 8 != 0) return -3;
  if ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(kc) |
       reinterpret_cast<uintptr_t>(vc) | reinterpret_cast<uintptr_t>(o)) % 16 != 0)
    return -3;
  if ((long)P * (H / Hkv) > 0x7fffffffL) return -1;
  const Plan pl = make_plan(P, start, H, Hkv, nsplit, nw, ks);
  const long need = pl.nsplit == 1 ? 0 : (long)pl.nsplit * P * H * (kD + 2) * 4;
  if (need > work_bytes || (need > 0 && (reinterpret_cast<uintptr_t>(work) % 16) != 0)) return -4;
  Args a;
  a.q = static_cast<const uint16_t*>(q);
  a.k = static_cast<const uint16_t*>(kc);
  a.v = static_cast<const uint16_t*>(vc);
  a.o = static_cast<uint16_t*>(o);
  a.opart = static_cast<float*>(work);
  a.ml = a.opart + (long)pl.nsplit * P * H * kD;
  a.sq_tok = sq_tok;
  a.sq_head = sq_head;
  a.so_tok = so_tok;
  a.so_head = so_head;
  a.skv_head = skv_head;
  a.P = P;
  a.start = start;
  a.H = H;
  a.Hkv = Hkv;
  a.group = H / Hkv;
  a.nrb = pl.nrb;
  a.nsplit = pl.nsplit;
  a.tps = pl.tps;
  a.c = scale * 1.4426950408889634f;
  if (dtype == 1) {
    if (pl.ks == 2) return pl.nw == 8 ? launch<true, 8, 2>(a, pl, stream) : launch<true, 4, 2>(a, pl, stream);
    return pl.nw == 8 ? launch<true, 8, 1>(a, pl, stream) : launch<true, 4, 1>(a, pl, stream);
  }
  if (pl.ks == 2) return pl.nw == 8 ? launch<false, 8, 2>(a, pl, stream) : launch<false, 4, 2>(a, pl, stream);
  return pl.nw == 8 ? launch<false, 8, 1>(a, pl, stream) : launch<false, 4, 1>(a, pl, stream);
}

}  // extern "C"
