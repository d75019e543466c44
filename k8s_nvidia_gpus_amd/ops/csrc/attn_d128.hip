// Flash-attention forward on 32x32x16 MFMAs for head dims 40 / 64 / 80 / 128 / 160 (Wan2.1 DiT:
// 128; SD1.5 UNet: 40 / 80 / 160 at 64² / 32² / 16² latents), gfx950.
//
//   O[n, q, h*D : (h+1)*D] = softmax(Q Kᵀ · scale) V   per (n, head), no mask, bf16 / fp16 I/O
//
// Built around v_mfma_f32_32x32x16 (one 32×32×16 product per instruction, half the instruction count
// of the 16×16×32 form for the same FLOPs) and the operand-swapped orientation, so the softmax never
// leaves registers:
//
//   Sᵀ[key][q] = K · Qᵀ     A = K fragment   (ds_read_b128, row-major K image, XOR-swizzled chunks)
//                           B = Qᵀ fragment  (registers for the whole kernel: 8 × 8 bf16 per lane)
//   Oᵀ[d][q]  += Vᵀ · Pᵀ    A = Vᵀ fragment  (ds_read_b64_tr_b16 transpose reads of a row-major V image)
//                           B = Pᵀ           (the Sᵀ accumulator converted in place: the 32×32 result
//                                             has its column (= query) on the lane and its rows (= keys)
//                                             in registers, which is exactly a B-operand fragment with a
//                                             permuted reduction order that the V reads reproduce)
//
// A lane therefore owns ONE query (lane & 31) and 32 of the 64 keys of a tile (its partner lane ^ 32
// holds the other 32): the row max is 31 local max ops, the row sum 32 adds, and the two halves meet
// only on the rare rescale (deferred max: P ≤ 2^8 between rescales, exact in bf16/fp16) and once in
// the epilogue.  Scores run in the exp2 domain with scale·log2(e) folded into one FMA per score.
//
// Work split: a workgroup = NW waves × 32 query rows; K/V tiles of 64 keys are staged through
// registers into a double-buffered LDS image (16 KiB K + 16 KiB V per buffer): the next tile's global
// loads are issued before this tile's MFMAs and written to the other buffer after them (one barrier
// per tile).  LDS images (256-byte rows, 16-byte chunks):
//   K: chunk c of key row r at c ^ (r & 15)        → the 32-row ds_read_b128 of a 32x32x16 A fragment
//                                                     hits 16 distinct chunks per lane group (no conflict)
//   V: chunk c of key row r at c ^ ((r & 3) << 2)  → the 4-row transpose read of a 32-lane half spans
//                                                     16 distinct chunks (no conflict)
// Workgroups are mapped XCD-major (consecutive block ids land on different XCDs), so the q-blocks of
// one head share an XCD's L2 for that head's K/V.
//
// The SD-family kernel (sd_attention.hip) keeps every other head dim; this file replaces it for d=128
// (reference workload: the Wan2.1 T2V DiT the reference's ComfyUI client drives,
// generate_wan_t2v.py:305-312, 347).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kKeys = 64;                    // keys per tile

// Per-head-dim geometry.  QK^T runs over DK = D rounded up to 16 (k-steps of the 32x32x16 MFMA),
// P·V over DV = D rounded up to 32 (32-row blocks of O^T); an LDS row holds max(DK, DV) elements,
// padded to RB = 128 / 256 / 512 bytes so one of two conflict-free swizzle families applies, and
// the pad columns stay zero (they add nothing to QK^T and produce O^T rows that are not stored).
template <int D>
struct Geo {
  static_assert(D % 8 == 0 && D >= 16 && D <= 256, "head dim: multiple of 8 in [16, 256]");
  static constexpr int DK = (D + 15) / 16 * 16;
  static constexpr int DV = (D + 31) / 32 * 32;
  static constexpr int DP = DK > DV ? DK : DV;
  static constexpr int RB = DP * 2 <= 128 ? 128 : DP * 2 <= 256 ? 256 : 512;
  static constexpr int KSTEPS = DK / 16;
  static constexpr int DBLK = DV / 32;
  static constexpr int CR = D / 8;             // 16-byte chunks of a global row
  static constexpr int TILE = kKeys * RB;      // bytes per operand tile
  static constexpr int BUF = 2 * TILE;         // K + V
  static constexpr int LDS = 2 * BUF;          // double buffered
  static constexpr bool PAD = CR * 16 < RB;
  // K image: the 32-row ds_read_b128 of an A fragment; V image: the 4-row transpose reads
  __device__ static constexpr int kswz(int row, int ch) {
    return RB == 128 ? ch ^ ((row >> 1) & 7) : ch ^ (row & 15);
  }
  __device__ static constexpr int vswz(int row, int ch) {
    return RB == 128 ? ch ^ (((row >> 1) & 1) << 2) : ch ^ ((row & 3) << 2);
  }
};

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
    const bf16x2 v = {(__bf16)lo, (__bf16)hi};   // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
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
  int H, Lq, Lk, nqb;
  long sqb, sqr, skb, skr, svb, svr, sob, sor;  // batch / row strides in elements
  float c;                                       // scale * log2(e)
  int causal;                                    // 1: query i sees keys 0 .. i (top-left aligned)
};

template <bool BF16, int NW, int D>
__global__ __launch_bounds__(NW * 64, 2) void attn_m32_kernel(const Args a) {
  using G = Geo<D>;
  constexpr int NT = NW * 64;
  constexpr int NCH = kKeys * G::CR;            // 16-byte chunks per operand tile
  constexpr int CH = (NCH + NT - 1) / NT;       // ... per thread
  __shared__ __attribute__((aligned(16))) char lds[G::LDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;

  // XCD-major block → (head, q-block): blocks b, b+8, b+16, … share an XCD; give each XCD a
  // contiguous run of work items (bijective for any grid size).
  int work;
  {
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, idx = bid >> 3;
    const int qn = nwg >> 3, rem = nwg & 7;
    work = (xcd < rem ? xcd * (qn + 1) : rem * (qn + 1) + (xcd - rem) * qn) + idx;
  }
  const int nh = work / a.nqb, qblk = work - nh * a.nqb;
  const int n = nh / a.H, head = nh - n * a.H;
  const int q0 = qblk * (NW * 32) + wave * 32;
  const uint16_t* qb = a.q + n * a.sqb + (long)head * D;
  const uint16_t* kb = a.k + n * a.skb + (long)head * D;
  const uint16_t* vb = a.v + n * a.svb + (long)head * D;

  // Qᵀ fragments (B operand of the k-steps over d): lane holds Q[q0 + r][16s + 8h .. +7] (zero
  // past D)
  s16x8 qf[G::KSTEPS];
  {
    const int qrow = min(q0 + r, a.Lq - 1);
#pragma unroll
    for (int s = 0; s < G::KSTEPS; ++s)
      qf[s] = (16 * s + 8 * h < D)
                  ? *reinterpret_cast<const s16x8*>(qb + qrow * a.sqr + 16 * s + 8 * h)
                  : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }

  f32x16 o[G::DBLK];
#pragma unroll
  for (int t = 0; t < G::DBLK; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[t][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  uint4 kr[CH], vr[CH];
  auto load_tile = [&](int kbase) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = tid + j * NT, row = c / G::CR, ch = c - row * G::CR;
      const int key = kbase + row;
      if (c < NCH && key < a.Lk) {
        kr[j] = *reinterpret_cast<const uint4*>(kb + key * a.skr + ch * 8);
        vr[j] = *reinterpret_cast<const uint4*>(vb + key * a.svr + ch * 8);
      } else {
        kr[j] = make_uint4(0, 0, 0, 0);
        vr[j] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* kl = lds + buf * G::BUF;
    char* vl = kl + G::TILE;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = tid + j * NT, row = c / G::CR, ch = c - row * G::CR;
      if (c < NCH) {
        *reinterpret_cast<uint4*>(kl + row * G::RB + (G::kswz(row, ch) << 4)) = kr[j];
        *reinterpret_cast<uint4*>(vl + row * G::RB + (G::vswz(row, ch) << 4)) = vr[j];
      }
    }
  };

  // per-lane LDS offsets that do not depend on the tile
  const int kofs = r * G::RB;                    // K row r (and r + 32: + 32 rows)
  const int g16 = lane >> 4, qq = (lane & 15) >> 2, p = lane & 3;
  // V transpose read: row (key) 4h + qq (+8, + 16·step), byte column 64·db + 32·(g16&1) + 8p
  const int vcol_chunk = 2 * (g16 & 1) + (p >> 1);
  const int vsub = 8 * (p & 1);
  const int vrow = 4 * h + qq;

  // causal: no key past the workgroup's last query row (workgroup-uniform)
  const int klim = a.causal ? min(a.Lk, qblk * (NW * 32) + NW * 32) : a.Lk;
  const int ntiles = (klim + kKeys - 1) / kKeys;
  const float thr = 8.f / a.c;                   // deferred-max margin in raw score units
  load_tile(0);
  if constexpr (G::PAD) {      // pad columns of both buffers read as zeros for the whole kernel
    for (int i = tid; i < G::LDS / 16; i += NT) reinterpret_cast<uint4*>(lds)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int kbase = kt * kKeys;
    const char* kl = lds + (kt & 1) * G::BUF;
    const char* vl = kl + G::TILE;
    if (kt + 1 < ntiles) load_tile(kbase + kKeys);   // in flight under this tile's MFMAs

    // ---- Sᵀ = K Qᵀ: two 32-key blocks × KSTEPS k-steps over d
    f32x16 s[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[b][i] = 0.f;
#pragma unroll
      for (int st = 0; st < G::KSTEPS; ++st) {
        const s16x8 kf = *reinterpret_cast<const s16x8*>(
            kl + b * 32 * G::RB + kofs + (G::kswz(r, 2 * st + h) << 4));
        s[b] = mfma32<BF16>(kf, qf[st], s[b]);
      }
    }
    // keys past Lk (zero rows in the image) score -inf; causal: so do keys past the query
    if (kbase + kKeys > a.Lk || (a.causal && kbase + kKeys - 1 > q0)) {
      const int qi = a.causal ? q0 + r : 0x7fffffff;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kbase + 32 * b + 8 * (i >> 2) + 4 * h + (i & 3);
          if (key >= a.Lk || key > qi) s[b][i] = -INFINITY;
        }
    }

    // ---- online softmax with a deferred max (rescale only when a score passes m + 8/c)
    float lmax = s[0][0];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) lmax = fmaxf(lmax, s[b][i]);
    if (__builtin_amdgcn_ballot_w64(lmax > m + thr) != 0) {    // wave-uniform, rare after tile 0
      const float tmax = fmaxf(lmax, __shfl_xor(lmax, 32, 64));
      const float mnew = fmaxf(m, tmax);
      const float alpha = __builtin_amdgcn_exp2f((m - mnew) * a.c);
      m = mnew;
      l *= alpha;
#pragma unroll
      for (int t = 0; t < G::DBLK; ++t) o[t] *= alpha;
    }
    const float mc = m * a.c;
    s16x8 pf[4];                                 // Pᵀ B fragments of the 4 16-key steps
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

    // ---- Oᵀ += Vᵀ Pᵀ: k-step ks covers keys 16ks + {4h + 0..3, 8 + 4h + 0..3} for lane half h
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int r0 = 16 * ks + vrow, r1 = r0 + 8;      // same swizzle row class for both
      const char* v0 = vl + r0 * G::RB + vsub;
      const char* v1 = vl + r1 * G::RB + vsub;
#pragma unroll
      for (int db = 0; db < G::DBLK; ++db) {
        const int c0 = G::vswz(r0, 4 * db + vcol_chunk), c1 = G::vswz(r1, 4 * db + vcol_chunk);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(v0 + (c0 << 4)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(v1 + (c1 << 4)));
        const s16x8 vf = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[db] = mfma32<BF16>(vf, pf[ks], o[db]);
      }
    }

    if (kt + 1 < ntiles) store_tile((kt + 1) & 1);   // other buffer: its last reads were a barrier ago
    __syncthreads();
  }

  // ---- epilogue: lane holds O[q0 + r][32db + 8(i>>2) + 4h + (i&3)]
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = 1.f / lt;
  const int q = q0 + r;
  if (q < a.Lq) {
    uint16_t* orow = a.o + n * a.sob + (long)head * D + (long)q * a.sor;
#pragma unroll
    for (int db = 0; db < G::DBLK; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (32 * db + 8 * g + 4 * h >= D) continue;     // pad rows of Oᵀ
        uint2 w;
        w.x = pack2<BF16>(o[db][4 * g] * inv, o[db][4 * g + 1] * inv);
        w.y = pack2<BF16>(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * db + 8 * g + 4 * h) = w;
      }
  }
}

template <bool BF16, int NW, int D>
int launch(const Args& a0, int NH, hipStream_t stream) {
  Args a = a0;
  a.nqb = (a.Lq + NW * 32 - 1) / (NW * 32);
  const long nwg = (long)a.nqb * NH;
  if (nwg <= 0 || nwg > 0x7fffffff) return -1;
  hipLaunchKernelGGL((attn_m32_kernel<BF16, NW, D>), dim3((unsigned)nwg), dim3(NW * 64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <bool BF16, int D>
int launch_nw(const Args& a, int NH, int nw, hipStream_t stream) {
  return nw == 8 ? launch<BF16, 8, D>(a, NH, stream) : launch<BF16, 4, D>(a, NH, stream);
}

template <bool BF16>
int dispatch_d(const Args& a, int d, int NH, int nw, hipStream_t stream) {
  switch (d) {
    case 40: return launch_nw<BF16, 40>(a, NH, nw, stream);
    case 64: return launch_nw<BF16, 64>(a, NH, nw, stream);
    case 80: return launch_nw<BF16, 80>(a, NH, nw, stream);
    case 128: return launch_nw<BF16, 128>(a, NH, nw, stream);
    case 160: return launch_nw<BF16, 160>(a, NH, nw, stream);
    default: return -1;
  }
}

int g_nw = 0;   // amdk8s_attention_d128_set_nw(): 0 = heuristic, 4 or 8 waves per workgroup

}  // namespace

extern "C" {

void amdk8s_attention_d128_set_nw(int nw) { g_nw = nw; }

int amdk8s_attention_m32_supported(int d) {
  return d == 40 || d == 64 || d == 80 || d == 128 || d == 160;
}

// Same contract as amdk8s_attention_fwd (sd_attention.hip): element strides, 16-byte aligned rows,
// output row stride `sor`, batch stride Lq*sor; dtype 0 = fp16, 1 = bf16.
static int m32_fwd(const void* q, const void* k, const void* v, void* o, int N, int H, int Lq,
                   int Lk, int d, int sqb, int sqr, int skb, int skr, int svb, int svr, int sor,
                   float scale, int dtype, int causal, hipStream_t stream);

int amdk8s_attention_m32_fwd(const void* q, const void* k, const void* v, void* o, int N, int H,
                             int Lq, int Lk, int d, int sqb, int sqr, int skb, int skr, int svb,
                             int svr, int sor, float scale, int dtype, hipStream_t stream) {
  return m32_fwd(q, k, v, o, N, H, Lq, Lk, d, sqb, sqr, skb, skr, svb, svr, sor, scale, dtype, 0,
                 stream);
}

// Causal self-attention (query i attends to keys 0 .. i; Lq == Lk): the CLIP text encoder of SD1.5
// (77 tokens, d = 64), same contract as amdk8s_attention_m32_fwd otherwise.
int amdk8s_attention_causal_fwd(const void* q, const void* k, const void* v, void* o, int N, int H,
                                int L, int d, int sqb, int sqr, int skb, int skr, int svb, int svr,
                                int sor, float scale, int dtype, hipStream_t stream) {
  return m32_fwd(q, k, v, o, N, H, L, L, d, sqb, sqr, skb, skr, svb, svr, sor, scale, dtype, 1,
                 stream);
}

static int m32_fwd(const void* q, const void* k, const void* v, void* o, int N, int H, int Lq,
                   int Lk, int d, int sqb, int sqr, int skb, int skr, int svb, int svr, int sor,
                   float scale, int dtype, int causal, hipStream_t stream) {
  if (N <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || !amdk8s_attention_m32_supported(d)) return -1;
  if (causal && Lq != Lk) return -1;
  if ((sqr | skr | svr | sqb | skb | svb | sor) % 8 != 0) return -3;
  if ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o)) % 16 != 0)
    return -3;
  Args a;
  a.q = static_cast<const uint16_t*>(q);
  a.k = static_cast<const uint16_t*>(k);
  a.v = static_cast<const uint16_t*>(v);
  a.o = static_cast<uint16_t*>(o);
  a.H = H;
  a.Lq = Lq;
  a.Lk = Lk;
  a.nqb = 0;
  a.sqb = sqb;
  a.sqr = sqr;
  a.skb = skb;
  a.skr = skr;
  a.svb = svb;
  a.svr = svr;
  a.sob = (long)Lq * sor;
  a.sor = sor;
  a.c = scale * 1.4426950408889634f;
  a.causal = causal;
  // 8 waves (256 query rows) per workgroup: at the Wan shapes it beats 4 waves even where it
  // leaves CUs idle (2x12 heads x 2560 tokens = 240 workgroups: 88 vs 99 us; 32 760 tokens:
  // 12.4 vs 13.6 ms — profiles/r03/attn_probe_v1.log); 4 waves only for very short sequences
  const long nh = (long)N * H;
  int nw = ((long)((Lq + 255) / 256) * nh >= 128) ? 8 : 4;
  if (g_nw == 4 || g_nw == 8) nw = g_nw;
  return dtype == 1 ? dispatch_d<true>(a, d, N * H, nw, stream)
                    : dispatch_d<false>(a, d, N * H, nw, stream);
}

int amdk8s_attention_d128_fwd(const void* q, const void* k, const void* v, void* o, int N, int H,
                              int Lq, int Lk, int sqb, int sqr, int skb, int skr, int svb, int svr,
                              int sor, float scale, int dtype, hipStream_t stream) {
  return amdk8s_attention_m32_fwd(q, k, v, o, N, H, Lq, Lk, 128, sqb, sqr, skb, skr, svb, svr, sor,
                                  scale, dtype, stream);
}

}  // extern "C"
