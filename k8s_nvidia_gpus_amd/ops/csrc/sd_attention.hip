// Flash-attention forward for the SD1.5 model family (gfx950, wave64, fp16 / bf16, fp32 softmax).
//
//   O[n, q, h*d : (h+1)*d] = softmax(Q Kᵀ · scale) V   per (n, head), no mask (SD attention)
//
// Shapes served: head dim d ∈ {40, 64, 80, 128, 160} (SD1.5 UNet: 40 / 80 / 160 at 64² / 32² / 16²
// latents), any Lq, any Lk (self-attention 64…4096 tokens, cross-attention 77 text tokens).  Q, K, V
// are read through row strides, so they can be column slices of ONE fused q|k|v projection output.
//
// Work split: a workgroup = 4 waves; each wave owns QT×16 query rows (QT = 1 or 2) and streams the
// keys in tiles of 64 staged in LDS.  All products run on v_mfma_f32_16x16x32_{f16,bf16}:
//   S  = Q Kᵀ : A = Q fragment (registers for the whole kernel, d zero-padded to 32·QK_STEPS),
//              B = K fragment (ds_read_b128 of 8 consecutive d of one key row);
//   O += P V  : A = P fragment, B = V fragment, both column reads of row-major LDS tiles via the
//              gfx950 transpose read ds_read_b64_tr_b16 (P is written to LDS as Pᵀ[key][q] with one
//              8-byte store per key: the accumulator already holds 4 consecutive q of one key).
// Online softmax in the exp2 domain (scale·log2e folded into one FMA per score).  The row max over
// the 16 lanes that share a row group is 4 DPP steps (quad_perm xor1 / xor2, row_half_mirror,
// row_mirror) — no LDS round trip; the row sum is kept per lane and reduced once at the end.
// EXEC stays full everywhere (DPP and the transpose read need it): out-of-range keys are zero
// rows in LDS and −inf scores, out-of-range query rows are computed and not stored.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) short lds_short;

constexpr int kKeys = 64;      // keys per tile
constexpr int kWaves = 4;
constexpr int kPad = 8;        // LDS row padding (elements) against bank conflicts

template <bool BF16>
__device__ __forceinline__ f32x4 mfma16(const s16x8 a, const s16x8 b, const f32x4 c) {
  if constexpr (BF16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

template <bool BF16>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  if constexpr (BF16) {
    // one v_cvt_pk_bf16_f32 (gfx950, round-to-nearest-even) instead of ~10 integer ops: P is
    // packed for every score, and this conversion was ~40 % of the softmax VALU work
    const bf16x2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
  } else {
    _Float16 a = (_Float16)lo, b = (_Float16)hi;
    uint16_t ua, ub;
    __builtin_memcpy(&ua, &a, 2);
    __builtin_memcpy(&ub, &b, 2);
    return (uint32_t)ua | ((uint32_t)ub << 16);
  }
}

template <bool BF16>
__device__ __forceinline__ uint16_t to16(float f) {
  if constexpr (BF16) {
    return (uint16_t)f32_to_bf16(f);
  } else {
    _Float16 a = (_Float16)f;
    uint16_t u;
    __builtin_memcpy(&u, &a, 2);
    return u;
  }
}

__device__ __forceinline__ float dpp_f(float v, int ctrl_sel) {
  int x = __float_as_int(v);
  int r;
  switch (ctrl_sel) {  // constant-folded at every call site
    case 0: r = __builtin_amdgcn_mov_dpp(x, 0xB1, 0xf, 0xf, false); break;   // quad_perm [1,0,3,2]
    case 1: r = __builtin_amdgcn_mov_dpp(x, 0x4E, 0xf, 0xf, false); break;   // quad_perm [2,3,0,1]
    case 2: r = __builtin_amdgcn_mov_dpp(x, 0x141, 0xf, 0xf, false); break;  // row_half_mirror
    default: r = __builtin_amdgcn_mov_dpp(x, 0x140, 0xf, 0xf, false); break; // row_mirror
  }
  return __int_as_float(r);
}

// max / sum over the 16 lanes of a DPP row (all lanes end with the result)
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f(v, 0));
  v = fmaxf(v, dpp_f(v, 1));
  v = fmaxf(v, dpp_f(v, 2));
  return fmaxf(v, dpp_f(v, 3));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f(v, 0);
  v += dpp_f(v, 1);
  v += dpp_f(v, 2);
  return v + dpp_f(v, 3);
}

struct AttnArgs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* o;
  int H, Lq, Lk, d;
  long sqb, sqr, skb, skr, svb, svr, sob, sor;  // batch / row strides in elements
  float c;                                       // scale * log2(e)
};

// QK_STEPS = ceil(d/32) (reduction steps of S), DT = ceil(d/16) (16-column tiles of O), QT = q tiles per wave
template <bool BF16, int QK_STEPS, int DT, int QT, int D>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const AttnArgs a) {
  constexpr int DK = QK_STEPS * 32;   // K row width in LDS (zero padded)
  constexpr int DV = DT * 16;         // V row width in LDS (zero padded)
  constexpr int KS = DK + kPad;       // LDS row strides (elements)
  constexpr int VS = DV + kPad;
  constexpr int QW = QT * 16;         // query rows per wave
  constexpr int PS = QW + 4;          // Pᵀ row stride (elements; keeps 8-byte alignment)
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* kl = smem;                          // [64][KS]
  uint16_t* vl = kl + kKeys * KS;               // [64][VS]
  uint16_t* pl = vl + kKeys * VS;               // [wave][64][PS]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;   // 16-lane group, lane in group
  const int nh = blockIdx.y, n = nh / a.H, head = nh % a.H;
  const int q0 = blockIdx.x * (kWaves * QW) + wave * QW;
  constexpr int d = D;                // head dim as a compile-time constant: the K/V tile loader's
                                      // row/column split below is shifts, not integer divisions
  const uint16_t* qb = a.q + n * a.sqb + (long)head * d;
  const uint16_t* kb = a.k + n * a.skb + (long)head * d;
  const uint16_t* vb = a.v + n * a.svb + (long)head * d;
  uint16_t* pw = pl + wave * (kKeys * PS);

  // zero the whole K/V image once: pad columns stay zero, partial tiles leave zero rows
  for (int i = tid; i < kKeys * (KS + VS) / 8; i += 256)
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(0, 0, 0, 0);

  // Q fragments (A operand): lane holds Q[q0 + 16qt + c16][32s + 8g .. +7]
  s16x8 qf[QT][QK_STEPS];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int qrow = min(q0 + qt * 16 + c16, a.Lq - 1);
#pragma unroll
    for (int s = 0; s < QK_STEPS; ++s) {
      const int col = 32 * s + 8 * g;
      if (col < d)
        qf[qt][s] = *reinterpret_cast<const s16x8*>(qb + qrow * a.sqr + col);
      else
        qf[qt][s] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }

  f32x4 o[QT][DT];
  float m[QT][4], l[QT][4];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
    for (int t = 0; t < DT; ++t) o[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m[qt][i] = -INFINITY;
      l[qt][i] = 0.f;
    }
  }

  // K/V tile loader: 16-byte chunks, CK = d/8 per row
  constexpr int CK = d / 8;
  constexpr int nchunks = kKeys * CK;
  constexpr int kMaxPer = QK_STEPS;  // chunks per thread: 64 rows * d/8 <= 256 * QK_STEPS
  uint4 kreg[kMaxPer], vreg[kMaxPer];
  auto load_tile = [&](int kbase) {
#pragma unroll
    for (int j = 0; j < kMaxPer; ++j) {
      const int ch = tid + j * 256;
      if (ch < nchunks) {
        const int r = ch / CK, cc = (ch - r * CK) * 8;
        const int key = kbase + r;
        if (key < a.Lk) {
          kreg[j] = *reinterpret_cast<const uint4*>(kb + key * a.skr + cc);
          vreg[j] = *reinterpret_cast<const uint4*>(vb + key * a.svr + cc);
        } else {
          kreg[j] = make_uint4(0, 0, 0, 0);
          vreg[j] = make_uint4(0, 0, 0, 0);
        }
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int j = 0; j < kMaxPer; ++j) {
      const int ch = tid + j * 256;
      if (ch < nchunks) {
        const int r = ch / CK, cc = (ch - r * CK) * 8;
        *reinterpret_cast<uint4*>(kl + r * KS + cc) = kreg[j];
        *reinterpret_cast<uint4*>(vl + r * VS + cc) = vreg[j];
      }
    }
  };

  const int ntiles = (a.Lk + kKeys - 1) / kKeys;
  constexpr float kThr = 8.f;              // P <= 2^8 between rescales (exact in fp16 / bf16)
  const float thr = kThr / a.c;            // the same margin in raw score units
  load_tile(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    const int kbase = kt * kKeys;
    __syncthreads();  // previous tile's LDS reads done (and the zero fill, on the first pass)
    store_tile();
    __syncthreads();
    if (kt + 1 < ntiles) load_tile(kbase + kKeys);  // in flight under this tile's MFMAs
    const bool partial = kbase + kKeys > a.Lk;

    // S = Q Kᵀ for QT × (16 q × 64 keys): each K fragment is read from LDS once and feeds the
    // MFMAs of all QT query tiles (the QT independent accumulators also hide MFMA latency)
    f32x4 sall[QT][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) sall[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < QK_STEPS; ++s) {
        const s16x8 kf = *reinterpret_cast<const s16x8*>(kl + (16 * t + c16) * KS + 32 * s + 8 * g);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) sall[qt][t] = mfma16<BF16>(qf[qt][s], kf, sall[qt][t]);
      }
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      f32x4* sacc = sall[qt];
      if (partial) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (kbase + 16 * t + c16 >= a.Lk) sacc[t] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      }
      // online softmax; this lane's rows are q = 4g + i.  Deferred max (T13): the row max and the
      // O / l rescale run only when some score of the wave exceeds its row's running max by more
      // than kThr (exp2 units), so P stays <= 2^kThr and exact; otherwise the old max is kept.
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float lmax = fmaxf(fmaxf(sacc[0][i], sacc[1][i]), fmaxf(sacc[2][i], sacc[3][i]));
        if (__builtin_amdgcn_ballot_w64(lmax > m[qt][i] + thr) != 0) {  // wave-uniform branch
          const float tmax = row16_max(lmax);
          const float mnew = fmaxf(m[qt][i], tmax);
          const float alpha = __builtin_amdgcn_exp2f((m[qt][i] - mnew) * a.c);
          m[qt][i] = mnew;
          l[qt][i] *= alpha;
#pragma unroll
          for (int t = 0; t < DT; ++t) o[qt][t][i] *= alpha;
        }
        const float mc = m[qt][i] * a.c;
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sacc[t][i], a.c, -mc));
          sacc[t][i] = p;
          rs += p;
        }
        l[qt][i] += rs;
      }
      // Pᵀ[key][q]: this lane holds keys 16t + c16, q = 4g .. 4g+3 of tile qt → one 8-byte store
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint2 w;
        w.x = pack2<BF16>(sacc[t][0], sacc[t][1]);
        w.y = pack2<BF16>(sacc[t][2], sacc[t][3]);
        *reinterpret_cast<uint2*>(pw + (16 * t + c16) * PS + qt * 16 + 4 * g) = w;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // O += P V over two 32-key steps; column reads via ds_read_b64_tr_b16:
    // lane 16g + 4qq + p supplies row (key) 32ks + 8g + qq (+4), columns 4p .. 4p+3 of the block
    const int qq = c16 >> 2, p4 = (c16 & 3) * 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int krow = 32 * ks + 8 * g + qq;
      s16x8 pf[QT];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((lds_short*)pw + krow * PS + qt * 16 + p4));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((lds_short*)pw + (krow + 4) * PS + qt * 16 + p4));
        pf[qt] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((lds_short*)vl + krow * VS + 16 * t + p4));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((lds_short*)vl + (krow + 4) * VS + 16 * t + p4));
        const s16x8 vf = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) o[qt][t] = mfma16<BF16>(pf[qt], vf, o[qt][t]);
      }
    }
  }

  // epilogue: row sums across the 16 lanes, normalise, store the d valid columns
  uint16_t* ob = a.o + n * a.sob + (long)head * d;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float inv = 1.f / row16_sum(l[qt][i]);
      const int q = q0 + qt * 16 + 4 * g + i;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        const int col = 16 * t + c16;
        if (q < a.Lq && col < d) ob[q * a.sor + col] = to16<BF16>(o[qt][t][i] * inv);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Transposed-score variant (default): S^T = K Q^T and O^T = V^T P^T on the same MFMA.  With the
// operands swapped, a lane's S accumulator holds 4 keys (16t + 4g + i) of ONE query (c16), which
// is exactly the B-operand layout P^T needs for the P·V MFMA (keys 4g..4g+3 of two 16-key tiles
// per 32-key step, a consistent permutation of the reduction index shared with V^T).  P therefore
// never leaves registers: no P store / transpose read through LDS and no wave barrier per tile,
// and the per-query max / sum live in one register per query tile (a 4-lane shuffle on the rare
// rescale and once in the epilogue).  V^T comes from the same ds_read_b64_tr_b16 column reads as
// before, only with the key rows permuted to match.
template <bool BF16, int QK_STEPS, int DT, int QT, int D>
__global__ __launch_bounds__(256) void attn_fwd_t_kernel(const AttnArgs a) {
  constexpr int DK = QK_STEPS * 32;
  constexpr int DV = DT * 16;
  constexpr int KS = DK + kPad;
  constexpr int VS = DV + kPad;
  constexpr int QW = QT * 16;
  constexpr int d = D;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* kl = smem;                // [64][KS]
  uint16_t* vl = kl + kKeys * KS;     // [64][VS]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int nh = blockIdx.y, n = nh / a.H, head = nh % a.H;
  const int q0 = blockIdx.x * (kWaves * QW) + wave * QW;
  const uint16_t* qb = a.q + n * a.sqb + (long)head * d;
  const uint16_t* kb = a.k + n * a.skb + (long)head * d;
  const uint16_t* vb = a.v + n * a.svb + (long)head * d;

  for (int i = tid; i < kKeys * (KS + VS) / 8; i += 256)
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(0, 0, 0, 0);

  // Q^T fragments (B operand): lane holds Q[q0 + 16qt + c16][32s + 8g .. +7]
  s16x8 qf[QT][QK_STEPS];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int qrow = min(q0 + qt * 16 + c16, a.Lq - 1);
#pragma unroll
    for (int s = 0; s < QK_STEPS; ++s) {
      const int col = 32 * s + 8 * g;
      if (col < d)
        qf[qt][s] = *reinterpret_cast<const s16x8*>(qb + qrow * a.sqr + col);
      else
        qf[qt][s] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }

  f32x4 o[QT][DT];                    // O^T: lane holds O[q = c16][16t + 4g + i]
  float m[QT], l[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
    for (int t = 0; t < DT; ++t) o[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    m[qt] = -INFINITY;
    l[qt] = 0.f;
  }

  constexpr int CK = d / 8;
  constexpr int nchunks = kKeys * CK;
  constexpr int kMaxPer = QK_STEPS;
  uint4 kreg[kMaxPer], vreg[kMaxPer];
  auto load_tile = [&](int kbase) {
#pragma unroll
    for (int j = 0; j < kMaxPer; ++j) {
      const int ch = tid + j * 256;
      if (ch < nchunks) {
        const int r = ch / CK, cc = (ch - r * CK) * 8;
        const int key = kbase + r;
        if (key < a.Lk) {
          kreg[j] = *reinterpret_cast<const uint4*>(kb + key * a.skr + cc);
          vreg[j] = *reinterpret_cast<const uint4*>(vb + key * a.svr + cc);
        } else {
          kreg[j] = make_uint4(0, 0, 0, 0);
          vreg[j] = make_uint4(0, 0, 0, 0);
        }
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int j = 0; j < kMaxPer; ++j) {
      const int ch = tid + j * 256;
      if (ch < nchunks) {
        const int r = ch / CK, cc = (ch - r * CK) * 8;
        *reinterpret_cast<uint4*>(kl + r * KS + cc) = kreg[j];
        *reinterpret_cast<uint4*>(vl + r * VS + cc) = vreg[j];
      }
    }
  };

  const int ntiles = (a.Lk + kKeys - 1) / kKeys;
  constexpr float kThr = 8.f;
  const float thr = kThr / a.c;
  const int qq = c16 >> 2, p4 = (c16 & 3) * 4;
  load_tile(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    const int kbase = kt * kKeys;
    __syncthreads();
    store_tile();
    __syncthreads();
    if (kt + 1 < ntiles) load_tile(kbase + kKeys);
    const bool partial = kbase + kKeys > a.Lk;

    // S^T tiles: sall[qt][t][i] = score(key 16t + 4g + i, query c16)
    f32x4 sall[QT][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) sall[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < QK_STEPS; ++s) {
        const s16x8 kf = *reinterpret_cast<const s16x8*>(kl + (16 * t + c16) * KS + 32 * s + 8 * g);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) sall[qt][t] = mfma16<BF16>(kf, qf[qt][s], sall[qt][t]);
      }
    }
    s16x8 pf[QT][2];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      if (partial) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (kbase + 16 * t + 4 * g + i >= a.Lk) sall[qt][t][i] = -INFINITY;
      }
      float lmax = sall[qt][0][0];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) lmax = fmaxf(lmax, sall[qt][t][i]);
      if (__builtin_amdgcn_ballot_w64(lmax > m[qt] + thr) != 0) {   // wave-uniform, rare
        float tmax = fmaxf(lmax, __shfl_xor(lmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mnew = fmaxf(m[qt], tmax);
        const float alpha = __builtin_amdgcn_exp2f((m[qt] - mnew) * a.c);
        m[qt] = mnew;
        l[qt] *= alpha;
#pragma unroll
        for (int t = 0; t < DT; ++t) o[qt][t] *= alpha;
      }
      const float mc = m[qt] * a.c;
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sall[qt][t][i], a.c, -mc));
          sall[qt][t][i] = p;
          rs += p;
        }
      l[qt] += rs;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f32x4 lo = sall[qt][2 * ks], hi = sall[qt][2 * ks + 1];
        const uint32_t w0 = pack2<BF16>(lo[0], lo[1]), w1 = pack2<BF16>(lo[2], lo[3]);
        const uint32_t w2 = pack2<BF16>(hi[0], hi[1]), w3 = pack2<BF16>(hi[2], hi[3]);
        pf[qt][ks] = __builtin_bit_cast(s16x8, make_uint4(w0, w1, w2, w3));
      }
    }

    // O^T += V^T P^T: reduction position 8g + j <-> key 32ks + 4g + j (j < 4), 32ks + 16 + 4g + j - 4
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int rlo = 32 * ks + 4 * g + qq;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((lds_short*)vl + rlo * VS + 16 * t + p4));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((lds_short*)vl + (rlo + 16) * VS + 16 * t + p4));
        const s16x8 vf = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) o[qt][t] = mfma16<BF16>(vf, pf[qt][ks], o[qt][t]);
      }
    }
  }

  uint16_t* ob = a.o + n * a.sob + (long)head * d;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float lt = l[qt] + __shfl_xor(l[qt], 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const float inv = 1.f / lt;
    const int q = q0 + qt * 16 + c16;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const int col = 16 * t + 4 * g;
      if (q < a.Lq && col < d) {
        uint2 w;
        w.x = pack2<BF16>(o[qt][t][0] * inv, o[qt][t][1] * inv);
        w.y = pack2<BF16>(o[qt][t][2] * inv, o[qt][t][3] * inv);
        *reinterpret_cast<uint2*>(ob + q * a.sor + col) = w;
      }
    }
  }
}

// amdk8s_attention_set_variant(): -1 = auto (head dims 40 / 64 / 80 / 128 / 160 → attn_d128.hip's
// 32x32x16 kernel, any other → the transposed kernel), 0 = transposed (P in registers),
// 1 = P via LDS, 2 = the 32x32x16 kernel
int g_variant = -1;

template <bool BF16, int QK, int DT, int QT, int D>
int launch(const AttnArgs& a, int NH, hipStream_t stream) {
  constexpr int KS = QK * 32 + kPad, VS = DT * 16 + kPad, PS = QT * 16 + 4;
  const int rows = kWaves * QT * 16;
  dim3 grid((a.Lq + rows - 1) / rows, NH);
  if (g_variant <= 0 || g_variant == 2) {
    const size_t lds = (size_t)(kKeys * KS + kKeys * VS) * 2;
    hipLaunchKernelGGL((attn_fwd_t_kernel<BF16, QK, DT, QT, D>), grid, dim3(256), lds, stream, a);
  } else {
    const size_t lds = (size_t)(kKeys * KS + kKeys * VS + kWaves * kKeys * PS) * 2;
    hipLaunchKernelGGL((attn_fwd_kernel<BF16, QK, DT, QT, D>), grid, dim3(256), lds, stream, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int g_qt_override = 0;   // amdk8s_attention_set_qt(): 0 = heuristic, else 1 / 2 / 4

template <bool BF16, int QK, int DT, int D>
int launch_qt(const AttnArgs& a, int NH, hipStream_t stream) {
  // K fragments (one LDS read per 16x32 step) and V fragments are shared by the QT query tiles of
  // a wave; QT = 2 wherever that still leaves >= 256 workgroups (one per CU), QT = 1 otherwise.
  // d = 128 (Wan2.1) takes QT = 4 when that still covers ~all CUs: with P kept in registers the
  // transposed kernel fits it without spills and reuses every K/V fragment 4x
  // (tools/attn_probe.py at 2x12 heads x 2560 tokens: QT 1 / 2 / 4 = 182 / 164 / 132 us).
  const long wg2 = (long)((a.Lq + 127) / 128) * NH;
  const long wg4 = (long)((a.Lq + 255) / 256) * NH;
  int qt = wg2 >= 256 ? 2 : 1;
  if constexpr (DT == 8) {
    if (g_variant <= 0 && wg4 >= 224) qt = 4;
  }
  if (g_qt_override == 1 || g_qt_override == 2) qt = g_qt_override;
  if constexpr (DT == 8) {
    if (g_qt_override == 4) qt = 4;
    if (qt == 4) return launch<BF16, QK, DT, 4, D>(a, NH, stream);
  }
  if (qt == 2) return launch<BF16, QK, DT, 2, D>(a, NH, stream);
  return launch<BF16, QK, DT, 1, D>(a, NH, stream);
}

template <bool BF16>
int dispatch(const AttnArgs& a, int NH, hipStream_t stream) {
  switch (a.d) {
    case 40: return launch_qt<BF16, 2, 3, 40>(a, NH, stream);
    case 64: return launch_qt<BF16, 2, 4, 64>(a, NH, stream);
    case 80: return launch_qt<BF16, 3, 5, 80>(a, NH, stream);
    case 128: return launch_qt<BF16, 4, 8, 128>(a, NH, stream);
    case 160: return launch_qt<BF16, 5, 10, 160>(a, NH, stream);
    default: return -1;
  }
}

}  // namespace

extern "C" int amdk8s_attention_m32_supported(int d);
extern "C" int amdk8s_attention_m32_fwd(const void* q, const void* k, const void* v, void* o, int N,
                                        int H, int Lq, int Lk, int d, int sqb, int sqr, int skb,
                                        int skr, int svb, int svr, int sor, float scale, int dtype,
                                        hipStream_t stream);

extern "C" {

void amdk8s_attention_set_qt(int qt) { g_qt_override = qt; }
void amdk8s_attention_set_variant(int v) { g_variant = v; }

int amdk8s_attention_supported(int d, int Lq, int Lk) {
  if (Lq <= 0 || Lk <= 0) return 0;
  return (d == 40 || d == 64 || d == 80 || d == 128 || d == 160) ? 1 : 0;
}

// q/k/v/o: fp16 or bf16 (dtype 0 / 1), element strides; o row stride `sor`, batch stride Lq*sor.
int amdk8s_attention_fwd(const void* q, const void* k, const void* v, void* o, int N, int H, int Lq,
                         int Lk, int d, int sqb, int sqr, int skb, int skr, int svb, int svr,
                         int sor, float scale, int dtype, hipStream_t stream) {
  if (!amdk8s_attention_supported(d, Lq, Lk) || N <= 0 || H <= 0) return -1;
  // 16-byte loads of 8 consecutive elements: every row start must stay 16-byte aligned
  if ((sqr | skr | svr | sqb | skb | svb | sor) % 8 != 0) return -3;
  // auto: the 32x32x16 kernel wherever its 128-row workgroups still fill the chip; tiny problems
  // (SD1.5 16² latents: 256 tokens) keep the 64-row legacy kernel (10.6 vs 16.2 us at d = 160,
  // profiles/r03/b/attn_probe.log)
  const bool m32 = g_variant == 2 ||
                   (g_variant == -1 && (long)((Lq + 127) / 128) * N * H >= 128);
  if (m32 && amdk8s_attention_m32_supported(d))
    return amdk8s_attention_m32_fwd(q, k, v, o, N, H, Lq, Lk, d, sqb, sqr, skb, skr, svb, svr, sor,
                                    scale, dtype, stream);
  if ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v)) % 16 != 0)
    return -3;
  AttnArgs a;
  a.q = static_cast<const uint16_t*>(q);
  a.k = static_cast<const uint16_t*>(k);
  a.v = static_cast<const uint16_t*>(v);
  a.o = static_cast<uint16_t*>(o);
  a.H = H;
  a.Lq = Lq;
  a.Lk = Lk;
  a.d = d;
  a.sqb = sqb;
  a.sqr = sqr;
  a.skb = skb;
  a.skr = skr;
  a.svb = svb;
  a.svr = svr;
  a.sob = (long)Lq * sor;
  a.sor = sor;
  a.c = scale * 1.4426950408889634f;
  return dtype == 1 ? dispatch<true>(a, N * H, stream) : dispatch<false>(a, N * H, stream);
}

}  // extern "C"
