// Decode-path kernels of the in-tree Qwen2 LLM engine (k8s_nvidia_gpus_amd/models/llm), gfx950.
//
// The reference serves a Qwen2.5-7B Q4_K_M GGUF with llama.cpp (reference
// cluster-config/apps/llm/deployment.yaml:31-34,61,76-84); decoding one token is a chain of
// matrix-vector products over ~4.4 GB of 4/6-bit weights, i.e. HBM-bound.  These kernels are laid
// out for that regime on MI355X:
//
// * Activations are quantised once per matrix input to int8 per 32 values ("Q8 act": x8, a fp32
//   scale per 32, and a pre-multiplied fp32 sum per 16 for the K-quant min / offset terms), fused
//   into the RMSNorm (amdk8s_llm_rmsnorm_q8) or the attention combine.  The GEMV inner product is
//   then v_dot4_i32_i8 on nibbles masked straight out of the weight words: ~0.5 VALU op per
//   weight, so the streaming load, not the ALU, is the bound.
// * One wavefront walks one weight row: 8 lanes x 16 B cover a 256-weight super-block, so each
//   wave-wide 16-byte load reads 8 consecutive super-blocks (1 KiB of quants) fully coalesced; a
//   wave's rows run as one software pipeline (next stage's loads in flight during this stage's
//   maths).
//   Both formats are repacked at load time into planes (Q4_K: nibbles + 16-byte block headers;
//   Q6_K: ql / qh / scales / d) so every load is aligned and a wave's header load covers 8
//   consecutive blocks in one 128-byte line.
// * The activations of the (<= 4) tokens are staged once per workgroup in LDS (x8 padded 32 B per
//   256 so the 16-lane groups of a ds_read_b128 hit disjoint banks); every wave of the workgroup
//   then streams its rows against them.
// * Epilogues are fused: bias add (q/k/v), residual add in place (o_proj, ffn_down), and the SwiGLU
//   pair mode that runs ffn_gate and ffn_up rows in the same wave and writes silu(g)*u.
// * Decode attention is split over the context (flash-decoding): per (kv head, 64-position chunk,
//   token) one workgroup scores all q heads of the GQA group with every K/V load of the chunk in
//   flight at once, and the combine kernel merges the chunks and emits the Q8 activations of the
//   o_proj input directly.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kWave = 64;
constexpr int kQ4KBytes = 144;
constexpr int kMaxTok = 4;          // tokens per GEMV launch (activations staged in LDS)
constexpr int kAttnChunk = 64;      // context positions per decode-attention workgroup
constexpr int kHeadDim = 128;
constexpr int kMaxGroup = 8;        // q heads per kv head

enum { kQ4K = 0, kQ6K = 1 };
enum { kStore = 0, kResid = 1, kPair = 2 };

__device__ __forceinline__ float h2f(uint16_t h) {
  _Float16 v;
  __builtin_memcpy(&v, &h, 2);
  return (float)v;
}

__device__ __forceinline__ uint16_t f2h(float f) {
  _Float16 v = (_Float16)f;
  uint16_t h;
  __builtin_memcpy(&h, &v, 2);
  return h;
}

__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// LDS offset of activation byte p of one token (32-byte pad per 256 bytes)
__device__ __forceinline__ int xoff(int p) { return (p >> 8) * 288 + (p & 255); }

// ---------------------------------------------------------------- split-context decode attention
// grid (Hkv, max_ctx/64, T); 256 threads.  One workgroup: the G = H/Hkv q heads of one kv head
// over the 64 positions [s*64, min(s*64+64, len)).  Scores: 4 lanes per position (32 dims each,
// all four 16-byte K loads in flight), softmax by one wave (lane = position), P.V: wave w takes
// 16 positions with all 16 V loads in flight, lane = 2 dims.  Writes the unnormalised partial
// output and (max, sum) per head.
template <int STOP>
__global__ void __launch_bounds__(256) attn_decode_kernel(const float* __restrict__ q,
                                                          const int* __restrict__ pos,
                                                          const int* __restrict__ slot,
                                                          const uint16_t* __restrict__ kc,
                                                          const uint16_t* __restrict__ vc,
                                                          int H, int Hkv, int max_ctx, int nsplit,
                                                          float scale, float* __restrict__ po,
                                                          float* __restrict__ pml) {
  __shared__ float qs[kMaxGroup][kHeadDim];
  __shared__ float ps[kMaxGroup][kAttnChunk];
  __shared__ float mls[kMaxGroup][2];
  __shared__ float opart[4][kMaxGroup][kHeadDim];
  const int kh = blockIdx.x, sp = blockIdx.y, t = blockIdx.z;
  const int G = H / Hkv;
  const int len = pos[t] + 1;
  const int p0 = sp * kAttnChunk;
  const long pidx = ((long)t * H + kh * G) * nsplit + sp;   // + g * nsplit
  if (p0 >= len) {
    if (threadIdx.x < G) {
      pml[(pidx + (long)threadIdx.x * nsplit) * 2] = -INFINITY;
      pml[(pidx + (long)threadIdx.x * nsplit) * 2 + 1] = 0.f;
    }
    return;
  }
  const int n = min(kAttnChunk, len - p0);
  const long cbase = ((long)slot[t] * Hkv + kh) * max_ctx * kHeadDim;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // K loads first (independent of q)
  const int pi = threadIdx.x >> 2, qd = threadIdx.x & 3;
  // every load is unconditional (positions clamped into the chunk): a load under a branch ends
  // its basic block and the join waits for it, which would serialise the HBM round trips
  uint4 kv[4];
  {
    const uint4* kr = reinterpret_cast<const uint4*>(kc + cbase + (long)(p0 + min(pi, n - 1))
                                                     * kHeadDim + qd * 32);
#pragma unroll
    for (int c = 0; c < 4; ++c) kv[c] = kr[c];
  }
  for (int i = threadIdx.x; i < G * kHeadDim; i += blockDim.x)
    qs[i / kHeadDim][i % kHeadDim] = q[(long)t * H * kHeadDim + (kh * G) * kHeadDim + i] * scale;
  __syncthreads();
  if (STOP == 1) { if (threadIdx.x == 0) po[blockIdx.x] = qs[0][0] + (float)kv[0].x; return; }
  float sc[kMaxGroup];
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) sc[g] = 0.f;
  {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t kw[4] = {kv[c].x, kv[c].y, kv[c].z, kv[c].w};
      float kf[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        kf[2 * e] = h2f(kw[e] & 0xffffu);
        kf[2 * e + 1] = h2f(kw[e] >> 16);
      }
#pragma unroll
      for (int g = 0; g < kMaxGroup; ++g) {
        if (g < G) {
#pragma unroll
          for (int e = 0; e < 8; ++e) sc[g] += kf[e] * qs[g][qd * 32 + c * 8 + e];
        }
      }
    }
  }
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) {
    sc[g] += __shfl_xor(sc[g], 1, kWave);
    sc[g] += __shfl_xor(sc[g], 2, kWave);
  }
  if (qd == 0) {
#pragma unroll
    for (int g = 0; g < kMaxGroup; ++g)
      if (g < G) ps[g][pi] = pi < n ? sc[g] : -INFINITY;
  }
  __syncthreads();
  if (STOP == 2) { if (threadIdx.x == 0) po[blockIdx.x] = ps[0][0]; return; }
  if (wave == 0) {
    for (int g = 0; g < G; ++g) {
      const float s = ps[g][lane];
      const float m = wave_max(s);
      const float p = lane < n ? __expf(s - m) : 0.f;
      ps[g][lane] = p;
      const float l = wave_sum(p);
      if (lane == 0) { mls[g][0] = m; mls[g][1] = l; }
    }
  }
  __syncthreads();
  if (STOP == 3) { if (threadIdx.x == 0) po[blockIdx.x] = ps[0][1]; return; }
  // P.V: wave w → positions w*16 .. w*16+15
  uint32_t vv[16];
  const uint32_t* vr = reinterpret_cast<const uint32_t*>(vc + cbase) + lane;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int p = min(wave * 16 + j, n - 1);        // ps[.][p >= n] == 0
    vv[j] = vr[(long)(p0 + p) * (kHeadDim / 2)];
  }
  float o[kMaxGroup][2];
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) o[g][0] = o[g][1] = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float v0 = h2f(vv[j] & 0xffffu), v1 = h2f(vv[j] >> 16);
#pragma unroll
    for (int g = 0; g < kMaxGroup; ++g) {
      if (g < G) {
        const float pw = ps[g][wave * 16 + j];
        o[g][0] += pw * v0;
        o[g][1] += pw * v1;
      }
    }
  }
  if (STOP == 4) { float z = 0.f; for (int g = 0; g < kMaxGroup; ++g) z += o[g][0] + o[g][1]; if (z == 123.f) po[threadIdx.x] = z; return; }
  if (STOP == 5) { float z = 0.f; for (int j = 0; j < 16; ++j) z += (float)vv[j]; if (z == 123.f) po[threadIdx.x] = z; return; }
#pragma unroll
  for (int g = 0; g < kMaxGroup; ++g) {
    if (g < G) {
      opart[wave][g][2 * lane] = o[g][0];
      opart[wave][g][2 * lane + 1] = o[g][1];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * kHeadDim; i += blockDim.x) {
    const int g = i / kHeadDim, dd = i % kHeadDim;
    const float v = opart[0][g][dd] + opart[1][g][dd] + opart[2][g][dd] + opart[3][g][dd];
    po[(pidx + (long)g * nsplit) * kHeadDim + dd] = v;
  }
  if (threadIdx.x < G) {
    const int g = threadIdx.x;
    pml[(pidx + (long)g * nsplit) * 2] = mls[g][0];
    pml[(pidx + (long)g * nsplit) * 2 + 1] = mls[g][1];
  }
}

}  // namespace
#include <cstdio>
#include <vector>
template <int S>
float run(const float* q, const int* pos, const int* slot, const uint16_t* kc, const uint16_t* vc, float* po, float* pml, int nsplit, int max_ctx) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(attn_decode_kernel<S>, dim3(4, nsplit, 1), dim3(256), 0, 0, q, pos, slot, kc, vc, 28, 4, max_ctx, nsplit, 0.088f, po, pml);
  hipEventRecord(e0);
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(attn_decode_kernel<S>, dim3(4, nsplit, 1), dim3(256), 0, 0, q, pos, slot, kc, vc, 28, 4, max_ctx, nsplit, 0.088f, po, pml);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); return ms / 200 * 1e3;
}
int main() {
  const int max_ctx = 4096;
  float *q, *po, *pml; int *pos, *slot; uint16_t *kc, *vc;
  hipMalloc(&q, 28 * 128 * 4); hipMalloc(&po, 28 * 64 * 128 * 4); hipMalloc(&pml, 28 * 64 * 8);
  hipMalloc(&pos, 4); hipMalloc(&slot, 4);
  hipMalloc(&kc, (size_t)4 * max_ctx * 128 * 2); hipMalloc(&vc, (size_t)4 * max_ctx * 128 * 2);
  hipMemset(q, 0, 28 * 128 * 4); hipMemset(kc, 0, (size_t)4 * max_ctx * 256); hipMemset(vc, 0, (size_t)4 * max_ctx * 256);
  hipMemset(slot, 0, 4);
  for (int p : {100, 1000, 4000}) {
    hipMemcpy(pos, &p, 4, hipMemcpyHostToDevice);
    int nsplit = 4; while (nsplit * 64 <= p) nsplit *= 2;
    printf("pos %d nsplit %d: vload %.2f pv %.2f\n", p, nsplit, run<5>(q, pos, slot, kc, vc, po, pml, nsplit, max_ctx), run<4>(q, pos, slot, kc, vc, po, pml, nsplit, max_ctx));
    printf("pos %d nsplit %d: kload %.2f us  scores %.2f  softmax %.2f  full %.2f\n", p, nsplit,
           run<1>(q, pos, slot, kc, vc, po, pml, nsplit, max_ctx), run<2>(q, pos, slot, kc, vc, po, pml, nsplit, max_ctx),
           run<3>(q, pos, slot, kc, vc, po, pml, nsplit, max_ctx), run<0>(q, pos, slot, kc, vc, po, pml, nsplit, max_ctx));
  }
  return 0;
}
