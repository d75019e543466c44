// Shared declarations for the native (C/C++/HIP) tools of the MI355X Kubernetes GPU stack.
#pragma once

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define AMDK8S_HIP_CHECK(expr)                                                              \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) {                                                                 \
      std::fprintf(stderr, "HIP error %s (%d) at %s:%d: %s\n", hipGetErrorString(_e),      \
                   (int)_e, __FILE__, __LINE__, #expr);                                     \
      std::exit(2);                                                                         \
    }                                                                                       \
  } while (0)

extern "C" {
// k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950.hip
int amdk8s_gemm_bf16_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                        int ldb, int ldc, hipStream_t stream);
int amdk8s_gemm_bf16_nt_w4(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                           int ldb, int ldc, hipStream_t stream);
int amdk8s_gemm_bf16_nt_w4a(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                            int ldb, int ldc, hipStream_t stream);
int amdk8s_gemm_f16_nt_w4a(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                           int ldb, int ldc, hipStream_t stream);
int amdk8s_gemm_bf16_nt_sample_check(const void* A, const void* B, const int* coords, float* out,
                                     int nsamples, int K, int lda, int ldb, hipStream_t stream);
// k8s_nvidia_gpus_amd/ops/csrc/gemm_fp8_gfx950.hip
int amdk8s_gemm_fp8_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                       int ldb, int ldc, hipStream_t stream);
int amdk8s_gemm_fp8_nt_f8a(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                           int ldb, int ldc, hipStream_t stream);
int amdk8s_gemm_fp8_nt_sample_check(const void* A, const void* B, const int* coords, float* out,
                                    int nsamples, int K, int lda, int ldb, hipStream_t stream);
// k8s_nvidia_gpus_amd/ops/csrc/vector_add.hip
int amdk8s_vector_add_f32(const float* a, const float* b, float* c, int n, hipStream_t stream);
int amdk8s_vector_add_f32_bw(const float* a, const float* b, float* c, long n, int num_cus,
                             hipStream_t stream);
int amdk8s_vector_add_blocks(int n);
// k8s_nvidia_gpus_amd/ops/csrc/loadgen.hip
int amdk8s_hbm_stream(int mode, const void* src, void* dst, long bytes, int num_cus,
                      int blocks_per_cu, uint32_t* sink, hipStream_t stream);
int amdk8s_fp32_fma(int blocks, int iters, float* sink, hipStream_t stream);
double amdk8s_fp32_fma_flop(int blocks, int iters);
int amdk8s_fp64_mfma(int blocks, int iters, double* sink, hipStream_t stream);
double amdk8s_fp64_mfma_flop(int blocks, int iters);
// k8s_nvidia_gpus_amd/ops/csrc/fill.hip
int amdk8s_fill_uniform_bf16(void* dst, long n, unsigned long long seed, float lo, float hi,
                             hipStream_t stream);
int amdk8s_fill_uniform_fp8(void* dst, long n, unsigned long long seed, float lo, float hi,
                            hipStream_t stream);
}
#endif  // __HIPCC__

#include <cstdint>
#include <string>
#include <vector>

namespace amdk8s {

// One GPU (or compute partition) as the KFD topology describes it.
// Parsed from /sys/class/kfd/kfd/topology/nodes/<id>/properties (+ gpu_id, name).
struct KfdNode {
  int node_id = -1;             // topology node index
  uint32_t gpu_id = 0;          // KFD gpu_id (0 for CPU nodes)
  std::string name;             // e.g. "gfx950" or the marketing name file content
  uint32_t gfx_target_version = 0;  // e.g. 90500 for gfx950
  int drm_render_minor = -1;    // /dev/dri/renderD<minor>
  uint64_t unique_id = 0;       // stable per-ASIC id (partitions of one ASIC share it)
  uint32_t location_id = 0;     // PCI BDF-derived location
  uint32_t domain = 0;          // PCI domain
  uint32_t simd_count = 0;
  uint32_t cu_count() const { return simd_count / 4; }  // CDNA: 4 SIMDs per CU
  uint32_t array_count = 0;
  uint32_t num_xcc = 0;         // XCDs owned by this node (8 = SPX, 1 = CPX on MI355X)
  uint64_t vram_bytes = 0;      // sum of mem_banks/*/properties size_in_bytes (heap_type 1/2)
  uint32_t vendor_id = 0;
  uint32_t device_id = 0;
  uint32_t max_engine_clk_fcompute = 0;
  uint32_t io_links_xgmi = 0;   // number of XGMI io_links (type 11)
  bool is_gpu() const { return gpu_id != 0 && simd_count > 0; }
  std::string pci_bdf() const;  // "dddd:bb:dd.f"
};

// Reads a KFD topology tree rooted at `sysfs_root` (default /sys/class/kfd/kfd/topology).
// Tests pass a fabricated tree.  Returns false and fills `err` on a malformed tree.
bool read_kfd_topology(const std::string& sysfs_root, std::vector<KfdNode>* nodes,
                       std::string* err);

std::string json_escape(const std::string& s);

}  // namespace amdk8s
