"""Hand-written gfx950 HIP kernels (MFMA GEMM, vectorAdd, device fills) and their bindings."""
from .kernels import (  # noqa: F401
    KernelLibraryError,
    fill_uniform_bf16,
    gemm_bf16,
    gemm_bf16_nt,
    gemm_sample_check,
    gemm_shape_supported,
    library,
    library_path,
    vector_add,
    vector_add_bandwidth,
)
