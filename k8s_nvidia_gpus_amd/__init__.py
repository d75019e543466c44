"""k8s_nvidia_gpus_amd — an MI355X-native Kubernetes GPU-enablement stack.

Same capabilities as christianshub/k8s-nvidia-gpus (Ansible → RKE2 → Flux → GPU operator →
validated GPU workloads), re-designed for AMD Instinct MI355X (gfx950):

* ``ops``       hand-written CDNA4 HIP kernels (bf16 MFMA GEMM, vectorAdd) + ctypes bindings
* ``parallel``  RCCL-over-xGMI collectives (torch.distributed, one process per GPU)
* ``models``    the workloads the operator schedules: validator, GEMM benchmark, SD1.5 service
* ``operator``  device plugin (amd.com/gpu), node labeller, metrics exporter, partition manager,
                validator orchestration, driver readiness, CDI / OCI-hook configuration
* ``utils``     KFD sysfs topology, config, Prometheus text format, logging

The Python package name is the importable spelling of ``k8s-nvidia-gpus_amd``.
"""

__version__ = "0.1.0"

RESOURCE_NAME = "amd.com/gpu"
RUNTIME_CLASS = "amd"
GFX_TARGET = "gfx950"
GFX_TARGET_VERSION = 90500
