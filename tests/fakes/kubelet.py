"""The fake kubelet of the CPU tests lives in the package (the bring-up rehearsal uses it too)."""
from k8s_nvidia_gpus_amd.operator.kubelet_stub import KubeletStub as FakeKubelet  # noqa: F401
