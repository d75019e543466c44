"""RCCL-over-xGMI collectives for multi-GPU validator / benchmark workloads (torch.distributed)."""
