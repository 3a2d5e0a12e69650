"""Multi-GPU workload plumbing (torch.distributed over RCCL/xGMI) for pods with several GPUs."""
