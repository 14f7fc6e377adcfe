"""Multi-GPU (RCCL over xGMI) load generators and the distributed bench harness helpers."""
