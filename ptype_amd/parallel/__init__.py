"""Multi-GPU data plane: RCCL (torch.distributed "nccl") exchange epochs."""
from .exchange import ActorExchange, capacity_for  # noqa: F401
