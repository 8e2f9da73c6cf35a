"""Multi-GPU data plane: RCCL (torch.distributed "nccl") exchange epochs, and the
elastic generation manager that survives rank failures."""
from .elastic import ElasticDataPlane, Excluded, RankFailure, ring_placement  # noqa: F401
from .exchange import ActorExchange, capacity_for  # noqa: F401
