"""The data plane's process group as a compiled object (VERDICT r4 Missing #3).

``NativeGroup`` wraps ``_core.DataPlane`` (csrc/core/dataplane.hpp): the RCCL
communicator of a service's GPUs, formed through the replicated store
(``ncclGetUniqueId`` published under ``store/_ptype/nccl/<service>/<gen>/uid``,
then ``ncclCommInitRank`` on every member), aborted with ``ncclCommAbort`` when
a generation fails, and re-formed over the lease-driven membership -- with no
torch process group and no TCPStore.  The native engines take its communicator
directly; the few host-level agreements of the exchange (a chunk geometry, a
re-send count) and the buddy-replica moves go through the same communicator.

Reference: Join brings a member up in one compiled call (cluster/cluster.go:28-84,
:161-196); a dead member is seen through its lapsed lease
(cluster/registry.go:51-86).
"""
from __future__ import annotations

import torch


class NativeGroup:
    """A formed ``_core.DataPlane`` generation, seen as a process group."""

    def __init__(self, dp):
        self.dp = dp

    @classmethod
    def join(cls, core_cluster, service: str, me: str, device_for_rank, world: int, timeout_s: float = 30.0):
        """Generation 0 over the first ``world`` registered nodes of ``service``;
        ``device_for_rank(rank)`` names this member's GPU once its rank is known."""
        from .. import _core

        dp = _core.DataPlane(core_cluster, service, me, -1, float(timeout_s))
        nodes = dp.wait_nodes(int(world))
        if me not in nodes:
            raise RuntimeError(f"{me} is not among the first {world} nodes of {service!r}: {nodes}")
        dev = device_for_rank(nodes.index(me))
        dp.set_device(int(dev.index if dev.index is not None else torch.cuda.current_device()))
        dp.form(0, nodes)
        return cls(dp)

    @staticmethod
    def available() -> bool:
        from .. import _core

        return bool(_core.DataPlane.available())

    # ------------------------------------------------------------------ group view
    @property
    def rank(self) -> int:
        return int(self.dp.rank)

    @property
    def size(self) -> int:
        return int(self.dp.size)

    @property
    def gen(self) -> int:
        return int(self.dp.gen)

    @property
    def members(self) -> list[str]:
        return list(self.dp.members)

    def comm_ptr(self) -> int:
        return int(self.dp.comm)

    def allreduce_max(self, values) -> list[int]:
        return [int(x) for x in self.dp.allreduce_max([int(v) for v in values])]

    def allreduce_max_dev(self, t: torch.Tensor, stream: int) -> None:
        """In place on an int64 device tensor, enqueued on ``stream``."""
        self.dp.allreduce_max_dev(t.data_ptr(), t.numel(), int(stream))

    def sendrecv(self, send: torch.Tensor | None, dst: int, recv: torch.Tensor | None, src: int) -> None:
        """One point-to-point exchange (synchronous): ``send`` to rank ``dst`` and
        ``recv`` from rank ``src`` (either may be None)."""
        torch.cuda.current_stream().synchronize()  # the tensors' producers are done
        self.dp.sendrecv(send.data_ptr() if send is not None else 0,
                         send.numel() * send.element_size() if send is not None else 0, dst if send is not None else -1,
                         recv.data_ptr() if recv is not None else 0,
                         recv.numel() * recv.element_size() if recv is not None else 0, src if recv is not None else -1)

    def barrier(self) -> None:
        self.dp.barrier()

    # ------------------------------------------------------------------ lifecycle
    def abort(self) -> None:
        self.dp.abort()

    def async_error(self) -> int:
        return int(self.dp.async_error())

    def recover(self, grace_s: float) -> list[str]:
        """Abort, wait for the lease-driven membership to settle, form the next generation."""
        return list(self.dp.recover(float(grace_s)))

    def form(self, gen: int, members: list[str]) -> int:
        return int(self.dp.form(int(gen), list(members)))
