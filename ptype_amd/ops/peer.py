"""GPU-initiated remote calls (csrc/hip/xcall.hpp).

``PeerCaller(shm_name, device)`` registers a lane on another process's
persistent dispatcher (same node: this GPU or a peer over xGMI) and runs calls
from a KERNEL on this process's GPU: the request goes into a lane of the
server's shared-memory segment and the reply comes back in the lane's reply
slot -- memory this process maps itself, so a dead server costs a timeout, not
a fault -- with no host on the path.  Every call's
round trip is stamped with the device clock (s_memrealtime, 100 MHz).

Reference: one remote request/reply, cluster/rpc.go:59-67.
"""
from __future__ import annotations

import torch

from . import hip
from .records import METHOD_CALC_MULTIPLY

TICK_NS = 10.0  # s_memrealtime runs at 100 MHz
_ATTACHED: list = []  # relays handed to a dispatcher (kept until process exit; see PeerRelay)


class PeerCaller:
    def __init__(self, shm_name: str, device=None, timeout_s: float = 10.0):
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._lane = hip().PeerLane(shm_name, self.device.index, timeout_s)

    @property
    def lane(self) -> int:
        return self._lane.lane

    def call(self, actor, a0=None, a1=None, a2=None, method: int | torch.Tensor = METHOD_CALC_MULTIPLY,
             timeout_s: float = 5.0):
        """Calls ``actor[k](a0[k], a1[k], a2[k])`` one after another from one
        GPU lane; returns ``(value int64, status int32, rtt_ns float64, done)``."""
        dev = self.device
        actor = torch.as_tensor(actor, dtype=torch.int32, device=dev).reshape(-1).contiguous()
        n = actor.numel()

        def col(x):
            if x is None:
                return None
            return torch.as_tensor(x, dtype=torch.int64, device=dev).reshape(-1).expand(n).contiguous()

        c0, c1, c2 = col(a0), col(a1), col(a2)
        mcol = None
        mu = 0
        if isinstance(method, torch.Tensor):
            mcol = method.to(device=dev, dtype=torch.int16).reshape(-1).contiguous()
        else:
            mu = int(method)
        val = torch.zeros(n, dtype=torch.int64, device=dev)
        st = torch.zeros(n, dtype=torch.int32, device=dev)
        ticks = torch.zeros(n, dtype=torch.int64, device=dev)
        p = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        stream = torch.cuda.current_stream(dev).cuda_stream
        done = self._lane.call(p(actor), p(mcol), mu, p(c0), p(c1), p(c2), n, p(val), p(st), p(ticks),
                               float(timeout_s), stream)
        return val, st, ticks.to(torch.float64) * TICK_NS, int(done)


class PeerRelay:
    """Handler-initiated remote calls: ``n_lanes``
    GPU peer lanes on another process's dispatcher, handed to ``server`` (this
    process's ``DeviceServer``) as its relay table.  A request to ``server``
    with method ``METHOD_RELAY`` -- actor = the REMOTE actor, a0 = the remote
    method, a1/a2 = its arguments -- is forwarded by the dispatcher wave itself:
    published into a free lane of the peer's segment and parked there while the
    wave keeps serving; the remote reply, when it lands, completes the call (a
    timed-out relay answers kStatusNotDelivered and fails that call only).  A
    handler that calls another server, with no host between the hops
    (reference: a handler dialling another node, cluster/rpc.go:59-67).

    The native relay (its lanes and device table) is kept for the life of the
    process once attached: the dispatcher wave reads the table until its next
    idle refresh, so freeing it earlier could pull memory out from under a
    running wave."""

    def __init__(self, server, shm_name: str, device=None, n_lanes: int = 8, timeout_s: float = 1.0):
        dev = torch.device(device if device is not None else "cuda")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self._relay = hip().PeerRelay(shm_name, dev.index, int(n_lanes), float(timeout_s))
        self._server = server
        server.set_relay(self._relay.table)
        _ATTACHED.append(self._relay)

    @property
    def lanes(self) -> int:
        return self._relay.lanes

    def slots(self) -> list[int]:
        """Per lane ``[seq, suspect]`` as the device table holds them (the dispatcher
        wave writes its slot words back when it parks or the table is replaced)."""
        return [int(x) for x in self._relay.slots()]

    def detach(self):
        self._server.set_relay(0)
