"""GPU-initiated remote calls (csrc/hip/xcall.hpp).

``PeerCaller(shm_name, device)`` registers a lane on another process's
persistent dispatcher (same node: this GPU or a peer over xGMI) and runs calls
from a KERNEL on this process's GPU: the request goes into the server's HBM
lane, the reply lands in this GPU's HBM, no host on the path.  Every call's
round trip is stamped with the device clock (s_memrealtime, 100 MHz).

Reference: one remote request/reply, cluster/rpc.go:59-67.
"""
from __future__ import annotations

import torch

from . import hip
from .records import METHOD_CALC_MULTIPLY

TICK_NS = 10.0  # s_memrealtime runs at 100 MHz


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
