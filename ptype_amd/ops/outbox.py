"""Device outbox: actor-to-actor sends emitted by GPU handlers.

A handler that sends (``kForward``, handlers.hpp) appends the message to an
outbox in HBM -- SoA columns exactly like a client ``MsgBatch`` -- reserving
slots with one atomic per wave.  ``ActorExchange.pump`` then routes the outbox
as the next epoch's batch, so chains of messages between actors anywhere in the
node run without the host touching a message (it reads one count per epoch).

Two banks: the epoch that routes bank A dispatches into bank B; ``take()``
returns A as a batch view and makes B the active bank.  A full bank counts
drops rather than overwriting (``dropped``).
"""
from __future__ import annotations

import torch

from . import _ptr
from .batch import MsgBatch


class DeviceOutbox:
    def __init__(self, capacity: int, device="cuda"):
        self.cap = int(capacity)
        self.device = torch.device(device)
        self.banks = [self._bank() for _ in range(2)]
        self.active = 0

    def _bank(self) -> dict:
        d, n = self.device, self.cap
        return {"actor": torch.zeros(n, dtype=torch.int32, device=d), "a0": torch.zeros(n, dtype=torch.int64, device=d),
                "a1": torch.zeros(n, dtype=torch.int64, device=d), "a2": torch.zeros(n, dtype=torch.int64, device=d),
                "method": torch.zeros(n, dtype=torch.int16, device=d),
                "count": torch.zeros(2, dtype=torch.int64, device=d)}  # [reserved, dropped]

    @property
    def bank(self) -> dict:
        return self.banks[self.active]

    def view(self):
        """(pointer list, capacity) of the active bank for the dispatch kernel."""
        b = self.bank
        return [_ptr(b["actor"]), _ptr(b["a0"]), _ptr(b["a1"]), _ptr(b["a2"]), _ptr(b["method"]),
                _ptr(b["count"])], self.cap

    def pending(self) -> int:
        """Messages waiting in the active bank (synchronises with the device)."""
        return min(int(self.bank["count"][0].item()), self.cap)

    @property
    def dropped(self) -> int:
        return int(sum(int(b["count"][1].item()) for b in self.banks))

    def take(self, n: int | None = None) -> MsgBatch:
        """The active bank's messages as a batch; the other bank becomes active (emptied)."""
        n = self.pending() if n is None else n
        b = self.bank
        self.active ^= 1
        self.bank["count"][0] = 0
        return MsgBatch(b["actor"][:n], b["a0"][:n], b["a1"][:n], b["a2"][:n], b["method"][:n])

    # ---- CPU reference (the plain-PyTorch dispatch appends here)
    def emit_cpu(self, actor: int, method: int, a0: int, a1: int, a2: int) -> None:
        b = self.bank
        slot = int(b["count"][0])
        b["count"][0] += 1
        if slot >= self.cap:
            b["count"][1] += 1
            return
        b["actor"][slot] = actor
        b["method"][slot] = method
        b["a0"][slot], b["a1"][slot], b["a2"][slot] = a0, a1, a2
