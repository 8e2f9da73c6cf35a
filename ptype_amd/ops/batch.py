"""Batch ``Send`` data path: route/bucket (K1), dispatch (K3), complete (K8).

See ``csrc/hip/batch.hip`` for the kernels and the epoch-slot layout.  Each op
takes optional pre-allocated outputs so the steady state (bench / exchange
epochs) allocates nothing and can be captured in a hipGraph.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _check, _ptr, _stream, hip
from .records import (FLAG_ROUTED, FLAG_VALID, METHOD_CALC_MULTIPLY, STATUS_NO_ACTOR, STATUS_OVERFLOW,
                      make_requests, split_requests)
from .table import RegistryTable, actor_keys, mix64

# workspace words (int64): [0:4) stats [nomatch, overflow, failed, -]
WS_WORDS = 4
STAT_NOMATCH, STAT_OVERFLOW, STAT_FAILED = 0, 1, 2
ROUTE_NO_ACTOR = 0xFF
MAX_MBOX = 1 << 24  # route word = rank | mbox << 8


def new_workspace(device) -> torch.Tensor:
    return torch.zeros(WS_WORDS, dtype=torch.int64, device=device)


def ws_stats(ws: torch.Tensor) -> torch.Tensor:
    return ws[0:4]


def stripe_capacity(M: int, R: int, slack: float = 0.05) -> int:
    """Per-destination slot capacity for uniformly spread traffic: mean + slack +
    an 8-sigma margin, so overflow is a statistical non-event at bench sizes."""
    import math

    mean = M / R
    return int(math.ceil(mean * (1 + slack) + 8 * math.sqrt(max(mean, 1.0)) + 64))


@dataclass
class MsgBatch:
    """Client-side batch of messages, structure-of-arrays (GPU-native layout).

    ``actor`` int32[M] global actor ids; ``a0``/``a1``/``a2`` int64[M] payload
    columns (``a1``/``a2`` optional -> 0); ``method`` one uniform method id or an
    int16[M] column.
    """

    actor: torch.Tensor
    a0: torch.Tensor
    a1: torch.Tensor | None = None
    a2: torch.Tensor | None = None
    method: int | torch.Tensor = METHOD_CALC_MULTIPLY

    @property
    def M(self) -> int:
        return self.actor.numel()

    @property
    def device(self):
        return self.actor.device

    def slice(self, lo: int, hi: int) -> "MsgBatch":
        f = (lambda t: None if t is None else t[lo:hi])
        m = self.method if isinstance(self.method, int) else self.method[lo:hi]
        return MsgBatch(self.actor[lo:hi], self.a0[lo:hi], f(self.a1), f(self.a2), m)

    def index_select(self, idx: torch.Tensor) -> "MsgBatch":
        f = (lambda t: None if t is None else t.index_select(0, idx))
        m = self.method if isinstance(self.method, int) else self.method.index_select(0, idx)
        return MsgBatch(self.actor.index_select(0, idx), self.a0.index_select(0, idx), f(self.a1), f(self.a2), m)

    @staticmethod
    def from_records(req: torch.Tensor) -> "MsgBatch":
        """AoS int64[M,4] records -> SoA batch."""
        actor, method, _, a0, a1, a2 = split_requests(req)
        return MsgBatch(actor.to(torch.int32).contiguous(), a0.contiguous(), a1.contiguous(), a2.contiguous(),
                        method.to(torch.int16).contiguous())

    def to_records(self) -> torch.Tensor:
        m = self.method if isinstance(self.method, int) else self.method.to(torch.int64)
        return make_requests(self.actor.to(torch.int64) & 0xFFFFFFFF, m, self.a0, self.a1, self.a2)


def gen_requests(M: int, n_actors: int, method: int = METHOD_CALC_MULTIPLY, seed: int = 0, device="cuda",
                 out: MsgBatch | None = None) -> MsgBatch:
    """Synthetic client load: M calls (A, B) to uniformly hashed actors in [0, n_actors)."""
    device = torch.device(device)
    if out is None:
        out = MsgBatch(torch.empty(M, dtype=torch.int32, device=device), torch.empty(M, dtype=torch.int64, device=device),
                       torch.empty(M, dtype=torch.int64, device=device), None, method)
    if device.type == "cuda":
        hip().gen_requests(_ptr(out.actor), _ptr(out.a0), _ptr(out.a1), M, int(n_actors), int(seed) & (2**64 - 1),
                           _stream(out.actor))
        return out
    i = np.arange(M, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = mix64(np.uint64(seed & (2**64 - 1)) ^ (i * np.uint64(0x9E3779B97F4A7C15)))
    out.actor.copy_(torch.from_numpy((h % np.uint64(n_actors)).astype(np.int64)).to(torch.int32))
    out.a0.copy_(torch.from_numpy(((h >> np.uint64(20)) & np.uint64(0xFFFF)).astype(np.int64) - 0x8000))
    out.a1.copy_(torch.from_numpy(((h >> np.uint64(40)) & np.uint64(0xFFFF)).astype(np.int64)))
    return out


class RouteWorkspace:
    """Per-epoch scratch of the route kernels (route words + block histograms)."""

    def __init__(self, M: int, R: int, device):
        device = torch.device(device)
        G, _ = hip().route_grid(max(M, 1)) if device.type == "cuda" else (1, M)
        self.M, self.R = M, R
        self.route = torch.empty(max(M, 1), dtype=torch.int32, device=device)
        self.hist = torch.empty(G * (R + 1), dtype=torch.int32, device=device)
        self.ws = new_workspace(device)


def route(batch: MsgBatch, table: RegistryTable, R: int, C: int, rank_self: int = 0,
          sendbuf: torch.Tensor | None = None, perm: torch.Tensor | None = None,
          rws: RouteWorkspace | None = None):
    """K1: resolve each message's actor in the GPU registry and place it, in
    message order, into its destination rank's epoch slot as a 32-B wire record.

    Returns ``(sendbuf int64[R*(C+1), 4], perm int32[M], stats int64[4])``.
    """
    M = batch.M
    dev = batch.device
    if batch.actor.dtype != torch.int32 or batch.a0.dtype != torch.int64:
        raise TypeError("MsgBatch: actor must be int32 and a0..a2 int64")
    if sendbuf is None:
        sendbuf = torch.empty(R * (C + 1), 4, dtype=torch.int64, device=dev)
    if perm is None:
        perm = torch.empty(M, dtype=torch.int32, device=dev)
    if rws is None or rws.M < M or rws.R != R:
        rws = RouteWorkspace(M, R, dev)
    rws.ws.zero_()
    uniform = isinstance(batch.method, int)
    if dev.type == "cuda":
        mcol = None if uniform else batch.method.to(torch.int16).contiguous()
        d, n_dir = table.directory()
        hip().route(_ptr(batch.actor), _ptr(batch.a0), _ptr(batch.a1), _ptr(batch.a2), _ptr(mcol),
                    int(batch.method) if uniform else 0, M, _ptr(table.table), table.cap, _ptr(d), n_dir, R, C,
                    _ptr(sendbuf),
                    _ptr(perm), _ptr(rws.route), _ptr(rws.hist), _ptr(rws.ws), rank_self, _stream(batch.actor))
        return sendbuf, perm, ws_stats(rws.ws)
    # ---- CPU reference: bit-identical layout (stable message order per destination) ----
    actor = batch.actor.to(torch.int64) & 0xFFFFFFFF
    rank, mbox = table.lookup(actor_keys(actor))
    rank = rank.to(torch.int64)
    mbox = mbox.to(torch.int64)
    ok = (rank >= 0) & (rank < R) & (mbox < MAX_MBOX)
    method = torch.full((M,), int(batch.method), dtype=torch.int64) if uniform else batch.method.to(torch.int64)
    z = torch.zeros(M, dtype=torch.int64)
    a1 = z if batch.a1 is None else batch.a1
    a2 = z if batch.a2 is None else batch.a2
    w0 = (mbox & 0xFFFFFFFF) | ((method & 0xFFFF) << 32) | ((FLAG_VALID | FLAG_ROUTED) << 48)
    routed = torch.stack([w0, batch.a0, a1, a2], dim=1)
    perm.fill_(-2)
    overflow = 0
    for d in range(R):
        idx = torch.nonzero(ok & (rank == d)).flatten()
        n = idx.numel()
        k = min(n, C)
        slot = d * (C + 1) + 1 + torch.arange(k, dtype=torch.int64)
        sendbuf[slot] = routed[idx[:k]]
        perm[idx[:k]] = slot.to(torch.int32)
        perm[idx[k:]] = -1
        overflow += n - k
        sendbuf[d * (C + 1)] = torch.tensor([k | (n << 32), rank_self | ((FLAG_VALID << 16) << 32), 0, 0])
    st = ws_stats(rws.ws)
    st[STAT_NOMATCH] = int((~ok).sum())
    st[STAT_OVERFLOW] = overflow
    return sendbuf, perm, st


def _handler_ref(method, actor, a0, a1, a2, state):
    """Plain-PyTorch reference of the device handler table (handlers.hpp)."""
    from .records import (METHOD_CALC_MULTIPLY as MUL, METHOD_COUNTER_ADD as CADD, METHOD_ECHO as ECHO,
                          METHOD_PRIME_CHECK as PRIME, METHOD_RETRY_TEST as RETRY, STATUS_FAILED,
                          STATUS_NO_METHOD)
    n = method.numel()
    value = torch.zeros(n, dtype=torch.int64)
    status = torch.full((n,), STATUS_NO_METHOD, dtype=torch.int64)
    m = method == MUL
    value[m] = a0[m] * a1[m]
    status[m] = 0
    m = method == ECHO
    value[m] = a0[m]
    status[m] = 0
    for i in torch.nonzero(method == PRIME).flatten().tolist():
        lo, hi, t = int(a0[i]), min(int(a1[i]), int(a2[i])), int(a2[i])
        v = t
        for c in range(lo, hi):
            if c != 0 and t % c == 0:
                v = c
                break
        value[i] = v
        status[i] = 0
    for i in torch.nonzero((method == RETRY) | (method == CADD)).flatten().tolist():
        a = int(actor[i])
        if state is None or a >= state.numel():
            status[i] = STATUS_NO_ACTOR
            continue
        if int(method[i]) == RETRY:
            state[a] += 1
            c = int(state[a])
            if c >= int(a0[i]):
                value[i], status[i] = c, 0
            else:
                status[i] = STATUS_FAILED
        else:
            state[a] += int(a0[i])
            value[i], status[i] = int(state[a]), 0
    return value, status


def dispatch(recv: torch.Tensor, R: int, C: int, state: torch.Tensor | None = None, delay_us: int = 0,
             reply: torch.Tensor | None = None, ws: torch.Tensor | None = None, expected_per_rank: int = 0):
    """K3 (batch form): run every delivered record through the handler table.

    ``recv`` is ``int64[R*(C+1), 4]`` epoch slots (one per source rank); returns
    replies ``int64[R*(C+1), 2]`` in the same geometry.
    """
    _check(recv, torch.int64, 2, "recv")
    dev = recv.device
    if reply is None:
        reply = torch.empty(R * (C + 1), 2, dtype=torch.int64, device=dev)
    if dev.type == "cuda":
        if ws is None:
            ws = new_workspace(dev)
        n_state = 0 if state is None else state.numel()
        hip().dispatch(_ptr(recv), R, C, _ptr(reply), _ptr(state), n_state, int(delay_us) * 100, _ptr(ws),
                       int(expected_per_rank), _stream(recv))
        return reply
    from .records import make_replies
    reply.zero_()
    for d in range(R):
        h = recv[d * (C + 1)]
        valid = ((int(h[1]) >> 48) & FLAG_VALID) != 0
        cnt = min(int(h[0]) & 0xFFFFFFFF, C) if valid else 0
        reply[d * (C + 1), 0] = cnt
        reply[d * (C + 1), 1] = cnt << 32
        if cnt == 0:
            continue
        lo = d * (C + 1) + 1
        rows = recv[lo:lo + cnt]
        w0 = rows[:, 0]
        actor = w0 & 0xFFFFFFFF
        method = (w0 >> 32) & 0xFFFF
        v, stt = _handler_ref(method, actor, rows[:, 1], rows[:, 2], rows[:, 3], state)
        reply[lo:lo + cnt] = make_replies(v, stt, actor)
    return reply


def complete(reply: torch.Tensor, perm: torch.Tensor, out_val: torch.Tensor | None = None,
             out_status: torch.Tensor | None = None, checksum: torch.Tensor | None = None):
    """K8: ``value[i], status[i] = reply[perm[i]]`` (overflow/no-actor statuses for perm < 0)."""
    M = perm.numel()
    dev = perm.device
    out_val = torch.empty(M, dtype=torch.int64, device=dev) if out_val is None else out_val
    out_status = torch.empty(M, dtype=torch.int32, device=dev) if out_status is None else out_status
    if dev.type == "cuda":
        hip().complete(_ptr(reply), _ptr(perm), M, _ptr(out_val), _ptr(out_status), _ptr(checksum), _stream(perm))
        return out_val, out_status
    p = perm.to(torch.int64)
    ok = p >= 0
    out_val.zero_()
    out_val[ok] = reply[p[ok], 0]
    st = reply[p.clamp(min=0), 1] & 0xFFFFFFFF
    st = torch.where(p == -1, torch.full_like(st, STATUS_OVERFLOW), st)
    st = torch.where(p == -2, torch.full_like(st, STATUS_NO_ACTOR), st)
    out_status.copy_(st.to(torch.int32))
    if checksum is not None:
        checksum += out_val.sum()
    return out_val, out_status
