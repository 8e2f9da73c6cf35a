"""Batch ``Send`` data path: route/bucket (K1), dispatch (K3), complete (K8).

See ``csrc/hip/batch.hip`` for the kernels and the epoch-slot layout.  Each op
takes optional pre-allocated outputs so the steady state (bench / exchange
epochs) allocates nothing and can be captured in a hipGraph.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _check, _ptr, _stream, hip
from .records import FLAG_ROUTED, FLAG_VALID, METHOD_CALC_MULTIPLY, STATUS_NO_ACTOR, STATUS_OVERFLOW
from .table import RegistryTable, actor_keys, mix64

# workspace words (int64): [0:32) counts as 64 x u32, [32] ticket (u32 in low half), [36:40) stats
WS_WORDS = 40
STAT_NOMATCH, STAT_OVERFLOW, STAT_FAILED = 0, 1, 2


def new_workspace(device) -> torch.Tensor:
    return torch.zeros(WS_WORDS, dtype=torch.int64, device=device)


def ws_counts(ws: torch.Tensor, R: int) -> torch.Tensor:
    return ws[0:32].view(torch.int32)[:R]


def ws_stats(ws: torch.Tensor) -> torch.Tensor:
    return ws[36:40]


def gen_requests(M: int, n_actors: int, method: int = METHOD_CALC_MULTIPLY, seed: int = 0, device="cuda",
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """Synthetic client load: M records to uniformly hashed actors in [0, n_actors)."""
    device = torch.device(device)
    out = torch.empty(M, 4, dtype=torch.int64, device=device) if out is None else out
    if device.type == "cuda":
        hip().gen_requests(_ptr(out), M, int(n_actors), int(method), int(seed) & (2**64 - 1), _stream(out))
        return out
    i = np.arange(M, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = mix64(np.uint64(seed & (2**64 - 1)) ^ (i * np.uint64(0x9E3779B97F4A7C15)))
    actor = (h % np.uint64(n_actors)).astype(np.int64)
    a0 = ((h >> np.uint64(20)) & np.uint64(0xFFFF)).astype(np.int64) - 0x8000
    a1 = ((h >> np.uint64(40)) & np.uint64(0xFFFF)).astype(np.int64)
    w0 = actor | (int(method) << 32) | (FLAG_VALID << 48)
    out.copy_(torch.from_numpy(np.stack([w0, a0, a1, np.zeros_like(a0)], axis=1)))
    return out


def route_bucket(req: torch.Tensor, table: RegistryTable, R: int, C: int, rank_self: int = 0,
                 sendbuf: torch.Tensor | None = None, perm: torch.Tensor | None = None,
                 ws: torch.Tensor | None = None):
    """K1: resolve each message's actor in the GPU registry and bucket it into
    its destination rank's epoch slot.

    Returns ``(sendbuf int64[R*(C+1), 4], perm int32[M], ws)``; ``ws_counts(ws, R)``
    holds raw per-destination counts and ``ws_stats(ws)`` [nomatch, overflow, failed].
    """
    _check(req, torch.int64, 2, "req")
    M = req.shape[0]
    dev = req.device
    if sendbuf is None:
        sendbuf = torch.empty(R * (C + 1), 4, dtype=torch.int64, device=dev)
    if perm is None:
        perm = torch.empty(M, dtype=torch.int32, device=dev)
    if ws is None:
        ws = new_workspace(dev)
    else:
        ws.zero_()
    if dev.type == "cuda":
        hip().route_bucket(_ptr(req), M, _ptr(table.table), table.cap, R, C, _ptr(sendbuf), _ptr(perm),
                           _ptr(ws), _ptr(ws[32:33]), _ptr(ws[36:40]), rank_self, _stream(req))
        return sendbuf, perm, ws
    # ---- CPU reference (stable order within a bucket) ----
    actor = req[:, 0] & 0xFFFFFFFF
    rank, mbox = table.lookup(actor_keys(actor))
    rank = rank.to(torch.int64)
    ok = (rank >= 0) & (rank < R)
    counts = torch.zeros(R, dtype=torch.int64)
    perm.fill_(-2)
    routed = req.clone()
    routed[:, 0] = (req[:, 0] & ~0xFFFFFFFF) | (mbox.to(torch.int64) & 0xFFFFFFFF) | (FLAG_ROUTED << 48)
    sendbuf.zero_()
    overflow = 0
    for d in range(R):
        idx = torch.nonzero(ok & (rank == d)).flatten()
        n = idx.numel()
        counts[d] = n
        k = min(n, C)
        base = d * (C + 1) + 1
        sendbuf[base:base + k] = routed[idx[:k]]
        perm[idx[:k]] = torch.arange(base, base + k, dtype=torch.int32)
        perm[idx[k:]] = -1
        overflow += n - k
        sendbuf[d * (C + 1), 0] = k | (FLAG_VALID << 48)
        sendbuf[d * (C + 1), 1] = n
        sendbuf[d * (C + 1), 2] = rank_self
    ws_counts(ws, R).copy_(counts.to(torch.int32))
    st = ws_stats(ws)
    st[STAT_NOMATCH] = int((~ok).sum())
    st[STAT_OVERFLOW] = overflow
    return sendbuf, perm, ws


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
        hip().dispatch(_ptr(recv), R, C, _ptr(reply), _ptr(state), n_state, int(delay_us) * 100, _ptr(ws[36:40]),
                       int(expected_per_rank), _stream(recv))
        return reply
    from .records import make_replies
    reply.zero_()
    for d in range(R):
        hdr = recv[d * (C + 1)]
        valid = (int(hdr[0]) >> 48) & FLAG_VALID
        cnt = min(int(hdr[0]) & 0xFFFFFFFF, C) if valid else 0
        reply[d * (C + 1), 0] = cnt
        reply[d * (C + 1), 1] = cnt << 32
        if cnt == 0:
            continue
        rows = recv[d * (C + 1) + 1:d * (C + 1) + 1 + cnt]
        w0 = rows[:, 0]
        actor = w0 & 0xFFFFFFFF
        method = (w0 >> 32) & 0xFFFF
        v, st = _handler_ref(method, actor, rows[:, 1], rows[:, 2], rows[:, 3], state)
        reply[d * (C + 1) + 1:d * (C + 1) + 1 + cnt] = make_replies(v, st, actor)
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
