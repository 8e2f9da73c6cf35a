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
from .records import (FLAG_IDENTITY, FLAG_VALID, METHOD_CALC_MULTIPLY, STATUS_NO_ACTOR, STATUS_OVERFLOW, make_requests,
                      split_requests)
from .table import RegistryTable, actor_keys, mix64

# workspace words (int64): [0:4) stats [nomatch, overflow, failed, route-error flag]
WS_WORDS = 8
STAT_NOMATCH, STAT_OVERFLOW, STAT_FAILED, STAT_ROUTE_ERROR = 0, 1, 2, 3
STAT_TOOWIDE = 4  # wire v3: replies wider than the agreed value plane (never, by construction)
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
    def from_records(req: torch.Tensor, mfma: bool = False) -> "MsgBatch":
        """AoS int64[M,4] records -> SoA batch (on the GPU: one kernel, see
        csrc/hip/transpose.hip; ``mfma`` selects the MFMA byte-transposition
        variant, kept for measurement -- the dwordx4 copy is faster)."""
        if req.device.type == "cuda":
            M = req.shape[0]
            d = req.device
            out = MsgBatch(torch.empty(M, dtype=torch.int32, device=d), torch.empty(M, dtype=torch.int64, device=d),
                           torch.empty(M, dtype=torch.int64, device=d), torch.empty(M, dtype=torch.int64, device=d),
                           torch.empty(M, dtype=torch.int16, device=d))
            req = req.contiguous()
            hip().records_to_soa(_ptr(req), M, _ptr(out.actor), _ptr(out.method), _ptr(out.a0), _ptr(out.a1),
                                 _ptr(out.a2), bool(mfma), _stream(req))
            return out
        actor, method, _, a0, a1, a2 = split_requests(req)
        return MsgBatch(actor.to(torch.int32).contiguous(), a0.contiguous(), a1.contiguous(), a2.contiguous(),
                        method.to(torch.int16).contiguous())

    def to_records(self) -> torch.Tensor:
        m = self.method if isinstance(self.method, int) else self.method.to(torch.int64)
        return make_requests(self.actor.to(torch.int64) & 0xFFFFFFFF, m, self.a0, self.a1, self.a2)


def gen_requests(M: int, n_actors: int, method: int = METHOD_CALC_MULTIPLY, seed: int = 0, device="cuda",
                 out: MsgBatch | None = None, seed_tensor: torch.Tensor | None = None, wide: bool = False) -> MsgBatch:
    """Synthetic client load: M calls (A, B) to uniformly hashed actors in [0, n_actors).
    A is a 16-bit signed and B a 16-bit unsigned value; ``wide``: both full-range
    int64 (products wrap, as the handler's do).  ``seed_tensor`` (GPU int64[1]) is
    read by the kernel instead of ``seed``, so a captured graph produces a fresh
    batch on every replay."""
    device = torch.device(device)
    if out is None:
        out = MsgBatch(torch.empty(M, dtype=torch.int32, device=device), torch.empty(M, dtype=torch.int64, device=device),
                       torch.empty(M, dtype=torch.int64, device=device), None, method)
    if device.type == "cuda":
        hip().gen_requests(_ptr(out.actor), _ptr(out.a0), _ptr(out.a1), M, int(n_actors), int(seed) & (2**64 - 1),
                           _ptr(seed_tensor), _stream(out.actor), bool(wide))
        return out
    if seed_tensor is not None:
        seed = int(seed_tensor.reshape(-1)[0])
    i = np.arange(M, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = mix64(np.uint64(seed & (2**64 - 1)) ^ (i * np.uint64(0x9E3779B97F4A7C15)))
    out.actor.copy_(torch.from_numpy((h % np.uint64(n_actors)).astype(np.int64)).to(torch.int32))
    if wide:
        with np.errstate(over="ignore"):
            out.a0.copy_(torch.from_numpy(mix64(h ^ np.uint64(0xA0761D6478BD642F)).view(np.int64)))
            out.a1.copy_(torch.from_numpy(mix64(h ^ np.uint64(0xE7037ED1A0B428DB)).view(np.int64)))
        return out
    out.a0.copy_(torch.from_numpy(((h >> np.uint64(20)) & np.uint64(0xFFFF)).astype(np.int64) - 0x8000))
    if out.a1 is not None:  # (a one-argument batch: no second column)
        out.a1.copy_(torch.from_numpy(((h >> np.uint64(40)) & np.uint64(0xFFFF)).astype(np.int64)))
    return out


_ZIPF_CDF: dict = {}


def zipf_actors(M: int, n_actors: int, s: float = 1.1, seed: int = 0, device="cuda",
                scatter_seed: int = 99) -> torch.Tensor:
    """Skewed client load: M actor ids with P(rank k) ~ 1 / k^s over n_actors (Zipf),
    the popularity ranks scattered over the id space by a fixed permutation (hot
    actors land on arbitrary GPUs).  int32[M] on ``device``."""
    device = torch.device(device)
    key = (int(n_actors), float(s), int(scatter_seed), str(device))
    if key not in _ZIPF_CDF:
        w = torch.arange(1, n_actors + 1, dtype=torch.float64).pow(-float(s))
        cdf = torch.cumsum(w, 0)
        cdf = (cdf / cdf[-1]).to(device)
        perm = torch.randperm(n_actors, generator=torch.Generator().manual_seed(scatter_seed)).to(device)
        _ZIPF_CDF[key] = (cdf, perm)
    cdf, perm = _ZIPF_CDF[key]
    g = torch.Generator(device=device).manual_seed(int(seed))
    u = torch.rand(M, dtype=torch.float64, device=device, generator=g)
    k = torch.searchsorted(cdf, u).clamp_(max=n_actors - 1)
    return perm[k].to(torch.int32)


def gen_zipf_requests(M: int, n_actors: int, s: float = 1.1, method: int = METHOD_CALC_MULTIPLY, seed: int = 0,
                      device="cuda") -> MsgBatch:
    """``gen_requests`` with Zipf(s) actor popularity."""
    device = torch.device(device)
    g = torch.Generator(device=device).manual_seed(int(seed) + 1)
    a0 = torch.randint(-0x8000, 0x8000, (M,), dtype=torch.int64, device=device, generator=g)
    a1 = torch.randint(0, 0x10000, (M,), dtype=torch.int64, device=device, generator=g)
    return MsgBatch(zipf_actors(M, n_actors, s, seed, device), a0, a1, None, method)


@dataclass(frozen=True)
class WireFormat:
    """Epoch wire format v2 (see csrc/hip/batch.hip): which payload columns a
    record carries.  ``nargs`` int64 args (1..3) and, with ``method_col``, a
    per-record method word; otherwise the method is uniform per slot (header).
    A calculator call (uniform Multiply, A, B) is 5 words = 20 B on the wire."""

    nargs: int = 3
    method_col: bool = True

    @property
    def stride(self) -> int:
        return 1 + int(self.method_col) + 2 * self.nargs

    def req_words(self, C: int) -> int:
        return (4 + C * self.stride + 3) & ~3

    @staticmethod
    def rep_words(C: int) -> int:
        return (4 + 2 * C + (C + 3) // 4 + 3) & ~3

    @staticmethod
    def for_batch(batch: "MsgBatch") -> "WireFormat":
        nargs = 3 if batch.a2 is not None else 2 if batch.a1 is not None else 1
        return WireFormat(nargs, not isinstance(batch.method, int))

    def admits(self, batch: "MsgBatch") -> bool:
        need = WireFormat.for_batch(batch)
        return need.nargs <= self.nargs and (self.method_col or not need.method_col)


FULL_FORMAT = WireFormat(3, True)  # 32-B records: any batch fits


class RouteWorkspace:
    """Per-epoch scratch of the route kernels: the single-pass route's look-back
    words (ticket/epoch + per-block per-destination prefix states, zeroed once)
    and the 3-pass route's route words + block histograms."""

    def __init__(self, M: int, R: int, device):
        device = torch.device(device)
        cuda = device.type == "cuda"
        G, _ = hip().route_grid(max(M, 1)) if cuda else (1, M)
        Gf, _ = hip().route_fused_grid(max(M, 1)) if cuda else (1, M)
        self.M, self.R = M, R
        self.lb = torch.zeros(1 + Gf * (R + 1), dtype=torch.int64, device=device)
        self.route = torch.empty(max(M, 1), dtype=torch.int32, device=device)
        self.hist = torch.empty(G * (R + 1), dtype=torch.int32, device=device)
        self.ws = new_workspace(device)


def route(batch: MsgBatch, table: RegistryTable, R: int, C: int, rank_self: int = 0,
          sendbuf: torch.Tensor | None = None, perm: torch.Tensor | None = None,
          rws: RouteWorkspace | None = None, fmt: WireFormat = FULL_FORMAT, reset_stats: bool = True,
          direct: tuple | None = None, write_perm: bool = True):
    """K1: resolve each message's actor in the GPU registry and place it, in
    message order, into its destination rank's epoch slot (wire format ``fmt``).

    Returns ``(sendbuf int32[R * fmt.req_words(C)], perm int32[M], stats int64[4])``;
    ``perm[i] = d * C + pos`` (-1 overflow, -2 no actor).  The no-actor /
    overflow counters accumulate in ``rws.ws`` unless ``reset_stats``.

    ``direct = (out_val, out_status, src)``: direct completion -- messages to
    ``rank_self`` get ``perm = -3`` and ``src[pos] = i`` (the own slot's dispatch
    then writes their replies straight into the outputs), and no-actor / overflow
    statuses are written into the outputs here.  ``write_perm=False`` (only valid
    with ``direct`` at R == 1, where nothing is completed later) skips ``perm``.
    """
    if not write_perm and (direct is None or R != 1):
        raise ValueError("write_perm=False needs direct completion at R == 1")
    M = batch.M
    dev = batch.device
    if batch.actor.dtype != torch.int32 or batch.a0.dtype != torch.int64:
        raise TypeError("MsgBatch: actor must be int32 and a0..a2 int64")
    if not fmt.admits(batch):
        raise ValueError(f"batch columns do not fit wire format {fmt}")
    W = fmt.req_words(C)
    if sendbuf is None:
        sendbuf = torch.empty(R * W, dtype=torch.int32, device=dev)
    _check(sendbuf, torch.int32, 1, "sendbuf")
    if sendbuf.numel() < R * W:
        raise ValueError("sendbuf too small for R x req_words(C)")
    if perm is None:
        perm = torch.empty(M, dtype=torch.int32, device=dev)
    if rws is None or rws.M < M or rws.R != R:
        rws = RouteWorkspace(M, R, dev)
    if reset_stats:
        rws.ws.zero_()
    uniform = isinstance(batch.method, int)
    method_u = int(batch.method) if uniform else 0
    if dev.type == "cuda":
        mcol = None if uniform else batch.method.to(torch.int16).contiguous()
        d, n_dir, affine = table.directory()
        dptr = [] if direct is None else [_ptr(direct[2]), _ptr(direct[0]), _ptr(direct[1])]
        hip().route(_ptr(batch.actor), _ptr(batch.a0), _ptr(batch.a1), _ptr(batch.a2), _ptr(mcol), method_u, M,
                    _ptr(table.table), table.cap, _ptr(d), n_dir, R, C, fmt.nargs, fmt.method_col, _ptr(sendbuf),
                    _ptr(perm) if write_perm else 0, _ptr(rws.route), _ptr(rws.hist), _ptr(rws.lb), _ptr(rws.ws),
                    rank_self, dptr, affine, _stream(batch.actor))
        return sendbuf, perm, ws_stats(rws.ws)
    # ---- CPU reference: bit-identical layout (stable message order per destination) ----
    actor = batch.actor.to(torch.int64) & 0xFFFFFFFF
    rank, mbox = table.lookup(actor_keys(actor))
    rank = rank.to(torch.int64)
    mbox = mbox.to(torch.int64)
    ok = (rank >= 0) & (rank < R) & (mbox < MAX_MBOX)
    cols = [mbox & 0xFFFFFFFF]
    if fmt.method_col:
        method = torch.full((M,), method_u, dtype=torch.int64) if uniform else batch.method.to(torch.int64)
        cols.append(method & 0xFFFF)
    z = torch.zeros(M, dtype=torch.int64)
    for a in [batch.a0, batch.a1, batch.a2][: fmt.nargs]:
        a = z if a is None else a
        cols += [a & 0xFFFFFFFF, (a >> 32) & 0xFFFFFFFF]
    words = _u32(torch.stack(cols, dim=1))  # [M, stride] int32
    perm.fill_(-2)
    overflow = 0
    for d in range(R):
        idx = torch.nonzero(ok & (rank == d)).flatten()
        n = idx.numel()
        k = min(n, C)
        region = sendbuf[d * W:(d + 1) * W]
        region[4:4 + k * fmt.stride] = words[idx[:k]].reshape(-1)
        if direct is not None and d == rank_self:
            perm[idx[:k]] = -3
            direct[2][:k] = idx[:k].to(torch.int32)
        else:
            perm[idx[:k]] = (d * C + torch.arange(k, dtype=torch.int64)).to(torch.int32)
        perm[idx[k:]] = -1
        overflow += n - k
        region[:4] = _u32(torch.tensor([k, n, rank_self, (FLAG_VALID << 16) | (method_u & 0xFFFF)]))
    if R == 1 and bool(ok.all()) and M <= C:  # gap-free single slot (as the device scan flags it)
        sendbuf[3] = sendbuf[3] | (FLAG_IDENTITY << 16)
    if direct is not None:
        neg = perm < 0
        neg &= perm != -3
        direct[0][neg] = 0
        direct[1][perm == -2] = STATUS_NO_ACTOR
        direct[1][perm == -1] = STATUS_OVERFLOW
    st = ws_stats(rws.ws)
    st[STAT_NOMATCH] += int((~ok).sum())
    st[STAT_OVERFLOW] += overflow
    return sendbuf, perm, st


def _u32(x: torch.Tensor) -> torch.Tensor:
    """int64 values in [0, 2^32) -> the same bits as int32."""
    return torch.from_numpy(x.numpy().astype(np.uint32).view(np.int32))


def _words_i64(lo: torch.Tensor, hi: torch.Tensor) -> torch.Tensor:
    return (lo.to(torch.int64) & 0xFFFFFFFF) | (hi.to(torch.int64) << 32)


def fold_step(prev: int, a0: int) -> int:
    """One kSeqFold application on int64 state: prev * FOLD_MUL + a0, wrapped to int64."""
    from .records import FOLD_MUL

    v = (prev * FOLD_MUL + a0) & 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= (1 << 63) else v


def _handler_ref(method, actor, a0, a1, a2, state, outbox=None):
    """Plain-PyTorch reference of the device handler table (handlers.hpp)."""
    from .records import (METHOD_CALC_MULTIPLY as MUL, METHOD_COUNTER_ADD as CADD, METHOD_ECHO as ECHO,
                          METHOD_FORWARD as FWD, METHOD_PRIME_CHECK as PRIME, METHOD_RETRY_TEST as RETRY,
                          METHOD_SEQ_FOLD as FOLD, STATUS_FAILED, STATUS_NO_METHOD)
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
    for i in torch.nonzero(method == FOLD).flatten().tolist():  # in message order: a serial execution
        a = int(actor[i])
        if state is None or a >= state.numel():
            status[i] = STATUS_NO_ACTOR
            continue
        value[i], status[i] = int(state[a]), 0
        state[a] = fold_step(int(state[a]), int(a0[i]))
    for i in torch.nonzero(method == FWD).flatten().tolist():
        a = int(actor[i])
        if state is None or a >= state.numel():
            status[i] = STATUS_NO_ACTOR
            continue
        state[a] += 1
        value[i], status[i] = int(state[a]), 0
        if int(a1[i]) > 0:
            if outbox is None:
                status[i] = STATUS_FAILED
                continue
            w = int(a2[i]) & 0xFFFFFFFFFFFFFFFF
            stride, n = w & 0xFFFFFFFF, w >> 32
            nxt = (int(a0[i]) + stride) % n if n else int(a0[i])
            outbox.emit_cpu(int(a0[i]) & 0xFFFFFFFF, FWD, nxt, int(a1[i]) - 1, int(a2[i]))
    return value, status


def dispatch(recv: torch.Tensor, R: int, C: int, state: torch.Tensor | None = None, delay_us: int = 0,
             reply: torch.Tensor | None = None, ws: torch.Tensor | None = None, expected_per_rank: int = 0,
             fmt: WireFormat = FULL_FORMAT, outbox=None, direct: tuple | None = None, rank_self: int = 0):
    """K3 (batch form): run every delivered record through the handler table.

    ``recv`` is ``int32[R * fmt.req_words(C)]`` (one request region per source
    rank); returns ``int32[R * rep_words(C)]`` reply regions (header, int64
    values, u8 statuses) in the same geometry.  Handlers that send (``Forward``)
    append to ``outbox`` (a ``DeviceOutbox``).  With ``direct = (out_val,
    out_status, src)`` the own slot (``rank_self``) replies into the outputs.
    """
    _check(recv, torch.int32, 1, "recv")
    dev = recv.device
    W, Wr = fmt.req_words(C), WireFormat.rep_words(C)
    if reply is None:
        reply = torch.empty(R * Wr, dtype=torch.int32, device=dev)
    if dev.type == "cuda":
        if ws is None:
            ws = new_workspace(dev)
        n_state = 0 if state is None else state.numel()
        ob, ob_cap = outbox.view() if outbox is not None else ([], 0)
        dptr = [] if direct is None else [_ptr(direct[2]), _ptr(direct[0]), _ptr(direct[1])]
        hip().dispatch(_ptr(recv), R, C, fmt.nargs, fmt.method_col, _ptr(reply), _ptr(state), n_state,
                       int(delay_us) * 100, _ptr(ws), int(expected_per_rank), ob, ob_cap, dptr, int(rank_self),
                       _stream(recv))
        return reply
    reply.zero_()
    for d in range(R):
        region = recv[d * W:(d + 1) * W]
        h = region[:4].to(torch.int64) & 0xFFFFFFFF
        valid = ((int(h[3]) >> 16) & FLAG_VALID) != 0
        cnt = min(int(h[0]), C) if valid else 0
        rr = reply[d * Wr:(d + 1) * Wr]
        rr[0] = cnt
        if cnt == 0:
            continue
        rows = region[4:4 + cnt * fmt.stride].reshape(cnt, fmt.stride)
        actor = rows[:, 0].to(torch.int64) & 0xFFFFFFFF
        o = 1 + int(fmt.method_col)
        method = (rows[:, 1].to(torch.int64) & 0xFFFF) if fmt.method_col else torch.full((cnt,), int(h[3]) & 0xFFFF)
        args = [_words_i64(rows[:, o + 2 * j], rows[:, o + 2 * j + 1]) for j in range(fmt.nargs)]
        args += [torch.zeros(cnt, dtype=torch.int64)] * (3 - fmt.nargs)
        v, stt = _handler_ref(method, actor, args[0], args[1], args[2], state, outbox)
        if direct is not None and d == rank_self:
            ident = ((int(h[3]) >> 16) & FLAG_IDENTITY) != 0
            src = torch.arange(cnt) if ident else direct[2][:cnt].to(torch.int64)
            direct[0][src] = v
            direct[1][src] = stt.to(torch.int32)
            continue
        rr[4:4 + 2 * C].view(torch.int64)[:cnt] = v
        rr[4 + 2 * C:].view(torch.uint8)[:cnt] = stt.to(torch.uint8)
    return reply


def complete(reply: torch.Tensor, perm: torch.Tensor, C: int, out_val: torch.Tensor | None = None,
             out_status: torch.Tensor | None = None, checksum: torch.Tensor | None = None, direct: bool = False):
    """K8: ``value[i], status[i]`` = the reply at ``perm[i] = d * C + pos`` (overflow /
    no-actor statuses for perm < 0).  ``direct``: entries with perm < 0 were
    already completed (route / own-slot dispatch) and are left alone."""
    M = perm.numel()
    dev = perm.device
    out_val = torch.empty(M, dtype=torch.int64, device=dev) if out_val is None else out_val
    out_status = torch.empty(M, dtype=torch.int32, device=dev) if out_status is None else out_status
    if dev.type == "cuda":
        hip().complete(_ptr(reply), C, _ptr(perm), M, _ptr(out_val), _ptr(out_status), _ptr(checksum), bool(direct),
                       _stream(perm))
        return out_val, out_status
    Wr = WireFormat.rep_words(C)
    R = reply.numel() // Wr
    regions = reply[:R * Wr].reshape(R, Wr)
    vals = regions[:, 4:4 + 2 * C].contiguous().view(torch.int64).reshape(-1)  # [R*C]
    sts = regions[:, 4 + 2 * C:].contiguous().view(torch.uint8)[:, :C].reshape(-1)
    p = perm.to(torch.int64)
    ok = p >= 0
    if direct:
        out_val[ok] = vals[p[ok]]
        out_status[ok] = sts[p[ok]].to(torch.int32)
        if checksum is not None:
            checksum += out_val.sum()
        return out_val, out_status
    out_val.zero_()
    out_val[ok] = vals[p[ok]]
    st = sts[p.clamp(min=0)].to(torch.int64)
    st = torch.where(p == -1, torch.full_like(st, STATUS_OVERFLOW), st)
    st = torch.where(p == -2, torch.full_like(st, STATUS_NO_ACTOR), st)
    out_status.copy_(st.to(torch.int32))
    if checksum is not None:
        checksum += out_val.sum()
    return out_val, out_status
