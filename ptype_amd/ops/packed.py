"""Wire format v3 ("packed"): width-adaptive bit-packed epoch records.

The layout, the reply-width rule and the region sizes are defined in
``csrc/hip/packed.hpp``; this module wraps the gfx950 kernels
(``csrc/hip/packed.hip``) and holds the CPU reference that the GPU tests compare
against bit for bit:

* ``meta_reference``  -- the column maxima a rank contributes to the agreement
* ``layout_reference`` -- field offsets/widths, dwords per record, reply bytes
* ``requests_from_v2`` / ``replies_from_v2`` -- re-encode v2 epoch regions (the
  existing, independently tested CPU reference of route / dispatch) into v3

The reference's wire is gob, whose integers are variable-length
(cluster/rpc.go:65 and :88 hand ``Args`` to net/rpc's gob codec); v3 is that
idea applied per exchange: every integer column is zigzag-coded at the width of
its largest value across the node.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _ptr, _stream, hip
from .batch import FLAG_VALID, MAX_MBOX, MsgBatch, RouteWorkspace, WireFormat, ws_stats
from .records import (METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, METHOD_ECHO, METHOD_FORWARD, METHOD_PRIME_CHECK,
                      METHOD_RETRY_TEST, STATUS_OK)
from .table import RegistryTable

META_WORDS = 16
META_MBOX, META_ARG0, META_METHOD, META_MCOL, META_CAP, META_FLAGS = 0, 1, 4, 5, 6, 8

_U64 = np.uint64


def zz(v: np.ndarray) -> np.ndarray:
    v = np.asarray(v, dtype=np.int64)
    return (v.astype(_U64) << _U64(1)) ^ (v >> np.int64(63)).astype(_U64)


def unzz(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=_U64)
    return ((z >> _U64(1)).astype(np.int64)) ^ -((z & _U64(1)).astype(np.int64))


def _bits(x: int) -> int:
    return int(x).bit_length()


# ----------------------------------------------------------------- reference
def meta_reference(batch: MsgBatch, n_dir: int = 0, affine_w: int = 0, nargs: int = 3) -> list[int]:
    """What ``packed_meta_kernel`` contributes for one rank's batch."""
    m = [0] * META_WORDS
    if batch.M == 0:
        return m
    actor = batch.actor.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    if affine_w:
        mb = np.where(actor < n_dir, actor // affine_w, MAX_MBOX - 1)
    else:
        mb = np.full(actor.shape, MAX_MBOX - 1)
    m[META_MBOX] = int(mb.max())
    for j, a in enumerate([batch.a0, batch.a1, batch.a2][:nargs]):
        if a is not None:
            m[META_ARG0 + j] = int(zz(a.cpu().numpy()).max())
    if isinstance(batch.method, int):
        meths = [int(batch.method)]
        m[META_METHOD] = int(batch.method)
    else:
        col = batch.method.cpu().numpy().astype(np.int64) & 0xFFFF
        meths = np.unique(col).tolist()
        m[META_METHOD] = int(col.max())
        m[META_MCOL] = 1
    for x in meths:
        m[META_FLAGS + min(int(x), 7)] = 1
    return m


def combine(metas) -> list[int]:
    """The node-wide agreement (ncclAllReduce MAX) of per-rank meta vectors."""
    return [max(col) for col in zip(*metas)]


def reply_bits_reference(meta) -> int:
    z0, z1, z2 = meta[META_ARG0], meta[META_ARG0 + 1], meta[META_ARG0 + 2]
    mag = lambda z: z // 2 + (z & 1)  # noqa: E731
    flag = lambda m: meta[META_FLAGS + m] != 0  # noqa: E731
    bits = 0
    if flag(METHOD_CALC_MULTIPLY):
        p = 2 * mag(z0) * mag(z1)
        bits = max(bits, 64 if p >> 64 else _bits(p))
    if flag(METHOD_ECHO):
        bits = max(bits, _bits(z0))
    if flag(METHOD_PRIME_CHECK):
        z = max(z0, z1, z2)
        bits = max(bits, 64 if z == 2**64 - 1 else _bits(z + 1))
    if flag(METHOD_RETRY_TEST) or flag(METHOD_COUNTER_ADD) or flag(METHOD_FORWARD) or meta[META_FLAGS + 7]:
        bits = 64
    return max(bits, 8)


def layout_reference(meta) -> dict:
    off, w, o = [], [], 0
    widths = [max(1, _bits(meta[META_METHOD])) if meta[META_MCOL] else 0, _bits(meta[META_MBOX])]
    widths += [_bits(meta[META_ARG0 + j]) for j in range(3)]
    for x in widths:
        off.append(o)
        w.append(x)
        o += x
    S = max(1, (o + 31) // 32)
    vbits = reply_bits_reference(meta)
    vb = 1 if vbits <= 8 else 2 if vbits <= 16 else 4 if vbits <= 32 else 8
    return {"off": off, "w": w, "S": S, "vb": vb}


def req_words(C: int, S: int) -> int:
    return (4 + C * S + 3) & ~3


def val_words(C: int, vb: int) -> int:
    return 2 * ((C * vb + 7) // 8)


def ok_words(n: int) -> int:
    return 2 * ((n + 63) // 64)


def rep_words(C: int, vb: int) -> int:
    """[header 4][ok bitmap ok_words(n)][values val_words(n, vb)] (packed.hpp)."""
    return (4 + ok_words(C) + val_words(C, vb) + 3) & ~3


def pack_reference(fields: list[np.ndarray], L: dict) -> np.ndarray:
    """fields = [method, mbox, zz(a0), zz(a1), zz(a2)] (uint64 arrays) -> uint32 [n, S]."""
    n = len(fields[1])
    out = np.zeros((n, L["S"]), dtype=np.uint32)
    for j in range(L["S"]):
        x = np.zeros(n, dtype=_U64)
        for q in range(5):
            wq = L["w"][q]
            if not wq:
                continue
            v = np.asarray(fields[q], dtype=_U64) & _U64((1 << wq) - 1 if wq < 64 else 2**64 - 1)
            sh = L["off"][q] - 32 * j
            if 0 <= sh < 32:
                x |= (v << _U64(sh)) & _U64(0xFFFFFFFF)
            elif -64 < sh < 0:
                x |= (v >> _U64(-sh)) & _U64(0xFFFFFFFF)
        out[:, j] = x.astype(np.uint32)
    return out


def requests_from_v2(send_v2: torch.Tensor, R: int, C: int, fmt: WireFormat, L: dict,
                     method_uniform: int = 0) -> list[tuple[np.ndarray, np.ndarray]]:
    """Per destination: (header uint32[4], packed records uint32[count, S]) of the
    v3 encoding of a v2 request buffer.  ``fmt`` is the v2 buffer's format."""
    W = fmt.req_words(C)
    buf = send_v2.cpu().numpy().view(np.uint32)
    out = []
    for d in range(R):
        reg = buf[d * W:(d + 1) * W]
        h = reg[:4].copy()
        valid = (int(h[3]) >> 16) & FLAG_VALID
        cnt = min(int(h[0]), C) if valid else 0
        rows = reg[4:4 + cnt * fmt.stride].reshape(cnt, fmt.stride).astype(_U64)
        mbox = rows[:, 0]
        o = 1 + int(fmt.method_col)
        meth = rows[:, 1] & _U64(0xFFFF) if fmt.method_col else np.full(cnt, int(h[3]) & 0xFFFF, dtype=_U64)
        args = [(rows[:, o + 2 * j] | (rows[:, o + 2 * j + 1] << _U64(32))).view(np.int64) for j in range(fmt.nargs)]
        args += [np.zeros(cnt, dtype=np.int64)] * (3 - fmt.nargs)
        out.append((h, pack_reference([meth, mbox] + [zz(a) for a in args], L)))
    return out


def replies_from_v2(rep_v2: torch.Tensor, R: int, C: int, vb: int, skip: int = -1):
    """Per source: (count, codes uint64[count], ok bool[count]) of the v3 encoding of
    v2 reply regions (``skip``: the own slot under direct completion)."""
    Wr = WireFormat.rep_words(C)
    buf = rep_v2.cpu().numpy().view(np.uint32)
    out = []
    for d in range(R):
        reg = buf[d * Wr:(d + 1) * Wr]
        cnt = int(reg[0])
        vals = reg[4:4 + 2 * C].view(np.int64)[:cnt]
        sts = reg[4 + 2 * C:].view(np.uint8)[:cnt].astype(np.int64)
        ok = sts == STATUS_OK
        codes = np.where(ok, vals.view(_U64) if vb == 8 else zz(vals), sts.astype(_U64))
        out.append((cnt, codes if d != skip else None, ok if d != skip else None))
    return out


# ----------------------------------------------------------------- GPU kernels
def meta(batch: MsgBatch, table: RegistryTable, out: torch.Tensor | None = None) -> torch.Tensor:
    """``packed_meta_kernel`` over one batch (int64[16] on the batch's device)."""
    dev = batch.device
    out = torch.empty(META_WORDS, dtype=torch.int64, device=dev) if out is None else out
    _, n_dir, affine = table.directory()
    uniform = isinstance(batch.method, int)
    mcol = None if uniform else batch.method.to(torch.int16).contiguous()
    hip().packed_meta(_ptr(batch.actor), _ptr(batch.a0), _ptr(batch.a1), _ptr(batch.a2), _ptr(mcol),
                      int(batch.method) if uniform else 0, batch.M, n_dir, affine, _ptr(out), _stream(batch.actor))
    return out


def meta_list(t: torch.Tensor) -> list[int]:
    return [int(x) & (2**64 - 1) for x in t.cpu().tolist()]


def layout(meta_words) -> dict:
    return hip().packed_layout([int(x) & (2**64 - 1) for x in meta_words])


def route(batch: MsgBatch, table: RegistryTable, R: int, C: int, L: dict, rank_self: int = 0,
          sendbuf: torch.Tensor | None = None, rws: RouteWorkspace | None = None, direct: tuple | None = None):
    """K1 with v3 records.  Returns ``(sendbuf int32[R * req_words(C, S)], perm, stats)``."""
    dev = batch.device
    M = batch.M
    W = req_words(C, L["S"])
    sendbuf = torch.empty(R * W, dtype=torch.int32, device=dev) if sendbuf is None else sendbuf
    perm = torch.empty(M, dtype=torch.int32, device=dev)
    rws = RouteWorkspace(M, R, dev) if rws is None else rws
    rws.ws.zero_()
    uniform = isinstance(batch.method, int)
    mcol = None if uniform else batch.method.to(torch.int16).contiguous()
    d, n_dir, affine = table.directory()
    dptr = [] if direct is None else [_ptr(direct[2]), _ptr(direct[0]), _ptr(direct[1])]
    hip().route_packed(_ptr(batch.actor), _ptr(batch.a0), _ptr(batch.a1), _ptr(batch.a2), _ptr(mcol),
                       int(batch.method) if uniform else 0, M, _ptr(table.table), table.cap, _ptr(d), n_dir, R, C, L,
                       _ptr(sendbuf), _ptr(perm), _ptr(rws.route), _ptr(rws.hist), _ptr(rws.ws), rank_self, dptr,
                       affine, _stream(batch.actor))
    return sendbuf, perm, ws_stats(rws.ws)


def dispatch(recv: torch.Tensor, R: int, C: int, L: dict, state: torch.Tensor | None = None,
             ws: torch.Tensor | None = None, expected_per_rank: int = 0, direct: tuple | None = None,
             rank_self: int = 0) -> torch.Tensor:
    """K3 over v3 request regions -> v3 reply regions (value plane + ok bitmap)."""
    from .batch import new_workspace

    dev = recv.device
    reply = torch.empty(R * rep_words(C, L["vb"]), dtype=torch.int32, device=dev)
    ws = new_workspace(dev) if ws is None else ws
    dptr = [] if direct is None else [_ptr(direct[2]), _ptr(direct[0]), _ptr(direct[1])]
    hip().dispatch_packed(_ptr(recv), R, C, L, _ptr(reply), _ptr(state), 0 if state is None else state.numel(), 0,
                          _ptr(ws), int(expected_per_rank), [], 0, dptr, int(rank_self), _stream(recv))
    return reply


def complete(reply: torch.Tensor, perm: torch.Tensor, C: int, vb: int, direct: bool = False,
             out_val: torch.Tensor | None = None, out_status: torch.Tensor | None = None):
    M = perm.numel()
    dev = perm.device
    out_val = torch.empty(M, dtype=torch.int64, device=dev) if out_val is None else out_val
    out_status = torch.empty(M, dtype=torch.int32, device=dev) if out_status is None else out_status
    R = reply.numel() // rep_words(C, vb)
    hip().complete_packed(_ptr(reply), C, R, vb, _ptr(perm), M, _ptr(out_val), _ptr(out_status), 0, bool(direct),
                          _stream(perm))
    return out_val, out_status


def reply_regions(reply: torch.Tensor, R: int, C: int, vb: int):
    """Decode v3 reply regions on the host: per source (count, codes, ok)."""
    Wr = rep_words(C, vb)
    buf = reply.cpu().numpy().view(np.uint32)
    dt = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[vb]
    out = []
    for d in range(R):
        reg = buf[d * Wr:(d + 1) * Wr]
        cnt = int(reg[0])
        ow = ok_words(cnt)
        codes = reg[4 + ow:4 + ow + val_words(cnt, vb)].view(dt)[:cnt].astype(_U64)
        okw = reg[4:4 + ow].view(_U64)
        ok = ((okw[np.arange(cnt) // 64] >> (np.arange(cnt) % 64).astype(_U64)) & _U64(1)).astype(bool)
        out.append((cnt, codes, ok))
    return out
