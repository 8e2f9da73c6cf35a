"""K4: gob value messages for batches of fixed-schema structs, on the GPU.

The reference's net/rpc carries every call's arguments and reply as
``encoding/gob`` values (cluster/rpc.go:59-67; the calculator's
``Args{A, B int}``, example/calculator/calculator.go:5-8).  For a batch held
as one int64 column per struct field in HBM, ``encode_structs`` produces the
value messages a gob stream carries after the type's definition (``uint(len)
int(type id)`` then the struct's non-zero fields as delta / zigzag pairs), byte
for byte as the host codec (``_core.gob_encode``, csrc/core/gob.cpp) and Go
write them; ``decode_structs`` parses such messages back into columns, one
message per lane, with a status per message (csrc/hip/gob.hip).

CPU tensors run the host codec itself (``encode_structs_ref`` /
``decode_structs_ref``), which is also the test oracle.
"""
from __future__ import annotations

import torch

from . import _ptr, _stream, hip

STATUS_OK, STATUS_TRUNCATED, STATUS_WRONG_TYPE, STATUS_BAD_FIELD, STATUS_TRAILING = 0, 1, 2, 3, 4
MAX_FIELDS = 8


def _check_cols(cols):
    if not 1 <= len(cols) <= MAX_FIELDS:
        raise ValueError(f"gob structs: 1..{MAX_FIELDS} int fields")
    M = cols[0].numel()
    for c in cols:
        if c.dtype != torch.int64 or c.numel() != M or not c.is_contiguous():
            raise ValueError("gob structs: contiguous int64 columns of one length")
    return M


def encode_structs(cols: list[torch.Tensor], type_id: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Columns -> (bytes uint8[total], offsets int64[M + 1]): message i is
    ``bytes[offsets[i]:offsets[i + 1]]``."""
    M = _check_cols(cols)
    dev = cols[0].device
    if dev.type != "cuda":
        return encode_structs_ref(cols, type_id)
    h = hip()
    out = torch.empty(max(1, h.gob_max_bytes(M, len(cols), int(type_id))), dtype=torch.uint8, device=dev)
    offsets = torch.empty(M + 1, dtype=torch.int64, device=dev)
    ws = torch.empty(h.gob_ws_words(M), dtype=torch.int64, device=dev)
    h.gob_encode([_ptr(c) for c in cols], M, int(type_id), _ptr(out), _ptr(offsets), _ptr(ws), _stream(cols[0]))
    total = int(offsets[M].item())
    return out[:total], offsets


def decode_structs(buf: torch.Tensor, offsets: torch.Tensor, nf: int, type_id: int):
    """(bytes, offsets int64[M + 1]) -> (columns int64[nf][M], status int32[M]).
    A malformed message decodes to zeros with a non-zero status."""
    M = offsets.numel() - 1
    if buf.device.type != "cuda":
        return decode_structs_ref(buf, offsets, nf, type_id)
    if not 1 <= nf <= MAX_FIELDS:
        raise ValueError(f"gob structs: 1..{MAX_FIELDS} int fields")
    dev = buf.device
    cols = [torch.empty(M, dtype=torch.int64, device=dev) for _ in range(nf)]
    status = torch.empty(M, dtype=torch.int32, device=dev)
    hip().gob_decode(_ptr(buf.contiguous()), _ptr(offsets.contiguous()), M, int(type_id), [_ptr(c) for c in cols],
                     _ptr(status), _stream(buf))
    return cols, status


# ------------------------------------------------------------------ host codec
def _struct_type(nf: int):
    from dataclasses import make_dataclass

    return make_dataclass("S", [(f"F{k}", int) for k in range(nf)])


def value_messages_ref(rows: list[tuple[int, ...]]) -> tuple[int, list[bytes]]:
    """The host codec's stream for ``rows`` (one struct each), split into the
    type id and the value messages (the leading type definition dropped)."""
    from .. import _core

    nf = len(rows[0])
    S = _struct_type(nf)
    stream = _core.gob_encode([S(*r) for r in rows])
    msgs, pos, type_id = [], 0, None
    while pos < len(stream):
        n, pos = _get_uint(stream, pos)
        body = stream[pos:pos + n]
        tid, _ = _get_uint(body, 0)
        tid = -((tid >> 1) + 1) if tid & 1 else tid >> 1
        if tid > 0:  # a value message (definitions carry the negated id)
            type_id = tid
            msgs.append(bytes([n]) + body if n < 128 else _put_uint(n) + body)
        pos += n
    return type_id, msgs


def _get_uint(b: bytes, pos: int) -> tuple[int, int]:
    c = b[pos]
    if c < 128:
        return c, pos + 1
    n = 256 - c
    return int.from_bytes(b[pos + 1:pos + 1 + n], "big"), pos + 1 + n


def _put_uint(x: int) -> bytes:
    if x < 128:
        return bytes([x])
    n = (x.bit_length() + 7) // 8
    return bytes([256 - n]) + x.to_bytes(n, "big")


def encode_structs_ref(cols: list[torch.Tensor], type_id: int):
    """Host codec encode of the columns' rows (type id must be the one the host
    codec assigns a fresh stream's first struct type)."""
    rows = list(zip(*[c.tolist() for c in cols]))
    if not rows:
        return torch.empty(0, dtype=torch.uint8), torch.zeros(1, dtype=torch.int64)
    tid, msgs = value_messages_ref(rows)
    if tid != type_id:
        raise ValueError(f"host codec assigns type id {tid}, not {type_id}")
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    return torch.tensor(list(b"".join(msgs)), dtype=torch.uint8), torch.tensor(offs, dtype=torch.int64)


def decode_structs_ref(buf: torch.Tensor, offsets: torch.Tensor, nf: int, type_id: int):
    """Per-message parse on the host (the same rules as the kernel)."""
    data = bytes(buf.tolist())
    offs = offsets.tolist()
    M = len(offs) - 1
    cols = [[0] * M for _ in range(nf)]
    status = [STATUS_OK] * M
    for i in range(M):
        lo, hi = offs[i], offs[i + 1]
        try:
            n, p = _get_uint(data[:hi], lo)
            if hi - p != n:
                raise IndexError
            t, p = _get_uint(data[:hi], p)
            if (-((t >> 1) + 1) if t & 1 else t >> 1) != type_id:
                status[i] = STATUS_WRONG_TYPE
                continue
            field, vals = -1, {}
            while True:
                d, p = _get_uint(data[:hi], p)
                if d == 0:
                    break
                field += d
                if field >= nf:
                    status[i] = STATUS_BAD_FIELD
                    break
                u, p = _get_uint(data[:hi], p)
                vals[field] = -((u >> 1) + 1) if u & 1 else u >> 1
            if status[i] == STATUS_OK and p != hi:
                status[i] = STATUS_TRAILING
            if status[i] == STATUS_OK:
                for f, v in vals.items():
                    cols[f][i] = v
        except IndexError:
            status[i] = STATUS_TRUNCATED
    return [torch.tensor(c, dtype=torch.int64) for c in cols], torch.tensor(status, dtype=torch.int32)
