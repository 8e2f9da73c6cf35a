"""Device ops of the actor runtime: thin wrappers over the gfx950 kernels in
``ptype_amd/_hip`` plus plain-PyTorch reference implementations.

Tensor conventions (all little-endian int64 views of the binary records in
``csrc/core/records.hpp``):

* message record  ``int64[M, 4]`` (32 B): ``col0 = actor | method << 32 | flags << 48``,
  ``col1..3 = a0, a1, a2``
* reply record    ``int64[M, 2]`` (16 B): ``col0 = value``, ``col1 = status | actor << 32``
* registry table  ``int64[cap, 2]`` (16 B entries): ``col0 = key``, ``col1 = rank | mbox << 32``

CUDA (HIP) tensors always run the hand-written kernels; if the extension is
missing on a GPU box the call raises -- there is no silent fallback.  CPU tensors
run the reference implementation (used by the numerics tests and by the gloo
multi-process CPU tests of the exchange).
"""
from __future__ import annotations

import torch

from . import records
from .records import (
    FLAG_ROUTED,
    FLAG_VALID,
    METHOD_CALC_MULTIPLY,
    METHOD_COUNTER_ADD,
    METHOD_ECHO,
    METHOD_PRIME_CHECK,
    METHOD_RETRY_TEST,
    STATUS_FAILED,
    STATUS_NO_ACTOR,
    STATUS_NO_METHOD,
    STATUS_OK,
    STATUS_OVERFLOW,
    make_requests,
    split_requests,
    split_replies,
)

_HIP = None


def hip():
    """Return the loaded ``_hip`` extension (raises loudly if it is missing)."""
    global _HIP
    if _HIP is None:
        try:
            from .. import _hip as mod  # noqa: WPS433
        except ImportError as e:  # pragma: no cover - exercised on a box without a build
            raise RuntimeError(
                "ptype_amd._hip is not built; run `python -m ptype_amd._build` (hipcc --offload-arch=gfx950)"
            ) from e
        _HIP = mod
    return _HIP


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def raw_stream(device) -> int:
    """The current HIP stream of ``device`` as an integer handle.  The raw
    accessor skips building a torch Stream object (~1.5 us on every Send)."""
    idx = device.index if isinstance(device, torch.device) else device
    if idx is None:
        idx = torch.cuda.current_device()
    if _raw_stream is not None:
        return _raw_stream(idx)
    return torch.cuda.current_stream(idx).cuda_stream


def _stream(t: torch.Tensor) -> int:
    return raw_stream(t.device)


def _ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def _check(t: torch.Tensor, dtype, ndim=None, name="tensor"):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim} dims, got {t.dim()}")


from .table import RegistryTable, actor_keys, mix64  # noqa: E402
from .batch import MsgBatch, RouteWorkspace, complete, dispatch, gen_requests, route  # noqa: E402

__all__ = [
    "hip", "records", "RegistryTable", "actor_keys", "mix64", "gen_requests", "route", "MsgBatch", "RouteWorkspace", "dispatch",
    "complete", "make_requests", "split_requests", "split_replies", "FLAG_VALID", "FLAG_ROUTED",
    "METHOD_CALC_MULTIPLY", "METHOD_PRIME_CHECK", "METHOD_ECHO", "METHOD_RETRY_TEST", "METHOD_COUNTER_ADD",
    "STATUS_OK", "STATUS_FAILED", "STATUS_NO_ACTOR", "STATUS_NO_METHOD", "STATUS_OVERFLOW",
]
