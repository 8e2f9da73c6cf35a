"""Tracing and latency observability.

* ``range(name)`` / ``mark(name)``: roctx ranges and markers around ``Send``,
  exchange chunks and calls -- visible with ``rocprofv3 --marker-trace``; no-ops
  when the roctx library is absent (CPU runs).
* ``DispatcherTrace``: the persistent dispatcher's device timestamp ring
  (``s_memrealtime``, 100 MHz) joined with the host publication time of each
  request, giving per-call queue (publish -> picked up by the wave) and service
  (picked up -> reply published) latency, plus the host round-trip histogram.
  The two clocks are tied together by a handshake with the running kernel
  (``DeviceServer.calibrate``: +-half the handshake window).
"""
from __future__ import annotations

import builtins
import contextlib

import numpy as np

TICK_NS = 10.0  # s_memrealtime: 100 MHz


def _hip_or_none():
    try:
        from ..ops import hip

        return hip()
    except Exception:
        return None


_H = None


def _h():
    global _H
    if _H is None:
        _H = _hip_or_none() or False
    return _H or None


def available() -> bool:
    h = _h()
    return bool(h and h.roctx_available())


class _Range:
    __slots__ = ("h", "name")

    def __init__(self, h, name):
        self.h, self.name = h, name

    def __enter__(self):
        self.h.roctx_push(self.name)
        return self

    def __exit__(self, *exc):
        self.h.roctx_pop()
        return False


_NULL = contextlib.nullcontext()
_ROCTX = None  # the module when the roctx library is loaded, else False (decided once)


def range(name: str):  # noqa: A001 - mirrors roctxRange naming
    """roctx range around a block; a shared no-op context (no allocation, no
    generator frame) when no roctx library is loaded -- it sits on every Send."""
    global _ROCTX
    if _ROCTX is None:
        h = _h()
        _ROCTX = h if (h is not None and h.roctx_available()) else False
    return _Range(_ROCTX, name) if _ROCTX else _NULL


def mark(name: str) -> None:
    h = _h()
    if h is not None:
        h.roctx_mark(name)


def percentiles(values, ps=(50, 90, 99)) -> dict:
    v = np.asarray(values, dtype=np.float64)
    if v.size == 0:
        return {f"p{p}": None for p in ps}
    return {f"p{p}": float(np.percentile(v, p)) for p in ps}


def hist_percentile(hist, p: float) -> float | None:
    """Percentile (ns, bucket upper bound) of a log2(ns) histogram."""
    h = np.asarray(hist, dtype=np.float64)
    tot = h.sum()
    if tot == 0:
        return None
    k = int(np.searchsorted(np.cumsum(h), tot * p / 100.0))
    return float(2 ** (k + 1))


class DispatcherTrace:
    """Per-call latency breakdown of a ``DeviceServer`` (the single-call path)."""

    def __init__(self, server, capacity: int = 4096):
        self.srv = server
        self.capacity = capacity

    def __enter__(self):
        self.srv.enable_trace(self.capacity)
        # keep the tightest of several handshakes (the kernel answers from its idle poll)
        self.calib = min((self.srv.calibrate() for _ in builtins.range(8)), key=lambda c: c[2])
        return self

    def __exit__(self, *exc):
        self.srv.disable_trace()

    def records(self) -> np.ndarray:
        raw = np.frombuffer(self.srv.trace_records(), dtype=np.uint64).reshape(-1, 4)
        return raw[raw[:, 1] != 0]  # written slots only

    def breakdown(self) -> dict:
        """Queue / service latency (us) of the traced calls, in host time."""
        host_ns, ticks, err_ns = (int(x) for x in self.calib)
        r = self.records().astype(np.float64)
        if r.shape[0] == 0:
            return {"n": 0}
        seen_ns = host_ns + (r[:, 2] - ticks) * TICK_NS
        done_ns = host_ns + (r[:, 3] - ticks) * TICK_NS
        queue = (seen_ns - r[:, 1]) / 1e3
        service = (done_ns - seen_ns) / 1e3
        return {"n": int(r.shape[0]), "clock_err_us": err_ns / 1e3,
                "queue_us": percentiles(queue), "service_us": percentiles(service),
                "rtt_us_p50_bucket": (hist_percentile(self.srv.rtt_histogram(), 50) or 0) / 1e3}
