"""The calculator workload (reference example/calculator).

``Args{A, B int}`` and ``Calculator.Multiply`` (example/calculator/calculator.go:3-12)
as (a) a host receiver for the net/rpc server -- what the reference runs -- and
(b) a GPU actor method (compiled-in handler ``kCalculatorMultiply``) reachable
through net/rpc (persistent dispatcher) and through batched ``Send``.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..ops.batch import MsgBatch
from ..ops.records import METHOD_CALC_MULTIPLY

SERVICE = "Calculator"
DEVICE_METHODS = {"Multiply": (METHOD_CALC_MULTIPLY, ["A", "B"])}


@dataclass
class Args:
    A: int
    B: int


class Calculator:
    """Host receiver: ``rpc.Register(new(Calculator))``."""

    def Multiply(self, args) -> int:
        return args.A * args.B


def serve_device(runtime, server) -> None:
    """Register ``Calculator.Multiply`` backed by the GPU handler."""
    runtime.serve(server, SERVICE, DEVICE_METHODS)


def make_batch(actors: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> MsgBatch:
    """A batch of ``Multiply(Args{A, B})`` messages to the given actors (SoA)."""
    return MsgBatch(actors.to(torch.int32).contiguous(), a.to(torch.int64).contiguous(),
                    b.to(torch.int64).contiguous(), None, METHOD_CALC_MULTIPLY)
