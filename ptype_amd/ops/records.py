"""Binary record layout helpers (mirror of ``csrc/core/records.hpp``)."""
from __future__ import annotations

import torch

METHOD_NONE = 0
METHOD_CALC_MULTIPLY = 1
METHOD_PRIME_CHECK = 2
METHOD_ECHO = 3
METHOD_RETRY_TEST = 4
METHOD_COUNTER_ADD = 5
METHOD_FORWARD = 6  # actor-to-actor tell: count the visit, emit Forward to a0 while a1 > 0
METHOD_SEQ_FOLD = 7  # ORDERED: reply = state; state = state * FOLD_MUL + a0 (mod 2**64)
# dispatcher-only: forwarded to another process's actor through a GPU peer lane (csrc/hip/xcall.hpp PeerRelay);
# actor = remote actor, a0 = remote method, a1 / a2 = its arguments
METHOD_RELAY = 0x7E
# handler-initiated: local actor A (a0 = n, a1 = workers W, a2 = first worker B) picks a worker,
# asks it PrimeCheck over the relay and tallies primes into its own state (csrc/core/records.hpp)
METHOD_COORD_PRIME = 0x7D

FOLD_MUL = 0x100000001B3
ORDERED_METHODS = frozenset({METHOD_SEQ_FOLD})  # one at a time per actor, in mailbox order


def method_ordered(m: int) -> bool:
    return int(m) in ORDERED_METHODS

FLAG_VALID = 1
FLAG_ROUTED = 2
FLAG_IDENTITY = 4  # slot header: slot position == message index (R = 1, no gaps)
FLAG_A2 = 8  # mailbox record: third argument in the ring's a2 side array

STATUS_OK = 0
STATUS_NO_METHOD = 1
STATUS_FAILED = 2
STATUS_NO_ACTOR = 3
STATUS_OVERFLOW = 4
STATUS_NOT_DELIVERED = 5
STATUS_RANK_LOST = 6  # the actor's rank died with the message in flight (re-homed since: re-send)

MSG_WORDS = 4    # int64 words per 32-B message record
REPLY_WORDS = 2  # int64 words per 16-B reply record

_U32 = 0xFFFFFFFF


def make_requests(actor, method, a0, a1=None, a2=None, flags: int = FLAG_VALID, device=None) -> torch.Tensor:
    """Pack message records ``int64[M, 4]`` from per-field tensors/scalars."""
    actor = torch.as_tensor(actor, dtype=torch.int64, device=device)
    M = actor.numel()
    dev = actor.device
    method = torch.as_tensor(method, dtype=torch.int64, device=dev).expand(M)
    a0 = torch.as_tensor(a0, dtype=torch.int64, device=dev).expand(M)
    a1 = torch.zeros(M, dtype=torch.int64, device=dev) if a1 is None else torch.as_tensor(a1, dtype=torch.int64, device=dev).expand(M)
    a2 = torch.zeros(M, dtype=torch.int64, device=dev) if a2 is None else torch.as_tensor(a2, dtype=torch.int64, device=dev).expand(M)
    w0 = (actor.reshape(M) & _U32) | ((method & 0xFFFF) << 32) | ((flags & 0xFFFF) << 48)
    return torch.stack([w0, a0, a1, a2], dim=1).contiguous()


def split_requests(req: torch.Tensor):
    """Unpack ``int64[M,4]`` into (actor, method, flags, a0, a1, a2)."""
    w0 = req[:, 0]
    return w0 & _U32, (w0 >> 32) & 0xFFFF, (w0 >> 48) & 0xFFFF, req[:, 1], req[:, 2], req[:, 3]


def make_replies(value, status, actor) -> torch.Tensor:
    value = torch.as_tensor(value, dtype=torch.int64)
    status = torch.as_tensor(status, dtype=torch.int64).expand_as(value)
    actor = torch.as_tensor(actor, dtype=torch.int64).expand_as(value)
    return torch.stack([value, (status & _U32) | ((actor & _U32) << 32)], dim=1).contiguous()


def split_replies(rep: torch.Tensor):
    """Unpack ``int64[M,2]`` into (value, status(int32 semantics), actor)."""
    st = rep[:, 1] & _U32
    st = torch.where(st >= 2**31, st - 2**32, st)
    return rep[:, 0], st, (rep[:, 1] >> 32) & _U32
