"""HBM actor mailboxes (SURVEY K2 ``mailbox_enqueue`` + K3 ``dispatch``).

Thin wrapper over ``_hip.Mailboxes`` (csrc/hip/mailbox.hpp): S shard rings of
Q tagged 32-B records per GPU.  A ``Send`` through the mailboxes is

* K2: every message resolved against the GPU registry mirror (route directory /
  hash probe), ranked per shard in LDS, reserved with one atomicAdd per
  (tile, shard) on the ring's tail and written as a tagged record;
* K3: the rings drained through the handler table, replies written back to the
  message's origin (its index in the batch).  Ordered methods
  (``records.ORDERED_METHODS``) run one at a time per actor in ring order; the
  rest run with the whole grid.

A persistent consumer (``start`` / ``stop``) drains the same rings while
producers on other streams keep enqueueing (``enqueue(live=True)``): the
asynchronous "tell" form.

Reference: the server's per-request goroutine of stdlib net/rpc
(example/calculator/server/server.go:16-20, :38) -- here the queue is explicit
and lives in HBM.

CPU tensors run ``send_ref``: a serial execution in message order (one valid
mailbox order), used by the CPU tests and the gloo pipeline.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _ptr, hip, raw_stream
from .batch import MsgBatch, _handler_ref, fold_step
from .records import STATUS_NO_ACTOR, STATUS_OK, method_ordered

STAT_NAMES = ("enqueued", "overflow", "no_actor", "processed", "failed", "holes", "serialised", "spilled", "reserved",
              "lookback_timeouts")
SORT_MAX_SHARDS = 1024  # csrc/hip/mailbox.hpp kMboxSortMaxShards


SORT_MODES = {"auto": 0, "onepass": 1, "twopass": 2}


def batch_ordered(batch: MsgBatch) -> bool:
    """Whether a batch may carry an ordered method (a method column: assume so)."""
    return method_ordered(batch.method) if isinstance(batch.method, int) else True


class Mailboxes:
    """The HBM mailboxes of one GPU."""

    def __init__(self, device, shards: int = 256, slots: int = 65536, with_a2: bool = True):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("Mailboxes live in HBM: use send_ref() for CPU tensors")
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self._m = hip().Mailboxes(idx, int(shards), int(slots), bool(with_a2))
        self.shards, self.slots = int(shards), int(slots)
        self.last_sharding = None  # the rings the last send() took ("actor" / "arrival")

    @property
    def bytes(self) -> int:
        return int(self._m.bytes)

    @property
    def last_record_bytes(self) -> int:
        """Ring record size of the last sorted Send: 8 (8-B records), 16 (compact) or 32."""
        return int(self._m.last_record_bytes)

    @property
    def last_view_shards(self) -> int:
        """Shards the last sorted Send viewed the rings as: the full count for ordered
        batches, a coarser view (8 by default) for stateless ones."""
        return int(self._m.last_view_shards)

    @property
    def last_route(self) -> int:
        """Route of the last sorted Send: 0 hash probe, 1 route directory, 2 affine rule,
        3 rank byte table (a stateless uniform batch; its records carry the actor id)."""
        return int(self._m.last_route)

    @property
    def handle(self) -> int:
        """Address of the native object: the epoch engine delivers received records into it."""
        return int(self._m.handle)

    def _stream(self) -> int:
        return raw_stream(self.device)

    def enqueue(self, batch: MsgBatch, table, out_val: torch.Tensor, out_status: torch.Tensor, rank_self: int = 0,
                origin_base: int = 0, live: bool = False, arrival: bool = False) -> None:
        """K2 on the current stream: replies for messages that never enter a ring
        (no actor on this rank, ring full -> STATUS_OVERFLOW) are written at once.
        ``arrival``: shard by arrival tile instead of by actor -- only for batches
        without ordered methods, whose actors need no single ring."""
        if batch.actor.dtype != torch.int32 or batch.a0.dtype != torch.int64:
            raise TypeError("MsgBatch: actor must be int32 and a0..a2 int64")
        uniform = isinstance(batch.method, int)
        mcol = None if uniform else batch.method.to(torch.int16).contiguous()
        d, n_dir, affine = table.directory()
        self._m.enqueue(_ptr(batch.actor), _ptr(batch.a0), _ptr(batch.a1), _ptr(batch.a2), _ptr(mcol),
                        int(batch.method) if uniform else 0, batch.M, _ptr(table.table), table.cap, _ptr(d), n_dir,
                        affine, int(rank_self), int(origin_base), _ptr(out_val), _ptr(out_status), out_val.numel(),
                        bool(live), self._stream(), bool(arrival))

    def drain(self, state: torch.Tensor | None, out_val: torch.Tensor, out_status: torch.Tensor,
              ordered: bool = True, delay_us: int = 0, outbox=None, fixed_method: int = 0) -> None:
        """K3 epoch form on the current stream: run everything queued.
        ``fixed_method``: every queued record is known to carry this method."""
        ob, ob_cap = outbox.view() if outbox is not None else ([], 0)
        self._m.drain(_ptr(state), 0 if state is None else state.numel(), int(delay_us) * 100, _ptr(out_val),
                      _ptr(out_status), out_val.numel(), bool(ordered), self._stream(), ob, ob_cap,
                      int(fixed_method))

    def send(self, batch: MsgBatch, table, state: torch.Tensor | None, out_val: torch.Tensor | None = None,
             out_status: torch.Tensor | None = None, rank_self: int = 0, delay_us: int = 0,
             ordered: bool | None = None, outbox=None, sharding: str = "actor", sort: bool | None = None,
             sort_mode: str = "auto"):
        """World-1 Send through the mailboxes: K2 + K3, replies in message order.

        ``sharding``: ``"actor"`` (every actor's messages in one ring, FIFO in
        message order) or ``"arrival"`` (a tile's messages in one ring: only for
        batches without ordered methods).  ``ordered`` (default: whether the batch
        may carry an ordered method): drain each actor's records one at a time in
        ring order; otherwise every record runs in parallel.  ``sort`` (default on):
        the sorted epoch kernels (csrc/hip/mailbox_sort.hip: counting-sort enqueue,
        16-B records); off: the tagged reservation kernels of mailbox.hip.
        ``sort_mode`` (actor sharding): ``"auto"``, ``"onepass"`` (run reservations for
        stateless batches, look-back for ordered ones) or ``"twopass"`` (count + scatter)."""
        M = batch.M
        out_val = torch.empty(M, dtype=torch.int64, device=self.device) if out_val is None else out_val
        out_status = torch.empty(M, dtype=torch.int32, device=self.device) if out_status is None else out_status
        if M == 0:
            return out_val, out_status
        if sharding not in ("actor", "arrival"):
            raise ValueError("sharding: 'actor' or 'arrival'")
        ordered = batch_ordered(batch) if ordered is None else bool(ordered)
        arrival = sharding == "arrival"
        self.last_sharding = sharding
        if arrival and ordered:
            raise ValueError("arrival sharding cannot serve ordered methods (an actor's messages meet in no one ring)")
        # the rings are empty between Sends, so a uniform batch fixes every queued method
        fixed = int(batch.method) if isinstance(batch.method, int) else 0
        if sort is None:
            sort = self.shards <= SORT_MAX_SHARDS
        # a stateless batch on the sorted kernels never answers STATUS_OVERFLOW: a
        # message whose ring is full spills to the drain, which runs it from the batch
        self.last_spills = bool(sort and not ordered)
        if not sort:
            self.enqueue(batch, table, out_val, out_status, rank_self=rank_self, arrival=arrival)
            self.drain(state, out_val, out_status, ordered=ordered, delay_us=delay_us, outbox=outbox,
                       fixed_method=fixed)
            return out_val, out_status
        if batch.actor.dtype != torch.int32 or batch.a0.dtype != torch.int64:
            raise TypeError("MsgBatch: actor must be int32 and a0..a2 int64")
        uniform = isinstance(batch.method, int)
        mcol = None if uniform else batch.method.to(torch.int16).contiguous()
        d, n_dir, affine = table.directory()
        ob, ob_cap = outbox.view() if outbox is not None else ([], 0)
        self._m.send_sorted(_ptr(batch.actor), _ptr(batch.a0), _ptr(batch.a1), _ptr(batch.a2), _ptr(mcol),
                            int(batch.method) if uniform else 0, M, _ptr(table.table), table.cap, _ptr(d), n_dir,
                            affine, int(rank_self), 0, _ptr(out_val), _ptr(out_status), out_val.numel(), _ptr(state),
                            0 if state is None else state.numel(), int(delay_us) * 100, ob, ob_cap, arrival, ordered,
                            fixed, self._stream(), SORT_MODES[sort_mode],
                            _ptr(table.dir_rank) if d is not None else 0,
                            _ptr(table.presence) if d is not None and table.presence is not None else 0,
                            table.presence_rank)
        return out_val, out_status

    # ---- persistent consumer ("tell" sessions)
    def start(self, state: torch.Tensor | None, out_val: torch.Tensor, out_status: torch.Tensor, blocks: int = 16,
              idle_ms: float = 0.0, max_s: float = 60.0, delay_us: int = 0) -> None:
        """Launch the persistent consumer (``blocks`` x 4 waves, each owning
        shards) on its own stream.  Earlier epoch enqueues must have completed."""
        self._m.start(_ptr(state), 0 if state is None else state.numel(), int(delay_us) * 100, _ptr(out_val),
                      _ptr(out_status), out_val.numel(), int(blocks), float(idle_ms), float(max_s))

    def stop(self) -> None:
        """Drain what is queued, then let the consumer exit (waits for it)."""
        self._m.stop()

    @property
    def running(self) -> bool:
        return bool(self._m.running)

    def reset(self) -> None:
        self._m.reset(self._stream())

    def stats(self) -> dict:
        v = self._m.stats()
        out = {k: int(v[i]) for i, k in enumerate(STAT_NAMES)}
        out["consumer_processed"] = int(self._m.consumer_processed)
        out["bytes"] = self.bytes
        return out

    def shard_counters(self) -> np.ndarray:
        """``[S, 3]``: tail, done, head per shard."""
        return np.asarray(self._m.shard_counters(), dtype=np.uint64).reshape(-1, 3)


def send_ref(batch: MsgBatch, route_rank: torch.Tensor, route_mbox: torch.Tensor, state: torch.Tensor | None,
             rank_self: int = 0):
    """CPU reference of a mailbox Send: every message to its actor, run serially
    in message order (one of the orders the rings allow).  ``route_rank`` /
    ``route_mbox`` are the registry's answer per message (rank -1: no actor)."""
    M = batch.M
    method = (torch.full((M,), int(batch.method), dtype=torch.int64) if isinstance(batch.method, int)
              else batch.method.to(torch.int64))
    a1 = batch.a1 if batch.a1 is not None else torch.zeros(M, dtype=torch.int64)
    a2 = batch.a2 if batch.a2 is not None else torch.zeros(M, dtype=torch.int64)
    mine = route_rank == rank_self
    val = torch.zeros(M, dtype=torch.int64)
    st = torch.full((M,), STATUS_NO_ACTOR, dtype=torch.int32)
    idx = torch.nonzero(mine).flatten()
    if idx.numel():
        v, s = _handler_ref(method[idx], route_mbox[idx].to(torch.int64), batch.a0[idx], a1[idx], a2[idx], state)
        val[idx] = v
        st[idx] = s.to(torch.int32)
    return val, st


def audit_fold(mbox, a0, reply, status, state_before, state_after):
    """Exactly-once + serialisation audit of ``SeqFold`` traffic.

    Every message to actor x replied the state it found; each actor's messages
    must chain from ``state_before[x]`` through ``fold_step`` to
    ``state_after[x]``, using every message exactly once.  Returns
    ``(ok, order)`` where ``order[x]`` lists the message indices in the order
    actor x ran them; ``ok`` is False with the first failure's description.
    """
    mbox = np.asarray(mbox, dtype=np.int64)
    a0 = np.asarray(a0, dtype=np.int64)
    reply = np.asarray(reply, dtype=np.int64)
    status = np.asarray(status)
    if (status != STATUS_OK).any():
        return False, f"{int((status != STATUS_OK).sum())} non-OK replies"
    by_actor: dict[int, dict[int, list[int]]] = {}
    for i in np.argsort(mbox, kind="stable"):
        by_actor.setdefault(int(mbox[i]), {}).setdefault(int(reply[i]), []).append(int(i))
    order = {}
    for x, by_reply in by_actor.items():
        s = int(state_before[x])
        seq = []
        n = sum(len(v) for v in by_reply.values())
        while len(seq) < n:
            cand = by_reply.get(s)
            if not cand:
                return False, f"actor {x}: no message saw state {s} after {len(seq)} of {n} (lost or duplicated)"
            i = cand.pop()
            seq.append(i)
            s = fold_step(s, int(a0[i]))
        if s != int(state_after[x]):
            return False, f"actor {x}: chain ends at {s}, state is {int(state_after[x])}"
        order[x] = seq
    return True, order
