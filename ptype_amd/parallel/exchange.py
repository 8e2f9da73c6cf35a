"""Exchange-epoch engine: remote `Send` between GPUs over RCCL (xGMI).

One process per GPU; every rank is both a client (it sends messages to actors
anywhere in the node) and a server (it hosts a shard of the actors).  The
reference moves each call over its own TCP connection (cluster/rpc.go:272-285,
`rpc.DialHTTP`; calls at :65 and :88).  Here traffic moves in *epochs*: each
rank buckets its outbound records by destination GPU (K1, deterministic
counting sort), one RCCL all-to-all moves every bucket at once over all 7 xGMI
links, the receiver runs the handler table over what it got (K3), a second
all-to-all returns the replies (8-B value + 1-B status) into the exact slots the
requests left from, and K8 scatters them back to message order.

Wire volume is what bounds an epoch on xGMI.  On the native engine with
collectives (N > 1), records use wire format v3 (``csrc/hip/packed.hpp``,
``ops/packed.py``): the ranks agree per Send, with one 16-word all-reduce, on
the bit widths of every column, and records are zigzag bit-packed at them.  A
calculator call is 8 B plus a 4-B reply, where v2 takes 20 + 9 B.  Elsewhere
(world 1, the Python/gloo pipeline, a captured graph), v2 records carry only the
columns the batch has (``WireFormat``).  For v2, every rank must send batches
with the same columns in the same call (the all-to-all is equal-split over the
format's slot size), or fix the format at construction with ``fmt=``.  v3
derives one layout from the agreed maxima, so ranks may differ in their columns.

Fixed-capacity slots (``C + 1`` records per peer, slot 0 a header with the
count) make both all-to-alls equal-split: no host round trip for sizes, so an
epoch is launch-only and the host never blocks inside it.  A bucket that
overflows ``C`` leaves the overflow in the caller's queue for the next epoch
(``STATUS_OVERFLOW`` until re-sent), which is the actor model's usual
at-least-once hand-off rather than an error.

Pipelining: ``send()`` splits a batch into chunks; chunk k's all-to-alls run on
a communication stream while chunk k+1 is routed and chunk k-1 is dispatched
on the compute stream (stream-level, not host-level, waits).

On a GPU the whole pipeline is enqueued by one native call
(``_hip.EpochEngine``, csrc/hip/engine.hpp; ``_hip.SortedExchange`` for mailbox
delivery): it calls RCCL on the communicator the control plane's DataPlane
formed (``NativeGroup``, csrc/core/dataplane.hpp -- through its CommCell, so a
watchdog abort never races an enqueue) and orders the streams with events.  The
Python pipeline below is the same schedule over ``torch.distributed`` and serves
CPU/gloo groups; tune ``engine=0`` (ops/tune.py) selects it on a GPU for comparison.
"""
from __future__ import annotations

import collections
import math
import threading
from dataclasses import dataclass

import torch
import torch.distributed as dist

from ..ops import batch as B
from ..ops import raw_stream, tune
from ..ops.packed import META_CAP, META_WORDS
from ..ops.records import STATUS_OVERFLOW, method_ordered
from ..ops.table import RegistryTable
from ..utils import trace


ARRIVAL_AUTO_MAX = 2 << 20  # world-1 mailbox Sends without ordered methods: arrival rings up to here


def capacity_for(msgs_per_chunk: int, world: int, slack: float = 0.01) -> int:
    """Per-peer slot capacity for uniformly spread traffic: mean + 1% + an 8-sigma
    margin (overflow probability ~1e-15 per slot), so overflow is a statistical
    non-event while padding -- which the all-to-all moves over xGMI -- stays ~2.5%
    at bench sizes.  Skewed traffic overflows into ``send_all``'s re-send epochs."""
    return B.stripe_capacity(msgs_per_chunk, world, slack)


@dataclass
class EpochStats:
    sent: int = 0  # messages handed to send()
    epochs: int = 0  # chunk epochs run (one request + one reply all-to-all each)
    wire_bytes: int = 0  # bytes this rank put on the all-to-alls (requests + replies, padded slots)
    resends: int = 0  # send_all re-send rounds
    overflow: int = 0  # device counters (cumulative): overflowed, no-actor, handler-failed
    nomatch: int = 0
    failed: int = 0
    toowide: int = 0  # wire v3 replies that did not fit the agreed value plane (must stay 0)
    pump_sealed: int = 0  # idle slots of device-pump epochs (routed as no-actor; not counted in nomatch)
    mailbox: dict | None = None  # HBM mailbox counters (mailbox delivery)


class _ChunkBufs:
    """Slot buffers of one in-flight chunk, sized for the widest wire format."""

    def __init__(self, R, C, M, device, separate=False, fmt: B.WireFormat = B.FULL_FORMAT):
        sep = R > 1 or separate
        self.send = torch.empty(R * fmt.req_words(C), dtype=torch.int32, device=device)
        self.recv = torch.empty_like(self.send) if sep else self.send
        self.reply = torch.empty(R * B.WireFormat.rep_words(C), dtype=torch.int32, device=device)
        self.back = torch.empty_like(self.reply) if sep else self.reply
        self.perm = torch.empty(M, dtype=torch.int32, device=device)
        self.src = torch.empty(C, dtype=torch.int32, device=device)  # own slot: position -> message index
        self.rws = B.RouteWorkspace(M, R, device)
        self.ws = self.rws.ws


class ActorExchange:
    """Epoch exchange over the default (or given) process group.

    ``table`` is this rank's GPU registry mirror (actor -> rank, mailbox);
    ``state`` the int64 actor state of the mailboxes this rank hosts.
    """

    def __init__(self, table: RegistryTable, max_batch: int, chunks: int = 1, group=None, state=None,
                 delay_us: int = 0, slack: float = 0.01, fmt: B.WireFormat | None = None,
                 packed: bool | None = None, fake=None, delivery: str = "auto", mailbox_shards: int = 256,
                 mailbox_slots: int = 0, mailbox_ordered: bool | None = None, comm: str = "rccl",
                 comm_timeout_s: float = 30.0):
        if delivery not in ("auto", "direct", "mailbox"):
            raise ValueError("delivery: 'auto', 'direct' or 'mailbox'")
        if comm not in ("rccl", "ipc"):
            raise ValueError("comm: 'rccl' (the process group's communicator) or 'ipc'")
        # How a message reaches its actor on the GPU that hosts it (world 1):
        #   direct  -- resolved and run in one streaming pass (no queue): stateless and
        #              commutative methods, and ordered ones as linearizable CAS updates
        #   mailbox -- through the HBM mailboxes (ops/mailbox.py): FIFO per actor, ordered
        #              methods one at a time per actor
        #   auto    -- mailbox for a uniform ordered method, direct otherwise
        # With more ranks the receiver cannot see what the other ranks sent, so there
        # the choice is the exchange's (same on every rank): "mailbox" delivers on
        # receipt (K2 from the request regions, v3 or v2 records) into actor-sharded rings with
        # the ordered drain -- unless `mailbox_ordered=False` promises that no ordered
        # method is ever sent (then arrival-sharded rings, streaming drain); "auto"
        # and "direct" dispatch directly (ordered methods as linearizable CAS updates).
        self.delivery = delivery
        self.mailbox_ordered = True if mailbox_ordered is None else bool(mailbox_ordered)
        self.mailbox_shards = int(mailbox_shards)
        self.mailbox_slots = int(mailbox_slots)
        self.mailboxes = None
        self.table = table
        self.device = table.device
        self.group = group
        # ``fake = (_hip.FakeComm(R), rank)``: one of R in-process ranks on one GPU
        # (tests drive each from its own thread and stream; geometry must match)
        self.fake = fake
        # a NativeGroup (parallel/native_group.py): the compiled DataPlane's communicator --
        # no torch process group behind it (RCCL, or IpcComm between processes of one GPU)
        self.native = group is not None and hasattr(group, "comm_ptr") and hasattr(group, "dp")
        if fake is not None:
            self.rank, self.world = int(fake[1]), int(fake[0].size)
        elif self.native:
            self.rank, self.world = group.rank, group.size
        elif dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1
        # comm="ipc": the native engines' collectives go through an IpcComm
        # (csrc/hip/ipc_comm.hpp) -- one rank per process, every rank's receive segment
        # a POSIX shared-memory file that all ranks map and register with HIP -- over a
        # group of any backend (gloo is enough: it only carries the segment names and
        # the host agreements).  It runs the multi-process pipeline where
        # RCCL cannot: several ranks on one GPU.  Built below, once the geometry is agreed.
        self.ipc = None
        if self.native and group.transport == "ipc":
            comm = "ipc"
        self.comm_kind = comm if fake is None and self.world > 1 else "rccl"
        # run the RCCL all-to-alls even on a single rank (validates the collective
        # path on a 1-GPU box; a 1-rank all-to-all is a device-local copy)
        self.force_collectives = bool(fake is None and self.world == 1 and self.native)
        self.chunks = max(1, int(chunks))
        self.max_chunk = int(math.ceil(max_batch / self.chunks))
        # every rank must use the same slot geometry (equal-split all-to-all):
        # agree on the largest chunk and the chunk count once, collectively
        if self.world > 1 and fake is None:
            if self.native:
                self.max_chunk, self.chunks = group.allreduce_max([self.max_chunk, self.chunks])
            else:
                t = torch.tensor([self.max_chunk, self.chunks], dtype=torch.int64, device=self._agree_device())
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
                self.max_chunk, self.chunks = int(t[0]), int(t[1])
        self.C = capacity_for(self.max_chunk, self.world, slack)
        self.state = state
        self.delay_us = delay_us
        self.fmt = fmt  # None: derived per send() from the batch's columns
        self.use_engine = self.device.type == "cuda" and tune.get("engine") != 0
        # wire format v3 (csrc/hip/packed.hpp): width-adaptive packed records on the
        # all-to-alls, agreed per Send by one 16-word all-reduce (native engine, collectives on)
        self.packed = tune.get("wire") != 2 if packed is None else bool(packed)
        # Adaptive slot capacity (native engine + wire v3): every Send's slots are sized
        # by the node's busiest (rank, destination) bucket, agreed in the layout
        # all-reduce; the buffers hold `skew_room` x the uniform share per peer, so
        # skewed (Zipf) traffic fits without re-send rounds and uniform traffic moves
        # less padding than the static mean + 8 sigma capacity
        # (tune adaptive_c=2: also at world 1 with forced collectives -- runs the
        # counts all-to-all and the grouped ncclSend / ncclRecv on a 1-GPU box)
        ad = tune.get("adaptive_c")
        self.adaptive = bool(self.use_engine and self.packed and self.chunks <= 8 and ad != 0
                             and (self.world > 1 or (ad == 2 and self.force_collectives)))
        room = tune.get("skew_room")
        self.C_alloc = (max(self.C, min(self.max_chunk, int(math.ceil(room * self.max_chunk / self.world))))
                        if self.adaptive else self.C)
        self.bufs = [_ChunkBufs(self.world, self.C_alloc, self.max_chunk, self.device, self.force_collectives,
                                fmt or B.FULL_FORMAT) for _ in range(min(self.chunks, 8))]
        if self.comm_kind == "ipc":
            if not self.use_engine:
                raise RuntimeError("comm='ipc' drives the native engines: it needs a GPU")
            if self.native:  # the DataPlane formed the IpcComm generation (csrc/core/dp_link.hpp)
                self.ipc = group.ipc_comm()
                if self.ipc.cap < self.ipc_cap_bytes():
                    raise RuntimeError(f"the group's IPC regions ({self.ipc.cap} B) are smaller than this exchange "
                                       f"needs ({self.ipc_cap_bytes()} B): form it with ipc_cap_for()")
            else:  # (tests: an IpcComm over a gloo group, tests/_ipc_worker.py)
                self.ipc = ipc_group_comm(self.group, self.device, self.ipc_cap_bytes(), comm_timeout_s)
        self.checksum = None  # optional int64[1] reply-value checksum (block-reduced)
        self.outbox = None  # DeviceOutbox that dispatched handlers send into (set by pump)
        # direct completion of self-directed messages (no reply staging, no
        # completion pass for them; at world 1 no completion kernel at all).
        # Default on at world 1 only: with more ranks the completion pass runs
        # anyway, and the own slot's replies written from the dispatcher land
        # scattered (message index through the inverse index, ~R messages apart)
        # -- the completion's gather writes them coalesced instead (bench
        # --loopback 8: 0.360 -> 0.337 ms/step).  Tune direct=0/1 overrides.
        d = tune.get("direct")
        self.direct = (d != 0) if d >= 0 else (self.world == 1)
        self.counters = EpochStats()
        self._engine = None  # native epoch engine, built on first GPU send
        self._capturing = False  # a captured graph cannot host the v3 agreement (host wait)
        self._last_mailbox = True  # whether the last send went through the mailboxes (until known: assume so)
        self._pump_graph = None  # (key, hipGraph of a group of device-pump epochs, its buffers)
        self.last_wire = None  # engine.last_wire() of the latest native send
        self._sorted = None  # _hip.SortedExchange: N > 1 mailbox delivery (csrc/hip/exchange_sorted.hpp)
        self._deferred = collections.deque()  # send_all(defer=True): (Send index, batch, val, st, rounds)
        self._last_sorted = False  # whether the last send() ran on it

    def _agree_device(self) -> torch.device:
        """Where host-level agreements' tensors live: CPU for a gloo group (its
        CUDA collectives are not universally available), else the exchange's device."""
        if getattr(self, "native", False):
            return self.device
        if self.device.type == "cuda" and dist.is_available() and dist.is_initialized():
            if dist.get_backend(self.group) == "gloo":
                return torch.device("cpu")
        return self.device

    def _sorted_c_alloc(self) -> int:
        # the sorted exchange's buffers hold 2.5x the uniform share per peer (skewed
        # traffic fits); the start-up capacity is the static mean + 8 sigma
        room = tune.get("sorted_room")
        return max(64, self.C, min(self.max_chunk, int(math.ceil(room * self.max_chunk / self.world))))

    def ipc_cap_bytes(self) -> int:
        """The largest region one collective moves per peer, over both native
        engines: the sorted exchange's request regions (widest layout, 8 dwords per
        record + the shard table: csrc/hip/packed.hpp packed_req_words,
        exchange_sorted.hpp kSxTableWords), the epoch engine's v2 slots (3
        arguments + a method column) and its agreement vector."""
        c = self._sorted_c_alloc()
        sorted_req = 4 * (((4 + c * 8 + 3) & ~3) + 68)
        epoch_req = 4 * int(B.hip().wire_req_words(self.C_alloc, 3, True))
        epoch_rep = 4 * int(B.hip().wire_rep_words(self.C_alloc))
        agree = 8 * (META_WORDS + self.world * self.world * self.chunks)
        return max(sorted_req, epoch_req, epoch_rep, agree)

    def _comm_ptr(self) -> int:
        """The DataPlane's CommCell of a NativeGroup (0 without collectives).  RCCL
        comes only from the compiled DataPlane: a torch process group's private
        communicator is never borrowed."""
        if self.world == 1 and not self.force_collectives:
            return 0
        if self.ipc is not None:
            return 0
        if self.native:
            return self.group.comm_ptr()
        raise RuntimeError("native epoch engine needs an RCCL communicator: a NativeGroup (Join with a gpu: "
                           "section, or parallel.native_group.solo_group) -- a torch/gloo group has none")

    def _get_engine(self):
        if self._engine is None:
            h = B.hip()
            dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
            if self.fake is not None or self.ipc is not None:
                eng = h.EpochEngine(dev, 0, self.world, self.rank, self.C_alloc, self.max_chunk, self.chunks,
                                    fake=self.fake[0] if self.fake is not None else self.ipc,
                                    adaptive=self.adaptive, c_fixed=self.C)
            else:
                eng = h.EpochEngine(dev, self._comm_ptr(), self.world, self.rank, self.C_alloc, self.max_chunk,
                                    self.chunks, adaptive=self.adaptive, c_fixed=self.C)
            for i, b in enumerate(self.bufs):
                eng.set_bufs(i, b.send.data_ptr(), b.recv.data_ptr(), b.reply.data_ptr(), b.back.data_ptr(),
                             b.perm.data_ptr(), b.src.data_ptr(), b.rws.route.data_ptr(), b.rws.hist.data_ptr(),
                             b.rws.lb.data_ptr(), b.ws.data_ptr())
            self._engine = eng
        return self._engine

    def _send_native(self, req: B.MsgBatch, out_val, out_status, fmt: B.WireFormat):
        """One native call enqueues every chunk's route/all-to-all/dispatch/complete."""
        if req.actor.dtype != torch.int32 or req.a0.dtype != torch.int64:
            raise TypeError("MsgBatch: actor must be int32 and a0..a2 int64")
        uniform = isinstance(req.method, int)
        mcol = None if uniform else req.method.to(torch.int16).contiguous()
        d, n_dir, affine = self.table.directory()
        ob, ob_cap = self.outbox.view() if self.outbox is not None else ([], 0)
        state = self.state
        mb = self._mailboxes().handle if self._mailbox_on_receipt() else 0
        self._get_engine().send(
            B._ptr(req.actor), B._ptr(req.a0), B._ptr(req.a1), B._ptr(req.a2), B._ptr(mcol),
            int(req.method) if uniform else 0, req.M, B._ptr(self.table.table), self.table.cap, B._ptr(d), n_dir,
            affine, fmt.nargs, fmt.method_col, B._ptr(out_val), B._ptr(out_status), B._ptr(state),
            0 if state is None else state.numel(), int(self.delay_us) * 100, ob, ob_cap, self.direct and not mb,
            B._ptr(self.checksum), raw_stream(self.device), self.packed_active(),
            mb, self.mailbox_ordered)
        if self.world > 1 or self.force_collectives:
            w = self._engine.last_wire()
            self.last_wire = w
            self.counters.wire_bytes += self.chunks * 4 * (w["req_words"] + w["rep_words"])
        return out_val, out_status

    def _use_sorted(self) -> bool:
        """Mailbox delivery across ranks through the sorted exchange: the sender's
        counting sort by (destination rank, actor shard) fills the receivers'
        mailboxes directly, with no host wait per Send (csrc/hip/exchange_sorted.hpp).
        It is the N > 1 path of delivery "mailbox" and of "auto" (Join's default:
        ordered methods keep per-(sender, actor) FIFO through its ordered drain,
        stateless ones run in parallel) -- "direct" keeps the epoch engine's fused
        dispatch.  Tune sorted_exchange=0 keeps the epoch engine everywhere."""
        if self.delivery == "direct" or not self.use_engine or self.device.type != "cuda":
            return False
        if self.delivery == "auto" and self.world == 1:  # world 1: the fused local pass / world-1 mailboxes
            return False
        if self.outbox is not None or self.checksum is not None or self.chunks > 4:
            return False
        if not (1 < self.world <= 16 or self.force_collectives):
            return False
        return tune.get("sorted_exchange") != 0

    def _get_sorted(self):
        if self._sorted is None:
            h = B.hip()
            dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
            c_alloc = self._sorted_c_alloc()
            fake = self.fake[0] if self.fake is not None else self.ipc
            self._sorted = h.SortedExchange(dev, 0 if fake is not None else self._comm_ptr(), self.world, self.rank,
                                            self.max_chunk, self.chunks, c_alloc, min(self.C, c_alloc), fake=fake)
            self._sorted_c_alloc_val = c_alloc
        return self._sorted

    def _send_sorted(self, req: B.MsgBatch, out_val, out_status):
        if req.actor.dtype != torch.int32 or req.a0.dtype != torch.int64:
            raise TypeError("MsgBatch: actor must be int32 and a0..a2 int64")
        uniform = isinstance(req.method, int)
        mcol = None if uniform else req.method.to(torch.int16).contiguous()
        d, n_dir, affine = self.table.directory()
        state = self.state
        eng = self._get_sorted()
        eng.send(B._ptr(req.actor), B._ptr(req.a0), B._ptr(req.a1), B._ptr(req.a2), B._ptr(mcol),
                 int(req.method) if uniform else 0, req.M, B._ptr(self.table.table), self.table.cap, B._ptr(d), n_dir,
                 affine, B._ptr(out_val), B._ptr(out_status), B._ptr(state), 0 if state is None else state.numel(),
                 int(self.delay_us) * 100, self.mailbox_ordered, raw_stream(self.device),
                 B._ptr(self.table.dir_rank) if d is not None else 0)
        w = eng.last_wire()
        # words moved per chunk, all peers (as the epoch engine reports it): padded
        # regions, or the per-pair prefixes when the agreed capacities differ
        w["req_words"] = w["req_moved"]
        w["rep_words"] = w["rep_moved"]
        w.update(engine="sorted", exact=False, adapted=bool(w["agreed"]), C_alloc=self._sorted_c_alloc_val)
        self.last_wire = w
        self.counters.wire_bytes += self.chunks * 4 * (w["req_words"] + w["rep_words"])
        return out_val, out_status

    def _mailbox_on_receipt(self) -> bool:
        """N > 1 (or forced collectives): received records go through the mailboxes."""
        return (self.delivery == "mailbox" and self.device.type == "cuda"
                and (self.world > 1 or self.force_collectives))

    def _use_mailbox(self, req: B.MsgBatch) -> bool:
        if self.device.type != "cuda" or self.world > 1 or self.force_collectives or self.delivery == "direct":
            return False
        if self.delivery == "mailbox":
            return True
        return isinstance(req.method, int) and method_ordered(req.method)

    def _mailboxes(self):
        if self.mailboxes is None:
            from ..ops.mailbox import Mailboxes

            S = self.mailbox_shards
            per = self.max_chunk * self.chunks / S
            # twice the uniform load per shard: a Send's messages fit at once; skew
            # overflows into send_all's re-send rounds
            Q = self.mailbox_slots or 1 << max(6, math.ceil(math.log2(2 * per + 256)))
            self.mailboxes = Mailboxes(self.device, S, Q, with_a2=True)
        return self.mailboxes

    def _send_mailbox(self, req: B.MsgBatch, out_val, out_status):
        """World-1 Send through the HBM mailboxes: K2 enqueue (a stable counting sort
        into the shard rings) + K3 drain (per-actor serial in ring order when the
        batch may carry ordered methods, else every record in parallel).
        Actor-sharded rings unless ``mailbox_ordered=False`` promised a batch
        without ordered methods (then arrival-sharded)."""
        from ..ops.mailbox import batch_ordered

        ordered = batch_ordered(req)
        sharding = "actor" if self.mailbox_ordered else "arrival"
        # A batch without ordered methods keeps no per-actor order, so the rings it
        # takes are free: up to 2 Mi messages the arrival rings (one enqueue + drain
        # launch, mbx_arrival_fused_kernel) beat the sorted ones at every measured size
        # (1 Mi: 0.039 vs 0.046 ms per step; profiles/r6_small_sends.md); above, the
        # one-pass sort with its 8-B records (8 Mi: 51.9 vs 50.0 G msg/s)
        if sharding == "actor" and not ordered and req.M <= ARRIVAL_AUTO_MAX and tune.get("auto_arrival"):
            sharding = "arrival"
        self._mailboxes().send(req, self.table, self.state, out_val, out_status, rank_self=self.rank,
                               delay_us=self.delay_us, outbox=self.outbox, ordered=ordered, sharding=sharding)
        return out_val, out_status

    def packed_active(self) -> bool:
        """Whether the next native send uses wire format v3."""
        return bool(self.packed and self.use_engine and not self._capturing
                    and (self.world > 1 or self.force_collectives))

    # ------------------------------------------------------------------
    def _a2a(self, out, inp):
        if self.world == 1 and not self.force_collectives:
            return None
        if self.native:  # (the Python pipeline beside a NativeGroup: world 1 only, a self copy)
            if self.world > 1:
                raise RuntimeError("the Python pipeline runs over torch groups; a NativeGroup drives the native engines")
            out.copy_(inp)
            return None
        return dist.all_to_all_single(out, inp, group=self.group, async_op=True)

    def send(self, req: B.MsgBatch, out_val: torch.Tensor | None = None, out_status: torch.Tensor | None = None):
        """Deliver every message of ``req`` (a SoA ``MsgBatch``) to its actor and return
        ``(value int64[M], status int32[M])`` in message order.  Collective:
        every rank of the group must call it (with its own, possibly empty, batch)
        the same number of times."""
        if self._deferred and not self._capturing:  # a deferred Send two Sends old: its agreement buffer is reused
            self._resolve_deferred(final=False)
        M = req.M
        if M > self.max_chunk * self.chunks:
            raise ValueError(f"batch of {M} exceeds max_batch {self.max_chunk * self.chunks}")
        dev = self.device
        out_val = torch.empty(M, dtype=torch.int64, device=dev) if out_val is None else out_val
        out_status = torch.empty(M, dtype=torch.int32, device=dev) if out_status is None else out_status
        self._last_mailbox = self._use_mailbox(req)
        if self._last_mailbox:  # world 1: one sorted mailbox pass over the whole batch (no wire, no chunks)
            self.counters.sent += M
            self.counters.epochs += 1
            with trace.range("ptype.send.mailbox"):
                return self._send_mailbox(req, out_val, out_status)
        n = self.chunks
        bounds = [min(M, i * self.max_chunk) for i in range(n + 1)]
        R, C = self.world, self.C
        fmt = self.fmt or B.WireFormat.for_batch(req)
        if not fmt.admits(req):
            raise ValueError(f"batch columns do not fit the exchange's wire format {fmt}")
        wq, wr = R * fmt.req_words(C), R * B.WireFormat.rep_words(C)
        self.counters.sent += M
        self.counters.epochs += n
        self._last_sorted = bool(self.use_engine and self._use_sorted())
        if self._last_sorted:
            with trace.range("ptype.send.sorted"):
                return self._send_sorted(req, out_val, out_status)
        if self.use_engine and self._engine is None:
            try:
                self._get_engine()
            except RuntimeError as e:  # e.g. a gloo group over CUDA tensors: no RCCL communicator
                if "RCCL" not in str(e):
                    raise
                self.use_engine = False
        if self.use_engine:
            with trace.range("ptype.send"):
                return self._send_native(req, out_val, out_status, fmt)
        if R > 1 or self.force_collectives:
            self.counters.wire_bytes += n * 4 * (wq + wr)
        pending_bwd = []  # (chunk index, work handle, bufs)

        direct = self.direct
        local_only = R == 1  # every message is self-directed: nothing comes back
        self._bounds, self._outs = bounds, (out_val, out_status)

        def finish(entry):
            i, work, bufs = entry
            if work is not None:
                work.wait()
            lo, hi = bounds[i], bounds[i + 1]
            if direct and local_only and self.checksum is None:
                return
            B.complete(bufs.back[:wr], bufs.perm[: hi - lo], C, out_val[lo:hi], out_status[lo:hi], self.checksum,
                       direct=direct)

        fwd = None
        with trace.range("ptype.send"):
            for i in range(n):
                bufs = self.bufs[i % len(self.bufs)]
                lo, hi = bounds[i], bounds[i + 1]
                # buffer reuse: chunk i-2's replies must be consumed before overwriting
                while pending_bwd and pending_bwd[0][0] <= i - len(self.bufs):
                    finish(pending_bwd.pop(0))
                with trace.range("ptype.route"):
                    dv = (out_val[lo:hi], out_status[lo:hi], bufs.src) if direct else None
                    B.route(req.slice(lo, hi), self.table, R, C, self.rank, sendbuf=bufs.send[:wq],
                            perm=bufs.perm[: hi - lo], rws=bufs.rws, fmt=fmt, reset_stats=False, direct=dv,
                            write_perm=not (direct and local_only and self.checksum is None))
                work = self._a2a(bufs.recv[:wq], bufs.send[:wq])
                if fwd is not None:
                    pending_bwd.append(self._serve(*fwd, fmt))
                fwd = (i, work, bufs, hi - lo)
            if fwd is not None:
                pending_bwd.append(self._serve(*fwd, fmt))
            with trace.range("ptype.complete"):
                for e in pending_bwd:
                    finish(e)
        return out_val, out_status

    def _serve(self, i, work, bufs, m, fmt):
        if work is not None:
            work.wait()
        wq, wr = self.world * fmt.req_words(self.C), self.world * B.WireFormat.rep_words(self.C)
        dv = None
        if self.direct:
            lo, hi = self._bounds[i], self._bounds[i + 1]
            dv = (self._outs[0][lo:hi], self._outs[1][lo:hi], bufs.src)
        with trace.range("ptype.dispatch"):
            B.dispatch(bufs.recv[:wq], self.world, self.C, self.state, self.delay_us, reply=bufs.reply[:wr], ws=bufs.ws,
                       expected_per_rank=max(1, m // self.world), fmt=fmt, outbox=self.outbox, direct=dv,
                       rank_self=self.rank)
        return (i, self._a2a(bufs.back[:wr], bufs.reply[:wr]), bufs)

    # ------------------------------------------------------------------
    def capture(self, req: B.MsgBatch, out_val: torch.Tensor, out_status: torch.Tensor, prologue=None,
                allow_collectives: bool = False, repeat: int = 1) -> "SendGraph":
        """Capture ``send(req)`` (plus an optional ``prologue()``, e.g. a kernel
        that refills ``req``) into a hipGraph for fixed-shape steady-state epochs:
        one graph launch replaces the ~6 kernel launches + host logic per chunk,
        which is what bounds small batches.  ``repeat``: that many (prologue +
        Send) rounds in one graph -- one replay per ``repeat`` steps, for batches
        small enough that the graph launch itself shows; ``prologue(j)`` then gets
        the step's index j within the replay.  Single rank by default;
        RCCL collectives are capturable but opt-in (``allow_collectives``)."""
        if (self.world > 1 or self.force_collectives) and not allow_collectives:
            raise RuntimeError("capture: collectives in a graph are opt-in (allow_collectives=True)")
        return SendGraph(self, req, out_val, out_status, prologue, repeat)

    # ------------------------------------------------------------------
    def pump(self, outbox, initial: B.MsgBatch | None = None, max_epochs: int = 1 << 20, check_every: int = 8):
        """Actor-to-actor messaging on the device: deliver ``initial`` (if any),
        then keep routing whatever the dispatched handlers emitted into
        ``outbox`` until every rank's outbox is empty.  Fire-and-forget ("tell")
        semantics: replies of emitted messages are discarded; overflowed slots are
        re-sent.  Collective; the host reads one count per epoch -- on one rank
        (native engine, direct delivery) once per ``check_every`` epochs: each
        epoch's kernel reads its batch length from the outbox bank's device
        counter, so epochs queue back to back without a host round trip.
        Returns ``(epochs, messages delivered by this rank's sends)``."""
        prev, self.outbox = self.outbox, outbox
        per_send = self.max_chunk * self.chunks
        epochs = delivered = 0
        try:
            if initial is not None:  # every rank passes one (possibly empty), same columns
                m0 = initial.M
                mx0 = self._agree_max(m0) if self.world > 1 else m0
                for lo in range(0, mx0, per_send):
                    self.send_all(initial.slice(min(lo, m0), min(m0, lo + per_send)))
                delivered += m0
            if self._device_pump_ok(outbox):
                e, d = self._pump_device(outbox, max_epochs, check_every)
                return epochs + e, delivered + d
            if self._device_pump_multi_ok(outbox):
                e, d = self._pump_device_multi(outbox, max_epochs, check_every)
                return epochs + e, delivered + d
            while epochs < max_epochs:
                n = outbox.pending()
                mx = self._agree_max(n) if self.world > 1 else n
                if mx == 0:
                    break
                batch = outbox.take(n)
                for lo in range(0, mx, per_send):  # same number of collective sends on every rank
                    self.send_all(batch.slice(min(lo, n), min(n, lo + per_send)))
                delivered += n
                epochs += 1
        finally:
            self.outbox = prev
        return epochs, delivered

    def _device_pump_ok(self, outbox) -> bool:
        """The single-rank local path (one fused kernel per epoch, no slots) with
        an outbox whose banks fit one Send."""
        return bool(self.use_engine and self.world == 1 and not self.force_collectives and self.direct
                    and self.delivery != "mailbox" and outbox.cap <= self.max_chunk * self.chunks
                    and tune.get("device_pump") != 0 and B.hip().tune()["local"] != 0)

    def _device_pump_multi_ok(self, outbox) -> bool:
        """Several ranks (RCCL, or FakeComm in-process ranks) on the native engine
        with an outbox whose bank fits one Send."""
        # (a destination slot holds a whole bank, so no tell can overflow: nothing to re-send)
        return bool(self.use_engine and self.device.type == "cuda" and (self.world > 1 or self.force_collectives)
                    and (self.fake is None or not self.fake[0].loopback)
                    and outbox.cap <= self.max_chunk * self.chunks and self.C >= outbox.cap
                    and tune.get("device_pump") != 0)

    def _pump_device_multi(self, outbox, max_epochs: int, check_every: int):
        """Multi-rank pump without a host round trip per epoch.
        Epoch j routes the active bank's FULL capacity -- the slots past its device
        count are sealed as no-actor messages, so no host size is needed -- over
        the padded all-to-all (wire v2: no agreement wait), the handlers emit into
        the other bank, and a tiny kernel records the count.  After a group of
        ``check_every`` epochs the group's counts and what is left pending are
        max-reduced over the ranks ON THE DEVICE (RCCL all-reduce / FakeComm) and
        copied to pinned memory; the host reads them while the next group already
        runs.  Every rank reads the same agreed vector, so all stop after the same
        group: when nothing is left anywhere."""
        from ..ops import hip

        k = max(2, check_every + (check_every & 1))
        cap = outbox.cap
        dev = self.device
        p0 = outbox.active
        val = torch.empty(cap, dtype=torch.int64, device=dev)  # replies of tells: discarded
        st = torch.empty(cap, dtype=torch.int32, device=dev)
        own = torch.zeros(2, k + 1, dtype=torch.int64, device=dev)  # per group: epoch counts + what is left
        agreed = torch.zeros(2, k + 1, dtype=torch.int64, device=dev)
        host = torch.zeros(2, 2, k + 1, dtype=torch.int64, pin_memory=True)  # [group buffer][own, agreed]
        ev = [torch.cuda.Event(), torch.cuda.Event()]
        start_count = outbox.banks[p0]["count"]  # active again after every (even) group
        # wire v2 (no agreement wait inside a Send), direct dispatch (no ring to overflow)
        prev = (self._capturing, self.delivery)
        self._capturing, self.delivery = True, "direct"

        def launch(h):
            stream = torch.cuda.current_stream(dev).cuda_stream
            for j in range(k):
                b = outbox.bank
                outbox.active ^= 1  # the handlers emit into the other bank (emptied when it was consumed)
                hip().outbox_seal(B._ptr(b["actor"]), cap, B._ptr(b["count"]), stream)
                self.send(B.MsgBatch(b["actor"], b["a0"], b["a1"], b["a2"], b["method"]), val, st)
                hip().outbox_advance(B._ptr(b["count"]), cap, B._ptr(own[h]), j, stream)
            own[h, k:].copy_(start_count[:1])  # pending after the group
            agreed[h].copy_(own[h])
            if self.fake is not None:  # max over the ranks, on the device side of the comm
                self.fake[0].allreduce_max(self.rank, agreed[h].data_ptr(), k + 1, stream)
            elif self.ipc is not None:
                self.ipc.allreduce_max(agreed[h].data_ptr(), k + 1, stream)
            elif self.native:
                self.group.allreduce_max_dev(agreed[h], stream)
            else:
                dist.all_reduce(agreed[h], op=dist.ReduceOp.MAX, group=self.group)
            host[h, 0].copy_(own[h], non_blocking=True)
            host[h, 1].copy_(agreed[h], non_blocking=True)
            ev[h].record()

        def account(h):
            mine = host[h, 0, :k].tolist()
            self.counters.pump_sealed += k * cap - sum(mine)  # sealed slots route as no-actor: kept out of stats()
            return sum(mine)

        epochs = delivered = 0
        try:
            launch(0)
            launched, h = k, 1
            while True:
                more = launched < max_epochs
                if more:  # the next group runs while this one's agreed counts are read
                    launch(h)
                    launched += k
                ev[h ^ 1].synchronize()
                counts = host[h ^ 1, 1, :k].tolist()  # agreed: the same on every rank
                left = int(host[h ^ 1, 1, k])
                n_ep = sum(1 for m in counts if m)
                epochs += n_ep
                self.counters.epochs += n_ep
                delivered += account(h ^ 1)
                if not more or left == 0:
                    if more:  # the group in flight (no-op: nothing was left) completes on every rank alike
                        ev[h].synchronize()
                        delivered += account(h)
                    break
                h ^= 1
        finally:
            self._capturing, self.delivery = prev
        return epochs, delivered

    def _pump_device(self, outbox, max_epochs: int, check_every: int):
        """World-1 pump without a host round trip per epoch.  Epoch j sends the
        active bank's full capacity with its device count as the length
        (``m_dev``); the handlers emit into the other bank; one tiny kernel
        records the count and empties the consumed bank.  Epochs go in groups of
        ``check_every`` (even: a group starts and ends on the same bank), and the
        host reads a group's counts -- copied to pinned memory behind an event --
        while the NEXT group already runs, so the GPU never waits for the host.
        After the first groups, a group is one hipGraph replay (cached while the
        buffers it points at are unchanged).  ``max_epochs`` is rounded up to a
        whole group; trailing epochs of an empty outbox are no-op launches."""
        from ..ops import hip

        k = max(2, check_every + (check_every & 1))
        cap = outbox.cap
        dev = self.device
        d, n_dir, affine = self.table.directory()
        state = self.state
        engine = self._get_engine()
        p0 = outbox.active
        key = (id(outbox), p0, cap, k, B._ptr(self.table.table), B._ptr(d), n_dir, affine, B._ptr(state),
               B._ptr(self.checksum), int(self.delay_us))
        c = self._pump_graph
        if c is None or c["key"] != key:
            c = self._pump_graph = {
                "key": key, "graphs": [None, None],
                "val": torch.empty(cap, dtype=torch.int64, device=dev),  # replies of tells: discarded
                "st": torch.empty(cap, dtype=torch.int32, device=dev),
                "ms": torch.zeros(2, k, dtype=torch.int64, device=dev),
                "host": torch.zeros(2, k + 1, dtype=torch.int64, pin_memory=True),
                "ev": [torch.cuda.Event(), torch.cuda.Event()]}
        val, st, ms, host, ev = c["val"], c["st"], c["ms"], c["host"], c["ev"]
        start_count = outbox.banks[p0]["count"]  # active again after every (even) group

        def group(h):
            stream = torch.cuda.current_stream(dev).cuda_stream
            for j in range(k):
                b = outbox.bank
                outbox.active ^= 1  # the handlers emit into the other bank (emptied when it was consumed)
                ob, ob_cap = outbox.view()
                engine.send(B._ptr(b["actor"]), B._ptr(b["a0"]), B._ptr(b["a1"]), B._ptr(b["a2"]),
                            B._ptr(b["method"]), 0, cap, B._ptr(self.table.table), self.table.cap, B._ptr(d), n_dir,
                            affine, 3, True, B._ptr(val), B._ptr(st), B._ptr(state),
                            0 if state is None else state.numel(), int(self.delay_us) * 100, ob, ob_cap, True,
                            B._ptr(self.checksum), stream, False, 0, False, B._ptr(b["count"]))
                hip().outbox_advance(B._ptr(b["count"]), cap, B._ptr(ms[h]), j, stream)

        def launch(h):
            if c["graphs"][h] is not None:
                c["graphs"][h].replay()
            else:
                group(h)
            host[h, :k].copy_(ms[h], non_blocking=True)
            host[h, k:].copy_(start_count[:1], non_blocking=True)  # what is left to pump
            ev[h].record()

        use_graphs = tune.get("pump_graph") != 0
        epochs = delivered = 0
        launch(0)
        launched, h = k, 1
        while True:
            more = launched < max_epochs
            if more:  # the next group runs while this one's counts are read
                launch(h)
                launched += k
            ev[h ^ 1].synchronize()
            counts = host[h ^ 1, :k].tolist()
            left = int(host[h ^ 1, k])
            n_ep = sum(1 for m in counts if m)
            epochs += n_ep
            delivered += sum(counts)
            self.counters.sent += sum(counts)
            self.counters.epochs += n_ep
            if not more:
                break
            if left == 0:  # the group in flight has nothing to deliver
                break
            if use_graphs and c["graphs"][h ^ 1] is None:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    group(h ^ 1)
                c["graphs"][h ^ 1] = g
            h ^= 1
        return epochs, delivered

    # ------------------------------------------------------------------
    def send_all(self, req: B.MsgBatch, max_epochs: int = 16, out: tuple | None = None, defer: bool = False):
        """`send` + re-send of overflowed messages until every one is delivered.
        Reads the overflow count once per epoch (a host round trip); with adaptive
        slot capacity (native engine, wire v3) skewed traffic fits in the first
        epoch and no re-send round runs.

        ``defer`` (sorted exchange, N > 1): return without waiting
        for this Send's overflow count.  The count arrives with the Send's own
        agreement, which Send k + 2 waits for anyway to pick its layout, so Send k
        is resolved right before Send k + 2 is issued (or by ``flush()``): when any
        rank overflowed, every rank runs the re-send rounds then -- the same point
        on every rank -- and writes the replies into Send k's output tensors.  Until
        then a message that overflowed reads STATUS_OVERFLOW ("pending re-send"),
        and the batch ``req`` must stay unchanged.  No host wait on the current
        Send."""
        val, st = self.send(req, *(out or ()))
        if self._fits_for_sure():
            return val, st
        if defer and self._last_sorted and out is None and not self._keeps_fifo(req):
            self._deferred.append((self._sorted.sends - 1, req, val, st, max_epochs))
            return val, st
        return self._resend_rounds(req, val, st, max_epochs, None)

    def _keeps_fifo(self, req: B.MsgBatch) -> bool:
        """Whether ``req``'s overflow must be re-sent before the next Send: a batch
        that may carry an ordered method on actor-sharded delivery keeps per-(sender,
        actor) FIFO, so its overflowed suffix runs before any later Send's messages
        to the same actors (a deferred re-send ran them after Send k + 1's).
        The reference's Call completes before its caller's next one (rpc.go:59-67)."""
        from ..ops.mailbox import batch_ordered

        return self.mailbox_ordered and batch_ordered(req)

    def flush(self) -> None:
        """Resolve every deferred Send (``send_all(defer=True)``): afterwards all
        their outputs are final.  Collective (re-send rounds may run)."""
        self._resolve_deferred(final=True)

    def pending(self) -> int:
        """Deferred Sends whose overflow is not resolved yet (``flush`` resolves them)."""
        return len(self._deferred)

    def drop_pending(self) -> int:
        """Forget deferred Sends without re-sending (their generation failed: the
        caller re-sends whole batches).  Returns how many were dropped."""
        n = len(self._deferred)
        self._deferred.clear()
        return n

    def _resolve_deferred(self, final: bool) -> None:
        # Send k is resolved just before Send k + 2 (its agreement buffer is reused
        # then); `final`: all of them.  The order and the points are the same on every
        # rank (every rank issues the same Sends), so the re-send rounds stay collective.
        while self._deferred:
            k, req, val, st, max_epochs = self._deferred[0]
            if not final and k > self._sorted.sends - 2:
                break
            self._deferred.popleft()
            n_over = int(self._sorted.overflow_of(k))
            if n_over:
                self._resend_rounds(req, val, st, max_epochs, n_over)

    def _resend_rounds(self, req, val, st, max_epochs: int, n_first):
        n_over = n_first
        for _ in range(max_epochs):
            over = st == STATUS_OVERFLOW
            if n_over is not None:
                pass  # (a deferred Send's count, already read)
            elif self._last_sorted:
                # the sorted exchange folds every rank's overflow count into its own
                # agreement all-reduce: one wait on that copy, no count pass, no collective
                n_over = int(self._sorted.last_overflow())
            else:
                n_over = int(over.sum())
                if self.world > 1:
                    n_over = self._agree_max(n_over)
            if n_over == 0:
                break
            n_over = None
            idx = torch.nonzero(over).flatten()
            self.counters.resends += 1
            v2, s2 = self.send(req.index_select(idx))
            val[idx] = v2
            st[idx] = s2
        return val, st

    def _fits_for_sure(self) -> bool:
        """Whether the last native send provably overflowed no slot on any rank: its
        capacity was sized from the agreed busiest (rank, destination) bucket of the
        node and that bucket fit.  Every rank holds the same agreed vector, so all
        take this exit together -- no count, no host round trip, no agreement."""
        if self.world == 1 and not self.force_collectives and not self._last_mailbox and self.C >= self.max_chunk:
            return True  # one destination whose slot holds a whole chunk: nothing can overflow
        if (self.world == 1 and not self.force_collectives and self._last_mailbox and self.mailboxes is not None
                and getattr(self.mailboxes, "last_spills", False)):
            return True  # stateless mailbox Send: full rings spill to the drain (no STATUS_OVERFLOW)
        if getattr(self, "_last_sorted", False):
            return False  # the agreement that sized it is two Sends old: read this Send's count (send_all)
        if self._mailbox_on_receipt():
            # the slots fit, but K2 on receipt can still answer STATUS_OVERFLOW when a
            # receiver's rings fill (skewed traffic to one shard): count them
            return False
        w = self.last_wire
        if not (self.use_engine and w is not None and w.get("adapted")):
            return False
        return int(w["meta"][META_CAP]) <= int(w["C"])

    def _agree_max(self, v: int) -> int:
        """Max of ``v`` over the group (every rank must take the same number of
        re-send rounds).  In-process FakeComm ranks agree through a barrier; the
        loopback stand-in is one rank that speaks for a symmetric node."""
        if self.fake is None and self.native:
            return int(self.group.allreduce_max([v])[0])
        if self.fake is None:
            t = torch.tensor([v], dtype=torch.int64, device=self._agree_device())
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            return int(t.item())
        fc = self.fake[0]
        if fc.loopback:
            return v
        return _FakeAgree.of(fc).max(self.rank, v)

    def stats(self) -> EpochStats:
        c = self.counters
        s = EpochStats(sent=c.sent, epochs=c.epochs, wire_bytes=c.wire_bytes, resends=c.resends,
                       pump_sealed=c.pump_sealed)
        s.nomatch -= c.pump_sealed
        for b in self.bufs:
            w = B.ws_stats(b.ws).tolist()
            s.nomatch += w[B.STAT_NOMATCH]
            s.overflow += w[B.STAT_OVERFLOW]
            s.failed += w[B.STAT_FAILED]
            s.toowide += int(b.ws[B.STAT_TOOWIDE])
            if w[B.STAT_ROUTE_ERROR]:
                raise RuntimeError("route look-back stalled: epoch results are invalid")
        if self._sorted is not None:
            f = self._sorted.stats()
            s.failed += int(f[0])
            s.toowide += int(f[1])
            if len(f) > 2 and f[2]:
                raise RuntimeError("sorted exchange: one-pass look-back stalled: results are invalid")
        if self.mailboxes is not None:
            m = self.mailboxes.stats()
            if m.get("lookback_timeouts"):
                raise RuntimeError("mailbox sort: one-pass look-back stalled: results are invalid")
            s.nomatch += m["no_actor"]
            s.overflow += m["overflow"]
            s.failed += m["failed"]
            s.mailbox = m
        return s


def ipc_cap_for(max_batch: int, chunks: int, world: int, slack: float = 0.01) -> int:
    """Bytes per peer region an IpcComm must move for an exchange of this
    geometry (``ActorExchange.ipc_cap_bytes``), for forming the group before the
    exchange exists (DeviceRuntime.for_cluster)."""
    chunks = max(1, int(chunks))
    max_chunk = int(math.ceil(max_batch / chunks))
    C = capacity_for(max_chunk, world, slack)
    room = tune.get("skew_room")
    c_alloc = max(C, min(max_chunk, int(math.ceil(room * max_chunk / world))))
    sroom = tune.get("sorted_room")
    c_sorted = max(64, C, min(max_chunk, int(math.ceil(sroom * max_chunk / world))))
    sorted_req = 4 * (((4 + c_sorted * 8 + 3) & ~3) + 68)
    epoch_req = 4 * int(B.hip().wire_req_words(c_alloc, 3, True))
    epoch_rep = 4 * int(B.hip().wire_rep_words(c_alloc))
    agree = 8 * (META_WORDS + world * world * chunks)
    return max(sorted_req, epoch_req, epoch_rep, agree, 1 << 20)


def ipc_group_comm(group, device: torch.device, cap_bytes: int, timeout_s: float = 30.0):
    """An ``_hip.IpcComm`` over the ranks of ``group`` (collective): every rank
    creates its receive segment (shared memory), the names travel through the
    group (``all_gather_object``; gloo is enough), every rank maps and registers
    the others', and once all have, the names are removed (nothing is left in
    /dev/shm when a rank is killed later)."""
    import uuid

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    token = [uuid.uuid4().hex[:12] if rank == 0 else None]
    dist.broadcast_object_list(token, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    c = B.hip().IpcComm(idx, world, rank, int(cap_bytes), float(timeout_s), f"ptype-ipc-{token[0]}-{rank}")
    names = [None] * world
    dist.all_gather_object(names, c.handle(), group=group)
    c.connect(names)
    dist.barrier(group=group)
    c.seal()
    return c


class _FakeAgree:
    """Max-agreement among the in-process ranks of one FakeComm (one thread each)."""

    _by_comm: dict = {}
    _lock = threading.Lock()

    def __init__(self, R: int):
        self.R = R
        self.vals = [0] * R
        self.barrier = threading.Barrier(R)

    @classmethod
    def of(cls, fc) -> "_FakeAgree":
        with cls._lock:
            a = cls._by_comm.get(id(fc))
            if a is None:
                a = cls._by_comm[id(fc)] = cls(int(fc.size))
            return a

    def max(self, rank: int, v: int) -> int:
        self.vals[rank] = v
        self.barrier.wait()
        out = max(self.vals)
        self.barrier.wait()  # nobody overwrites a value before every rank has read them
        return out


class SendGraph:
    """A captured ``ActorExchange.send`` over fixed buffers (``torch.cuda.CUDAGraph``
    is a hipGraph on ROCm).  ``replay()`` re-runs every kernel of the epoch(s) on
    whatever ``req`` holds at that moment."""

    def __init__(self, ex: ActorExchange, req: B.MsgBatch, out_val, out_status, prologue=None, repeat: int = 1):
        if repeat < 1:
            raise ValueError("repeat >= 1")
        self.ex, self.req, self.M, self.repeat = ex, req, req.M, int(repeat)
        dev = ex.device

        def one(j=0):
            if prologue is not None:
                if self.repeat > 1:
                    prologue(j)  # the step's index within the replay
                else:
                    prologue()
            ex.send(req, out_val, out_status)

        def body():
            for j in range(self.repeat):
                one(j)

        ex.table.directory()  # build outside the capture if dirty
        # fixed-geometry v2 slots inside the graph (no host wait); the flag covers
        # only the warm-up and the capture, so eager sends afterwards keep wire v3
        prev, ex._capturing = ex._capturing, True
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):  # warm allocations / lazy state outside the graph
                    one()
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                body()
        finally:
            ex._capturing = prev
        self.replays = 0

    def replay(self) -> None:
        """One graph launch: ``repeat`` steps."""
        self.graph.replay()
        self.replays += 1
        self.ex.counters.sent += self.M * self.repeat
        self.ex.counters.epochs += self.ex.chunks * self.repeat

