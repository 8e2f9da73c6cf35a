"""Watch-driven GPU registry mirror (SURVEY C9, K5 + K6).

The authoritative placement of a service's actors is in the replicated store:
every node that hosts actors keeps one shard record,
``store/_ptype/actors/<service>/<node>`` -> ``{"rank", "world", "count", "node"}``
(actor ``a`` of the shard: ``a = rank + world * mbox``, ``mbox < count``),
attached to a 2 s lease the node keeps alive -- exactly how the reference keeps
``services/<svc>/<node>/`` (cluster/registry.go:51-86).  A node that dies stops
refreshing; its lease expires and the record is deleted.

The mirror follows those records into the GPU hash table the route kernels
read, the way the reference's clients follow ``WatchService``
(cluster/registry.go:119-150) with a debounce (cluster/rpc.go:197-244):

* a watch thread collects PUT / DELETE events of the prefix (plus a periodic
  re-list, which also refreshes when each shard was last seen alive), and
* ``apply()`` -- called by the runtime at the start of every Send, on the
  caller's stream, so no kernel reads a table that is being rebuilt under it --
  upserts or deletes the shards' actors with K5 batch kernels and drives K6:
  every entry carries the deadline ``last seen + TTL + grace`` and a sweep
  tombstones the ones whose node has not been seen since (the backstop when no
  DELETE event arrives, e.g. a broken watch stream).

So a node that joins after this one becomes routable at the next Send, and one
whose lease lapses disappears within TTL + the re-list period.

After a rank failure (runtime.py ``recover``) the survivors form data-plane
generation g + 1 and re-home the dead rank's actors (parallel/elastic.py
``ring_placement``): a record then carries ``"gen"`` and ``"blocks"`` -- the
original ranks whose actors the node hosts, block j in mailboxes
``[j * count, (j + 1) * count)`` (actor ``b + world * k`` of original rank b in
mailbox ``j * count + k``, ``world`` the original world).  The mirror drops the
records of older generations without touching the table (the recovering
runtime rebuilt it for the new placement), so a dead node's late DELETE can not
unroute actors that were adopted meanwhile.

``apply()`` is constant-time when nothing changed: the watch thread bumps a
version on every event / re-list, and apply returns at once while the version
is the one it applied and no shard deadline has passed.
"""
from __future__ import annotations

import json
import threading
import time

import torch

from .ops.table import actor_keys

ACTORS_PREFIX = "_ptype/actors"
STORE_PREFIX = "store/"
LEASE_TTL_S = 2  # the reference's service lease (cluster/registry.go:59)


def _prefix_end(p: str) -> str:
    b = bytearray(p.encode())
    b[-1] += 1
    return b.decode()


def _now_ms() -> int:
    return int(time.monotonic() * 1000)


def record_ids(rec: dict) -> tuple[torch.Tensor, torch.Tensor]:
    """(actor ids, mailboxes) of a shard record: actor ``b + world * k`` of every
    hosted original rank b (``blocks``, default ``[rank]``) in mailbox
    ``j * count + k`` (j = the block's index)."""
    P, W = int(rec["count"]), int(rec["world"])
    blocks = rec.get("blocks") or [int(rec["rank"])]
    k = torch.arange(P, dtype=torch.int64)
    ids = torch.cat([int(b) + W * k for b in blocks])
    mbox = torch.cat([j * P + k for j in range(len(blocks))])
    return ids, mbox


class ShardLease:
    """This node's shard record, attached to a lease kept alive until ``close()``
    (graceful close revokes it: the shard disappears at once)."""

    def __init__(self, kv, service: str, node: str, rank: int, world: int, count: int, ttl_s: int = LEASE_TTL_S,
                 **extra):
        from ._core import Context

        self.kv = kv
        self.key = f"{STORE_PREFIX}{ACTORS_PREFIX}/{service}/{node}"
        self.record = {"rank": int(rank), "world": int(world), "count": int(count), "node": node, **extra}
        self.lease, _ = kv.grant(int(ttl_s))
        kv.put(self.key, json.dumps(self.record).encode(), self.lease)
        self._ctx = Context.with_cancel()
        self._ka = kv.keepalive(self._ctx, self.lease)
        self._th = threading.Thread(target=self._drain, daemon=True, name="ptype-shard-keepalive")
        self._th.start()

    def _drain(self):
        while self._ka.recv(1.0) is not None or not self._ka.closed:
            pass

    def update(self, **fields) -> None:
        """Re-publish the record (same lease) with ``fields`` changed -- a new
        data-plane generation's rank and hosted blocks."""
        self.record = dict(self.record, **fields)
        self.kv.put(self.key, json.dumps(self.record).encode(), self.lease)

    def stop_keepalive(self) -> None:
        """Stop refreshing without revoking: the record expires with the lease (a crash, for tests)."""
        self._ctx.cancel()

    def close(self) -> None:
        self._ctx.cancel()
        try:
            self.kv.revoke(self.lease)
        except Exception:
            pass


class RegistryMirror:
    def __init__(self, table, kv, service: str, ttl_ms: int = LEASE_TTL_S * 1000, grace_ms: int = 1000,
                 relist_s: float = 0.5, watch: bool = True):
        from ._core import Context, RangeOpts

        self.table = table
        self.kv = kv
        self.service = service
        self.prefix = f"{STORE_PREFIX}{ACTORS_PREFIX}/{service}/"
        self.ttl_ms, self.grace_ms, self.relist_s = int(ttl_ms), int(grace_ms), float(relist_s)
        self.shards: dict[str, dict] = {}  # applied: key -> {record, deadline}
        self.applies = 0
        self.min_gen = 0  # records of older data-plane generations are ignored
        self._version = 0  # bumped by the watch thread on every change it queues
        self._applied = -1
        self._next_expiry = 0
        self._lock = threading.Lock()
        self._pending: list[tuple[str, str, dict | None]] = []
        self._seen: dict[str, int] = {}  # key -> monotonic ms it was last listed (lease alive)
        self._opts = RangeOpts()
        self._opts.end = _prefix_end(self.prefix)
        res = kv.get(self.prefix, self._opts)
        now = _now_ms()
        for kv_ in res.kvs:
            self._pending.append(("PUT", kv_.key, json.loads(kv_.value)))
            self._seen[kv_.key] = now
        self._version += 1
        self._stop = threading.Event()
        self._ctx = Context.with_cancel()
        self._watch = kv.watch(self._ctx, self.prefix, self._opts.end, res.rev + 1) if watch else None
        self._th = threading.Thread(target=self._run, daemon=True, name="ptype-registry-mirror")
        self._th.start()

    # ------------------------------------------------------------------ watch thread
    def _run(self) -> None:
        next_list = time.monotonic() + self.relist_s
        while not self._stop.is_set():
            if self._watch is not None and not self._watch.closed:
                resp = self._watch.recv(min(0.1, self.relist_s))
                if resp is not None:
                    with self._lock:
                        for ev in resp.events:
                            if ev.type == "PUT":
                                self._pending.append(("PUT", ev.kv.key, json.loads(ev.kv.value)))
                                self._seen[ev.kv.key] = _now_ms()
                            else:
                                self._pending.append(("DELETE", ev.kv.key, None))
                                self._seen.pop(ev.kv.key, None)
                        self._version += 1
            else:
                self._stop.wait(min(0.1, self.relist_s))
            if time.monotonic() >= next_list:
                next_list = time.monotonic() + self.relist_s
                self._relist()

    def _relist(self) -> None:
        try:
            res = self.kv.get(self.prefix, self._opts)
        except Exception:
            return  # control plane electing: keep the last view; K6 deadlines keep running
        now = _now_ms()
        listed = {kv_.key: kv_ for kv_ in res.kvs}
        with self._lock:
            for k, kv_ in listed.items():
                self._seen[k] = now
                if k not in self.shards and not any(p[1] == k and p[0] == "PUT" for p in self._pending):
                    self._pending.append(("PUT", k, json.loads(kv_.value)))  # a missed PUT
            for k in list(self.shards):
                if k not in listed and not any(p[1] == k for p in self._pending):
                    self._pending.append(("DELETE", k, None))  # a missed DELETE
                    self._seen.pop(k, None)
            self._version += 1

    # ------------------------------------------------------------------ applied on the runtime's stream
    @staticmethod
    def _ids(rec: dict) -> tuple[torch.Tensor, torch.Tensor]:
        return record_ids(rec)

    def set_generation(self, gen: int) -> None:
        """Data-plane generation ``gen`` formed: forget the records of older ones
        (without deleting their actors: the runtime re-homed them)."""
        with self._lock:
            self.min_gen = int(gen)
            self._pending = [p for p in self._pending if p[0] == "DELETE" or int(p[2].get("gen", 0)) >= gen]
            self._version += 1
        for k in [k for k, sh in self.shards.items() if int(sh["record"].get("gen", 0)) < gen]:
            self.shards.pop(k)

    def _put(self, key: str, rec: dict, deadline: int) -> None:
        if int(rec.get("gen", 0)) < self.min_gen:
            return
        old = self.shards.get(key)
        if old is not None and old["record"] != rec:
            self._delete(key)
        if self.table is None:  # records only (a replica set: parallel/replicas.py)
            self.shards[key] = {"record": rec, "deadline": deadline}
            return
        ids, mbox = self._ids(rec)
        n = ids.numel()
        self.table.upsert(actor_keys(ids), torch.full((n,), int(rec["rank"]), dtype=torch.int32),
                          mbox.to(torch.int32), torch.full((n,), deadline, dtype=torch.int64))
        self.shards[key] = {"record": rec, "deadline": deadline}

    def _delete(self, key: str) -> None:
        sh = self.shards.pop(key, None)
        if sh is not None and self.table is not None:
            ids, _ = self._ids(sh["record"])
            self.table.delete(actor_keys(ids))

    def apply(self) -> int:
        """Apply pending registry changes and expiries to the table; returns the
        number of shards added, changed or removed."""
        now = _now_ms()
        if self._version == self._applied and now < self._next_expiry:
            return 0  # nothing new since the last apply (a plain int compare: no lock)
        with self._lock:
            ops, self._pending = self._pending, []
            seen = dict(self._seen)
            version = self._version
        changed = 0
        for op, key, rec in ops:
            if op == "PUT":
                self._put(key, rec, seen.get(key, now) + self.ttl_ms + self.grace_ms)
            else:
                self._delete(key)
            changed += 1
        # K6: refresh the deadlines of shards seen alive since; sweep the rest
        for key, sh in list(self.shards.items()):
            dl = seen.get(key, 0) + self.ttl_ms + self.grace_ms
            if dl - sh["deadline"] > self.ttl_ms // 2:
                self._put(key, sh["record"], dl)
        live_before = len(self.shards)
        expired = [k for k, sh in self.shards.items() if sh["deadline"] < now]
        if expired:
            if self.table is not None:
                self.table.sweep(now)
            for k in expired:
                self.shards.pop(k, None)
            changed += live_before - len(self.shards)
        if changed:
            self.applies += 1
        self._applied = version
        self._next_expiry = min((sh["deadline"] for sh in self.shards.values()), default=now + self.ttl_ms)
        return changed

    def wait_shards(self, n: int, timeout_s: float = 60.0) -> None:
        """Apply until at least ``n`` shards are mirrored."""
        deadline = time.monotonic() + timeout_s
        while True:
            self.apply()
            if len(self.shards) >= n:
                return
            if time.monotonic() > deadline:
                raise TimeoutError(f"registry mirror of {self.service!r}: {len(self.shards)} of {n} shards")
            time.sleep(0.02)

    @property
    def actors(self) -> int:
        return sum(int(sh["record"]["count"]) * len(sh["record"].get("blocks") or [0])
                   for sh in self.shards.values())

    def close(self) -> None:
        self._stop.set()
        self._ctx.cancel()
        self._th.join(2.0)
