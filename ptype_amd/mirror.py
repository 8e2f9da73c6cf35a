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
version on every event / re-list, and ``quiet(now)`` (two loads, no lock) is
true while the version is the one applied and no shard deadline has passed.
"""
from __future__ import annotations

import json
import time

import torch

from .ops.table import actor_keys

ACTORS_PREFIX = "_ptype/actors"
STORE_PREFIX = "store/"
LEASE_TTL_S = 2  # the reference's service lease (cluster/registry.go:59)


def _prefix_end(p: str) -> str:
    """etcd's prefix range end (clientv3.GetPrefixRangeEnd for a non-empty prefix)."""
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
    (graceful close revokes it: the shard disappears at once).  A thin handle on
    the compiled ``_core.ShardLease``."""

    def __init__(self, kv, service: str, node: str, rank: int, world: int, count: int, ttl_s: int = LEASE_TTL_S,
                 **extra):
        from ._core import ShardLease as _Lease

        self.key = f"{STORE_PREFIX}{ACTORS_PREFIX}/{service}/{node}"
        self.record = {"rank": int(rank), "world": int(world), "count": int(count), "node": node, **extra}
        self._l = _Lease(kv, self.key, json.dumps(self.record), int(ttl_s))
        self.lease = self._l.lease

    def update(self, **fields) -> None:
        """Re-publish the record (same lease) with ``fields`` changed -- a new
        data-plane generation's rank and hosted blocks."""
        self.record = dict(self.record, **fields)
        self._l.update(json.dumps(self.record))

    def stop_keepalive(self) -> None:
        """Stop refreshing without revoking: the record expires with the lease (a crash, for tests)."""
        self._l.stop_keepalive()

    def close(self) -> None:
        self._l.close()


class RegistryMirror:
    """Device table <- compiled follower (``_core.RegistryFollower``).  ``table``
    None: records only (a replica set, parallel/replicas.py)."""

    def __init__(self, table, kv, service: str, ttl_ms: int = LEASE_TTL_S * 1000, grace_ms: int = 1000,
                 relist_s: float = 0.5, watch: bool = True):
        from ._core import RegistryFollower

        self.table = table
        self.service = service
        self.prefix = f"{STORE_PREFIX}{ACTORS_PREFIX}/{service}/"
        self._f = RegistryFollower(kv, self.prefix, int(ttl_ms), int(grace_ms), float(relist_s), bool(watch))

    def apply(self) -> int:
        """Apply pending registry changes and expiries to the table; returns the
        number of shards added, changed or removed."""
        now = _now_ms()
        if self._f.quiet(now):
            return 0  # nothing new since the last apply
        ops, sweep, changed = self._f.take(now)
        if self.table is not None:
            for kind, _key, rank, deadline, ids, mbox in ops:
                keys = actor_keys(torch.from_numpy(ids))
                if kind == 0:
                    n = ids.shape[0]
                    self.table.upsert(keys, torch.full((n,), rank, dtype=torch.int32), torch.from_numpy(mbox),
                                      torch.full((n,), deadline, dtype=torch.int64))
                else:
                    self.table.delete(keys)
            if sweep:
                self.table.sweep(now)
        return changed

    def set_generation(self, gen: int) -> None:
        """Data-plane generation ``gen`` formed: forget the records of older ones
        (without deleting their actors: the runtime re-homed them)."""
        self._f.set_generation(int(gen))

    @property
    def shards(self) -> dict[str, dict]:
        """Applied shards: key -> {"record", "deadline"} (a snapshot, not the hot path)."""
        return {k: {"record": json.loads(rec), "deadline": dl} for k, rec, dl in self._f.shards()}

    @property
    def applies(self) -> int:
        return int(self._f.applies)

    def wait_shards(self, n: int, timeout_s: float = 60.0) -> None:
        """Apply until at least ``n`` shards are mirrored."""
        deadline = time.monotonic() + timeout_s
        while True:
            self.apply()
            if len(self._f.shards()) >= n:
                return
            if time.monotonic() > deadline:
                raise TimeoutError(f"registry mirror of {self.service!r}: {len(self._f.shards())} of {n} shards")
            time.sleep(0.02)

    @property
    def actors(self) -> int:
        return int(self._f.actors)

    def close(self) -> None:
        self._f.close()
