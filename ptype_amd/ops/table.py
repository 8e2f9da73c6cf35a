"""GPU registry mirror: open-addressing hash table in HBM.

Wraps kernels K5 (upsert/delete/lookup), K6 (lease sweep) and K7 (snapshot pack)
from ``csrc/hip/registry_table.hip``.  The CPU path is a NumPy reference of the
exact same probing scheme (same hash, same slots), so GPU results can be checked
slot-for-slot.

Reference semantics mirrored: ``Register`` puts a leased key under
``services/<svc>/<node>/`` (cluster/registry.go:51-86); lease expiry removes it
(registry.go:59, TTL 2 s).  Keys here are 64-bit: actor id + 1 on the batch path
(``actor_keys``), or a 64-bit FNV-1a of ``"<svc>/<node>"`` for service nodes.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _ptr, _stream, hip

KEY_EMPTY = 0
KEY_TOMB = -1  # ~0 as int64

STAT_LIVE, STAT_TOMB, STAT_GEN, STAT_MAXPROBE = 0, 1, 2, 3

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer, bit-identical to ``ptype::mix64`` on the device."""
    x = np.asarray(x).astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return x


GROUP = 4  # probe group (kGroup): probing starts at the 64-B line the hash lands in


def probe_start(h: np.ndarray, mask: int) -> np.ndarray:
    return h & np.uint64(mask) & ~np.uint64(GROUP - 1)


def actor_keys(actor_ids: torch.Tensor) -> torch.Tensor:
    """Table keys of batch-path actors: id + 1 (0 means empty)."""
    return actor_ids.to(torch.int64) + 1


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    if h in (0, 0xFFFFFFFFFFFFFFFF):
        h = 1
    return h - (1 << 64) if h >= (1 << 63) else h


def _pow2(n: int) -> int:
    c = 1
    while c < n:
        c <<= 1
    return c


class RegistryTable:
    """Open-addressing registry table resident on one device (HBM) or the CPU."""

    def __init__(self, capacity: int, device="cuda"):
        self.device = torch.device(device)
        self.cap = _pow2(max(16, int(capacity)))
        self.table = torch.zeros(self.cap, 2, dtype=torch.int64, device=self.device)
        self.expiry = torch.zeros(self.cap, dtype=torch.int64, device=self.device)
        self.stats = torch.zeros(8, dtype=torch.int64, device=self.device)
        self.dir = None  # route directory (K5b), GPU only; see enable_directory
        self.dir_rank = None  # its rank byte table (K5c): one byte per id, built with it
        self.dir_n = 0
        self.affine_world = 0  # strided-rule candidate W (0: no check)
        self.affine = 0  # W when the last build verified the rule for every id of the range
        self._astats = None
        self._dir_dirty = True
        # route mode 4 (csrc/hip/mailbox_sort_dev.hpp): the directory folded into 2 bits
        # per id for rank `presence_rank` -- here / probe the table / not here -- rebuilt
        # with the directory, for directories that fit a sort block's LDS (<= 2^18 ids)
        self.presence = None
        self.presence_rank = 0

    # ------------------------------------------------------------------ directory
    def enable_directory(self, n_ids: int, affine_world: int = 0) -> None:
        """Keep a dense route directory for actor ids ``[0, n_ids)``: the registry
        flattened to one 4-B route word per id (K5b), rebuilt lazily after any
        mutation.  The data path reads it instead of probing the hash table; ids
        outside the range still probe the table, so results are identical.

        ``affine_world = W``: each rebuild also verifies, on the device, whether
        every id of the range is registered at rank ``id % W``, mailbox ``id // W``
        (the runtime's strided placement).  While that holds the route computes
        the route words -- no directory gathers -- and the first mutation that
        breaks it (a re-homed or removed actor) falls back to the directory."""
        if not self.is_gpu or n_ids <= 0:
            return
        if n_ids > (1 << 30):
            raise ValueError("directory range too large")
        self.dir_n = int(n_ids)
        self.dir = torch.empty(self.dir_n, dtype=torch.int32, device=self.device)
        # the rank byte of every id (0xff: not registered, 0xfe: probe the table):
        # what a stateless batch's sender needs, at a quarter of the directory's lines
        self.dir_rank = torch.empty(self.dir_n, dtype=torch.uint8, device=self.device)
        self.affine_world = int(affine_world)
        self._astats = torch.zeros(2, dtype=torch.int64, device=self.device) if affine_world else None
        words = int(hip().presence_words(self.dir_n))
        self.presence = torch.empty(words, dtype=torch.int32, device=self.device) if words else None
        self._dir_dirty = True

    def set_presence_rank(self, rank: int) -> None:
        """Keep the presence map for ``rank`` (the world-1 runtime's rank 0 by default)."""
        if int(rank) != self.presence_rank:
            self.presence_rank = int(rank)
            self._dir_dirty = True

    def directory(self):
        """``(dir tensor | None, n, affine W or 0)`` -- rebuilt on device if the table changed."""
        if self.dir is None:
            return None, 0, 0
        if self._dir_dirty:
            hip().table_build_dir(_ptr(self.table), self.cap, _ptr(self.dir), self.dir_n, self.affine_world,
                                  _ptr(self._astats), _stream(self.table), _ptr(self.dir_rank))
            if self.presence is not None:
                hip().presence_build(_ptr(self.dir_rank), self.dir_n, self.presence_rank, _ptr(self.presence),
                                     _stream(self.table))
            self.affine = 0
            if self.affine_world:
                present, bad = (int(x) for x in self._astats.tolist())  # one sync per rebuild
                self.affine = self.affine_world if present == self.dir_n and bad == 0 else 0
            self._dir_dirty = False
        return self.dir, self.dir_n, self.affine

    # ------------------------------------------------------------------ props
    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    def _stat(self, i: int) -> int:
        return int(self.stats[i].item())

    @property
    def live(self) -> int:
        return self._stat(STAT_LIVE)

    @property
    def tombstones(self) -> int:
        return self._stat(STAT_TOMB)

    @property
    def generation(self) -> int:
        return self._stat(STAT_GEN)

    # ------------------------------------------------------------------ ops
    def upsert(self, keys: torch.Tensor, ranks: torch.Tensor, mboxes: torch.Tensor, expiry: torch.Tensor | None = None):
        keys = keys.to(self.device, torch.int64).contiguous()
        ranks = ranks.to(self.device, torch.int32).contiguous()
        mboxes = mboxes.to(self.device, torch.int32).contiguous()
        if expiry is not None:
            expiry = expiry.to(self.device, torch.int64).contiguous()
        n = keys.numel()
        if not (ranks.numel() == n and mboxes.numel() == n and (expiry is None or expiry.numel() == n)):
            raise ValueError("upsert: keys/ranks/mboxes/expiry must have equal length")
        if self.live + self.tombstones + n > self.cap * 3 // 4:
            self._grow(self.live + n)
        self._dir_dirty = True
        if self.is_gpu:
            hip().table_upsert(_ptr(self.table), self.cap, _ptr(keys), _ptr(ranks), _ptr(mboxes), _ptr(expiry),
                               _ptr(self.expiry), n, _ptr(self.stats), _stream(self.table))
        else:
            self._cpu_upsert(keys, ranks, mboxes, expiry)

    def delete(self, keys: torch.Tensor) -> torch.Tensor:
        keys = keys.to(self.device, torch.int64).contiguous()
        found = torch.zeros(keys.numel(), dtype=torch.uint8, device=self.device)
        self._dir_dirty = True
        if self.is_gpu:
            hip().table_delete(_ptr(self.table), self.cap, _ptr(keys), keys.numel(), _ptr(self.stats), _ptr(found),
                               _stream(self.table))
        else:
            self._cpu_delete(keys, found)
        return found.bool()

    def lookup(self, keys: torch.Tensor):
        keys = keys.to(self.device, torch.int64).contiguous()
        n = keys.numel()
        rank = torch.empty(n, dtype=torch.int32, device=self.device)
        mbox = torch.empty(n, dtype=torch.int32, device=self.device)
        if self.is_gpu:
            hip().table_lookup(_ptr(self.table), self.cap, _ptr(keys), n, _ptr(rank), _ptr(mbox), _stream(self.table))
        else:
            r, m = self._cpu_lookup(keys.numpy())
            rank.copy_(torch.from_numpy(r))
            mbox.copy_(torch.from_numpy(m))
        return rank, mbox

    def sweep(self, now_ms: int) -> None:
        """K6: tombstone entries whose deadline (host monotonic ms) has passed."""
        self._dir_dirty = True
        if self.is_gpu:
            hip().table_sweep(_ptr(self.table), self.cap, _ptr(self.expiry), int(now_ms), _ptr(self.stats),
                              _stream(self.table))
        else:
            keys = self.table[:, 0]
            dead = (self.expiry != 0) & (self.expiry < now_ms) & (keys != KEY_EMPTY) & (keys != KEY_TOMB)
            n = int(dead.sum())
            keys[dead] = KEY_TOMB
            if n:
                self.stats[STAT_LIVE] -= n
                self.stats[STAT_TOMB] += n
                self.stats[STAT_GEN] += 1

    def pack(self):
        """K7: compact live entries -> (entries int64[n,2], expiry int64[n]) on the table's device."""
        out = torch.empty(self.cap, 2, dtype=torch.int64, device=self.device)
        out_exp = torch.empty(self.cap, dtype=torch.int64, device=self.device)
        cnt = torch.zeros(1, dtype=torch.int64, device=self.device)
        if self.is_gpu:
            hip().table_pack(_ptr(self.table), self.cap, _ptr(self.expiry), _ptr(out), _ptr(out_exp), _ptr(cnt),
                             _stream(self.table))
        else:
            keys = self.table[:, 0]
            live = (keys != KEY_EMPTY) & (keys != KEY_TOMB)
            n = int(live.sum())
            out[:n] = self.table[live]
            out_exp[:n] = self.expiry[live]
            cnt[0] = n
        n = int(cnt.item())
        return out[:n], out_exp[:n]

    def clear(self) -> None:
        self._dir_dirty = True
        self.table.zero_()
        self.expiry.zero_()
        self.stats[STAT_LIVE] = 0
        self.stats[STAT_TOMB] = 0
        self.stats[STAT_GEN] += 1

    def load_packed(self, entries: torch.Tensor, expiry: torch.Tensor | None = None) -> None:
        """Re-insert packed K7 records (``int64[n, 2]`` = TableEntry, + deadlines).
        On a GPU table: one host->device copy of each array (pinned sources copy
        asynchronously) and one upsert kernel reading the records as they are."""
        n = entries.shape[0]
        if n == 0:
            return
        if not self.is_gpu:
            keys = entries[:, 0].contiguous()
            v = entries[:, 1]
            self.upsert(keys, (v & 0xFFFFFFFF).to(torch.int32), ((v >> 32) & 0xFFFFFFFF).to(torch.int32), expiry)
            return
        ent = entries.to(self.device, non_blocking=True).contiguous()
        exp = expiry.to(self.device, non_blocking=True).contiguous() if expiry is not None else None
        if self.live + self.tombstones + n > self.cap * 3 // 4:
            self._grow(self.live + n)
        self._dir_dirty = True
        hip().table_upsert_packed(_ptr(self.table), self.cap, _ptr(ent), _ptr(exp), _ptr(self.expiry), n,
                                  _ptr(self.stats), _stream(self.table))

    def rebuild(self, min_capacity: int | None = None) -> None:
        """Drop tombstones: pack -> (resize) -> clear -> re-insert."""
        entries, exp = self.pack()
        entries, exp = entries.clone(), exp.clone()
        if min_capacity and _pow2(min_capacity) > self.cap:
            self.cap = _pow2(min_capacity)
            self.table = torch.zeros(self.cap, 2, dtype=torch.int64, device=self.device)
            self.expiry = torch.zeros(self.cap, dtype=torch.int64, device=self.device)
            self.stats[STAT_LIVE] = 0
            self.stats[STAT_TOMB] = 0
        else:
            self.clear()
        if entries.numel():
            self.load_packed(entries, exp)

    def _grow(self, need: int) -> None:
        self.rebuild(min_capacity=max(self.cap, 2 * need))

    # ---------------------------------------------------------- snapshot
    def snapshot_to_host(self, stream: "torch.cuda.Stream | None" = None):
        """K7 straight into pinned host DRAM: the pack kernel writes the live
        entries and deadlines over PCIe into pinned buffers allocated ONCE per
        table (reused by every later snapshot), so a snapshot is one kernel + an
        8-B count read back -- no device staging, no per-snapshot pinned
        allocation.  Runs on ``stream`` (default: a side stream behind the
        current one); returns views ``(entries int64[n, 2], expiry int64[n])``
        valid until the next snapshot of this table."""
        if not self.is_gpu:
            entries, exp = self.pack()
            return entries.clone(), exp.clone()
        if getattr(self, "_snap_cap", 0) < self.cap:
            self._snap_ent = torch.empty(self.cap, 2, dtype=torch.int64, pin_memory=True)
            self._snap_exp = torch.empty(self.cap, dtype=torch.int64, pin_memory=True)
            self._snap_cnt = torch.zeros(1, dtype=torch.int64, device=self.device)
            self._snap_cnt_h = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            self._snap_cap = self.cap
        side = stream if stream is not None else torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            self._snap_cnt.zero_()
            # the kernel stores through the pinned buffers' device mapping (UVA)
            hip().table_pack(_ptr(self.table), self.cap, _ptr(self.expiry), _ptr(self._snap_ent),
                             _ptr(self._snap_exp), _ptr(self._snap_cnt), side.cuda_stream)
            self._snap_cnt_h.copy_(self._snap_cnt, non_blocking=True)
        side.synchronize()
        n = int(self._snap_cnt_h[0])
        return self._snap_ent[:n], self._snap_exp[:n]

    # ---------------------------------------------------------- CPU reference
    def _slots(self):
        return self.table[:, 0].numpy(), self.table[:, 1].numpy()

    def _cpu_upsert(self, keys, ranks, mboxes, expiry):
        tk, tv = self._slots()
        mask = self.cap - 1
        k_np = keys.numpy()
        h_all = mix64(k_np.view(np.uint64))
        added = 0
        maxp = self._stat(STAT_MAXPROBE)
        for i in range(k_np.shape[0]):
            key = int(k_np[i])
            if key in (KEY_EMPTY, KEY_TOMB):
                continue
            h = int(h_all[i]) & mask & ~(GROUP - 1)
            for probe in range(self.cap):
                cur = int(tk[h])
                if cur == key:
                    break
                if cur == KEY_EMPTY:
                    tk[h] = key
                    added += 1
                    break
                h = (h + 1) & mask
            else:
                continue
            v = (int(ranks[i]) & 0xFFFFFFFF) | ((int(mboxes[i]) & 0xFFFFFFFF) << 32)
            tv[h] = v - (1 << 64) if v >= (1 << 63) else v
            self.expiry[h] = int(expiry[i]) if expiry is not None else 0
            maxp = max(maxp, probe)
        self.stats[STAT_LIVE] += added
        self.stats[STAT_MAXPROBE] = maxp
        self.stats[STAT_GEN] += 1

    def _cpu_delete(self, keys, found):
        tk, _ = self._slots()
        mask = self.cap - 1
        k_np = keys.numpy()
        h_all = mix64(k_np.view(np.uint64))
        removed = 0
        for i in range(k_np.shape[0]):
            key = int(k_np[i])
            if key in (KEY_EMPTY, KEY_TOMB):
                continue
            h = int(h_all[i]) & mask & ~(GROUP - 1)
            for _ in range(self.cap):
                cur = int(tk[h])
                if cur == KEY_EMPTY:
                    break
                if cur == key:
                    tk[h] = KEY_TOMB
                    found[i] = 1
                    removed += 1
                    break
                h = (h + 1) & mask
        if removed:
            self.stats[STAT_LIVE] -= removed
            self.stats[STAT_TOMB] += removed
            self.stats[STAT_GEN] += 1

    def _cpu_lookup(self, k_np: np.ndarray):
        """Vectorised probe loop: every key advances one slot per iteration."""
        tk, tv = self._slots()
        mask = self.cap - 1
        n = k_np.shape[0]
        rank = np.full(n, -1, dtype=np.int32)
        mbox = np.full(n, -1, dtype=np.int32)
        valid = (k_np != KEY_EMPTY) & (k_np != KEY_TOMB)
        h = probe_start(mix64(k_np.view(np.uint64)), mask).astype(np.int64)
        pending = np.nonzero(valid)[0]
        for _ in range(self.cap):
            if pending.size == 0:
                break
            cur = tk[h[pending]]
            hit = cur == k_np[pending]
            empty = cur == KEY_EMPTY
            idx = pending[hit]
            v = tv[h[idx]]
            rank[idx] = (v & 0xFFFFFFFF).astype(np.int32)
            mbox[idx] = ((v >> 32) & 0xFFFFFFFF).astype(np.int32)
            pending = pending[~hit & ~empty]
            h[pending] = (h[pending] + 1) & mask
        return rank, mbox
