"""ptype_amd -- an MI355X-native actor-cluster runtime with the capabilities of
edegens/ptype.

* ``ptype_amd.cluster`` -- the reference's API (Join/New, ConfigFromFile,
  Registry, KVStore, Client.Call/Go/Send, Serve) over a C++ control plane
  (Raft + MVCC + leases + watch, TCP transport, Go net/rpc + gob wire format).
* ``ptype_amd.ops`` -- hand-written gfx950 HIP kernels: GPU registry hash table,
  route/dispatch/complete of 32-B message records, persistent dispatcher.
* ``ptype_amd.parallel`` -- RCCL (torch.distributed "nccl") exchange epochs
  between the GPUs of a node, one process per GPU.
* ``ptype_amd.runtime`` -- the per-process device runtime tying them together.
* ``ptype_amd.models`` -- the reference workloads (calculator, optimus).
"""
from __future__ import annotations

__version__ = "0.1.0"

# The public API needs the native control plane (``_core``).  It is imported
# lazily so that ``python -m ptype_amd._build`` (and the driver's build())
# works on a fresh checkout where no extension has been compiled yet.
_API = (
    "Client",
    "Cluster",
    "Config",
    "ConfigFromFile",
    "ConnConfig",
    "Context",
    "DefaultConnConfig",
    "ErrNoClientAvailable",
    "ErrNoKey",
    "GetPrefixRangeEnd",
    "GoStruct",
    "GoUint",
    "Join",
    "KVStore",
    "New",
    "Node",
    "Registry",
    "Serve",
    "Server",
    "SortAscend",
    "SortByCreateRevision",
    "SortByKey",
    "SortByModRevision",
    "SortByValue",
    "SortByVersion",
    "SortDescend",
    "SortNone",
    "WithCountOnly",
    "WithFromKey",
    "WithKeysOnly",
    "WithLease",
    "WithLimit",
    "WithPrefix",
    "WithRange",
    "WithRev",
    "WithSerializable",
    "WithSort",
)

__all__ = list(_API)


def __getattr__(name):
    if name in _API:
        from . import cluster

        return getattr(cluster, name)
    raise AttributeError(f"module 'ptype_amd' has no attribute {name!r}")
