"""The ptype ``cluster`` API for Python, backed by the C++ control plane.

Names follow the reference package (``cluster.Join``, ``ConfigFromFile``,
``Cluster.Registry`` / ``Store`` / ``MemberList`` / ``NewClient`` / ``Close``,
``Client.Call`` / ``Go`` / ``Close`` / ``ConnectionErrs``, ``Registry.Register`` /
``Services`` / ``WatchService``, ``KVStore.Get`` / ``Put`` / ``Delete``, the
``With*`` option helpers, ``ErrNoKey``, ``ErrNoClientAvailable``,
``DefaultConnConfig``), plus the north-star entry points ``New`` (= ``Join``),
``Client.Send`` (batched device-native submit) and ``Serve`` (server-side
registration, which the reference leaves to stdlib net/rpc).

Reference: cluster/cluster.go, cluster/config.go, cluster/registry.go,
cluster/store.go, cluster/store_config.go, cluster/rpc.go.
"""
from __future__ import annotations

import inspect
from typing import Any, Callable, Iterable

from . import _core
from ._core import (  # noqa: F401  (re-exported API surface)
    CallChannel,
    ConfigError,
    ConnConfig,
    Context,
    ErrChannel,
    IntChannel,
    KvClient,
    LearnerNotReadyError,
    MemberConfig,
    MemberError,
    NoClientAvailableError,
    NoKeyError,
    Node,
    NodesChannel,
    PtypeError,
    RpcError,
    RpcServer,
    ShutdownError,
    TimeoutError,
    UnavailableError,
)
from .gobtypes import GoSlice, GoStruct, GoUint  # noqa: F401

# ---------------------------------------------------------------- sentinels
ErrNoKey = NoKeyError                       # cluster/store.go:15
ErrNoClientAvailable = NoClientAvailableError  # cluster/rpc.go:16
ErrLearnerNotReady = LearnerNotReadyError

# ---------------------------------------------------------------- options (store_config.go)
SortByKey, SortByVersion, SortByCreateRevision, SortByModRevision, SortByValue = range(5)
SortNone, SortAscend, SortDescend = range(3)

WithPrefix = _core.with_prefix
WithLimit = _core.with_limit
WithRev = _core.with_rev
WithRange = _core.with_range
WithFromKey = _core.with_from_key
WithSerializable = _core.with_serializable
WithKeysOnly = _core.with_keys_only
WithCountOnly = _core.with_count_only
WithLease = _core.with_lease


def WithSort(target: int, order: int):
    return _core.with_sort(int(target), int(order))


def GetPrefixRangeEnd(prefix: str | bytes) -> str | bytes:
    """Range end of a prefix on its bytes (store_config.go:41-58); returns str
    when the result is valid UTF-8, else bytes ("\\x00" when no end exists)."""
    b = bytearray(prefix.encode() if isinstance(prefix, str) else prefix)
    for i in range(len(b) - 1, -1, -1):
        if b[i] < 0xFF:
            b[i] += 1
            out = bytes(b[: i + 1])
            break
    else:
        out = b"\x00"
    if isinstance(prefix, str):
        try:
            return out.decode()
        except UnicodeDecodeError:
            return out
    return out


def DefaultConnConfig() -> ConnConfig:
    """{MaxConnections 3, InitialNodeTimeout 5 s, DebounceTime 3 s, Retries 2} (rpc.go:33-38)."""
    return _core.default_conn_config()


def background() -> Context:
    return Context.background()


def _ctx(ctx) -> Context:
    return ctx if ctx is not None else Context.background()


# ---------------------------------------------------------------- config
Config = _core.Config


def ConfigFromFile(path: str) -> Config:
    """Load the ptype YAML and its member (etcd) YAML (cluster/config.go:23-46)."""
    return _core.config_from_file(path)


config_from_file = ConfigFromFile


# ---------------------------------------------------------------- registry
class Registry:
    """Service registry over the Raft-replicated store (cluster/registry.go)."""

    def __init__(self, core):
        self._r = core

    def Register(self, ctx, serviceName: str, nodeName: str, host: str, port: int) -> None:
        self._r.register(_ctx(ctx), serviceName, nodeName, host, int(port))

    def Services(self, ctx=None) -> dict:
        return self._r.services(_ctx(ctx))

    def WatchService(self, ctx, serviceName: str) -> NodesChannel:
        return self._r.watch_service(_ctx(ctx), serviceName)

    def nodes(self, ctx, serviceName: str):
        return self._r.nodes(_ctx(ctx), serviceName)

    register = Register
    services = Services
    watch_service = WatchService

    @property
    def kv(self):
        return self._r.kv

    def close(self):
        self._r.close()


def new_etcd_registry(endpoints: list[str]) -> Registry:
    return Registry(_core.EtcdRegistry(list(endpoints)))


class KVStore:
    """Shared KV store under the ``store/`` prefix (cluster/store.go)."""

    def __init__(self, core):
        self._s = core

    def Get(self, ctx, key: str, *opts) -> list[str]:
        return self._s.get(_ctx(ctx), key, *opts)

    def Put(self, ctx, key: str, value: str, *opts) -> None:
        self._s.put(_ctx(ctx), key, value, *opts)

    def Delete(self, ctx, key: str, *opts) -> None:
        self._s.delete(_ctx(ctx), key, *opts)

    get, put, delete = Get, Put, Delete

    def close(self):
        self._s.close()


def new_kv_store(endpoints: list[str]) -> KVStore:
    return KVStore(_core.KVStore(list(endpoints)))


# ---------------------------------------------------------------- client
class Client:
    """RPC client with the reference's balancer semantics (cluster/rpc.go).

    ``Call`` returns the reply (Go writes it through a pointer); ``Go`` returns
    a call handle whose ``done`` channel later delivers it; ``Send`` is the
    batched device-native path (see ``ptype_amd.runtime``).
    """

    def __init__(self, core: _core.RpcClient, runtime=None, service: str = "", local_addr: str = "",
                 max_connections: int = 3):
        self._c = core
        self._rt = runtime
        self.service = service
        self._local_addr, self._max_connections = local_addr, int(max_connections)
        self._router = None  # replica routing of Send (parallel/replicas.py), when the service is replicated
        self._router_checked = False

    def _replica_router(self):
        if not self._router_checked:
            self._router_checked = True
            if self._rt.has_replicas(self.service):
                self._router = self._rt.replica_router(self.service, self._max_connections, self._local_addr)
        return self._router

    def Call(self, serviceMethod: str, args: Any) -> Any:
        return self._c.call(serviceMethod, args)

    def Go(self, serviceMethod: str, args: Any, done: CallChannel | None = None):
        return self._c.go(serviceMethod, args, done)

    def Send(self, batch, **kw):
        """Batched submit of a ``MsgBatch`` to GPU actors of this service:
        RCCL epoch exchange across ranks, device dispatch, replies in order.

        Asynchronous like ``Go`` (cluster/rpc.go:69-105): it returns device tensors
        ``(value, status)`` as soon as the Send is enqueued, with no host wait on
        it.  With more than one rank, a message that overflowed its region (skewed
        traffic beyond the agreed capacity) reads STATUS_OVERFLOW until its re-send
        -- at most two Sends later, or at ``Flush()`` -- writes its reply into the
        same tensors; keep ``batch`` unchanged until then."""
        if self._rt is None:
            raise RuntimeError("Client.Send needs the cluster's device runtime (Join with a gpu: section)")
        return self._rt.send(self.service, batch, router=self._replica_router(), **kw)

    def Flush(self) -> None:
        """Every earlier ``Send``'s replies final (pending re-sends run now)."""
        if self._rt is not None:
            self._rt.flush()

    def Tell(self, batch, **kw):
        """Batched fire-and-forget to GPU actors of this service; handlers may send
        on to other actors (device outbox), which is pumped until quiescent."""
        if self._rt is None:
            raise RuntimeError("Client.Tell needs the cluster's device runtime (Join with a gpu: section)")
        return self._rt.tell(batch, **kw)

    def Close(self) -> None:
        if self._router is not None:
            self._router.close()
        self._c.close()

    def ConnectionErrs(self) -> ErrChannel:
        return self._c.connection_errs()

    call, go, send, tell, close, flush = Call, Go, Send, Tell, Close, Flush

    @property
    def conns_updated(self) -> IntChannel:
        return self._c.conns_updated

    def selected_nodes(self):
        return self._c.selected_nodes()

    @property
    def cfg(self) -> ConnConfig:
        return self._c.cfg


def new_client(host: str, serviceName: str, nodes: NodesChannel, cfg: ConnConfig | None = None) -> Client:
    """newClient(host, serviceName, registry, cfg) taking the WatchService channel."""
    return Client(_core.RpcClient(host, serviceName, nodes, cfg if cfg is not None else DefaultConnConfig()),
                  service=serviceName)


# ---------------------------------------------------------------- server side
def _exported_methods(receiver) -> list[tuple[str, Callable]]:
    out = []
    for name, fn in inspect.getmembers(receiver, predicate=callable):
        if name[:1].isupper() and not name.startswith("_"):
            out.append((name, fn))
    return out


class Server:
    """net/rpc-compatible server (HTTP CONNECT + gob) for host and GPU actors.

    ``Register(receiver)`` mirrors ``rpc.Register``: every exported (capitalised)
    method of the receiver becomes ``"<TypeName>.<Method>"``; a method takes the
    decoded args and returns the reply, raising to return an RPC error.
    ``RegisterDevice`` binds a method to a compiled-in GPU handler through the
    persistent dispatcher.
    """

    def __init__(self):
        self._s = RpcServer()

    def Register(self, receiver, name: str | None = None) -> None:
        tname = name or type(receiver).__name__
        methods = _exported_methods(receiver)
        if not methods:
            raise ValueError(f"rpc.Register: type {tname} has no exported methods of suitable type")
        for mname, fn in methods:
            self._s.register_method(f"{tname}.{mname}", fn)

    def RegisterFunc(self, service_method: str, fn: Callable) -> None:
        self._s.register_method(service_method, fn)

    def RegisterDevice(self, service_method: str, device_server, method_id: int, fields: Iterable[str] = (),
                       actor: int = 0, actor_field: str = "") -> None:
        fn, ctx = device_server.submit_handle()
        self._s.register_device_method(service_method, fn, ctx, int(method_id), int(actor), list(fields), actor_field)
        if getattr(device_server, "shm_name", ""):  # same-node processes call it through shared memory
            device_server.export_method(service_method, int(method_id), int(actor), list(fields), actor_field)
            self._s.set_shm_segment(device_server.shm_name)

    def RegisterDeviceBatch(self, service_method: str, batch_handle, fields: Iterable[str] = (), actor_field: str = "",
                            max_batch: int = 1 << 16) -> None:
        """Serve ``service_method`` (registered for single calls first) in
        batches: the pipelined requests a connection has buffered are decoded
        together -- on the GPU with ``batch_handle = DeviceRuntime.gob_bridge(...).handle()``
        (K4, csrc/hip/gob_bridge.hpp), or on the host with ``_core.host_batch_multiply()``."""
        fn, ctx = batch_handle
        self._s.register_device_batch(service_method, fn, ctx, list(fields), actor_field, int(max_batch))

    @property
    def batches(self) -> int:
        return self._s.batches

    @property
    def batched_calls(self) -> int:
        return self._s.batched_calls

    def Listen(self, port: int = 0, host: str = "0.0.0.0", local: bool = True) -> int:
        return self._s.listen(host, int(port), local)

    def Close(self) -> None:
        self._s.close()

    def Dispatch(self, service_method: str, args: Any) -> Any:
        return self._s.dispatch(service_method, args)

    @property
    def port(self) -> int:
        return self._s.port

    def call_counts(self) -> dict:
        return self._s.call_counts()

    def debug_page(self) -> str:
        return self._s.debug_page()

    def ServeDebug(self, stats: Callable[[], dict], path: str = "/debug/ptype") -> None:
        """``GET <path>`` on this server's port answers ``json.dumps(stats())``
        (next to net/rpc's ``/debug/rpc``); e.g. ``server.ServeDebug(cluster.Stats)``."""
        import json

        self._s.set_debug_handler(path, lambda: json.dumps(stats(), default=str))

    register, register_func, register_device, listen, close = Register, RegisterFunc, RegisterDevice, Listen, Close
    serve_debug = ServeDebug


def Serve(port: int, *receivers, host: str = "0.0.0.0") -> Server:
    """rpc.Register(each receiver) + rpc.HandleHTTP + ListenAndServe(":port")
    (example/calculator/server/server.go:16-20, :38), non-blocking."""
    s = Server()
    for r in receivers:
        s.Register(r)
    s.Listen(port, host)
    return s


# ---------------------------------------------------------------- cluster
class Cluster:
    """Handle returned by ``Join`` (cluster/cluster.go:20-26)."""

    def __init__(self, core: _core.Cluster, cfg: Config, runtime=None):
        self._c = core
        self.cfg = cfg
        self.Registry = Registry(core.registry)
        self.Store = KVStore(core.store)
        self.runtime = runtime
        self._clients: list[Client] = []

    def MemberList(self, ctx=None):
        return self._c.member_list(_ctx(ctx))

    def NewClient(self, serviceName: str, cfg: ConnConfig | None = None) -> Client:
        mc = cfg.max_connections if cfg is not None else _core.default_conn_config().max_connections
        c = Client(self._c.new_client(serviceName, cfg), self.runtime, serviceName, self.local_addr, mc)
        self._clients.append(c)
        return c

    def Stats(self) -> dict:
        """Observability snapshot: control-plane member status, the
        clients' call/attempt counters and selected nodes, and -- with a GPU
        runtime -- dispatcher, registry-mirror and exchange counters plus the
        single-call round-trip histogram.  Served as JSON by ``Server.ServeDebug``."""
        st = self._c.member_status()
        out = {
            "service": self.cfg.service_name, "node": self.cfg.node_name, "local_addr": self.local_addr,
            "member": {"id": st.id, "leader": st.leader, "term": st.term, "commit": st.commit,
                       "applied": st.applied, "revision": st.revision, "is_learner": st.is_learner},
            "clients": [{"service": c.service, "calls": c._c.calls, "attempts": c._c.attempts,
                         "nodes": [f"{n.address}:{n.port}" for n in c.selected_nodes()]} for c in self._clients],
        }
        if self.runtime is not None:
            out["runtime"] = self.runtime.stats()
        return out

    def Close(self) -> None:
        if self.runtime is not None:
            self.runtime.close()
        self._c.close()

    @property
    def local_addr(self) -> str:
        return self._c.local_addr

    @property
    def member_id(self) -> int:
        return self._c.member_id

    def status(self):
        return self._c.member_status()

    registry = property(lambda self: self.Registry)
    store = property(lambda self: self.Store)
    member_list, new_client, close, stats = MemberList, NewClient, Close, Stats

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.Close()


def Join(ctx, cfg: Config, runtime: bool | None = None) -> Cluster:
    """Join the cluster: start the local control-plane member (as a learner via
    ``initial_cluster_client_urls`` when ``initial-cluster-state: existing``,
    promoted once caught up), then register ``services/<service>/<node>/`` with
    a 2 s lease.  With a ``gpu:`` section (or ``runtime=True``) the process also
    brings up its GPU actor runtime (persistent dispatcher, registry mirror)."""
    core = _core.Cluster.join(_ctx(ctx), cfg)
    rt = None
    want = cfg.has_gpu if runtime is None else runtime
    if want:
        from .runtime import DeviceRuntime

        try:
            if cfg.gpu.tune:  # the config's path switches (ops/tune.py, csrc/hip/tune.hpp)
                from .ops import tune

                tune.set(cfg.gpu.tune)
            rt = DeviceRuntime.for_cluster(core, cfg)
        except Exception:
            core.close()
            raise
    return Cluster(core, cfg, rt)


def New(cfg: Config, ctx=None, runtime: bool | None = None) -> Cluster:
    """North-star entry point: ``cluster.New(cfg)`` == ``Join(ctx, cfg)``."""
    return Join(ctx, cfg, runtime)


join = Join
new = New


def member_config(**kw) -> MemberConfig:
    """Programmatic member config (the reference's tests set the unexported
    etcdConfig fields directly, cluster/cluster_test.go:73-87)."""
    m = MemberConfig()
    for k, v in kw.items():
        if not hasattr(m, k):
            raise AttributeError(f"MemberConfig has no field {k}")
        setattr(m, k, v)
    return m
