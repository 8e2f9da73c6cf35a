"""The integrated runtime on a real MI355X: control plane + GPU actors.

* net/rpc (HTTP CONNECT + gob over TCP) -> device handler through the
  persistent dispatcher: the reference's calculator call, served by a GPU actor;
* Client.Send of a large batch through route/dispatch/complete;
* registry mirror built from the replicated store;
* optimus fan-out as one device batch;
* snapshot of actor state + registry mirror to pinned host DRAM and back.
"""
import pytest
import torch

from ptype_amd import cluster as C
from ptype_amd.models import calculator, optimus
from ptype_amd.ops import batch as B
from ptype_amd.ops.records import METHOD_RETRY_TEST, STATUS_FAILED, STATUS_OK

pytestmark = pytest.mark.gpu


@pytest.fixture
def gpu_cluster(tmp_path, ports, monkeypatch):
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    pp, pc = ports(), ports()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "calculator", "gpu0", ports()
    cfg.member = C.member_config(name="m0", dir=str(tmp_path / "m0"), lpurls=[f"http://127.0.0.1:{pp}"],
                                 apurls=[f"http://127.0.0.1:{pp}"], lcurls=[f"http://127.0.0.1:{pc}"],
                                 acurls=[f"http://127.0.0.1:{pc}"], initial_cluster=f"m0=http://127.0.0.1:{pp}",
                                 heartbeat_ms=50, election_ms=500, unsafe_no_fsync=True)
    cfg.has_gpu = True
    cfg.gpu.device = 0
    cfg.gpu.actors = 4096
    cfg.gpu.max_batch = 1 << 20
    c = C.Join(C.background(), cfg)
    yield c, cfg
    c.Close()


def test_netrpc_call_served_by_gpu_actor(gpu_cluster):
    c, cfg = gpu_cluster
    rt = c.runtime
    assert rt is not None and rt.table.live == cfg.gpu.actors  # mirror synced from the store
    server = C.Server()
    calculator.serve_device(rt, server)
    server.RegisterDevice("Retry.Call", rt.server, METHOD_RETRY_TEST, ["Passes"], actor=5)
    server.Listen(cfg.port, "127.0.0.1", local=False)
    try:
        client = c.NewClient("calculator", C.ConnConfig(retries=0, allow_local=False))
        assert client.Call("Calculator.Multiply", calculator.Args(7, 8)) == 56
        assert client.Call("Calculator.Multiply", calculator.Args(-3, 1 << 40)) == -3 << 40
        with pytest.raises(C.RpcError, match="failed"):
            client.Call("Retry.Call", C.GoStruct("Args", Passes=3))  # actor 5 counts 1 -> fails
        client.Close()
        # the same call over the node-local path: the server listens with local=False,
        # so this reaches the GPU actor through the shared-memory rings (no socket, no
        # net/rpc dispatch -- the server's counter does not move)
        fast = c.NewClient("calculator", C.ConnConfig(retries=0))
        assert fast.Call("Calculator.Multiply", calculator.Args(6, 7)) == 42
        fast.Close()
        assert server.call_counts()["Calculator.Multiply"] == 2
    finally:
        server.Close()


def test_client_send_large_batch(gpu_cluster):
    c, cfg = gpu_cluster
    server = C.Server()  # NewClient dials the registered node, as the reference does
    calculator.serve_device(c.runtime, server)
    server.Listen(cfg.port, "127.0.0.1")
    try:
        client = c.NewClient("calculator", None)
        M = 1 << 20
        req = B.gen_requests(M, c.runtime.total_actors, seed=7, device="cuda")
        val, st = client.Send(req)
        torch.cuda.synchronize()
        assert bool((st == STATUS_OK).all()) and torch.equal(val, req.a0 * req.a1)
        client.Close()
    finally:
        server.Close()


def test_optimus_on_device(gpu_cluster):
    c, _ = gpu_cluster
    assert optimus.check_device(c.runtime, 221) == 13
    assert optimus.check_device(c.runtime, 97) == 97
    assert optimus.check_device(c.runtime, 1000003) == 1000003  # prime: 100k ranges in one batch


def test_runtime_latency_call_and_stateful_actor(gpu_cluster):
    rt = gpu_cluster[0].runtime
    assert rt.call(calculator.DEVICE_METHODS["Multiply"][0], 0, 9, 9) == (81, STATUS_OK)
    statuses = [rt.call(METHOD_RETRY_TEST, 11, 3)[1] for _ in range(3)]
    assert statuses == [STATUS_FAILED, STATUS_FAILED, STATUS_OK]


def test_snapshot_roundtrip(gpu_cluster, tmp_path):
    rt = gpu_cluster[0].runtime
    rt.state.copy_(torch.arange(rt.actors, device=rt.device) * 3)
    info = rt.save(str(tmp_path / "snap.safetensors"))
    assert info["bytes"] > rt.actors * 8
    rt.state.zero_()
    rt.table.clear()
    rt.restore(str(tmp_path / "snap.safetensors"))
    assert torch.equal(rt.state.cpu(), torch.arange(rt.actors) * 3)
    assert rt.table.live == rt.actors
    r, _ = rt.table.lookup(torch.arange(1, 100, device=rt.device))
    assert bool((r == 0).all())


def test_client_tell_token_ring(gpu_cluster):
    """Client.Tell: GPU actors pass tokens on through the device outbox."""
    from ptype_amd.ops.records import METHOD_FORWARD

    c, cfg = gpu_cluster
    rt = c.runtime
    server = C.Server()
    server.Listen(cfg.port, "127.0.0.1")
    try:
        client = c.NewClient("calculator", None)
        n, T, H = rt.total_actors, 1000, 5
        starts = torch.arange(T, dtype=torch.int64) * 3 % n
        batch = B.MsgBatch(starts.to(torch.int32).cuda(), ((starts + 1) % n).cuda(),
                           torch.full((T,), H, dtype=torch.int64, device="cuda"),
                           torch.full((T,), 1 | (n << 32), dtype=torch.int64, device="cuda"), METHOD_FORWARD)
        rt.state.zero_()
        epochs, delivered = client.Tell(batch)
        torch.cuda.synchronize()
        assert epochs == H and delivered == T * (H + 1) and int(rt.state.sum()) == T * (H + 1)
        client.Close()
    finally:
        server.Close()
