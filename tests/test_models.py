"""The reference examples end to end on the host path (CPU): calculator
(example/calculator: server + client processes sharing a cluster) and optimus
(example/optimus: coordinator fan-out over prime workers, HTTP /test)."""
import threading
import urllib.request

import pytest

from ptype_amd import cluster as C
from ptype_amd.models import calculator, optimus


def member(name, ports, d, initial=None, state="new"):
    pp, pc = ports(), ports()
    m = C.member_config(name=name, dir=str(d / name), lpurls=[f"http://127.0.0.1:{pp}"],
                        apurls=[f"http://127.0.0.1:{pp}"], lcurls=[f"http://127.0.0.1:{pc}"],
                        acurls=[f"http://127.0.0.1:{pc}"], heartbeat_ms=20, election_ms=200,
                        cluster_state=state, unsafe_no_fsync=True)
    return m


def cfg_for(service, node, port, m):
    c = C.Config()
    c.service_name, c.node_name, c.port = service, node, port
    c.member = m
    return c


@pytest.fixture(autouse=True)
def _loopback(monkeypatch):
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")


def _join_static(cfgs):
    """Both processes of example/calculator/run start together (static 2-member cluster)."""
    out = [None] * len(cfgs)

    def go(i):
        out[i] = C.Join(C.background(), cfgs[i])

    ths = [threading.Thread(target=go, args=(i,)) for i in range(len(cfgs))]
    [t.start() for t in ths]
    [t.join(30) for t in ths]
    assert all(out), "join failed"
    return out


def test_calculator_example(tmp_path, ports):
    ms = [member("calculator_etcd_1", ports, tmp_path), member("calculator_etcd_2", ports, tmp_path)]
    ic = ",".join(f"{m.name}={m.apurls[0]}" for m in ms)
    for m in ms:
        m.initial_cluster = ic
    server_port = ports()
    srv_cfg = cfg_for("calculator", "calculator_node_1", server_port, ms[0])
    cli_cfg = cfg_for("calculator_client", "calculator_client_node_1", ports(), ms[1])
    # server: rpc.Register(calculator) + ListenAndServe(":port"); client: Join + NewClient
    server = C.Serve(server_port, calculator.Calculator())
    srv, cli = _join_static([srv_cfg, cli_cfg])
    try:
        services = cli.Registry.Services(C.background())
        assert set(services) >= {"calculator", "calculator_client"}
        client = cli.NewClient("calculator", None)
        try:
            assert client.Call("Calculator.Multiply", calculator.Args(7, 8)) == 56
        finally:
            client.Close()
    finally:
        cli.Close()
        srv.Close()
        server.Close()


def test_optimus_split_and_gather():
    assert optimus.split_work(25) == [(2, 10), (10, 20), (20, 30)]
    assert optimus.split_work(10) == [(2, 10)]
    assert optimus.split_work(3) == [(2, 10)]
    assert optimus.watch_replies(97, [97, 97]) == 97
    assert optimus.watch_replies(91, [91, 7, 13]) == 7
    p = optimus.Prime(delay=0)
    assert p.Check(optimus.Args(2, 10, 91)) == 7
    assert p.Check(optimus.Args(10, 20, 91)) == 13
    assert p.Check(optimus.Args(2, 10, 97)) == 97
    assert p.Check(optimus.Args(0, 3, 5)) == 1  # i == 0 is skipped; 1 divides everything (as prime.go)


def test_optimus_fan_out_over_workers(tmp_path, ports):
    """Two prime workers + a coordinator in one static 3-member cluster;
    per-candidate delay 0 (the reference's 250 ms is a parameter)."""
    names = ["worker_etcd_1", "worker_etcd_2", "coordinator_etcd_1"]
    ms = [member(n, ports, tmp_path) for n in names]
    ic = ",".join(f"{m.name}={m.apurls[0]}" for m in ms)
    for m in ms:
        m.initial_cluster = ic
    wports = [ports(), ports()]
    servers = [C.Serve(p, optimus.Prime(delay=0.0)) for p in wports]
    cfgs = [cfg_for("prime_worker", f"prime_worker_{i + 1}", wports[i], ms[i]) for i in range(2)]
    cfgs.append(cfg_for("coordinator", "coordinator_1", ports(), ms[2]))
    clusters = _join_static(cfgs)
    coord = None
    try:
        conn = C.ConnConfig(max_connections=0, initial_node_timeout=5.0, debounce_time=0.5, retries=0)
        worker = clusters[2].NewClient("prime_worker", conn)
        assert len(worker.selected_nodes()) == 2  # mesh over both replicas
        assert optimus.check_host(worker, 97) == 97
        assert optimus.check_host(worker, 91) == 7
        assert optimus.check_host(worker, 221) == 13
        coord = optimus.Coordinator(lambda t: optimus.check_host(worker, t), port=0)
        req = urllib.request.Request(f"http://127.0.0.1:{coord.port}/test", data=b"target=221", method="POST")
        assert urllib.request.urlopen(req, timeout=10).read() == b"13"
        with pytest.raises(urllib.error.HTTPError):
            urllib.request.urlopen(f"http://127.0.0.1:{coord.port}/test", timeout=10)
        counts = servers[0].call_counts().get("Prime.Check", 0) + servers[1].call_counts().get("Prime.Check", 0)
        assert counts >= 2
        worker.Close()
    finally:
        if coord:
            coord.close()
        for c in reversed(clusters):
            c.Close()
        for s in servers:
            s.Close()


def test_optimus_fanout_gather_reference():
    """FanOut: every target's splitWork ranges in one batch; the gather returns the
    first non-target reply in range order (the smallest divisor) or the target."""
    import torch

    from ptype_amd.models.optimus import FanOut
    from ptype_amd.ops import batch as B
    from ptype_amd.ops.records import METHOD_PRIME_CHECK

    f = FanOut(torch.tensor([221, 97, 100, 1009 * 1013, 2]), 64, "cpu")
    b = f.batch
    assert f.M == sum((t + 9) // 10 for t in (221, 97, 100, 1009 * 1013, 2))
    val, st = B._handler_ref(torch.full((f.M,), METHOD_PRIME_CHECK), b.actor.long(), b.a0, b.a1, b.a2, None)
    ans, status = f.gather(val, st.to(torch.int32))
    assert ans.tolist() == [13, 97, 2, 1009, 2] and status.tolist() == [0] * 5
