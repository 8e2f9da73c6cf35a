"""Observability: Cluster.Stats over /debug/ptype, roctx
ranges, the dispatcher's device timestamp ring and round-trip histogram."""
import json
import urllib.request

import pytest
import torch

from ptype_amd import cluster as C
from ptype_amd.models import calculator
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, STATUS_OK
from ptype_amd.utils import trace


@pytest.fixture
def one_member(tmp_path, ports, monkeypatch):
    monkeypatch.setenv("PTYPE_ADVERTISE_ADDR", "127.0.0.1")
    pp, pc = ports(), ports()
    cfg = C.Config()
    cfg.service_name, cfg.node_name, cfg.port = "calculator", "n1", ports()
    cfg.member = C.member_config(name="m0", dir=str(tmp_path / "m0"), lpurls=[f"http://127.0.0.1:{pp}"],
                                 apurls=[f"http://127.0.0.1:{pp}"], lcurls=[f"http://127.0.0.1:{pc}"],
                                 acurls=[f"http://127.0.0.1:{pc}"], initial_cluster=f"m0=http://127.0.0.1:{pp}",
                                 heartbeat_ms=20, election_ms=200, unsafe_no_fsync=True)
    return cfg


def test_cluster_stats_on_debug_endpoint(one_member):
    cfg = one_member
    server = C.Server()
    server.Register(calculator.Calculator())
    server.Listen(cfg.port, "127.0.0.1")
    c = C.Join(C.background(), cfg)
    try:
        server.ServeDebug(c.Stats)
        client = c.NewClient("calculator", C.ConnConfig(allow_local=False))
        for i in range(5):
            assert client.Call("Calculator.Multiply", calculator.Args(i, 3)) == 3 * i
        body = urllib.request.urlopen(f"http://127.0.0.1:{cfg.port}/debug/ptype", timeout=10).read()
        st = json.loads(body)
        assert st["service"] == "calculator" and st["member"]["leader"] == st["member"]["id"] != 0
        assert st["member"]["revision"] >= 1 and st["member"]["applied"] >= st["member"]["commit"] > 0
        assert st["clients"][0]["calls"] == 5 and st["clients"][0]["nodes"] == [f"127.0.0.1:{cfg.port}"]
        assert b"Calculator.Multiply" in urllib.request.urlopen(f"http://127.0.0.1:{cfg.port}/debug/rpc",
                                                                 timeout=10).read()
        # a failing provider answers 500, the server keeps serving
        server.ServeDebug(lambda: 1 / 0, path="/debug/bad")
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(f"http://127.0.0.1:{cfg.port}/debug/bad", timeout=10)
        assert e.value.code == 500
        assert client.Call("Calculator.Multiply", calculator.Args(2, 2)) == 4
        client.Close()
    finally:
        c.Close()
        server.Close()


def test_trace_helpers():
    with trace.range("ptype.test"):  # no profiler attached: a cheap no-op
        trace.mark("ptype.mark")
    h = [0] * 40
    h[11] = 90  # 2-4 us
    h[14] = 10  # 16-32 us
    assert trace.hist_percentile(h, 50) == 4096.0 and trace.hist_percentile(h, 99) == 32768.0
    assert trace.hist_percentile([0] * 40, 50) is None
    assert trace.percentiles([1, 2, 3])["p50"] == 2.0


@pytest.mark.gpu
def test_dispatcher_timestamp_ring():
    from ptype_amd.ops import hip

    state = torch.zeros(16, dtype=torch.int64, device="cuda")
    srv = hip().DeviceServer(0, 1024, state.data_ptr(), 16, 0, 200.0, 30.0)
    try:
        with trace.DispatcherTrace(srv, capacity=1024) as t:
            for i in range(300):
                v, s, _ = srv.call(METHOD_CALC_MULTIPLY, i % 16, i, 2)
                assert (v, s) == (2 * i, STATUS_OK)
            b = t.breakdown()
        assert b["n"] == 300
        assert b["clock_err_us"] < 50
        # picked up within a poll interval (absolute placement is good to the handshake
        # window); a multiply is far below a microsecond of device service time
        err = b["clock_err_us"] + 1.0
        assert -err < b["queue_us"]["p50"] < 100 + err and 0 <= b["service_us"]["p50"] < 20
        assert sum(srv.rtt_histogram()) == 300 and b["rtt_us_p50_bucket"] < 200
    finally:
        srv.close()
