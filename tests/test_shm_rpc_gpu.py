"""Same-node cross-process calls to GPU actors through shared-memory rings.

A server process hosts calculator actors on the GPU (DeviceRuntime: the
dispatcher's rings live in a POSIX shared-memory segment) and serves net/rpc on
a port; a separate client process -- no GPU, no HIP -- dials that port and gets
a connection that publishes device calls straight into the ring the GPU polls.
The server's net/rpc method counter stays at zero for them (no socket, no gob),
non-device methods still go over TCP, and the round trip is a fraction of TCP's.

By default the request ring is the server GPU's device memory: the client maps
its dma-buf (fd handed over a unix socket, no HIP in the client) and writes
requests through the BAR, so the polling wave never reads host memory (VERDICT
r1 X3).  PTYPE_XPROC_RING=host on the server keeps the ring in the segment.
"""
import os
import time

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _server(port, q, stop, placement):
    if placement == "host":
        os.environ["PTYPE_XPROC_RING"] = "host"
    import torch

    from ptype_amd import cluster as C
    from ptype_amd.models import calculator
    from ptype_amd.runtime import DeviceRuntime

    rt = DeviceRuntime(torch.device("cuda", 0), actors=64, idle_ms=50.0)
    server = C.Server()
    calculator.serve_device(rt, server)
    server.RegisterFunc("Host.Echo", lambda a: a)
    server.Listen(port, "127.0.0.1")
    q.put(("ready", rt.server.shm_name))
    stop.wait(120)
    q.put(("counts", (server.call_counts(), rt.server.ring_fds_handed, rt.server.ring_on_device)))
    server.Close()
    rt.close()


def _client(port, q):
    os.environ["HIP_VISIBLE_DEVICES"] = ""  # the client process never touches a GPU
    from ptype_amd import _core
    from ptype_amd.models.calculator import Args

    conn = _core.dial_http("127.0.0.1", port, 5.0, True)
    tcp = _core.dial_http("127.0.0.1", port, 5.0, False)
    out = {"transport": conn.transport, "tcp_transport": tcp.transport, "ring": conn.ring_placement,
           "mul": conn.call("Calculator.Multiply", Args(7, 8)), "echo": conn.call("Host.Echo", 5)}
    for name, c in (("shm", conn), ("tcp", tcp)):
        for i in range(200):
            c.call("Calculator.Multiply", Args(i, 2))
        lat = []
        for i in range(2000):
            t = time.perf_counter()
            c.call("Calculator.Multiply", Args(i, 3))
            lat.append(time.perf_counter() - t)
        lat.sort()
        out[name + "_p50_us"] = lat[len(lat) // 2] * 1e6
    conn.close()
    tcp.close()
    q.put(("client", out))


@pytest.mark.parametrize("placement", ["device", "host"])
def test_cross_process_call_through_shared_memory(placement):
    from conftest import free_port

    ctx = mp.get_context("spawn")
    q, stop = ctx.Queue(), ctx.Event()
    port = free_port()
    sp = ctx.Process(target=_server, args=(port, q, stop, placement))
    sp.start()
    kind, seg = q.get(timeout=180)
    assert kind == "ready" and seg
    cp = ctx.Process(target=_client, args=(port, q))
    cp.start()
    kind, out = q.get(timeout=180)
    cp.join(30)
    stop.set()
    _, (counts, handed, on_device) = q.get(timeout=60)
    sp.join(60)
    assert out["transport"] == "shm" and out["tcp_transport"] == "tcp"
    assert out["ring"] == placement and bool(on_device) == (placement == "device")
    assert handed == (1 if placement == "device" else 0)
    assert out["mul"] == 56 and out["echo"] == 5
    # device calls over shm never reached the net/rpc server; the TCP ones (200 + 2000) did
    assert counts.get("Calculator.Multiply", 0) == 2200 and counts.get("Host.Echo") == 1
    assert out["shm_p50_us"] < out["tcp_p50_us"], out
    print("cross-process p50 RTT (us), %s ring: shm %.2f vs tcp %.1f" % (placement, out["shm_p50_us"], out["tcp_p50_us"]))
