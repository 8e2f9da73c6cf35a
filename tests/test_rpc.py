"""RPC client + connection balancer parity (reference cluster/rpc_test.go).

The reference uses a mock registry with a scriptable node channel
(rpc_test.go:16-40), real net/rpc servers on 127.0.0.1:0 (:478-490), an echo
receiver (RPCTest) and a fault injector that fails until `callsBeforePass`
(RPCRetryTest, :55-77).  Same here, over our Go-wire-compatible net/rpc server
(HTTP CONNECT + gob over TCP); `allow_local=False` keeps every call on TCP.
The documented retry fix: at most 1 + Retries attempts (rpc.go:107-116 loops
forever when Retries > 0); all reference expectations use Retries = 0.
"""
import threading
import time

import pytest

from ptype_amd import _core
from ptype_amd import cluster as C


class RPCTest:
    def Call(self, x):
        return "who's " + x

    def Go(self, x):
        time.sleep(1)
        return "who's " + x


class RPCRetryTest:
    def __init__(self, calls_before_pass):
        self.called = 0
        self.calls_before_pass = calls_before_pass
        self.lock = threading.Lock()

    def _hit(self):
        with self.lock:
            self.called += 1
            c = self.called
        if c >= self.calls_before_pass:
            return c
        raise RuntimeError("failed")

    def Call(self, arg):
        return self._hit()

    def Go(self, arg):
        time.sleep(1)
        return self._hit()


def serve(*receivers):
    s = C.Server()
    for r in receivers:
        s.Register(r)
    port = s.Listen(0, "127.0.0.1", local=False)
    return C.Node("127.0.0.1", port), s


def mock_registry(initial):
    """newMockRegistry: an unbuffered channel, the initial list sent from a goroutine."""
    ch = C.NodesChannel(0)
    threading.Thread(target=lambda: ch.send(initial), daemon=True).start()
    return ch


def conn_cfg():
    return C.ConnConfig(max_connections=3, initial_node_timeout=1.0, debounce_time=1.0, retries=0, allow_local=False)


@pytest.fixture
def servers():
    made = []

    def make(*receivers):
        n, s = serve(*receivers)
        made.append(s)
        return n

    yield make
    for s in made:
        s.Close()


def test_client_default_conn_config():
    c = C.new_client("", "foo", mock_registry([]), None)
    try:
        assert c.cfg == C.DefaultConnConfig()
        d = C.DefaultConnConfig()
        assert (d.max_connections, d.initial_node_timeout, d.debounce_time, d.retries) == (3, 5.0, 3.0, 2)
    finally:
        c.Close()


def test_client_call(servers):
    node = servers(RPCTest())
    c = C.new_client("", "foo", mock_registry([node]), conn_cfg())
    try:
        assert c.Call("RPCTest.Call", "joe") == "who's joe"
    finally:
        c.Close()


def test_client_call_with_retry_multi_node(servers):
    n1 = servers(RPCRetryTest(2))
    n2 = servers(RPCRetryTest(0))
    c = C.new_client("", "foo", mock_registry([n1, n2]), conn_cfg())
    try:
        # round robin starts at index 1: node2 (passes at once) is hit first
        assert c.Call("RPCRetryTest.Call", "") == 1
    finally:
        c.Close()


def test_client_call_with_retry_error(servers):
    n1 = servers(RPCRetryTest(10))
    c = C.new_client("", "foo", mock_registry([n1]), conn_cfg())
    try:
        with pytest.raises(C.RpcError, match="failed"):
            c.Call("RPCRetryTest.Call", "")
    finally:
        c.Close()


def test_client_call_bounded_retries(servers):
    """Fixed semantics: Retries=2 means at most 3 attempts, re-selected round robin."""
    r = RPCRetryTest(10)
    n1 = servers(r)
    cfg = conn_cfg()
    cfg.retries = 2
    c = C.new_client("", "foo", mock_registry([n1]), cfg)
    try:
        with pytest.raises(C.RpcError):
            c.Call("RPCRetryTest.Call", "")
        assert r.called == 3
        r2 = RPCRetryTest(3)
        n2 = servers(r2)
    finally:
        c.Close()
    c = C.new_client("", "foo", mock_registry([n2]), cfg)
    try:
        assert c.Call("RPCRetryTest.Call", "") == 3  # fails twice, third attempt passes
    finally:
        c.Close()


def test_client_go(servers):
    node = servers(RPCTest())
    c = C.new_client("", "foo", mock_registry([node]), conn_cfg())
    try:
        call = c.Go("RPCTest.Go", "joe")
        assert call is not None and call.error is None
        done = call.done.recv(5.0)
        assert done.reply == "who's joe"
    finally:
        c.Close()


def test_client_go_with_retry_multi_node(servers):
    n1 = servers(RPCRetryTest(2))
    n2 = servers(RPCRetryTest(0))
    c = C.new_client("", "foo", mock_registry([n1, n2]), conn_cfg())
    try:
        call = c.Go("RPCRetryTest.Go", "")
        assert call.error is None
        resp = call.done.recv(5.0)
        assert resp.error is None and resp.reply == 1
    finally:
        c.Close()


def test_client_go_with_retry_error(servers):
    n1 = servers(RPCRetryTest(10))
    c = C.new_client("", "foo", mock_registry([n1]), conn_cfg())
    try:
        call = c.Go("RPCRetryTest.Go", "")
        assert call.error is None
        resp = call.done.recv(5.0)
        assert resp.error is not None and "failed" in resp.error  # the final error is delivered
        assert resp.reply is None or resp.reply == 0
    finally:
        c.Close()


def test_client_no_client_available():
    c = C.new_client("", "foo", mock_registry([]), conn_cfg())
    try:
        with pytest.raises(C.ErrNoClientAvailable):
            c.Call("RPCTest.Call", "joe")
    finally:
        c.Close()


def test_new_connection_balancer_successful_initial_connect(servers):
    node = servers()  # an empty server still accepts connections
    b = _core.ConnectionBalancer("", "foo", mock_registry([node]), conn_cfg())
    try:
        assert b.selected_nodes() == [node]
        assert len(b.errs) == 0
    finally:
        b.close()


def test_new_connection_balancer_with_no_available_server():
    ch = C.NodesChannel(0)  # nothing is ever sent
    t0 = time.time()
    with pytest.raises(C.PtypeError, match="no initial nodes provided for foo"):
        _core.ConnectionBalancer("", "foo", ch, conn_cfg())
    assert 0.9 < time.time() - t0 < 3.0


def test_new_connection_balancer_with_servers_failing_to_connect():
    from conftest import free_port

    dead = free_port()  # closed port
    with pytest.raises(C.UnavailableError, match="failed to dial service address"):
        _core.ConnectionBalancer("", "foo", mock_registry([C.Node("127.0.0.1", dead)]), conn_cfg())


def test_connection_balancer_watch_for_new_nodes(servers):
    node = servers()
    ch = mock_registry([node])
    b = _core.ConnectionBalancer("", "foo", ch, conn_cfg())
    try:
        assert b.selected_nodes() == [node]
        node2, node3, node4 = servers(), servers(), servers()

        # more than MaxConnections nodes: FNV picks indices 3, 0, 1 for localAddr ""
        threading.Thread(target=lambda: ch.send([node, node2, node3, node4]), daemon=True).start()
        assert b.conns_updated.recv(5.0) is not None
        assert b.selected_nodes() == [node4, node, node2]

        # a connected node is removed
        threading.Thread(target=lambda: ch.send([node, node3, node4]), daemon=True).start()
        assert b.conns_updated.recv(5.0) is not None
        assert b.selected_nodes() == [node, node3, node4]

        # debounce: four rapid lists, only the last applies
        def burst():
            ch.send([node])
            ch.send([node2])
            ch.send([node3])
            ch.send([node, node2, node3])

        threading.Thread(target=burst, daemon=True).start()
        assert b.conns_updated.recv(5.0) is not None
        assert b.selected_nodes() == [node, node2, node3]
        assert len(b.errs) == 0
    finally:
        b.close()


def test_connection_balancer_ignores_empty_lists(servers):
    node = servers()
    ch = mock_registry([node])
    b = _core.ConnectionBalancer("", "foo", ch, conn_cfg())
    try:
        threading.Thread(target=lambda: ch.send([]), daemon=True).start()
        assert b.conns_updated.recv(1.6) is None  # an empty list keeps the old clients
        assert b.selected_nodes() == [node] and b.client_count() == 1
    finally:
        b.close()


def test_connection_balancer_round_robin_select(servers):
    nodes = [servers() for _ in range(5)]
    cfg = conn_cfg()
    cfg.max_connections = 0
    b = _core.ConnectionBalancer("", "foo", mock_registry(nodes), cfg)
    try:
        targets = [f"127.0.0.1:{n.port}" for n in nodes]
        got = [b.get_target() for _ in range(len(nodes))]
        assert got == targets[1:] + targets[:1]  # first pick is index 1
        assert b.get_target() == targets[1]      # wraps (overflow)
        # concurrency: N concurrent picks hit every client exactly once
        seen = []
        lock = threading.Lock()

        def pick():
            t = b.get_target()
            with lock:
                seen.append(t)

        ths = [threading.Thread(target=pick) for _ in range(len(nodes))]
        [t.start() for t in ths]
        [t.join() for t in ths]
        assert sorted(seen) == sorted(targets)
    finally:
        b.close()


def test_connection_balancer_mesh_network(servers):
    node, node2 = servers(), servers()
    ch = mock_registry([node, node2])
    cfg = conn_cfg()
    cfg.max_connections = 0
    b = _core.ConnectionBalancer("", "foo", ch, cfg)
    try:
        assert b.selected_nodes() == [node, node2]
        node3, node4 = servers(), servers()
        threading.Thread(target=lambda: ch.send([node, node2, node3]), daemon=True).start()
        assert b.conns_updated.recv(5.0) is not None
        assert b.selected_nodes() == [node, node2, node3]
        threading.Thread(target=lambda: ch.send([node, node2, node3, node4]), daemon=True).start()
        assert b.conns_updated.recv(5.0) is not None
        assert b.selected_nodes() == [node, node2, node3, node4]  # all nodes are connected to
    finally:
        b.close()


def test_select_nodes_golden():
    ns = [C.Node(f"h{i}", i) for i in range(4)]
    assert _core.ConnectionBalancer.select_nodes("", ns, 3) == [ns[3], ns[0], ns[1]]
    assert _core.ConnectionBalancer.select_nodes("", ns, 0) == ns
    assert _core.ConnectionBalancer.select_nodes("", ns, 4) == ns
    assert [_core.ConnectionBalancer.hash_index("", i, 4) for i in range(3)] == [3, 0, 1]
    # duplicates allowed when the hash collides
    sel = _core.ConnectionBalancer.select_nodes("10.0.0.7", ns[:2], 1)
    assert len(sel) == 1


def test_server_errors_and_debug_page(servers):
    node = servers(RPCTest())
    conn = _core.dial_http("127.0.0.1", node.port)
    try:
        with pytest.raises(C.RpcError, match="rpc: can't find method RPCTest.Nope"):
            conn.call("RPCTest.Nope", "x")
        with pytest.raises(C.RpcError, match="rpc: can't find service Missing.Call"):
            conn.call("Missing.Call", "x")
        with pytest.raises(C.RpcError, match="ill-formed"):
            conn.call("NoDot", "x")
        assert conn.call("RPCTest.Call", "bob") == "who's bob"  # the stream survives errors
    finally:
        conn.close()
    import socket

    s = socket.create_connection(("127.0.0.1", node.port))
    s.sendall(b"GET /debug/rpc HTTP/1.0\r\n\r\n")
    page = s.recv(65536).decode()
    s.close()
    assert "RPCTest.Call" in page and "200 OK" in page
    s = socket.create_connection(("127.0.0.1", node.port))
    s.sendall(b"POST /_goRPC_ HTTP/1.0\r\n\r\n")
    assert "405" in s.recv(4096).decode()
    s.close()


def test_local_fast_path_same_semantics():
    s = C.Server()
    s.Register(RPCTest())
    port = s.Listen(0, "127.0.0.1", local=True)
    try:
        cfg = conn_cfg()
        cfg.allow_local = True
        c = C.new_client("", "foo", mock_registry([C.Node("127.0.0.1", port)]), cfg)
        try:
            assert c.Call("RPCTest.Call", "amy") == "who's amy"
            with pytest.raises(C.RpcError, match="can't find method"):
                c.Call("RPCTest.Missing", "")
        finally:
            c.Close()
    finally:
        s.Close()


def test_concurrent_calls_pipelined(servers):
    node = servers(RPCTest())
    c = C.new_client("", "foo", mock_registry([node]), conn_cfg())
    try:
        calls = [c.Go("RPCTest.Call", f"n{i}") for i in range(200)]
        got = sorted(call.done.recv(10.0).reply for call in calls)
        assert got == sorted(f"who's n{i}" for i in range(200))
    finally:
        c.Close()


def test_rebalance_keeps_in_flight_calls(servers):
    """a re-balance must not cut calls in flight.  Connections of nodes
    that stay selected are kept; a deselected node's connection closes only after
    its pending call returned -- so a non-idempotent handler runs exactly once."""
    slow = RPCRetryTest(0)
    n1, n2 = servers(slow), servers(RPCTest())
    ch = mock_registry([n1])
    cfg = C.ConnConfig(max_connections=0, initial_node_timeout=1.0, debounce_time=0.2, retries=2, allow_local=False)
    c = C.new_client("", "foo", ch, cfg)
    try:
        call = c.Go("RPCRetryTest.Go", "")  # sleeps 1 s on n1
        time.sleep(0.1)
        ch.send([n1, n2])  # n1 stays selected
        assert c.conns_updated.recv(3.0) is not None
        time.sleep(0.1)
        ch.send([n2])  # n1 deselected while its call is still running
        assert c.conns_updated.recv(3.0) is not None
        assert c._c.retired_conns == 1
        done = call.done.recv(5.0)
        assert done.error is None and done.reply == 1  # completed on the retired connection
        assert slow.called == 1  # ran once: no retry after a cut connection
        deadline = time.time() + 3
        while c._c.retired_conns and time.time() < deadline:
            time.sleep(0.05)
        assert c._c.retired_conns == 0  # closed once idle
        assert c.Call("RPCTest.Call", "x") == "who's x"
    finally:
        c.Close()
