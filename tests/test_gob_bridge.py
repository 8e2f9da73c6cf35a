"""K4 on the net/rpc serving path: batched gob requests.

A Go-protocol client pipelines 10 K ``Calculator.Multiply`` calls on one TCP
connection; the server keeps each request header on the host, captures the
argument value messages raw and answers a connection's buffered requests as one
batch -- decoded on the GPU into mailbox columns (``gob_bridge``), or here on the
host by its CPU twin.  Replies equal the single-call host path's, and the
server counts fewer batches than calls (the pipelining was used)."""
import pytest

from ptype_amd import _core
from ptype_amd import cluster as C
from ptype_amd.models.calculator import Args


class Calculator:
    def Multiply(self, args):
        return args["A"] * args["B"] if isinstance(args, dict) else args.A * args.B


def _serve(batch_handle=None):
    srv = C.Server()
    srv.Register(Calculator())
    if batch_handle is not None:
        srv.RegisterDeviceBatch("Calculator.Multiply", batch_handle, ["A", "B"])
    port = srv.Listen(0, host="127.0.0.1", local=False)
    return srv, port


@pytest.mark.timeout(120)
def test_pipelined_gob_calls_are_served_in_batches():
    n = 10_000
    args = [Args(A=i - 5000, B=(i % 97) - 40) for i in range(n)]
    want = [a.A * a.B for a in args]
    ref_srv, ref_port = _serve()
    bat_srv, bat_port = _serve(_core.host_batch_multiply())
    try:
        ref = _core.dial_http("127.0.0.1", ref_port, allow_local=False).call_many("Calculator.Multiply", args)
        got = _core.dial_http("127.0.0.1", bat_port, allow_local=False).call_many("Calculator.Multiply", args)
        assert ref == want and got == want
        assert bat_srv.batched_calls == n and 0 < bat_srv.batches < n, (bat_srv.batches, bat_srv.batched_calls)
        assert bat_srv.call_counts()["Calculator.Multiply"] == n
        # a non-struct argument on the batched method falls back to the single-call path
        one = _core.dial_http("127.0.0.1", bat_port, allow_local=False)
        assert one.call("Calculator.Multiply", Args(A=6, B=7)) == 42
    finally:
        ref_srv.Close()
        bat_srv.Close()


def test_register_batch_needs_the_single_call_method():
    srv = C.Server()
    with pytest.raises(Exception, match="single calls first"):
        srv.RegisterDeviceBatch("Calculator.Multiply", _core.host_batch_multiply(), ["A", "B"])


@pytest.mark.timeout(60)
def test_uint_struct_fields_fall_back_to_the_single_call_path():
    """the batch path's decoders zigzag every field, which is
    right only for gob ``int`` (type 2).  A struct with a ``uint`` field (gob type
    3) is not captured for the batch path: the host single-call path answers it,
    with the right value."""
    from ptype_amd.gobtypes import GoStruct, GoUint

    srv, port = _serve(_core.host_batch_multiply())
    try:
        cli = _core.dial_http("127.0.0.1", port, allow_local=False)
        calls = [GoStruct("Args", [("A", 6 + i), ("B", GoUint(7 + i))]) for i in range(50)]
        got = cli.call_many("Calculator.Multiply", calls)
        assert got == [(6 + i) * (7 + i) for i in range(50)]
        assert srv.batched_calls == 0 and srv.call_counts()["Calculator.Multiply"] == 50
    finally:
        srv.Close()
