"""K4 on the serving path, on the GPU: a gob client's 10 K
pipelined Calculator.Multiply calls over one TCP connection are decoded by
``gob_decode_kernel`` straight into mailbox columns and served through the HBM
mailboxes (``DeviceRuntime.serve(..., batch=True)``); every reply equals the
host path's, and the bridge saw fewer batches than calls."""
import pytest
import torch

from ptype_amd import _core
from ptype_amd import cluster as C
from ptype_amd.models.calculator import Args
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY
from ptype_amd.runtime import DeviceRuntime


@pytest.mark.gpu
def test_gpu_gob_bridge_serves_pipelined_calls():
    rt = DeviceRuntime(torch.device("cuda", 0), actors=1024, service="Calculator", shm=False)
    srv = C.Server()
    rt.serve(srv, "Calculator", {"Multiply": (METHOD_CALC_MULTIPLY, ["A", "B"])}, batch=True)
    port = srv.Listen(0, host="127.0.0.1", local=False)
    try:
        n = 10_000
        args = [Args(A=(i * 7919) % 200_003 - 100_000, B=(i % 113) - 50) for i in range(n)]
        want = [a.A * a.B for a in args]
        conn = _core.dial_http("127.0.0.1", port, allow_local=False)
        got = conn.call_many("Calculator.Multiply", args)
        assert got == want
        bridge = rt._bridges[0][1]
        assert bridge.calls == n and 0 < bridge.batches < n, (bridge.batches, bridge.calls)
        assert srv.batched_calls == n
        # the single-call device path (persistent dispatcher) agrees
        assert conn.call("Calculator.Multiply", Args(A=-12345, B=678)) == -12345 * 678
        print("gob bridge:", {"calls": bridge.calls, "batches": bridge.batches})
    finally:
        srv.Close()
        rt.close()
