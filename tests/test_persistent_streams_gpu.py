"""Persistent kernels must not block other streams' work.

HIP maps ordinary streams round-robin onto a small pool of hardware queues
(GPU_MAX_HW_QUEUES = 4 on the box).  A persistent kernel (the dispatcher wave,
the mailbox consumer) launched on a pooled stream sits in an in-order queue, and
work that a later stream puts on the same queue waits behind it -- until the
dispatcher's idle exit, or the consumer's lifetime bound (a live mailbox session
whose producer lands there stalls outright).  Observed: the live-enqueue mailbox
test finishing with nothing processed.  The persistent kernels now run on
low-priority queues of their own (common.hpp dedicated_stream); here every one of 12
fresh streams gets a kernel through while each persistent kernel is resident
(tools/pstream_probe.py, profiles/r2_persistent_stream_probe.jsonl: on a pooled
stream one of 12 streams waited 2975 ms -- the wave's 3 s idle exit).
"""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _each_stream_completes(n_streams=12):
    # (stream syncs only: a device-wide synchronize waits for the resident wave too)
    x = torch.zeros(1024, device=DEV)
    torch.cuda.current_stream().synchronize()
    worst = 0.0
    for k in range(n_streams):
        s = torch.cuda.Stream(DEV)
        t = time.perf_counter()
        with torch.cuda.stream(s):
            x.add_(1)
            v = float(x[0].item())  # read back on s: waits for this stream's add only
        worst = max(worst, time.perf_counter() - t)
        assert v == k + 1
    return worst


def test_dispatcher_wave_does_not_block_other_streams():
    from ptype_amd.ops import hip
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY

    state = torch.zeros(64, dtype=torch.int64, device=DEV)
    # idle exit after 8 s: a stream queued behind the wave would wait that long
    srv = hip().DeviceServer(0, 256, state.data_ptr(), state.numel(), 0, 8000.0, 30.0, "")
    try:
        assert srv.call(METHOD_CALC_MULTIPLY, 1, 6, 7)[0] == 42  # the wave is resident now
        assert srv.running
        worst = _each_stream_completes()
        assert srv.running  # still resident: the streams did not wait for its exit
        assert worst < 1.5, worst
    finally:
        srv.close()


def test_mailbox_consumer_does_not_block_other_streams():
    from ptype_amd.ops.mailbox import Mailboxes

    mb = Mailboxes(torch.device(DEV), shards=64, slots=1024)
    state = torch.zeros(64, dtype=torch.int64, device=DEV)
    out_v = torch.zeros(16, dtype=torch.int64, device=DEV)
    out_s = torch.zeros(16, dtype=torch.int32, device=DEV)
    mb.start(state, out_v, out_s, blocks=2, max_s=8.0)
    try:
        time.sleep(0.05)
        assert mb.running
        worst = _each_stream_completes()
        assert mb.running
        assert worst < 1.5, worst
    finally:
        mb.stop()
