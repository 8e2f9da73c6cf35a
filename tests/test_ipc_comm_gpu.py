"""The native N > 1 engines across real PROCESSES on one GPU.

RCCL refuses two ranks on one device, so a one-GPU box could only run the
multi-rank pipelines as in-process FakeComm ranks.  IpcComm
(csrc/hip/ipc_comm.hpp) moves their collectives through shared-memory segments
that every rank maps and registers with HIP, stream-ordered on the device:
each rank here is its own Python process (torch.distributed gloo group for the
host side), exactly the one-process-per-rank shape of a node -- only the
transport differs from RCCL over xGMI.

Numerics: calculator replies compared exactly with A * B; ordered SeqFold
traffic audited exactly-once with per-(sender, actor) FIFO (ops.mailbox.audit_fold)
across every process's replies; a killed rank is detected within the comm's
timeout and surfaces as a peer failure the elastic path recovers from."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, free_port

pytestmark = pytest.mark.gpu
WORKER = os.path.join(ROOT, "tests", "_ipc_worker.py")


def _launch(scenario, R, timeout=300, expect_dead=()):
    port = free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, WORKER, scenario, str(r), str(R), str(port)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(R)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, (so, se)) in enumerate(zip(procs, outs)):
        if r in expect_dead:
            assert p.returncode == -9, (r, p.returncode, se[-2000:])
        else:
            assert p.returncode == 0, (r, p.returncode, so[-1000:], se[-3000:])
    line = [x for x in outs[0][0].splitlines() if x.startswith("RESULT ")]
    assert line, outs[0]
    return json.loads(line[0][7:])


@pytest.mark.parametrize("R", [2, 4])
def test_ipc_comm_collectives_exact(R):
    out = _launch("raw", R)
    assert out["ops"] == 24


@pytest.mark.parametrize("R", [2, 4])
def test_sorted_exchange_across_processes_calculator_exact(R):
    out = _launch("sorted_calc", R)
    assert out["mailbox"]["S"] <= 2 and out["auto"]["S"] <= 2
    assert sum(out["zipf_resend_rounds"][3:]) == 0


@pytest.mark.parametrize("R", [2, 3])
def test_sorted_exchange_across_processes_seqfold_exactly_once_fifo(R):
    out = _launch("sorted_fold", R)
    assert out["messages"] == R * 3 * 50_000 and out["actors"] > 0


@pytest.mark.parametrize("R", [2, 3])
def test_ordered_sends_keep_fifo_across_deferred_resends(R):
    out = _launch("sorted_fold_defer", R)
    print("fold_defer", out)
    assert out["messages"] == R * 7 * 60_000 and out["actors"] > 0
    # re-send rounds ran (skewed start-up capacity, the wide Send), more than one in total
    assert sum(sum(r) for r in out["rounds"]) > 1, out


def test_deferred_resend_has_no_host_wait_on_the_current_send():
    out = _launch("sorted_defer", 2)
    print("defer", out)
    assert out["resend_rounds"] >= 1  # the skewed start-up Sends overflowed and were re-sent late
    # steady state: every overflow read before flush() was of a Send two Sends old (K - 2 of them)
    assert out["steady_resend_rounds"] == 0 and out["steady_overflow_waits"] == out["deferred_sends"] - 2, out
    # host time of the native Send with IpcComm: ~2 kernels per collective op, 5 ops per Send
    assert out["host_us_per_native_send"] < 1000.0, out


def test_epoch_engine_across_processes_exact_size_exchange():
    out = _launch("epoch_direct", 2)
    assert out["exact"] and out["S"] > 0


def test_killed_rank_is_a_peer_failure_within_the_timeout():
    out = _launch("kill", 3, expect_dead=(2,))
    assert "IpcComm: peer" in out["raised"] and out["waited_s"] < 30
