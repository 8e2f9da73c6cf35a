"""Request-ring liveness (csrc/core/ringproto.hpp): takeovers and rescues are
decided by whether a caller's PROCESS is alive, never by how long it took.

A CPU dispatcher (_core.HostDispatcher) serves the same shared-memory protocol
the GPU dispatcher does; client processes call it through _core.ShmClient.  A
victim process freezes itself (SIGSTOP, test hook PTYPE_RING_TEST_STOP) at one
point of a call -- after taking its sequence number, after claiming its slot,
or after its reply landed but before reading it -- while other processes keep
calling through a small ring (slots are reused many times over).

* SIGSTOP for 2 s, then SIGCONT: every call of every process -- the victim's
  included -- returns its correct reply (a stopped caller is
  alive, so nothing is taken over or rescued behind its back).
* SIGKILL while stopped: the others still finish every call (the dead caller's
  number is rescued, its slot taken over).

Reference behaviour this protects: a net/rpc client call either returns its
reply or an error (cluster/rpc.go:59-67); nothing answers it with another
call's reply.
"""
import os
import signal
import subprocess
import sys
import time
import uuid

import pytest

from ptype_amd import _core

CALLER = r"""
import os, sys
from ptype_amd import _core
name, n, timeout, tag = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
c = _core.ShmClient(name)
bad = []
for i in range(n):
    a = tag * 100000 + i
    try:
        v, s = c.call(1, 0, a, 3, 0, timeout)   # Calculator.Multiply(a, 3)
        if (v, s) != (3 * a, 0):
            bad.append((i, v, s))
    except Exception as e:
        bad.append((i, repr(e)))
print("BAD", len(bad), bad[:3], flush=True)
sys.exit(1 if bad else 0)
"""

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _spawn(name, n, tag, timeout=30.0, stop=None):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.pop("PTYPE_RING_TEST_STOP", None)
    if stop:
        env["PTYPE_RING_TEST_STOP"] = stop
    return subprocess.Popen([sys.executable, "-c", CALLER, name, str(n), str(timeout), str(tag)], env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def _state(pid):
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0]
    except OSError:
        return "gone"


def _wait_stopped(p, timeout=60.0):
    t_end = time.monotonic() + timeout
    while time.monotonic() < t_end:
        if p.poll() is not None:
            raise AssertionError("victim exited before stopping: " + p.stdout.read())
        if _state(p.pid) == "T":
            return
        time.sleep(0.01)
    raise AssertionError("victim never stopped itself")


@pytest.mark.parametrize("point", ["took", "claimed", "landed"])
def test_sigstopped_caller_completes_and_nobody_fails(point):
    d = _core.HostDispatcher(f"/ptype-live-{uuid.uuid4().hex[:12]}", 16)
    victim = _spawn(d.name, 40, 9, stop=point)
    _wait_stopped(victim)
    others = [_spawn(d.name, 300, t) for t in range(3)]
    time.sleep(2.0)  # the others pile up behind the frozen caller (their timeouts are longer)
    os.kill(victim.pid, signal.SIGCONT)
    outs = [p.communicate(timeout=120)[0] for p in [victim] + others]
    assert [p.returncode for p in [victim] + others] == [0, 0, 0, 0], outs
    assert d.processed >= 940 and d.noops == 0  # nothing was rescued: every caller stayed alive


@pytest.mark.parametrize("point", ["took", "claimed", "landed"])
def test_killed_caller_cannot_wedge_the_ring(point):
    d = _core.HostDispatcher(f"/ptype-live-{uuid.uuid4().hex[:12]}", 16)
    victim = _spawn(d.name, 40, 9, stop=point)
    _wait_stopped(victim)
    others = [_spawn(d.name, 200, t) for t in range(3)]
    time.sleep(0.5)
    victim.kill()  # SIGKILL while stopped
    victim.wait()
    outs = [p.communicate(timeout=120)[0] for p in others]
    assert [p.returncode for p in others] == [0, 0, 0], outs
    if point != "landed":  # its number was taken but never published: a rescuer published a no-op
        assert d.noops >= 1
