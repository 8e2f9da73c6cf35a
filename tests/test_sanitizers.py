"""Host control plane under ThreadSanitizer and AddressSanitizer+UBSan.

The reference runs every test with Go's race detector (`go test -race`,
Makefile:2).  Here the C++ control plane (channels, Raft members,
MVCC/leases/watch, KV client, net/rpc server + balancer client, Cluster facade)
is linked into a native stress program (tests/native/core_stress.cpp) built with
each sanitizer -- the sanitizer runtime has to own the process, which a Python
extension module cannot give it -- and run concurrently-loaded scenarios:
3-member Raft with concurrent writers, a prefix watch, lease keepalive and a
leader failover; concurrent Call/Go with retries and a live re-balance; Join ->
register -> NewClient -> Call -> Close; a learner join + promotion; the same-node shared-memory call path;
the Send watchdog retiring the data plane's communicator while engine threads enqueue.  Any sanitizer report fails the test.
"""
import os
import subprocess

import pytest

from ptype_amd import _build

REPORTS = ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:")


@pytest.mark.parametrize("sanitizer", ["thread", "address"])
def test_core_under_sanitizer(sanitizer, tmp_path):
    exe = _build.build_native_test(sanitizer)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0", ASAN_OPTIONS="detect_leaks=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path)], env=env, capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    found = [x for x in REPORTS if x in out]
    assert not found, f"{sanitizer} sanitizer reports {found}:\n{out[-6000:]}"
    assert r.returncode == 0, out[-4000:]
    for s in ("channel", "raft", "rpc", "api", "learner", "shm", "commcell"):
        assert f"OK {s}" in r.stdout
