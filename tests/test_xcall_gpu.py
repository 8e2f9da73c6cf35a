"""GPU-initiated remote call between two processes on one GPU (SURVEY X3,
VERDICT r2 #7): the server process runs the persistent dispatcher with its
peer lanes in its shared-memory segment; the client process maps and registers
that segment and a KERNEL publishes each call into a lane and spins on the
lane's reply slot -- memory each process reaches through its own mapping, so a
killed peer faults nobody (the SIGKILL tests below).  Relays
(METHOD_RELAY) are asynchronous: the dispatcher parks them and keeps serving,
so two servers relaying to each other at once do not deadlock.
Replies are checked against the handlers' definitions; device-clock and host
round trip p50s are reported (and bounded loosely)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

from conftest import ROOT

_SERVER = textwrap.dedent("""
    import os, sys, time, torch
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import hip
    state = torch.zeros(1024, dtype=torch.int64, device="cuda")
    srv = hip().DeviceServer(0, 1024, state.data_ptr(), 1024, 0, 2000.0, 60.0, f"ptype-xcall-{os.getpid()}")
    print("SHM " + srv.shm_name + " " + str(int(srv.xlanes)), flush=True)
    sys.stdin.readline()  # until the client is done
    torch.cuda.synchronize()
    print("STATE " + str(int(state[7].item())) + " PROCESSED " + str(srv.processed), flush=True)
    srv.close()
""")

_CLIENT = textwrap.dedent("""
    import json, os, sys, torch
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops.peer import PeerCaller
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, STATUS_OK
    pc = PeerCaller(sys.argv[1], "cuda:0")
    n = 4000
    a = torch.arange(n, dtype=torch.int64) - 2000
    b = torch.arange(n, dtype=torch.int64) % 97 + 3
    val, st, rtt, done = pc.call(torch.arange(n) % 1024, a, b, method=METHOD_CALC_MULTIPLY)
    ok_mul = done == n and bool((st == STATUS_OK).all()) and torch.equal(val.cpu(), a * b)
    # stateful: 100 CounterAdd(+2) to actor 7, in order: values 2, 4, ..., 200
    v2, s2, _, d2 = pc.call(torch.full((100,), 7), torch.full((100,), 2), method=METHOD_COUNTER_ADD)
    ok_add = d2 == 100 and bool((s2 == STATUS_OK).all()) and v2.cpu().tolist() == list(range(2, 202, 2))
    r = rtt[200:].cpu().sort().values
    out = {"lane": pc.lane, "ok_mul": ok_mul, "ok_add": ok_add, "p50_us": float(r[len(r) // 2]) / 1e3,
           "p99_us": float(r[int(len(r) * 0.99)]) / 1e3}
    print("RESULT " + json.dumps(out), flush=True)
""")


@pytest.mark.gpu
def test_gpu_initiated_call_between_processes():
    env = dict(os.environ, PTYPE_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    srv = subprocess.Popen([sys.executable, "-c", _SERVER], env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    try:
        line = srv.stdout.readline().split()
        assert line and line[0] == "SHM", (line, srv.stderr.read()[-2000:] if srv.poll() is not None else "")
        assert line[2] == "1", "the server exported no GPU peer lanes"
        c = subprocess.run([sys.executable, "-c", _CLIENT, line[1]], env=env, capture_output=True, text=True,
                           timeout=180)
        assert c.returncode == 0, c.stderr[-3000:]
        res = [x for x in c.stdout.splitlines() if x.startswith("RESULT ")]
        assert res, c.stdout[-2000:] + c.stderr[-2000:]
        out = json.loads(res[0][7:])
        srv.stdin.write("done\n")
        srv.stdin.flush()
        tail = srv.stdout.readline().split()
        assert srv.wait(60) == 0
    finally:
        if srv.poll() is None:
            srv.kill()
    print("xcall", out, tail)
    assert out["ok_mul"] and out["ok_add"], out
    assert tail[0] == "STATE" and int(tail[1]) == 200, tail  # the server's actor state saw every add
    assert out["p50_us"] < 50.0, out  # a GPU->GPU round trip, no host: single-digit microseconds expected


_RELAYER = textwrap.dedent("""
    import json, os, sys, time, torch, numpy as np
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import hip
    from ptype_amd.ops.peer import PeerRelay
    from ptype_amd.ops.records import METHOD_RELAY, METHOD_CALC_MULTIPLY, METHOD_COUNTER_ADD, STATUS_OK
    state = torch.zeros(1024, dtype=torch.int64, device="cuda")
    srv = hip().DeviceServer(0, 1024, state.data_ptr(), 1024, 0, 2000.0, 60.0, f"ptype-relay-{os.getpid()}")
    relay = PeerRelay(srv, sys.argv[1], "cuda:0", n_lanes=8)
    # stateful through the relay: 100 CounterAdd(+2) on the REMOTE actor 7, in order
    adds, lat = [], []
    for _ in range(100):
        t = time.perf_counter()
        v, st, _ = srv.call(METHOD_RELAY, 7, METHOD_COUNTER_ADD, 2)
        lat.append(time.perf_counter() - t)
        adds.append((v, st))
    ok_add = [v for v, _ in adds] == list(range(2, 202, 2)) and all(st == STATUS_OK for _, st in adds)
    # a batch: 64 relayed Multiply calls served by one dispatcher pass (8 slots, 8 rounds)
    n = 256
    req = np.zeros((n, 4), dtype=np.int64)
    a = np.arange(n, dtype=np.int64) - 100
    b = np.arange(n, dtype=np.int64) % 13 + 2
    req[:, 0] = (np.arange(n) % 1024) | (METHOD_RELAY << 32) | (1 << 48)
    req[:, 1] = METHOD_CALC_MULTIPLY
    req[:, 2] = a
    req[:, 3] = b
    rep = np.zeros((n, 2), dtype=np.int64)
    t = time.perf_counter()
    srv.call_many(req.ctypes.data, rep.ctypes.data, n)
    batch_s = time.perf_counter() - t
    ok_mul = bool((rep[:, 0] == a * b).all()) and bool(((rep[:, 1] & 0xff) == STATUS_OK).all())
    # a local (non-relayed) call on the same dispatcher still runs its own handler
    v, st, _ = srv.call(METHOD_COUNTER_ADD, 7, 5)
    ok_local = v == 5 and st == STATUS_OK
    srv.close()
    del relay
    lat = sorted(lat[10:])
    print("RESULT " + json.dumps({"ok_add": ok_add, "ok_mul": ok_mul, "ok_local": ok_local,
                                  "p50_us": lat[len(lat) // 2] * 1e6, "batch_us": batch_s * 1e6}), flush=True)
""")


@pytest.mark.gpu
def test_handler_initiated_remote_call_relays_through_the_dispatcher():
    """A's dispatcher forwards METHOD_RELAY requests to B's actors over GPU peer
    lanes: B's state sees every relayed add, replies are exact,
    and A's own handlers keep working alongside."""
    env = dict(os.environ, PTYPE_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    srv = subprocess.Popen([sys.executable, "-c", _SERVER], env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    try:
        line = srv.stdout.readline().split()
        assert line and line[0] == "SHM", (line, srv.stderr.read()[-2000:] if srv.poll() is not None else "")
        assert line[2] == "1", "the server exported no GPU peer lanes"
        c = subprocess.run([sys.executable, "-c", _RELAYER, line[1]], env=env, capture_output=True, text=True,
                           timeout=180)
        assert c.returncode == 0, c.stderr[-3000:]
        res = [x for x in c.stdout.splitlines() if x.startswith("RESULT ")]
        assert res, c.stdout[-2000:] + c.stderr[-2000:]
        out = json.loads(res[0][7:])
        srv.stdin.write("done\n")
        srv.stdin.flush()
        tail = srv.stdout.readline().split()
        assert srv.wait(60) == 0
    finally:
        if srv.poll() is None:
            srv.kill()
    print("relay", out, tail)
    assert out["ok_add"] and out["ok_mul"] and out["ok_local"], out
    assert tail[0] == "STATE" and int(tail[1]) == 200, tail  # B's actor 7 saw the relayed adds only


_COORD = textwrap.dedent("""
    import json, os, sys, time, torch, numpy as np
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import hip
    from ptype_amd.ops.peer import PeerRelay
    from ptype_amd.ops.records import METHOD_COORD_PRIME, STATUS_OK
    state = torch.zeros(1024, dtype=torch.int64, device="cuda")
    srv = hip().DeviceServer(0, 1024, state.data_ptr(), 1024, 0, 2000.0, 60.0, f"ptype-coord-{os.getpid()}")
    relay = PeerRelay(srv, sys.argv[1], "cuda:0", n_lanes=8)
    N, W, B, A = 3000, 16, 100, 5
    req = np.zeros((N, 4), dtype=np.int64)
    req[:, 0] = A | (METHOD_COORD_PRIME << 32) | (1 << 48)
    req[:, 1] = np.arange(N)
    req[:, 2] = W
    req[:, 3] = B
    rep = np.zeros((N, 2), dtype=np.int64)
    t = time.perf_counter()
    srv.call_many(req.ctypes.data, rep.ctypes.data, N)
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    v, st, _ = srv.call(METHOD_COORD_PRIME, A, 7919, W, B)  # one more prime, one call
    srv.close()
    del relay
    sieve = np.ones(N, dtype=bool); sieve[:2] = False
    for p in range(2, int(N ** 0.5) + 1):
        if sieve[p]:
            sieve[p * p::p] = False
    n_primes = int(sieve.sum())
    prime_replies = sorted(int(x) for x in rep[sieve, 0])
    print("RESULT " + json.dumps({"all_ok": bool(((rep[:, 1] & 0xff) == STATUS_OK).all()),
                                  "tally": int(state[A].item()), "n_primes": n_primes,
                                  "prime_replies_exact": prime_replies == list(range(1, n_primes + 1)),
                                  "last": [int(v), int(st)], "us_per_call": dt / N * 1e6}), flush=True)
""")


@pytest.mark.gpu
def test_actor_handler_decides_its_remote_call_and_continues_on_the_reply():
    """not a host-chosen forward -- the coordinator actor's
    handler picks the worker (hash of the candidate), builds the PrimeCheck, and
    its continuation tallies primes into its own state when the reply lands
    (optimus coordinator.go:75-89).  3000 candidates over 16 remote workers: the
    tally is the prime count, every prime's reply is a distinct tally value."""
    env = dict(os.environ, PTYPE_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    srv = subprocess.Popen([sys.executable, "-c", _SERVER], env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    try:
        line = srv.stdout.readline().split()
        assert line and line[0] == "SHM", (line, srv.stderr.read()[-2000:] if srv.poll() is not None else "")
        c = subprocess.run([sys.executable, "-c", _COORD, line[1]], env=env, capture_output=True, text=True,
                           timeout=180)
        assert c.returncode == 0, c.stderr[-3000:]
        res = [x for x in c.stdout.splitlines() if x.startswith("RESULT ")]
        assert res, c.stdout[-2000:] + c.stderr[-2000:]
        out = json.loads(res[0][7:])
        srv.stdin.write("done\n")
        srv.stdin.flush()
        tail = srv.stdout.readline().split()
        assert srv.wait(60) == 0
    finally:
        if srv.poll() is None:
            srv.kill()
    print("coord", out, tail)
    assert out["all_ok"] and out["tally"] == out["n_primes"] + 1 == 431, out  # pi(2999) = 430, + 7919
    assert out["prime_replies_exact"] and out["last"] == [431, 0], out


# ---------------------------------------------------------------- r5: duplex relays, SIGKILLs
def _spawn(src, *args, env=None):
    return subprocess.Popen([sys.executable, "-c", src, *args], env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)


def _expect(p, word, timeout=120):
    """Next stdout line of `p` starting with `word` (split), or a failure with its stderr."""
    import select

    deadline = __import__("time").time() + timeout
    while __import__("time").time() < deadline:
        r, _, _ = select.select([p.stdout], [], [], 1.0)
        if r:
            line = p.stdout.readline()
            if not line:
                break
            if line.startswith(word):
                return line.split()
    if p.poll() is None:  # still running: stop it to read what it said
        p.kill()
        p.wait(30)
    raise AssertionError(f"no {word!r} from the child (rc {p.returncode}): stdout tail "
                         + p.stdout.read()[-1500:] + " stderr " + p.stderr.read()[-3000:])


def _unlink_shm(name):
    try:
        os.unlink("/dev/shm/" + name.lstrip("/"))
    except OSError:
        pass


_DUPLEX = textwrap.dedent("""
    import json, os, sys, time, threading, torch, numpy as np
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import hip
    from ptype_amd.ops.peer import PeerRelay
    from ptype_amd.ops.records import METHOD_RELAY, METHOD_CALC_MULTIPLY, METHOD_ECHO, STATUS_OK
    state = torch.zeros(1024, dtype=torch.int64, device="cuda")
    srv = hip().DeviceServer(0, 4096, state.data_ptr(), 1024, 0, 2000.0, 120.0, f"ptype-duplex-{os.getpid()}")
    print("SHM " + srv.shm_name, flush=True)
    peer = sys.stdin.readline().strip()
    relay = PeerRelay(srv, peer, "cuda:0", n_lanes=16, timeout_s=5.0)

    def local_calls(k, out, stop=None):  # single calls to a LOCAL actor of this dispatcher
        i = 0
        while (stop is None and i < k) or (stop is not None and not stop.is_set()):
            t = time.perf_counter()
            v, st, _ = srv.call(METHOD_ECHO, 3, i)
            out.append(time.perf_counter() - t)
            assert v == i and st == STATUS_OK, (v, st)
            i += 1

    base = []
    local_calls(3000, base)
    print("READY", flush=True)
    sys.stdin.readline()  # GO: both processes have their relays
    n = 10000
    a = np.arange(n, dtype=np.int64) - 5000
    b = np.arange(n, dtype=np.int64) % 101 + 1
    req = np.zeros((n, 4), dtype=np.int64)
    req[:, 0] = (np.arange(n) % 1024) | (METHOD_RELAY << 32) | (1 << 48)
    req[:, 1] = METHOD_CALC_MULTIPLY
    req[:, 2] = a
    req[:, 3] = b
    rep = np.zeros((n, 2), dtype=np.int64)
    stop, during = threading.Event(), []
    th = threading.Thread(target=local_calls, args=(0, during, stop))
    th.start()
    t = time.perf_counter()
    srv.call_many(req.ctypes.data, rep.ctypes.data, n, 120.0)
    relay_s = time.perf_counter() - t
    # keep relays in flight (batches of 10 K, both ways) for at least half a second, so the
    # local callers' p50 is measured while the dispatcher has parked relays
    more, exact_more = 0, True
    rep2 = np.zeros((n, 2), dtype=np.int64)
    while time.perf_counter() - t < 0.5 or more < 3:
        srv.call_many(req.ctypes.data, rep2.ctypes.data, n, 120.0)
        exact_more = exact_more and bool((rep2[:, 0] == a * b).all()) and bool(((rep2[:, 1] & 0xff) == STATUS_OK).all())
        more += 1
    relay_total_s = time.perf_counter() - t
    stop.set()
    th.join()
    st = rep[:, 1] & 0xff
    base = sorted(base[200:])
    during = sorted(during[50:]) or [0.0]
    out = {"exact": bool((rep[:, 0] == a * b).all()) and bool((st == STATUS_OK).all()) and exact_more,
           "not_delivered": int((st == 5).sum()), "relay_s": relay_s, "relays_per_s": n * (1 + more) / relay_total_s,
           "relay_batches": 1 + more,
           "local_p50_us": base[len(base) // 2] * 1e6, "local_p50_during_us": during[len(during) // 2] * 1e6,
           "local_calls_during": len(during), "slots": [int(x) for x in relay.slots()]}
    print("RESULT " + json.dumps(out), flush=True)
    sys.stdin.readline()  # DONE: the peer finished too (its relays target this dispatcher)
    relay.detach()
    srv.close()
""")


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_duplex_relays_do_not_block_the_dispatchers():
    """A relays 10 K Multiply calls to B while B relays 10 K to A, at the same
    time: exact values, zero timeouts, and each dispatcher keeps
    answering its own local callers while its relays are parked."""
    env = dict(os.environ, PTYPE_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    ps = [_spawn(_DUPLEX, env=env) for _ in range(2)]
    names = []
    try:
        names = [_expect(p, "SHM")[1] for p in ps]
        for p, peer in zip(ps, reversed(names)):
            p.stdin.write(peer + "\n")
            p.stdin.flush()
        for p in ps:
            _expect(p, "READY")
        for p in ps:
            p.stdin.write("go\n")
            p.stdin.flush()
        outs = [json.loads(" ".join(_expect(p, "RESULT", 240)[1:])) for p in ps]
        for p in ps:
            p.stdin.write("done\n")
            p.stdin.flush()
        rcs = [p.wait(60) for p in ps]
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
        for nm in names:
            _unlink_shm(nm)
    print("duplex", outs)
    assert rcs == [0, 0], [p.stderr.read()[-2000:] for p in ps]
    for o in outs:
        assert o["exact"] and o["not_delivered"] == 0, o
        assert o["local_calls_during"] > 100, o  # the dispatcher served its own ring while relays were parked
        # other callers' p50 while relays are in flight: within a few microseconds of the quiet p50
        assert o["local_p50_during_us"] < max(3 * o["local_p50_us"], o["local_p50_us"] + 30.0), o


_SLOW_SERVER = textwrap.dedent("""
    import os, sys, threading, time, torch
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import hip
    from ptype_amd.ops.records import METHOD_PRIME_CHECK
    state = torch.zeros(1024, dtype=torch.int64, device="cuda")
    # Prime.Check spins 50 ms per candidate here (the reference's per-candidate sleep, scaled)
    srv = hip().DeviceServer(0, 1024, state.data_ptr(), 1024, 50000, 2000.0, 60.0, f"ptype-slow-{os.getpid()}")
    print("SHM " + srv.shm_name, flush=True)
    cmd = sys.stdin.readline().strip()
    if cmd == "busy":  # the wave is busy with a long call of this process's own (a relay to it must wait)
        threading.Thread(target=lambda: srv.call(METHOD_PRIME_CHECK, 1, 2, 200, 1000003, 60.0), daemon=True).start()
        time.sleep(0.3)
        print("BUSY", flush=True)
    for line in sys.stdin:
        if line.startswith("done"):
            break
    v, st, _ = srv.call(3, 5, 77)  # Echo: the dispatcher still answers after its peer died
    print("ALIVE " + str(v) + " " + str(st) + " " + str(srv.processed), flush=True)
    srv.close()
""")

_SLOW_CALLER = textwrap.dedent("""
    import json, os, signal, sys, threading, time, torch
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops.peer import PeerCaller
    from ptype_amd.ops.records import METHOD_CALC_MULTIPLY, METHOD_PRIME_CHECK, STATUS_OK
    pc = PeerCaller(sys.argv[1], "cuda:0")
    mode = sys.argv[2]
    if mode == "die":  # SIGKILL this caller while its kernel spins on a 2 s Prime.Check
        threading.Timer(0.5, lambda: os.kill(os.getpid(), signal.SIGKILL)).start()
        print("LANE " + str(pc.lane), flush=True)
        pc.call([1], [2], [40], [1000003], method=METHOD_PRIME_CHECK, timeout_s=30.0)
        print("UNREACHED", flush=True)
        sys.exit(3)
    if mode == "again":  # a new caller after a dead one: its lane works
        v, st, _, done = pc.call(torch.arange(64), torch.arange(64), torch.full((64,), 3), method=METHOD_CALC_MULTIPLY)
        ok = done == 64 and bool((st == STATUS_OK).all()) and torch.equal(v.cpu(), torch.arange(64) * 3)
        print("RESULT " + json.dumps({"ok": ok, "lane": pc.lane}), flush=True)
        sys.exit(0)
    # mode "server_dies": the server is SIGKILLed mid-call; this kernel times out without a fault
    print("CALLING", flush=True)
    t = time.time()
    v, st, _, done = pc.call([1], [2], [80], [1000003], method=METHOD_PRIME_CHECK, timeout_s=6.0)
    waited = time.time() - t
    x = (torch.arange(1 << 20, device="cuda") * 2).sum().item()  # the GPU is healthy for this process
    print("RESULT " + json.dumps({"status": int(st[0]), "done": int(done), "waited_s": waited,
                                  "gpu_ok": x == (1 << 20) * ((1 << 20) - 1)}), flush=True)
""")


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_peer_lane_survives_a_killed_server():
    """The server is SIGKILLed while a GPU caller's kernel waits on its reply slot:
    the caller's spin ends at its timeout with kStatusNotDelivered and the
    caller's GPU keeps working (the lane is the caller's own mapping of the
    segment, not the dead process's HBM)."""
    env = dict(os.environ, PTYPE_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    srv = _spawn(_SLOW_SERVER, env=env)
    name = None
    try:
        name = _expect(srv, "SHM")[1]
        cl = _spawn(_SLOW_CALLER, name, "server_dies", env=env)
        _expect(cl, "CALLING")
        __import__("time").sleep(1.0)
        srv.kill()
        srv.wait(30)
        out = json.loads(" ".join(_expect(cl, "RESULT", 60)[1:]))
        assert cl.wait(60) == 0, cl.stderr.read()[-2000:]
    finally:
        for p in (srv,):
            if p.poll() is None:
                p.kill()
        if name:
            _unlink_shm(name)
    print("server killed", out)
    assert out["status"] == 5 and out["done"] == 1 and out["gpu_ok"], out  # NotDelivered, no fault
    assert 4.0 < out["waited_s"] < 30.0, out


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_killed_caller_lane_is_reclaimed():
    """A caller process is SIGKILLed with a call in flight: the server finishes the
    call (its reply lands in the segment, nobody faults), reclaims the dead
    caller's lane once quiet, and a new caller registers and calls exactly."""
    env = dict(os.environ, PTYPE_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    srv = _spawn(_SLOW_SERVER, env=env)
    name = None
    try:
        name = _expect(srv, "SHM")[1]
        srv.stdin.write("plain\n")
        srv.stdin.flush()
        dead = _spawn(_SLOW_CALLER, name, "die", env=env)
        lane = int(_expect(dead, "LANE")[1])
        assert dead.wait(60) == -9
        __import__("time").sleep(3.0)  # the in-flight Prime.Check (~2 s) completes into the segment
        again = subprocess.run([sys.executable, "-c", _SLOW_CALLER, name, "again"], env=env, capture_output=True,
                               text=True, timeout=120)
        assert again.returncode == 0, again.stderr[-2000:]
        out = json.loads([x for x in again.stdout.splitlines() if x.startswith("RESULT ")][0][7:])
        srv.stdin.write("done\n")
        srv.stdin.flush()
        alive = _expect(srv, "ALIVE", 60)
        assert srv.wait(60) == 0, srv.stderr.read()[-2000:]
    finally:
        if srv.poll() is None:
            srv.kill()
        if name:
            _unlink_shm(name)
    print("caller killed", lane, out, alive)
    assert out["ok"] and out["lane"] == lane, (out, lane)  # the dead caller's lane, reclaimed and reused
    assert alive[1] == "77" and alive[2] == "0", alive


_RELAY_TO_DYING = textwrap.dedent("""
    import json, os, sys, time, torch
    sys.path.insert(0, os.environ["PTYPE_ROOT"])
    from ptype_amd.ops import hip
    from ptype_amd.ops.peer import PeerRelay
    from ptype_amd.ops.records import METHOD_RELAY, METHOD_CALC_MULTIPLY, METHOD_ECHO, STATUS_OK
    state = torch.zeros(1024, dtype=torch.int64, device="cuda")
    srv = hip().DeviceServer(0, 1024, state.data_ptr(), 1024, 0, 2000.0, 60.0, f"ptype-rdie-{os.getpid()}")
    relay = PeerRelay(srv, sys.argv[1], "cuda:0", n_lanes=1, timeout_s=2.0)
    print("RELAYING", flush=True)
    t = time.time()
    v1, s1, _ = srv.call(METHOD_RELAY, 7, METHOD_CALC_MULTIPLY, 6, 7, 30.0)  # parked: the target is busy, then killed
    w1 = time.time() - t
    print("CALL1", s1, round(w1, 3), flush=True)
    t = time.time()
    v2, s2, _ = srv.call(METHOD_RELAY, 7, METHOD_CALC_MULTIPLY, 6, 7, 30.0)  # the only slot is suspect: fails at once
    w2 = time.time() - t
    print("CALL2", s2, round(w2, 3), flush=True)
    v3, s3, _ = srv.call(METHOD_ECHO, 3, 99)  # local calls unaffected
    print("CALL3", v3, s3, flush=True)
    x = (torch.arange(1 << 20, device="cuda") * 2).sum().item()
    time.sleep(2.5)  # the wave parks after 2 s idle and writes its slot words back to the table
    out = {"s1": s1, "w1": w1, "s2": s2, "w2": w2, "local": [v3, s3], "slots": [int(q) for q in relay.slots()],
           "gpu_ok": x == (1 << 20) * ((1 << 20) - 1)}
    print("RESULT " + json.dumps(out), flush=True)
    relay.detach()
    srv.close()
""")


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_relay_target_killed_mid_relay():
    """A's dispatcher has a relay parked on B when B is SIGKILLed: the call answers
    kStatusNotDelivered at the relay's deadline, the slot stays suspect (later
    relays on it fail at once instead of holding A's ring), A's own actors keep
    answering and A's GPU takes no fault."""
    env = dict(os.environ, PTYPE_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    b = _spawn(_SLOW_SERVER, env=env)
    name = None
    try:
        name = _expect(b, "SHM")[1]
        b.stdin.write("busy\n")
        b.stdin.flush()
        _expect(b, "BUSY")
        a = _spawn(_RELAY_TO_DYING, name, env=env)
        _expect(a, "RELAYING")
        __import__("time").sleep(0.5)
        b.kill()
        b.wait(30)
        out = json.loads(" ".join(_expect(a, "RESULT", 90)[1:]))
        assert a.wait(60) == 0, a.stderr.read()[-2000:]
    finally:
        if b.poll() is None:
            b.kill()
        if name:
            _unlink_shm(name)
    print("relay target killed", out)
    assert out["s1"] == 5 and 1.0 < out["w1"] < 20.0, out  # NotDelivered at the deadline
    assert out["s2"] == 5 and out["w2"] < 0.5, out          # no slot can free: fails fast
    assert out["local"] == [99, 0] and out["gpu_ok"], out
    assert out["slots"] == [0, 1], out                       # call 0 unanswered: the slot is suspect
