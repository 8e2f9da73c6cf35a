"""The optimus scatter/gather workload (reference example/optimus).

``Prime.Check(Args{Min, Max, Target})`` returns the first divisor of Target in
[Min, min(Max, Target)) or Target (example/optimus/prime.go:15-25), sleeping
250 ms per candidate in the reference.  The coordinator splits [2, Target) into
10-wide ranges, fans them out concurrently and returns the first reply that is
not Target (coordinator.go:46-99).

Three execution paths with the same answers:
* host: the reference's shape -- a net/rpc fan-out with ``Client.Go`` and a
  gather that returns early;
* device batch: the whole fan-out as ONE ``Send`` of ``ceil(T/10)`` 32-B
  records, bucketed to worker GPUs and exchanged by RCCL all-to-all, gathered
  by a min over non-Target replies;
* HTTP: ``POST /test`` with form ``target=<int>`` (coordinator.go:42-65).
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs

import torch

from ..ops.batch import MsgBatch
from ..ops.records import METHOD_PRIME_CHECK, STATUS_OK

SERVICE = "Prime"
DEVICE_METHODS = {"Check": (METHOD_PRIME_CHECK, ["Min", "Max", "Target"])}
CHUNK = 10  # coordinator.go:69


@dataclass
class Args:
    Min: int
    Max: int
    Target: int


class Prime:
    """Host receiver (prime.go:15-25); ``delay`` is the per-candidate sleep."""

    def __init__(self, delay: float = 0.25):
        self.delay = delay

    def Check(self, args) -> int:
        for i in range(args.Min, min(args.Max, args.Target)):
            if self.delay:
                time.sleep(self.delay)
            if i != 0 and args.Target % i == 0:
                return i
        return args.Target


def split_work(target: int) -> list[tuple[int, int]]:
    """splitWork (coordinator.go:67-73): ranges [2,10), [10,20), ... up to < target+10."""
    out, lo = [], 2
    for i in range(10, target + 10, CHUNK):
        out.append((lo, i))
        lo = i
    return out


def watch_replies(target: int, replies) -> int:
    """watchReplies (coordinator.go:91-98): the first reply != target wins."""
    for r in replies:
        if r != target:
            return r
    return target


def check_host(client, target: int) -> int:
    """Fan out with Client.Go, gather in completion order with early exit."""
    calls = [client.Go("Prime.Check", Args(lo, hi, target)) for lo, hi in split_work(target)]

    def replies():
        for c in calls:
            r = c.done.recv(600.0)
            if r is None or r.error is not None:
                raise RuntimeError(f"coordinator error: {None if r is None else r.error}")
            yield r.reply

    return watch_replies(target, replies())


def make_batch(target: int, n_actors: int, device) -> MsgBatch:
    """The fan-out as one batch: range k goes to actor k % n_actors."""
    ranges = split_work(target)
    n = len(ranges)
    lo = torch.tensor([r[0] for r in ranges], dtype=torch.int64)
    hi = torch.tensor([r[1] for r in ranges], dtype=torch.int64)
    actors = torch.arange(n, dtype=torch.int32) % max(1, n_actors)
    return MsgBatch(actors.to(device), lo.to(device), hi.to(device), torch.full((n,), target, dtype=torch.int64,
                                                                             device=device), METHOD_PRIME_CHECK)


class FanOut:
    """The coordinator for many targets at once (BASELINE config 4): every
    target's 10-wide ranges (splitWork, coordinator.go:67-73) in ONE batch,
    range r of the batch to actor r % n_actors, and the gather (watchReplies,
    :91-98) on the device -- ``csrc/hip/optimus.hip``: one wave per target scans
    its ranges in order and stops at the first non-target reply."""

    def __init__(self, targets: torch.Tensor, n_actors: int, device):
        device = torch.device(device)
        tg = targets.to(device=device, dtype=torch.int64)
        self.targets, self.T, self.device = tg, int(tg.numel()), device
        self.n = (tg + 9) // 10  # ranges per target: i = 10, 20, ... < target + 10
        self.M = int(self.n.sum()) if self.T else 0
        tid = torch.repeat_interleave(torch.arange(self.T, device=device), self.n)
        self.first = torch.cumsum(self.n, 0) - self.n
        k = torch.arange(self.M, device=device) - self.first[tid]
        lo = torch.where(k == 0, torch.full_like(k, 2), k * 10)
        actors = (torch.arange(self.M, device=device) % max(1, n_actors)).to(torch.int32)
        self.batch = MsgBatch(actors, lo, (k + 1) * 10, tg[tid], METHOD_PRIME_CHECK)
        self.answer = torch.empty(self.T, dtype=torch.int64, device=device)
        self.status = torch.empty(self.T, dtype=torch.int32, device=device)

    def gather(self, val: torch.Tensor, st: torch.Tensor):
        """Per target: its smallest divisor (the first non-target reply in range
        order) or the target itself; a failed range's status in ``status``."""
        if self.device.type == "cuda":
            from ..ops import hip, raw_stream

            hip().prime_gather(val.data_ptr(), st.data_ptr(), self.first.data_ptr(), self.n.data_ptr(),
                               self.targets.data_ptr(), self.T, self.answer.data_ptr(), self.status.data_ptr(), 0,
                               raw_stream(self.device))
            return self.answer, self.status
        return gather_ref(val, st, self.first, self.n, self.targets)


def gather_ref(val, st, first, n, targets):
    """Host reference of the device gather (same decision per target)."""
    ans = targets.clone()
    status = torch.zeros(targets.numel(), dtype=torch.int32)
    for j in range(targets.numel()):
        f, c, t = int(first[j]), int(n[j]), int(targets[j])
        for i in range(f, f + c):
            if int(st[i]) != STATUS_OK:
                status[j] = int(st[i])
                break
            if int(val[i]) != t:
                ans[j] = int(val[i])
                break
    return ans, status


def check_device(runtime, target: int) -> int:
    """One batched Send + the device-side gather (the first non-target reply in
    range order: the smallest divisor).  The prime workers are co-hosted on the
    runtime's GPU actors."""
    runtime.host(SERVICE)
    f = FanOut(torch.tensor([target], dtype=torch.int64), runtime.total_actors, runtime.device)
    val, st = runtime.send(SERVICE, f.batch)
    ans, status = f.gather(val, st)
    if int(status[0]) != STATUS_OK:
        raise RuntimeError("prime check failed on device")
    return int(ans[0])


class Coordinator:
    """HTTP front end: POST /test target=<int> -> decimal answer (coordinator.go:42-65)."""

    def __init__(self, check, port: int = 8082, host: str = "127.0.0.1"):
        check_fn = check

        class H(BaseHTTPRequestHandler):
            def do_POST(self):  # noqa: N802
                if self.path != "/test":
                    self.send_response(404)
                    self.end_headers()
                    return
                n = int(self.headers.get("Content-Length", "0"))
                form = parse_qs(self.rfile.read(n).decode())
                try:
                    target = int(form.get("target", ["0"])[0])
                except ValueError:
                    target = 0  # strconv.Atoi error is ignored in the reference
                try:
                    body = str(check_fn(target)).encode()
                except Exception as e:  # the reference log.Fatal()s the coordinator; answer 500 instead
                    self.send_response(500)
                    self.end_headers()
                    self.wfile.write(str(e).encode())
                    return
                self.send_response(200)
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):  # noqa: N802
                self.send_response(405)
                self.end_headers()
                self.wfile.write(b"invalid_http_method")

            def log_message(self, *a):
                pass

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.thread.start()

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()
