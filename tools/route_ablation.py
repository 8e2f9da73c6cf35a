"""Diagnostic: time route_bucket variants (production vs no-lookup) with HIP events."""
import sys, torch
sys.path.insert(0, '.')
from ptype_amd.ops import batch as B, hip, _ptr, _stream
from ptype_amd.ops.table import RegistryTable, actor_keys

def run(M, n_actors, R, cap_mult, ablate, reps=10):
    dev = torch.device('cuda')
    t = RegistryTable(cap_mult * n_actors, device=dev)
    ids = torch.arange(n_actors)
    t.upsert(actor_keys(ids), (ids % R).to(torch.int32), (ids // R).to(torch.int32))
    req = B.gen_requests(M, n_actors, 1, seed=3, device=dev)
    C = B.stripe_capacity(M, R)
    send = torch.empty(R * (C + 1), 4, dtype=torch.int64, device=dev)
    perm = torch.empty(M, dtype=torch.int32, device=dev)
    ws = B.new_workspace(dev)
    evs = []
    for i in range(reps + 2):
        ws.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        hip().route_bucket(_ptr(req), M, _ptr(t.table), t.cap, R, C, _ptr(send), _ptr(perm), _ptr(ws), _ptr(ws[256:257]), _ptr(ws[260:264]), 0, _stream(req), ablate)
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs[2:])
    return ts[len(ts) // 2]

M = 8 * 1024 * 1024
for R in (1, 8):
    for cm in (2, 4):
        for ab in (0, 1):
            print(f"R={R} cap={cm}x ablate={ab}: {run(M, 131072 * R, R, cm, ab):.1f} us", flush=True)
