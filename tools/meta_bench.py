"""Width pass (wire v3 agreement input) time vs block count, 8 Mi calculator messages.
usage: PTYPE_META_BLOCKS=N python tools/meta_bench.py  (one process per setting: the knob is read once)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ptype_amd.ops import batch as B  # noqa: E402
from ptype_amd.ops import packed as P  # noqa: E402
from ptype_amd.ops.records import METHOD_CALC_MULTIPLY  # noqa: E402
from ptype_amd.ops.table import RegistryTable, actor_keys  # noqa: E402

M, n = 8 * 1024 * 1024, 131072
g = RegistryTable(2 * n, device="cuda")
ids = torch.arange(n)
g.upsert(actor_keys(ids), torch.zeros(n, dtype=torch.int32), ids.to(torch.int32))
g.enable_directory(n, affine_world=1)
req = B.gen_requests(M, n, METHOD_CALC_MULTIPLY, seed=1, device="cuda")
out = torch.empty(16, dtype=torch.int64, device="cuda")
for _ in range(3):
    P.meta(req, g, out)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    P.meta(req, g, out)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
print(json.dumps({"blocks": os.environ.get("PTYPE_META_BLOCKS", "2048"), "us": round(us, 2),
                  "GBps": round(M * 20 / us / 1e3, 1)}))
