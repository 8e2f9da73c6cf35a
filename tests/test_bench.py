"""bench.py contract: one JSON line from rank 0 with the BASELINE.json metric, the
whole-job aggregate, and the fields the round driver reads.

CPU: the same pipeline on gloo (world 1 and 2, torchrun on 127.0.0.1).  GPU: the
real multi-process RCCL path at 2..8 ranks -- only where the box has that many
GPUs (a 1-GPU box skips it: RCCL refuses two ranks on one device)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, free_port

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "p50_rtt_us"}


def _run(nproc, extra, timeout=600, launcher="torchrun"):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    if nproc == 1 or launcher == "self":  # bench.py starts torch.distributed.run itself for N > 1
        cmd = [sys.executable, "bench.py"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py"]
    cmd += ["--gpus", str(nproc)] + extra
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


SMALL = ["--steps", "2", "--warmup", "1", "--msgs-per-gpu", "20000", "--actors-per-gpu", "1024", "--rtt-calls", "0"]


@pytest.mark.parametrize("nproc,launcher", [(1, "self"), (2, "torchrun"), (2, "self")])
def test_bench_json_contract_cpu(nproc, launcher):
    out = _run(nproc, ["--cpu"] + SMALL, launcher=launcher)
    assert REQUIRED <= set(out)
    assert out["metric"] == "messages/sec" and out["unit"] == "msg/s" and out["higher_is_better"] is True
    assert out["n_gpus"] == nproc and out["steps"] == 2 and out["warmup"] == 1 and out["scaling"] == "weak"
    assert out["data"] == "synthetic"
    assert out["config"]["global_batch"] == 20000 * nproc
    # headline placement reads the registry mirror; the strided figure is secondary only
    assert out["config"]["placement"] == "random" and out["config"]["registry_lookup"] != "computed (verified strided rule)"
    assert out["secondaries"]["affine_placement"]["placement"] == "affine"
    # value is the whole-job aggregate: every rank's messages over the max rank time
    assert out["value"] == pytest.approx(20000 * nproc * 2 / (out["ms_per_step"] * 2 / 1e3), rel=1e-6)


def _gpus() -> int:
    try:
        import torch

        return torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception:
        return 0


@pytest.mark.gpu
@pytest.mark.parametrize("nproc", [2, 4, 8])
def test_bench_multi_gpu(nproc):
    if _gpus() < nproc:
        pytest.skip(f"needs {nproc} GPUs (RCCL refuses two ranks on one device)")
    out = _run(nproc, ["--steps", "3", "--warmup", "2", "--rtt-calls", "200"], timeout=900)
    assert out["n_gpus"] == nproc and out["value"] > 0  # (the bench verifies every reply itself)
    # the N > 1 mailbox path is the sorted exchange (csrc/hip/exchange_sorted.hpp): wire-v3
    # records through padded RCCL all-to-alls at the capacity agreed two Sends earlier (or,
    # when the agreed per-pair capacities differ enough, their prefixes by grouped send / recv)
    c = out["config"]
    assert c["wire"] == "v3-packed" and c["engine"] == "sorted", c
    assert c["exchange"] in ("padded", "per-pair prefixes"), c
    # the communicator Join's compiled DataPlane formed (no torch process group)
    assert c["comm"] == "DataPlane/RCCL" and c["record_bytes"] <= 8
    assert out["p50_rtt_remote_us"] is not None
    assert out["rtt_error"] is None and out["rtt_remote_request_ring"] == "device"
    # skewed traffic: once the agreement of Send k - 2 sizes the regions (from Send 2 on),
    # no re-send rounds -- the warm-up's start-up Sends may re-send, the timed ones must not
    z = _run(nproc, ["--steps", "3", "--warmup", "3", "--rtt-calls", "0", "--zipf", "1.1", "--no-secondary"],
             timeout=900)
    assert z["config"]["resend_rounds"] == 0 and z["value"] > 0, z["config"]


@pytest.mark.gpu
@pytest.mark.parametrize("nproc", [2, 4])
def test_bench_multi_process_on_one_gpu_ipc(nproc):
    """The bench's N > 1 path across real processes on ONE GPU:
    torchrun ranks, a control-plane member per rank and the compiled DataPlane
    with the IpcComm transport (shared-memory segments every rank maps and
    registers; no torch process group) carrying the sorted exchange's
    all-to-alls and agreement --
    every reply verified by the bench itself, the cross-process RTT through the
    next rank's dispatcher ring, and skewed (Zipf) traffic without re-sends once
    the agreement applies."""
    small = ["--msgs-per-gpu", str(1 << 18), "--actors-per-gpu", "8192", "--comm", "ipc"]
    out = _run(nproc, ["--steps", "4", "--warmup", "3", "--rtt-calls", "200", "--no-secondary"] + small,
               timeout=600, launcher="self")
    c = out["config"]
    assert out["n_gpus"] == nproc and out["value"] > 0
    assert c["comm"] == "DataPlane/IpcComm" and c["engine"] == "sorted" and c["wire"] == "v3-packed"
    assert c["record_bytes"] <= 8
    assert out["rtt_error"] is None and out["p50_rtt_remote_us"] > 0
    z = _run(nproc, ["--steps", "4", "--warmup", "3", "--rtt-calls", "0", "--zipf", "1.1", "--no-secondary"] + small,
             timeout=600, launcher="self")
    assert z["config"]["resend_rounds"] == 0 and z["value"] > 0, z["config"]


@pytest.mark.gpu
def test_bench_force_dist_remote_rtt():
    """World 1 with the compiled DataPlane's RCCL communicator up: the multi-rank
    RTT phase (store barriers, the "next rank's" dispatcher mapped from its dma-buf
    -- here this rank's own) runs as it does at N > 1."""
    out = _run(1, ["--force-dist", "--steps", "2", "--warmup", "1", "--rtt-calls", "200", "--no-secondary"],
               timeout=300)
    assert out["rtt_error"] is None, out["rtt_error"]
    assert out["p50_rtt_remote_us"] is not None and out["p50_rtt_remote_us"] > 0
    assert out["rtt_remote_request_ring"] == "device"
    assert out["config"]["comm"] == "DataPlane/RCCL"


def test_bench_zipf_cpu():
    """Skewed load (Zipf 1.1, pre-generated) through the 2-rank gloo pipeline."""
    out = _run(2, ["--cpu", "--zipf", "1.1", "--no-secondary"] + SMALL, launcher="self")
    assert out["config"]["load"] == "zipf(1.1)" and out["config"]["pregenerated"] is True
    assert out["value"] > 0


def test_api_send_secondary_runs_join_newclient_send_on_cpu():
    """bench.py's api_send secondary (Join -> NewClient -> Client.Send), CPU twin."""
    import torch

    from ptype_amd.utils import benchmarks as BM

    out = BM.api_send(torch.device("cpu"), [2048], 512, 2, 1)
    assert out["2048"]["msgs_per_step"] == 2048 and out["2048"]["value"] > 0


_API_RANK = r"""
import json, os, sys, torch
import torch.distributed as dist
sys.path.insert(0, os.environ["PTYPE_ROOT"])
from ptype_amd.utils import benchmarks as BM
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)

def mx(x):
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

out = BM.api_send(torch.device("cpu"), [4096], 512, 3, 1, rank=rank, world=world, barrier=dist.barrier,
                  max_over_ranks=mx)
print("RESULT " + json.dumps(out), flush=True)
dist.destroy_process_group()
"""


def test_api_send_secondary_across_ranks_on_cpu():
    """the api_send secondary at N > 1 -- one control-plane member
    per rank (static cluster from MASTER_PORT), every rank's runtime on the
    existing process group, Client.Send from every rank (deferred re-sends, the
    timed loop ends with Flush), the replies verified on every rank."""
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, PTYPE_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-c", _API_RANK], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, e[-3000:]
        line = [x for x in o.splitlines() if x.startswith("RESULT ")]
        assert line, o[-2000:] + e[-2000:]
        outs.append(json.loads(line[0][7:]))
    for out in outs:
        assert out["ranks"] == 2 and out["4096"]["msgs_per_step"] == 4096 and out["4096"]["value"] > 0, out


@pytest.mark.gpu
def test_bench_api_send_secondary_at_n2_over_ipc():
    """The api_send secondary in the N > 1 bench line: two torchrun
    ranks on one GPU (IpcComm), Join -> NewClient -> Client.Send on both, replies
    verified, no host wait per Send beyond the deferred re-send resolution."""
    small = ["--msgs-per-gpu", str(1 << 18), "--actors-per-gpu", "8192", "--comm", "ipc"]
    out = _run(2, ["--steps", "3", "--warmup", "2", "--rtt-calls", "0"] + small, timeout=600, launcher="self")
    api = out["secondaries"]["api_send"]
    assert "error" not in api, api
    assert api["ranks"] == 2 and api[str(1 << 18)]["value"] > 0, api
