"""Multi-process runs of the HIP path, on the one GPU of a test box.

- Two torch.distributed ranks (gloo: RCCL cannot put two ranks on one device) each run
  their instance shard through libpsg on cuda:0, the summaries are all-reduced with
  round_amd.dist exactly as bench.py does, and the node-level result must equal one
  process running the whole range (bit-exact counters and digest).
- bench.py under torch.distributed.run (world size 1): the RCCL ("nccl") process group,
  the all-reduce of the counters and the max-over-ranks timing on real hardware.
The N = 2..8 scaling runs are the driver's (one rank per GPU on an 8-GPU node).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CASES = {  # name -> (algorithm factory, n, instances per rank, make_config kwargs)
    "otr": (lambda psync: psync.OTR(), 64, 20_000, dict(value_range=64, seed=5)),
    "floodmin": (lambda psync: psync.FloodMin(8), 256, 4_000, dict(seed=6)),
    "benor": (lambda psync: psync.BenOr(), 128, 4_000, dict(seed=7, rounds=32)),
}


def _worker(rank, world, port, name, out_q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from round_amd import abi, psync
    from round_amd import dist as rdist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    mk, n, per_rank, kw = CASES[name]
    begin, count = rdist.shard(rank, world, per_rank)
    with psync.GpuRound(mk(psync), n, device=0, batch_capacity=count, **kw) as gr:
        s = gr.run(begin, count).summary
    torch.cuda.synchronize()
    tot = rdist.allreduce_summary(s)  # gloo: CPU tensors
    if rank == 0:
        out_q.put(abi.summary_to_list(tot))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", sorted(CASES))
def test_two_rank_shards_equal_one_process(name):
    import torch.multiprocessing as mp
    from round_amd import abi, psync
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mk, n, per_rank, kw = CASES[name]
    with psync.GpuRound(mk(psync), n, device=0, batch_capacity=2 * per_rank, **kw) as gr:
        whole = abi.summary_to_list(gr.run(0, 2 * per_rank).summary)
    assert got[:-1] == whole[:-1]  # every counter, histogram and the digest (kernel_ns is a max)


def test_bench_under_torchrun_world1():
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--instances", "200000", "--variants=",
           "--no-cpu-baseline"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["checks"]["process_rounds_counted"] == 200000 * 64 * 20
    assert all(v == 0 for v in d["checks"]["violations"].values())


def test_bench_device_list_two_devices():
    """`bench.py --device-list 0,0` runs one context over two device slots
    (psg_config.devices), reports n_gpus = 2, and its node counters equal one context over
    the same 2 x I instances."""
    from round_amd import psync
    per = 100_000
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device-list", "0,0", "--steps", "2", "--warmup", "1",
           "--instances", str(per), "--variants=", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    c = d["checks"]
    assert c["process_rounds_counted"] == 2 * per * 64 * 20
    with psync.GpuRound(psync.OTR(), 64, rounds=20, seed=2, value_range=64,
                        schedule=psync.HOSchedule(drop_log2=3, good_round=0.25), device=0,
                        batch_capacity=2 * per) as gr:
        s = gr.run(0, 2 * per).summary
    assert c["decided_processes"] == s.decided_processes
    assert c["termination_hist"] == [s.term_hist[i] for i in range(22)]
    assert c["process_rounds_active"] == s.active_process_rounds
    assert c["instance_rounds_live"] == s.live_instance_rounds
