"""World-size-2 gloo test of the multi-GPU path (round_amd/dist.py).

bench.py shards instance ids across ranks and all-reduces the psg_summary
counters (RCCL on the GPU node). Here each gloo rank runs its shard on the CPU
oracle (standing in for the per-GPU executor, test infrastructure only) and the
reduced node-level summary must equal a single-process run of the whole range.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, per_rank, out_q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    import oracle
    from round_amd import abi, psync
    from round_amd import dist as rdist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    cfg = psync.make_config(psync.OTR(), 16, seed=5, value_range=6)
    begin, count = rdist.shard(rank, world, per_rank)
    s, _, _ = oracle.run(cfg, begin, count, threads=2)
    s.kernel_ns = 1000 * (rank + 1)
    tot = rdist.allreduce_summary(s)
    lo, cnt = rdist.shard_strong(rank, world, 1001)
    s2, _, _ = oracle.run(cfg, lo, cnt, threads=2)
    tot2 = rdist.allreduce_summary(s2)
    mx = rdist.allreduce_max(float(rank))
    if rank == 0:
        out_q.put((abi.summary_to_list(tot), abi.summary_to_list(tot2), mx))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_reduction(oracle_mod):
    from round_amd import abi, psync
    per_rank = 700
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, per_rank, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, got2, mx = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg = psync.make_config(psync.OTR(), 16, seed=5, value_range=6)
    whole, _, _ = oracle_mod.run(cfg, 0, 2 * per_rank, threads=4)
    assert got[:-1] == abi.summary_to_list(whole)[:-1]
    assert got[-1] == 2000  # kernel_ns reduced with MAX
    whole2, _, _ = oracle_mod.run(cfg, 0, 1001, threads=4)
    assert got2[:-1] == abi.summary_to_list(whole2)[:-1]
    assert mx == 1.0


def test_shard_helpers():
    from round_amd import dist as rdist
    assert rdist.shard(3, 8, 10) == (30, 10)
    parts = [rdist.shard_strong(r, 3, 10) for r in range(3)]
    assert sum(c for _, c in parts) == 10 and parts[0][0] == 0
    assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(2))
    with pytest.raises(ValueError):
        rdist.shard(2, 2, 5)
