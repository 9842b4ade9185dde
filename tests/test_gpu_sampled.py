"""Sampled parity at the instance ids the real runs use (north_star: bit-exact "on a
sampled subset"; SURVEY §8b psg_fetch_instances is the parity path).

The batch parity tests run ids near 1000; the benchmark configurations run ids up
to 1e7 (C2, one GPU) and 1e8 (C3, sharded over 8 ranks), and every Philox draw is
keyed on the 64-bit instance id (counter words inst_lo, inst_hi). These tests fetch
~512 ids spread over those ranges, across the shard boundaries and past 2^32
(inst_hi != 0), and compare each one bit for bit with the oracle: the per-instance
summary (digest, first failing check point per slot, termination round) and every
process's record (decision, decision round, halt round, final state).
"""
import random

import numpy as np
import pytest

from round_amd import psync

pytestmark = pytest.mark.gpu

TWO32 = 1 << 32


def _ids(rng, total, k, shards=1, extra=()):
    out = set(rng.randrange(total) for _ in range(k))
    out.update(range(max(0, total - 8), total))  # the tail of the range
    for r in range(1, shards):  # both sides of every rank's shard boundary
        b = r * total // shards
        out.update(range(b - 3, b + 3))
    out.update(extra)
    return sorted(out)


def _check(gr, ids, oracle_mod, threads=8):
    sums, recs = gr.fetch(ids)
    _, opi, orec = oracle_mod.run(gr.cfg, ids=ids, per_instance=True, records=True, threads=threads)
    n = gr.cfg.n
    for j, inst in enumerate(ids):
        g, o = sums[j], opi[j]
        assert (g.digest, tuple(g.first_fail), g.term_round, g.n_decided) == \
               (o.digest, tuple(o.first_fail), o.term_round, o.n_decided), inst
        for p in range(n):
            a, b = recs[j * n + p], orec[j * n + p]
            assert (a.decision, a.decision_round, a.halt_round, a.final_x) == \
                   (b.decision, b.decision_round, b.halt_round, b.final_x), (inst, p)


HIGH = list(range(TWO32 - 3, TWO32 + 5)) + [TWO32 + 300, 3 * TWO32 + 17, (1 << 40) + 5, (1 << 63) + 11,
                                              (1 << 64) - 2]


def test_c2_otr_ids_over_the_run(oracle_mod):
    """C2 (bench.py workload): OTR n=64, V=64, 1e7 instances, seed 2."""
    rng = random.Random(2)
    ids = _ids(rng, 10_000_000, 440, extra=HIGH)
    with psync.GpuRound(psync.OTR(), 64, rounds=20, seed=2, value_range=64,
                        schedule=psync.HOSchedule(drop_log2=3, good_round=0.25), batch_capacity=len(ids)) as gr:
        _check(gr, ids, oracle_mod)


def test_c3_lastvoting_shard_boundaries(oracle_mod):
    """C3: LastVoting n=64 crash-stop, 1e8 instances over 8 ranks (1.25e7 each)."""
    rng = random.Random(3)
    ids = _ids(rng, 100_000_000, 400, shards=8, extra=HIGH)
    with psync.GpuRound(psync.LastVoting(), 64, seed=7, batch_capacity=len(ids)) as gr:
        _check(gr, ids, oracle_mod)


@pytest.mark.parametrize("f", [0, 8, 64])
def test_c4_floodmin_f(f, oracle_mod):
    rng = random.Random(40 + f)
    ids = _ids(rng, 1_000_000, 40, extra=HIGH[:6])
    with psync.GpuRound(psync.FloodMin(f), 256, seed=7, batch_capacity=len(ids)) as gr:
        _check(gr, ids, oracle_mod)


@pytest.mark.parametrize("f", [0, 1, 8, 32, 64])
def test_c4_kset_f(f, oracle_mod):
    """C4 KSet n=256 k=2 crash-stop sweep (bench_configs.py C4_kset_n256_k2_f*): f = 0 (no crash
    schedule at all, psg_api.hip make_args), the default f < k, two inner points and the f = 64 end."""
    rng = random.Random(50 + f)
    ids = _ids(rng, 200_000, 24, extra=HIGH[:4])
    sched = psync.HOSchedule(drop_log2=0, good_round=0.0, crash_fmax=f)
    with psync.GpuRound(psync.KSetAgreement(2), 256, seed=7, schedule=sched, batch_capacity=len(ids)) as gr:
        _check(gr, ids, oracle_mod)


def test_c5_benor_r64(oracle_mod):
    """C5: BenOr n=128, 64 rounds, |HO(p)| > n/2."""
    rng = random.Random(5)
    ids = _ids(rng, 1_000_000, 120, extra=HIGH)
    with psync.GpuRound(psync.BenOr(), 128, rounds=64, seed=7, batch_capacity=len(ids)) as gr:
        _check(gr, ids, oracle_mod)


def test_batch_across_2_32(oracle_mod):
    """A contiguous batch whose ids cross 2^32 (inst_hi changes inside one launch)."""
    begin, count = TWO32 - 150, 300
    with psync.GpuRound(psync.OTR(), 64, seed=2, value_range=64, batch_capacity=count) as gr:
        res = gr.run(begin, count, per_instance=True)
    osum, opi, _ = oracle_mod.run(gr.cfg, begin, count, per_instance=True, threads=8)
    assert res.summary.digest == osum.digest
    assert list(res.summary.fail_count) == list(osum.fail_count)
    assert [(s.digest, tuple(s.first_fail), s.term_round) for s in res.per_instance] == \
           [(s.digest, tuple(s.first_fail), s.term_round) for s in opi]


def test_fetch_equals_batch_rows():
    """A fetched id reproduces the row the batch produced for it (same kernel, ids path)."""
    n, begin, count = 64, 9_990_000, 10_000
    with psync.GpuRound(psync.OTR(), n, seed=2, value_range=64, batch_capacity=count) as gr:
        res = gr.run(begin, count, per_instance=True)
        pick = np.random.default_rng(1).choice(count, 256, replace=False)
        sums, _ = gr.fetch([begin + int(i) for i in pick])
    for j, i in enumerate(pick):
        a, b = sums[j], res.per_instance[int(i)]
        assert (a.digest, tuple(a.first_fail), a.term_round) == (b.digest, tuple(b.first_fail), b.term_round)
