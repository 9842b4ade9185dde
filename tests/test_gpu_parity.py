"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Every comparison is bit-exact: per-instance summaries (digest of every
process's decision / decision round / halt round / final state, first failing
check point of every Spec slot, termination round), batch counters,
per-process decide results and fetched per-process records.
"""
import pytest

from round_amd import abi, psync

pytestmark = pytest.mark.gpu

H = psync.HOSchedule

# (id, algorithm, n, instances, make_config kwargs)
CASES = [
    ("otr-c1-n4", psync.OTR(), 4, 1000, dict(rounds=10, value_range=4, seed=1)),
    ("otr-n64-V64", psync.OTR(), 64, 2000, dict(value_range=64, seed=2)),
    ("otr-n64-V2", psync.OTR(), 64, 2000, dict(value_range=2, seed=3)),
    ("otr-n64-V4-after3", psync.OTR(afterDecision=3), 64, 1000, dict(value_range=4, seed=4)),
    ("otr-n17-ragged", psync.OTR(), 17, 2000, dict(value_range=5, seed=5)),
    ("otr-n100-W2", psync.OTR(), 100, 300, dict(value_range=8, seed=6)),
    ("otr-n200-W4", psync.OTR(), 200, 100, dict(value_range=3, seed=6)),
    ("otr-n1", psync.OTR(), 1, 100, dict(value_range=3, seed=7)),
    ("otr-mutant-n8", psync.OTR(variant=1), 8, 3000, dict(schedule=H(drop_log2=1, good_round=0.0), seed=8)),
    ("otr-pureho", psync.OTR(), 12, 2000, dict(schedule=H(drop_log2=2, self_bit=False), seed=9)),
    ("otr-crash", psync.OTR(), 64, 500, dict(schedule=H(drop_log2=3, crash_fmax=20), seed=10)),
    # at most 0 crashes: the library passes "no crash schedule" to the kernels (psg_api.hip make_args)
    ("otr-crash-f0", psync.OTR(), 64, 1000, dict(schedule=H(drop_log2=3, crash_fmax=0), seed=30)),
    ("lv-n64-f0", psync.LastVoting(), 64, 1000, dict(seed=31, schedule=H(drop_log2=3, crash_fmax=0))),
    ("lv-n64-crash", psync.LastVoting(), 64, 2000, dict(seed=11)),
    ("lv-n64-minpid", psync.LastVoting(), 64, 1000, dict(seed=12, tiebreak=abi.PSG_TIE_MIN_PID)),
    ("lv-n5", psync.LastVoting(), 5, 3000, dict(seed=13, value_range=4)),
    ("lv-n64-loss", psync.LastVoting(), 64, 1000, dict(seed=14, value_range=3,
                                                      schedule=H(drop_log2=1, good_round=0.0))),
    ("lv-mutant-n6", psync.LastVoting(variant=1), 6, 3000, dict(seed=15, value_range=5)),
    ("lv-n130-W3", psync.LastVoting(), 130, 100, dict(seed=16)),
    ("fm-n256-f4", psync.FloodMin(4), 256, 300, dict(seed=17)),
    ("fm-n64-f8", psync.FloodMin(8), 64, 1000, dict(seed=18)),
    ("fm-mutant-n16", psync.FloodMin(3, variant=1), 16, 2000, dict(seed=19)),
    ("fm-n256-loss", psync.FloodMin(2), 256, 100, dict(seed=20, schedule=H(drop_log2=2, crash_fmax=2))),
    # lane-packed crash-stop path (n > 64, seeded crash-only schedules): ragged n, every W
    ("fm-n65-f3", psync.FloodMin(3), 65, 400, dict(seed=60)),
    ("fm-n128-f0", psync.FloodMin(0), 128, 300, dict(seed=61)),
    ("fm-n130-mutant", psync.FloodMin(6, variant=1), 130, 300, dict(seed=62, value_range=5)),
    ("fm-n200-f16", psync.FloodMin(16), 200, 200, dict(seed=63, value_range=40)),
    ("fm-n256-f64", psync.FloodMin(64), 256, 60, dict(seed=64)),
    ("fm-n256-f8-V3", psync.FloodMin(8), 256, 300, dict(seed=65, value_range=3)),
    ("kset-n256-k2", psync.KSetAgreement(2), 256, 24, dict(seed=21)),
    ("kset-n64-k3-crash", psync.KSetAgreement(3), 64, 400, dict(seed=22, schedule=H(drop_log2=0, crash_fmax=10,
                                                                                       good_round=0.0))),
    ("kset-n16-loss", psync.KSetAgreement(2), 16, 2000, dict(seed=23, schedule=H(drop_log2=2, good_round=0.0))),
    ("kset-n16-minpid", psync.KSetAgreement(2), 16, 2000, dict(seed=24, tiebreak=abi.PSG_TIE_MIN_PID,
                                                              schedule=H(drop_log2=2, good_round=0.0))),
    # lane-packed KSet path (n > 64, seeded schedules): ragged n, every W, losses, good rounds,
    # both Map tie-break modes (CHAMP find on divergent decider candidates), mutant
    ("kset-n65-k2", psync.KSetAgreement(2), 65, 300, dict(seed=80)),
    ("kset-n130-k3-loss", psync.KSetAgreement(3), 130, 150, dict(seed=81, schedule=H(drop_log2=2, good_round=0.0,
                                                                                     crash_fmax=5))),
    ("kset-n200-minpid", psync.KSetAgreement(2), 200, 100, dict(seed=82, tiebreak=abi.PSG_TIE_MIN_PID,
                                                                schedule=H(drop_log2=1, good_round=0.3))),
    ("kset-n256-k4-champ", psync.KSetAgreement(4), 256, 60, dict(seed=83, schedule=H(drop_log2=1, good_round=0.2,
                                                                                      crash_fmax=3))),
    ("kset-n192-mutant", psync.KSetAgreement(2, variant=1), 192, 100, dict(seed=84)),
    ("kset-n256-k2-V3", psync.KSetAgreement(2), 256, 100, dict(seed=85, value_range=3)),
    # the uniform-t tail kernel (round 6): loss-free crash schedules (its uniform-mailbox form),
    # pure HO, good rounds, at most 0 crashes, and ho_min (the general form)
    ("kset-n256-f64-lossfree", psync.KSetAgreement(2), 256, 200, dict(seed=86, schedule=H(
        drop_log2=0, good_round=0.0, crash_fmax=64))),
    ("kset-n130-lossfree-pureho", psync.KSetAgreement(2), 130, 300, dict(seed=87, schedule=H(
        drop_log2=0, good_round=0.0, crash_fmax=20, self_bit=False))),
    ("kset-n200-lossfree-good", psync.KSetAgreement(3), 200, 200, dict(seed=88, value_range=4, schedule=H(
        drop_log2=0, good_round=0.3, crash_fmax=30))),
    ("kset-n256-f0", psync.KSetAgreement(2), 256, 200, dict(seed=89, schedule=H(drop_log2=0, good_round=0.0,
                                                                                 crash_fmax=0))),
    ("kset-n160-homin", psync.KSetAgreement(2), 160, 150, dict(seed=95, schedule=H(
        drop_log2=3, good_round=0.1, crash_fmax=12, ho_min=120))),
    ("benor-n128", psync.BenOr(), 128, 300, dict(seed=25)),
    ("benor-n4", psync.BenOr(), 4, 3000, dict(seed=26)),
    ("benor-n64-mutant", psync.BenOr(variant=1), 64, 500, dict(seed=27)),
    ("benor-n200-W4", psync.BenOr(), 200, 60, dict(seed=28, rounds=20)),
    # lane-packed built-in-checker path (n > 64, seeded schedules): ragged n, every W, every schedule family
    ("benor-n65", psync.BenOr(), 65, 400, dict(seed=66)),
    ("benor-n128-R64", psync.BenOr(), 128, 200, dict(seed=67, rounds=64)),
    ("benor-n100-crash-good", psync.BenOr(), 100, 300, dict(seed=68, schedule=H(drop_log2=1, good_round=0.3,
                                                                                 crash_fmax=30))),
    ("benor-n150-pureho", psync.BenOr(), 150, 200, dict(seed=69, schedule=H(drop_log2=2, good_round=0.0,
                                                                           self_bit=False))),
    ("benor-n192-mutant", psync.BenOr(variant=1), 192, 150, dict(seed=70)),
    ("benor-n256-W4", psync.BenOr(), 256, 80, dict(seed=71, rounds=24)),
    # second wave
    ("otr2-n64-V4", psync.OTR2(), 64, 2000, dict(value_range=4, seed=40)),
    ("otr2-mutant-n8", psync.OTR2(variant=1), 8, 3000, dict(schedule=H(drop_log2=1, good_round=0.0), seed=41)),
    ("otr2-n100-W2", psync.OTR2(), 100, 300, dict(value_range=8, seed=42)),
    ("slv-n64", psync.ShortLastVoting(), 64, 2000, dict(seed=43)),
    ("slv-n16-loss", psync.ShortLastVoting(), 16, 3000, dict(value_range=5, seed=44, schedule=H(
        drop_log2=1, good_round=0.0, crash_fmax=7))),
    ("slv-mutant-n16", psync.ShortLastVoting(variant=1), 16, 3000, dict(value_range=5, seed=45, schedule=H(
        drop_log2=1, good_round=0.0, crash_fmax=7))),
    ("slv-n16-minpid", psync.ShortLastVoting(), 16, 2000, dict(value_range=5, seed=46, tiebreak=abi.PSG_TIE_MIN_PID,
                                                               schedule=H(drop_log2=1, good_round=0.0))),
    ("slv-n130-W3", psync.ShortLastVoting(), 130, 100, dict(seed=47)),
    ("slv-n256-W4-loss", psync.ShortLastVoting(), 256, 40, dict(value_range=3, seed=48,
                                                                schedule=H(drop_log2=1, good_round=0.0))),
    ("kses-n64-t8k2", psync.KSetEarlyStopping(8, 2), 64, 1000, dict(seed=49)),
    ("kses-n256-t16k3", psync.KSetEarlyStopping(16, 3), 256, 100, dict(seed=50)),
    ("kses-mutant-n16", psync.KSetEarlyStopping(4, 2, variant=1), 16, 3000, dict(seed=51)),
    # lane-packed KSetEarlyStopping path (n > 64, seeded schedules)
    ("kses-n65-t8k2", psync.KSetEarlyStopping(8, 2), 65, 300, dict(seed=90)),
    ("kses-n130-loss", psync.KSetEarlyStopping(16, 3), 130, 150, dict(seed=91, schedule=H(
        drop_log2=2, good_round=0.2, crash_fmax=10))),
    ("kses-n200-pureho", psync.KSetEarlyStopping(8, 2), 200, 100, dict(seed=92, schedule=H(
        drop_log2=1, good_round=0.0, crash_fmax=6, self_bit=False))),
    ("kses-n256-mutant", psync.KSetEarlyStopping(16, 2, variant=1), 256, 60, dict(seed=93)),
    ("kses-n192-t64k2", psync.KSetEarlyStopping(64, 2), 192, 60, dict(seed=94)),
    ("kses-pureho", psync.KSetEarlyStopping(4, 2), 16, 2000, dict(seed=52, schedule=H(
        drop_log2=2, good_round=0.0, crash_fmax=4, self_bit=False))),
]


def _cmp_summary(g, o, rounds):
    assert g.instances == o.instances
    assert g.process_rounds == o.process_rounds
    assert (g.active_process_rounds, g.live_instance_rounds) == (o.active_process_rounds, o.live_instance_rounds)
    assert list(g.fail_count) == list(o.fail_count)
    assert g.decided_processes == o.decided_processes
    assert g.digest == o.digest
    assert list(g.term_hist)[: rounds + 2] == list(o.term_hist)[: rounds + 2]


def _inst_tuple(s):
    return (s.digest, tuple(s.first_fail), s.term_round, s.n_checks, s.n_decided)


def _rec_tuple(r):
    return (r.decision, r.decision_round, r.halt_round, r.final_x)


@pytest.mark.parametrize("cid,alg,n,count,kw", CASES, ids=[c[0] for c in CASES])
def test_gpu_matches_oracle(cid, alg, n, count, kw, oracle_mod):
    begin = 1000  # non-zero instance ids
    with psync.GpuRound(alg, n, batch_capacity=count, **kw) as gr:
        res = gr.run(begin, count, per_instance=True)
        dec, dround = gr.decisions()
        sample = [begin + i for i in range(0, count, max(1, count // 37))]
        fsums, frecs = gr.fetch(sample)
    cfg = gr.cfg
    osum, opi, orec = oracle_mod.run(cfg, begin, count, per_instance=True, records=True, threads=8)
    _cmp_summary(res.summary, osum, cfg.rounds)
    mism = [i for i in range(count) if _inst_tuple(res.per_instance[i]) != _inst_tuple(opi[i])]
    assert not mism, f"{len(mism)} instance summaries differ, first {mism[:5]}"
    for i in range(count):
        for p in range(n):
            r = orec[i * n + p]
            assert dec[i * n + p] == r.decision and dround[i * n + p] == r.decision_round, (i, p)
    for j, inst in enumerate(sample):
        i = inst - begin
        assert _inst_tuple(fsums[j]) == _inst_tuple(opi[i])
        for p in range(n):
            assert _rec_tuple(frecs[j * n + p]) == _rec_tuple(orec[i * n + p]), (inst, p)


def test_host_supplied_inputs(oracle_mod):
    """psg_load_inputs with caller-provided initial values (ConsensusIO.initialValue)."""
    n, count = 64, 200
    init = [[(i * 7 + p * 13) % 5 + 1 for p in range(n)] for i in range(count)]
    with psync.GpuRound(psync.OTR(), n, seed=31, batch_capacity=count) as gr:
        gr.load_inputs(50, count, init)
        res = gr.run(50, count, per_instance=True)
    osum, opi, _ = oracle_mod.run(gr.cfg, 50, count, init=init, per_instance=True)
    _cmp_summary(res.summary, osum, gr.cfg.rounds)
    assert [_inst_tuple(s) for s in res.per_instance] == [_inst_tuple(s) for s in opi]


@pytest.mark.parametrize("drop", [3, 5])
@pytest.mark.parametrize("alg", [psync.OTR(), psync.OTR2()], ids=["otr", "otr2"])
@pytest.mark.parametrize("n", [64, 40, 9])
def test_otr_round0_value_classes(alg, n, drop, oracle_mod):
    """Round 0's mmor folds values by holder classes (h >= 3, h = 2, h = 1) when the initial
    values fit the X0 bitmap and more than 8 are distinct: inputs where every value is held
    once (the singleton pass must run), twice, mixed with ties across classes, values at the
    edges of the 64-wide bitmap window (negative too), and spread-out values (hash mode, one
    pass), with links lost w.p. 1/8 and 1/32 (mailboxes above the 2n/3 quorum), against the
    oracle; the test also requires that round 0 updated x in most instances."""
    import random
    rng = random.Random(1000 + n)
    count = 240
    init = []
    for i in range(count):
        fam = i % 6
        if fam == 0:    # all distinct (n <= 64): only singletons
            row = rng.sample(range(1, 65), n)
        elif fam == 1:  # every value held twice
            row = [1 + (p // 2) for p in range(n)]
            rng.shuffle(row)
        elif fam == 2:  # mixed classes with ties
            row = [rng.choice([3, 3, 3, 7, 7, 11, 11]) if p % 3 == 0 else rng.randint(1, 64) for p in range(n)]
        elif fam == 3:  # the whole 64-wide window, negative base
            row = [-1000 + rng.randint(0, 63) for _ in range(n)]
            row[0], row[-1] = -1000, -937
        elif fam == 4:  # hash mode: values spread over more than 64
            row = [rng.randint(0, 40) * 1000 for _ in range(n)]
        else:           # near Int.MaxValue, within one window
            row = [2147483647 - rng.randint(0, 63) for _ in range(n)]
        init.append(row)
    sched = H(drop_log2=drop, good_round=0.0)
    with psync.GpuRound(alg, n, seed=33 + n, schedule=sched, batch_capacity=count) as gr:
        gr.load_inputs(90, count, init)
        res = gr.run(90, count, per_instance=True)
    osum, opi, orec = oracle_mod.run(gr.cfg, 90, count, init=init, per_instance=True, records=True)
    _cmp_summary(res.summary, osum, gr.cfg.rounds)
    assert [_inst_tuple(s) for s in res.per_instance] == [_inst_tuple(s) for s in opi]
    # the mmor path ran: most instances end with some x different from its initial value
    moved = sum(any(orec[i * n + p].final_x != init[i][p] for p in range(n)) for i in range(count))
    assert moved > count // 2, moved


@pytest.mark.parametrize("alg,n", [(psync.FloodMin(5), 256), (psync.FloodMin(3), 100), (psync.BenOr(), 128),
                                   (psync.KSetAgreement(2), 256), (psync.KSetAgreement(3), 90),
                                   (psync.KSetEarlyStopping(16, 2), 256)],
                         ids=["fm-n256", "fm-n100", "benor-n128", "kset-n256", "kset-n90", "kses-n256"])
def test_host_supplied_inputs_wide(alg, n, oracle_mod):
    """Caller-provided initial values on the wide fast paths (lane-packed kernels)."""
    count = 150
    vr = 2 if isinstance(alg, psync.BenOr) else 1000
    init = [[(i * 7 + p * 13) % vr + (0 if vr == 2 else -500) for p in range(n)] for i in range(count)]
    with psync.GpuRound(alg, n, seed=32, batch_capacity=count) as gr:
        gr.load_inputs(70, count, init)
        res = gr.run(70, count, per_instance=True)
    osum, opi, _ = oracle_mod.run(gr.cfg, 70, count, init=init, per_instance=True)
    _cmp_summary(res.summary, osum, gr.cfg.rounds)
    assert [_inst_tuple(s) for s in res.per_instance] == [_inst_tuple(s) for s in opi]


def test_sharding_invariance_and_determinism():
    """Any split of the instance range gives the same node-level sums (RNG keyed on global ids)."""
    n, N = 64, 200_000
    with psync.GpuRound(psync.OTR(), n, value_range=64, seed=41, batch_capacity=N) as gr:
        whole = gr.run(0, N).summary
        again = gr.run(0, N).summary
        a = gr.run(0, N // 3).summary
        b = gr.run(N // 3, N - N // 3).summary
    for s in (again,):
        assert abi.summary_to_list(s)[:-1] == abi.summary_to_list(whole)[:-1]
    merged = [x + y for x, y in zip(abi.summary_to_list(a)[:-1], abi.summary_to_list(b)[:-1])]
    merged = abi.summary_to_list(abi.summary_from_list(merged + [0]))[:-1]
    assert merged == abi.summary_to_list(whole)[:-1]


@pytest.mark.parametrize("V", [2, 4, 64])
def test_otr_full_size_zero_false_positives(V):
    """C2 shape at 1e6 instances: the verified OTR never violates its Spec."""
    n, N = 64, 1_000_000
    with psync.GpuRound(psync.OTR(), n, value_range=V, seed=100 + V, batch_capacity=N) as gr:
        res = gr.run(0, N)
    v = res.violations()
    assert all(c == 0 for c in v.values()), v
    s = res.summary
    assert s.process_rounds == N * n * 20
    assert sum(s.term_hist[i] for i in range(22)) == N


def test_lastvoting_full_size_zero_false_positives():
    n, N = 64, 500_000
    with psync.GpuRound(psync.LastVoting(), n, seed=7, batch_capacity=N) as gr:
        res = gr.run(0, N)
    assert all(c == 0 for c in res.violations().values()), res.violations()


def test_invalid_config_raises():
    from round_amd.lib import PsgError
    with pytest.raises((PsgError, ValueError)):
        psync.GpuRound(psync.OTR(), 300)
    cfg = psync.make_config(psync.OTR(), 8)
    cfg.abi_version = 99
    from round_amd import lib
    with pytest.raises(PsgError):
        lib.Context(cfg)


def test_gpu_map_head_matches_oracle(oracle_mod):
    """champ_first (per-receiver mailbox.head, psg_slv.hip) vs the oracle's Scala Map order."""
    import random
    from round_amd import lib
    rng = random.Random(5)
    sets = [0, 1, 0b11111, (1 << 64) - 1, (1 << 63) | 1]
    for _ in range(3000):
        m = 0
        for q in range(64):
            if rng.random() < rng.choice([0.05, 0.2, 0.5, 0.9]):
                m |= 1 << q
        sets.append(m)
    for tb in (abi.PSG_TIE_CHAMP, abi.PSG_TIE_MIN_PID):
        got = lib.selftest_map_head(sets, tb)
        for m, h in zip(sets, got):
            pids = [q for q in range(64) if (m >> q) & 1]
            want = oracle_mod.scala_map_order(pids, tb)[0] if pids else -1
            assert h == want, (hex(m), tb, h, want)


# --------------------------------------------------------------------------- EpsilonConsensus (Double)
# Values: every step is the same IEEE operation in the same order on both sides, so
# the GPU reproduces the oracle bit for bit; the stated tolerance covers libm log()
# differing by an ulp (which can move maxR only when r1 sits within an ulp of an
# integer). Integer results (rounds, first failing check points) must match exactly.
F64_ABS_TOL = 1e-12

EPS_CASES = [
    ("eps-n7-f1", psync.EpsilonConsensus(1, 0.1), 7, 4000, dict(seed=60)),
    ("eps-n16-f2", psync.EpsilonConsensus(2, 1e-3), 16, 2000, dict(seed=61)),
    ("eps-n64-f5", psync.EpsilonConsensus(5, 1e-6), 64, 1000, dict(seed=62)),
    ("eps-n64-loss-nan", psync.EpsilonConsensus(3, 1e-3), 64, 1000, dict(seed=63, schedule=psync.HOSchedule(
        drop_log2=1, good_round=0.0))),
    ("eps-n7-pureho", psync.EpsilonConsensus(1, 0.05), 7, 3000, dict(seed=64, schedule=psync.HOSchedule(
        drop_log2=2, good_round=0.0, self_bit=False))),
    ("eps-n40-crash", psync.EpsilonConsensus(4, 1e-4), 40, 1000, dict(seed=65, schedule=psync.HOSchedule(
        drop_log2=3, good_round=0.0, crash_fmax=4))),
    ("eps-mutant-n7", psync.EpsilonConsensus(1, 0.01, variant=1), 7, 3000, dict(seed=66, schedule=psync.HOSchedule(
        drop_log2=2, good_round=0.0, ho_min=5))),
    # W = 1 rank select (RankSel) extremes: f = 1 selects every other member (~30 selects per
    # lane per round, every byte of the position mask), f = 10 steps 20 positions at a time
    ("eps-n64-f1", psync.EpsilonConsensus(1, 1e-9), 64, 500, dict(seed=69)),
    ("eps-n64-f10", psync.EpsilonConsensus(10, 1e-4), 64, 500, dict(seed=71)),
    ("eps-n100-W2", psync.EpsilonConsensus(10, 1e-5), 100, 300, dict(seed=67, rounds=16)),
    ("eps-n256-W4", psync.EpsilonConsensus(40, 1e-3), 256, 60, dict(seed=68, rounds=16)),
]


def _close(a, b, tol=F64_ABS_TOL):
    import math
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b)
    return abs(a - b) <= tol


def _check_eps(gr, res, dec, dround, begin, count, init=None, oracle_mod=None):
    n = gr.cfg.n
    osum, opi, orec, odec, ofx = oracle_mod.run_real(gr.cfg, begin, count, init=init, per_instance=True,
                                                     records=True, threads=8)
    _cmp_summary(res.summary, osum, gr.cfg.rounds)
    for i in range(count):
        g, o = res.per_instance[i], opi[i]
        assert (tuple(g.first_fail), g.term_round, g.n_decided) == (tuple(o.first_fail), o.term_round, o.n_decided), i
        assert g.digest == o.digest, i
    for c in range(count * n):
        assert dround[c] == orec[c].decision_round, c
        assert _close(dec[c], odec[c]), (c, dec[c], odec[c])
    return opi, orec, odec, ofx


@pytest.mark.parametrize("cid,alg,n,count,kw", EPS_CASES, ids=[c[0] for c in EPS_CASES])
def test_gpu_epsilon_matches_oracle(cid, alg, n, count, kw, oracle_mod):
    begin = 777
    with psync.GpuRound(alg, n, batch_capacity=count, **kw) as gr:
        res = gr.run(begin, count, per_instance=True)
        dec, dround = gr.decisions()
        sample = [begin + i for i in range(0, count, max(1, count // 23))]
        fsums, frecs, fdec, ffx = gr.fetch_real(sample)
    opi, orec, odec, ofx = _check_eps(gr, res, dec, dround, begin, count, oracle_mod=oracle_mod)
    for j, inst in enumerate(sample):
        i = inst - begin
        assert _inst_tuple(fsums[j]) == _inst_tuple(opi[i])
        for p in range(n):
            assert _rec_tuple(frecs[j * n + p]) == _rec_tuple(orec[i * n + p]), (inst, p)
            assert _close(fdec[j * n + p], odec[i * n + p]) and _close(ffx[j * n + p], ofx[i * n + p]), (inst, p)


@pytest.mark.parametrize("n,f,dup", [(16, 2, 0.3), (33, 3, 0.6), (64, 5, 0.9)])
def test_gpu_epsilon_host_inputs(n, f, dup, oracle_mod):
    """psg_load_inputs_f64: caller Doubles incl. negatives, -0.0 / 0.0, duplicates and NaN.
    n = 33 crosses the 32-position halves of the sorted-membership mask; n = 64 with 90 %
    pooled values is tie-heavy (equal sort keys ordered by pid in the bitonic network)."""
    import random
    rng = random.Random(9 + n)
    count = 400
    pool = [0.0, -0.0, 1.0, -1.0, 0.5, 0.5, 1e-300, -1e300, float("nan")]
    init = [[rng.choice(pool) if rng.random() < dup else rng.uniform(-5, 5) for _ in range(n)]
            for _ in range(count)]
    with psync.GpuRound(psync.EpsilonConsensus(f, 1e-3), n, seed=70, batch_capacity=count) as gr:
        gr.load_inputs(5, count, init)
        res = gr.run(5, count, per_instance=True)
        dec, dround = gr.decisions()
    _check_eps(gr, res, dec, dround, 5, count, init=init, oracle_mod=oracle_mod)


@pytest.mark.gpu
@pytest.mark.parametrize("n,f", [(64, 5), (40, 4)])
def test_gpu_epsilon_keys_within_64_ulp_against_pid_order(n, f, oracle_mod):
    """Initial values a few ulp apart, descending by pid: the one-word sort (top 58 key bits,
    ties by pid) leaves them against their (key, pid) order, so its adjacent-key test must send
    every such round to the (key, pid) network (psg_epsilon.hip). Later rounds' means are
    also within a few ulp of each other."""
    import random
    import struct
    rng = random.Random(31 + n)
    count = 200

    def ulps(x, k):
        return struct.unpack("<d", struct.pack("<q", struct.unpack("<q", struct.pack("<d", x))[0] + k))[0]

    init = []
    for i in range(count):
        base = rng.uniform(0.1, 4.0) * (-1 if i % 3 == 0 else 1)
        init.append([ulps(base, (n - p) * (1 + i % 3)) for p in range(n)])
    with psync.GpuRound(psync.EpsilonConsensus(f, 1e-15), n, seed=71, batch_capacity=count) as gr:
        gr.load_inputs(0, count, init)
        res = gr.run(0, count, per_instance=True)
        dec, dround = gr.decisions()
    _check_eps(gr, res, dec, dround, 0, count, init=init, oracle_mod=oracle_mod)
