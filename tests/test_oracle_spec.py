"""Spec evaluation properties of the CPU oracle.

1. The hand-lowered evaluator (what the GPU kernels implement) agrees with the
   Formula-tree interpreter (mirror of psync/formula/Formula.scala, lowering of
   psync/macros/FormulaExtractor.scala) on every check point of random runs.
2. Zero false positives: the verified algorithms never violate their Spec on
   schedules that satisfy the Spec's environment assumptions.
3. Mutation tests: weakened algorithms are caught.
"""
import pytest

from round_amd import abi, psync

H = psync.HOSchedule
NEVER = abi.PSG_NEVER


@pytest.mark.parametrize("alg,n,kw", [
    (psync.OTR(), 4, {}),
    (psync.OTR(), 6, dict(value_range=3, schedule=H(drop_log2=1))),
    (psync.OTR(variant=1), 8, dict(schedule=H(drop_log2=1, good_round=0.0))),
    (psync.OTR(), 5, dict(schedule=H(drop_log2=2, self_bit=False))),
    (psync.LastVoting(), 4, dict(value_range=4)),
    (psync.LastVoting(), 5, dict(value_range=3, schedule=H(drop_log2=1, good_round=0.0, crash_fmax=2))),
    (psync.LastVoting(variant=1), 6, dict(value_range=5)),
    (psync.LastVoting(), 7, dict(tiebreak=abi.PSG_TIE_MIN_PID)),
    (psync.BenOr(), 4, {}),
    (psync.BenOr(), 7, dict(schedule=H(drop_log2=1, good_round=0.0, ho_min=3))),
    (psync.BenOr(variant=1), 6, {}),
    (psync.OTR2(), 4, {}),
    (psync.OTR2(), 6, dict(value_range=3, schedule=H(drop_log2=1))),
    (psync.OTR2(variant=1), 8, dict(schedule=H(drop_log2=1, good_round=0.0))),
], ids=lambda v: getattr(v, "class_name", None) or None)
def test_lowered_spec_matches_formula_interpreter(alg, n, kw, oracle_mod):
    cfg = psync.make_config(alg, n, seed=11, **kw)
    # SPEC_BOTH raises on the first check point where the two evaluators disagree
    oracle_mod.run(cfg, 0, 400, spec_mode=oracle_mod.SPEC_BOTH, threads=8)


@pytest.mark.parametrize("alg,n,kw", [
    (psync.OTR(), 64, dict(value_range=64)),
    (psync.OTR(), 64, dict(value_range=2, schedule=H(drop_log2=1, good_round=0.1))),
    (psync.OTR(), 16, dict(schedule=H(drop_log2=2, crash_fmax=8))),
    (psync.LastVoting(), 64, {}),
    (psync.LastVoting(), 16, dict(value_range=3, schedule=H(drop_log2=1, good_round=0.0, crash_fmax=12))),
    (psync.FloodMin(4), 64, {}),
    (psync.FloodMin(8), 32, dict(schedule=H(drop_log2=0, good_round=0.0, crash_fmax=8))),
    (psync.KSetAgreement(2), 32, {}),
    (psync.KSetAgreement(3), 24, dict(schedule=H(drop_log2=0, good_round=0.0, crash_fmax=2))),
    (psync.OTR2(), 64, dict(value_range=64)),
    (psync.OTR2(), 16, dict(schedule=H(drop_log2=2, crash_fmax=8))),
    (psync.ShortLastVoting(), 64, {}),
    (psync.ShortLastVoting(), 16, dict(value_range=5, schedule=H(drop_log2=1, good_round=0.0, crash_fmax=7))),
    (psync.KSetEarlyStopping(8, 2), 64, {}),
    (psync.KSetEarlyStopping(4, 2), 16, {}),
])
def test_zero_false_positives(alg, n, kw, oracle_mod):
    cfg = psync.make_config(alg, n, seed=21, **kw)
    s, _, _ = oracle_mod.run(cfg, 0, 1500, threads=8)
    bad = {abi.CHECK_NAMES[alg.alg_id][i]: s.fail_count[i] for i in alg.violation_slots if s.fail_count[i]}
    assert not bad, bad


@pytest.mark.parametrize("alg,n,kw", [
    (psync.EpsilonConsensus(1, 0.1), 7, {}),
    (psync.EpsilonConsensus(2, 1e-3), 16, {}),
    (psync.EpsilonConsensus(5, 1e-6), 64, {}),
    (psync.EpsilonConsensus(1, 0.1), 7, dict(schedule=H(drop_log2=1, good_round=0.0))),
])
def test_epsilon_violations_only_after_safety_predicate_breaks(alg, n, kw, oracle_mod):
    """Approximate agreement / validity hold in every instance whose processes always had
    |V| >= n - f values (Epsilon.scala:57); with heavy loss the assumption breaks and
    violations appear only after it has."""
    cfg = psync.make_config(alg, n, seed=33, **kw)
    _, pi, _, _, _ = oracle_mod.run_real(cfg, 0, 1500, per_instance=True, threads=8)
    for s in pi:
        for slot in (0, 1):
            if s.first_fail[slot] != NEVER:
                assert s.first_fail[2] != NEVER and s.first_fail[2] <= s.first_fail[slot]


def test_epsilon_mutant_is_caught(oracle_mod):
    cfg = psync.make_config(psync.EpsilonConsensus(1, 0.01, variant=1), 7, seed=34,
                            schedule=H(drop_log2=2, good_round=0.0, ho_min=5))
    s, pi, _, _, _ = oracle_mod.run_real(cfg, 0, 2000, per_instance=True, threads=8)
    assert sum(1 for x in pi if x.first_fail[0] != NEVER and x.first_fail[2] == NEVER) > 0


@pytest.mark.parametrize("n", [4, 8, 16])
def test_benor_violations_only_after_safety_predicate_breaks(n, oracle_mod):
    """BenOr's invariant assumes |HO(p)| > n/2 (BenOr.scala:92). Deciders exit, so
    the effective heard-of sets shrink and the assumption can break; no
    violation may precede that."""
    cfg = psync.make_config(psync.BenOr(), n, seed=31)
    _, pi, _ = oracle_mod.run(cfg, 0, 2000, per_instance=True, threads=8)
    viol = 0
    for s in pi:
        pred = s.first_fail[4]
        for slot in (0, 2, 3):
            if s.first_fail[slot] != NEVER:
                viol += 1
                assert pred != NEVER and pred <= s.first_fail[slot]
    assert viol > 0  # the situation does occur at these sizes


@pytest.mark.parametrize("alg,n,kw,slots", [
    (psync.OTR(variant=1), 8, dict(schedule=H(drop_log2=1, good_round=0.0)), [0, 4]),
    (psync.LastVoting(variant=1), 16, dict(value_range=5, schedule=H(drop_log2=1, good_round=0.0, crash_fmax=7)),
     [0, 3]),
    (psync.BenOr(variant=1), 8, {}, [0, 2]),
    (psync.KSetAgreement(2, variant=1), 16, dict(schedule=H(drop_log2=0, good_round=0.0, crash_fmax=4)), [0]),
    (psync.OTR2(variant=1), 8, dict(schedule=H(drop_log2=1, good_round=0.0)), [0, 4]),
    (psync.ShortLastVoting(variant=1), 16, dict(value_range=5, schedule=H(drop_log2=1, good_round=0.0,
                                                                          crash_fmax=7)), [0]),
    (psync.KSetEarlyStopping(4, 2, variant=1), 16, {}, [0]),
])
def test_mutants_are_caught(alg, n, kw, slots, oracle_mod):
    cfg = psync.make_config(alg, n, seed=77, **kw)
    s, _, _ = oracle_mod.run(cfg, 0, 3000, threads=8)
    for slot in slots:
        assert s.fail_count[slot] > 0, abi.CHECK_NAMES[alg.alg_id][slot]


def test_floodmin_early_decision_mutant_explicit(oracle_mod):
    """FloodMin deciding after f exchange rounds instead of f+2 (variant 1) disagrees
    when each round hides the minimum behind a crash: p0 holds 1 and crashes in
    round 0 reaching only p1, which crashes in round 1 reaching only p2 ..."""
    n, f = 6, 3
    cfg = psync.make_config(psync.FloodMin(f, variant=1), n, rounds=f + 2, value_range=100,
                            schedule=H(drop_log2=0, good_round=0.0, crash_fmax=-1))
    full = (1 << n) - 1
    # round k: processes 0..k-1 silent (crashed before), process k reaches only k+1
    ho = []
    for k in range(f + 2):
        row = []
        for p in range(n):
            m = full
            for q in range(min(k, n)):
                m &= ~(1 << q)
            if k < n and p != k + 1:
                m &= ~(1 << k)
            row.append(m | (1 << p))
        ho.append(row)
    s, rec, _ = oracle_mod.run_explicit(cfg, [1, 50, 60, 70, 80, 90], ho, spec_mode=oracle_mod.SPEC_DIRECT)
    decided = {r.decision for r in rec if r.decision_round >= 0}
    assert len(decided) > 1  # early deciders disagree
    cfg0 = psync.make_config(psync.FloodMin(f), n, rounds=f + 2, value_range=100,
                             schedule=H(drop_log2=0, good_round=0.0, crash_fmax=-1))
    s0, rec0, _ = oracle_mod.run_explicit(cfg0, [1, 50, 60, 70, 80, 90], ho, spec_mode=oracle_mod.SPEC_DIRECT)
    assert len({r.decision for r in rec0[f + 1:]}) == 1
