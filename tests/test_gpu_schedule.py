"""GPU parity of explicit HO schedules (psg_load_schedule / psg_materialize_schedule),
the adversary search and record-file replay.

Bit-exact against the CPU oracle under the same explicit schedules: per-instance
summaries (digest, first failing check point of every slot, termination round),
batch counters and per-process decide results. Seeded schedules exported by
the GPU equal the oracle's restatement of the generator word for word, and
replaying them as explicit schedules reproduces the seeded run.
"""
import os

import numpy as np
import pytest

from round_amd import abi, adversary as A, lib, psync, records, schedules as S

pytestmark = pytest.mark.gpu

H = psync.HOSchedule

ALGS = [
    ("otr-n64", psync.OTR(), 64, 12, 4, "omission"),
    ("otr-n17", psync.OTR(), 17, 10, 3, "omission"),
    ("otr-n200", psync.OTR(), 200, 8, 3, "omission"),
    ("otr2-n100", psync.OTR2(), 100, 8, 3, "omission"),
    ("lv-n64", psync.LastVoting(), 64, 16, 5, "omission"),
    ("lv-n130", psync.LastVoting(), 130, 12, 5, "omission"),
    ("slv-n64", psync.ShortLastVoting(), 64, 15, 5, "omission"),
    ("benor-n128", psync.BenOr(), 128, 16, 2, "omission"),
    ("benor-n8", psync.BenOr(), 8, 20, 2, "omission"),
    ("eps-n40", psync.EpsilonConsensus(f=2, epsilon=1e-3), 40, 8, 0, "omission"),
    ("fm-n256", psync.FloodMin(3), 256, 5, 1000, "crash"),
    ("fm-n64", psync.FloodMin(4), 64, 6, 1000, "crash"),
    ("kset-n100", psync.KSetAgreement(3), 100, 10, 1000, "crash"),
    ("kses-n70", psync.KSetEarlyStopping(t=4, k=2), 70, 5, 1000, "crash"),
]


def _schedule(rng, alg, n, R, I, family):
    if family == "crash":
        fmax = max(1, alg.param)
        crash, partial = S.random_crash(rng, I, R, n, fmax, p_partial=(0.1, 0.5, 0.9))
        ho = S.crash_to_ho(crash, partial, R, n)
        # a little benign loss on top, so explicit sets are not crash patterns only
        ho &= ~(S.random_bits(rng, ho.shape, 1 / 64) & ~S.self_mask(n)[None, None])
        return ho, crash
    ho = S.random_omission(rng, I, R, n, 0.8)
    if alg.alg_id == abi.PSG_ALG_BENOR:
        S.repair_min_size(ho, rng, n, n // 2 + 1)
    if alg.alg_id == abi.PSG_ALG_EPSILON:
        S.repair_min_size(ho, rng, n, n - alg.param)
    return ho, None


def _init(rng, alg, I, n, V):
    if alg.real:
        return rng.random((I, n))
    if alg.alg_id == abi.PSG_ALG_BENOR:
        return rng.integers(0, 2, (I, n), dtype=np.int32)
    return rng.integers(1, V + 1, (I, n), dtype=np.int32)


def _cmp_summaries(gpu_pi, opi, k):
    for j, (a, b) in enumerate(zip(gpu_pi, opi)):
        assert int(a["digest"]) == b.digest, f"instance {j}: digest"
        assert list(a["first_fail"][:k]) == list(b.first_fail)[:k], f"instance {j}: first_fail"
        assert int(a["term_round"]) == b.term_round, f"instance {j}: term_round"


@pytest.mark.parametrize("name,alg,n,R,V,family", ALGS, ids=[a[0] for a in ALGS])
def test_explicit_schedule_matches_oracle(name, alg, n, R, V, family, oracle_mod):
    rng = np.random.default_rng(abs(hash(name)) % 2 ** 32)
    I = 300 if n <= 64 else 80
    begin = 1000
    ho, crash = _schedule(rng, alg, n, R, I, family)
    init = _init(rng, alg, I, n, V)
    with psync.GpuRound(alg, n, R, seed=5, value_range=max(V, 1), batch_capacity=I) as g:
        ctx = g._ctx
        ctx.load_inputs(begin, I, init)
        ctx.load_schedule(begin, I, ho, crash)
        s, pi = ctx.run_batch_np(begin, I)
        dec, dr = ctx.copy_decisions_np()
        # fetch: staged inputs + loaded schedule, any subset of ids in range
        ids = [begin + 7, begin + I - 1, begin]
        fs, fr = ctx.fetch_np(ids)
    osum, opi, orec, odec, _ = oracle_mod.run_schedule(g.cfg, begin, I, ho, crash, init, per_instance=True,
                                                        records=True)
    k = len(alg.check_names)
    _cmp_summaries(pi, opi, k)
    assert list(s.fail_count) == list(osum.fail_count)
    assert s.digest == osum.digest
    assert list(s.term_hist)[:R + 2] == list(osum.term_hist)[:R + 2]
    ord_ = np.array([(r.decision, r.decision_round) for r in orec]).reshape(I, n, 2)
    assert (dr == ord_[:, :, 1]).all()
    if alg.real:
        assert np.allclose(dec, odec.reshape(I, n), atol=1e-12, rtol=0, equal_nan=True)
    else:
        assert (dec == ord_[:, :, 0]).all()
    for j, iid in enumerate(ids):
        assert int(fs[j]["digest"]) == int(pi[iid - begin]["digest"])
        assert list(fr[j]["decision_round"]) == list(ord_[iid - begin, :, 1])


CFG_CASES = [
    ("otr", psync.OTR(), 64, dict(value_range=4)),
    ("otr-goodmin", psync.OTR(), 100, dict(schedule=H(drop_log2=2, good_round=0.5, good_min=70))),
    ("lv-crash", psync.LastVoting(), 64, {}),
    ("benor-homin", psync.BenOr(), 128, {}),
    ("fm-crash", psync.FloodMin(4), 256, {}),
    ("kset-crash-loss", psync.KSetAgreement(3), 130, dict(schedule=H(drop_log2=2, crash_fmax=5, good_round=0.3))),
    ("eps", psync.EpsilonConsensus(f=2, epsilon=1e-3), 40, {}),
    ("pure-ho", psync.OTR(), 12, dict(schedule=H(drop_log2=2, self_bit=False))),
]


@pytest.mark.parametrize("name,alg,n,kw", CFG_CASES, ids=[c[0] for c in CFG_CASES])
def test_materialized_schedule_matches_oracle_and_replays(name, alg, n, kw, oracle_mod):
    I, begin = 64, 555
    with psync.GpuRound(alg, n, seed=9, batch_capacity=I, **kw) as g:
        ho, crash = g.materialize_schedule(begin, I)
        oho, ocrash = oracle_mod.materialize_schedule(g.cfg, begin, I)
        assert (ho == oho).all() and (crash == ocrash).all()
        seeded = g.run(begin, I, per_instance=True)
        g.load_schedule(begin, I, ho, crash)
        replay = g.run(begin, I, per_instance=True)
        g.clear_schedule()
        again = g.run(begin, I, per_instance=True)
    assert seeded.summary.digest == replay.summary.digest == again.summary.digest
    for a, b in zip(seeded.per_instance, replay.per_instance):
        assert a.digest == b.digest and bytes(a.first_fail) == bytes(b.first_fail) and a.term_round == b.term_round


def test_schedule_range_errors():
    n, R, I = 16, 6, 10
    with psync.GpuRound(psync.OTR(), n, R, batch_capacity=I) as g:
        ho = S.random_omission(np.random.default_rng(0), I, R, n, 0.9)
        g.load_schedule(100, I, ho)
        with pytest.raises(lib.PsgError) as e:
            g.run(95, I)
        assert e.value.rc == abi.PSG_ERANGE
        with pytest.raises(lib.PsgError):
            g.fetch([100, 110])
        g.run(102, 5)  # a sub-range is fine
        with pytest.raises(lib.PsgError):
            g.load_schedule(0, I + 1, np.zeros((I + 1, R, n, 1), np.uint64))  # > batch_capacity
        with pytest.raises(ValueError):
            g.load_schedule(0, I, np.zeros((I, R, n + 1, 1), np.uint64))
        g.clear_schedule()
        g.run(95, I)


@pytest.mark.parametrize("mode", ["vm", "fused"])
def test_spec_program_under_explicit_schedule(oracle_mod, mode):
    """psg_run_batch_spec reads the loaded schedule too: the reference OTR Spec
    compiled from the DSL (interpreted, or fused into the explicit-schedule round
    kernel) equals the built-in checks on the same explicit sets."""
    from round_amd import formula
    n, R, I = 64, 10, 200
    rng = np.random.default_rng(3)
    ho = S.random_omission(rng, I, R, n, 0.75)
    init = rng.integers(1, 4, (I, n), dtype=np.int32)
    with psync.GpuRound(psync.OTR(), n, R, value_range=3, batch_capacity=I) as g:
        g._ctx.load_inputs(0, I, init)
        g.load_schedule(0, I, ho)
        _, pi = g._ctx.run_batch_np(0, I)
        spec = formula.otr_spec() if mode == "vm" else formula.compile_native(formula.otr_spec(), abi.PSG_ALG_OTR,
                                                                               fused=True, n=n)
        sr = g.run_spec(0, I, spec, per_instance=True)
    for a, b in zip(pi, sr.per_instance):
        assert list(a["first_fail"][:8]) == list(b.first_fail)[:8]
        assert int(a["term_round"]) == b.term_round


SEARCH_CASES = [
    ("otr-mutant-n64", psync.OTR(variant=1), 64, 8, ["Safety"], 3),
    ("otr-mutant-n16", psync.OTR(variant=1), 16, 8, ["Agreement"], 2),
    ("lv-mutant-n8", psync.LastVoting(variant=1), 8, 12, ["Agreement"], 3),
    ("fm-mutant-n8", psync.FloodMin(2, variant=1), 8, 4, None, 3),
    ("benor-mutant-n8", psync.BenOr(variant=1), 8, 12, None, 2),
    ("kses-mutant-n8", psync.KSetEarlyStopping(t=2, k=2, variant=1), 8, 4, None, 3),
]


@pytest.mark.parametrize("name,alg,n,R,targets,V", SEARCH_CASES, ids=[c[0] for c in SEARCH_CASES])
def test_adversary_finds_shrinks_and_replays(name, alg, n, R, targets, V, tmp_path, oracle_mod):
    with A.Adversary(alg, n, R, targets=targets, population=2048, values=V, seed=11) as adv:
        res = adv.search(generations=60, want=2)
        assert res.counterexamples, f"{name}: no counterexample in {res.schedules_evaluated} schedules"
        path = str(tmp_path / "cex.psgr")
        rec = A.save(path, adv, res.counterexamples, meta={"test": name})
    back = records.read(path)
    assert back.count == len(res.counterexamples) and back.class_name == alg.class_name
    # GPU replay from the file reproduces every recorded summary (raises otherwise)
    records.replay(path)
    # and the oracle agrees with the file under the same schedule
    for j in range(back.count):
        _, opi, _, _, _ = oracle_mod.run_schedule(back.cfg, int(back.ids[j]), 1, back.ho[j:j + 1],
                                                  None if back.crash is None else back.crash[j:j + 1],
                                                  back.init[j:j + 1], per_instance=True)
        assert opi[0].digest == int(back.summary[j]["digest"])
        assert bytes(opi[0].first_fail)[:len(back.slot_names)] == bytes(back.summary[j]["first_fail"])[
            :len(back.slot_names)]
    for c in res.counterexamples:
        assert c.violated and c.check_point < abi.PSG_NEVER


@pytest.mark.parametrize("alg,n,R", [(psync.OTR(), 64, 8), (psync.LastVoting(), 16, 12),
                                     (psync.FloodMin(2), 16, 4)], ids=["otr", "lv", "floodmin"])
def test_adversary_reference_algorithms_hold(alg, n, R):
    """The reference algorithms under their fault models: no violation found."""
    with A.Adversary(alg, n, R, population=4096, values=3, seed=12) as adv:
        res = adv.search(generations=15, want=1, shrink=False)
    assert not res.counterexamples, A.describe(res.counterexamples[0], n)
    assert res.schedules_evaluated == 15 * 4096


def test_adversary_benor_respects_safety_predicate():
    """BenOr under its safetyPredicate (|HO(p)| > n/2 on the given sets): every
    violation found has the predicate already broken on the effective sets
    (deciders exit), so none counts as a counterexample."""
    n, R = 16, 16
    with A.Adversary(psync.BenOr(), n, R, population=4096, seed=13) as adv:
        res = adv.search(generations=10, want=1, shrink=False)
    assert not res.counterexamples


def test_adversary_liveness_otr_two_good_rounds():
    """OTR's livenessPredicate (two good rounds, example/Otr.scala:96-97) at rounds
    0 and 1: every instance terminates (the progress VCs of the Verifier, concretely)."""
    n, R = 32, 6
    with A.Adversary(psync.OTR(), n, R, mode="liveness", live_at=[0, 1], population=2048, seed=14) as adv:
        res = adv.search(generations=5, want=1, shrink=False)
    assert not res.counterexamples


# ---------------------------------------------------------------- device-resident search populations

def _pop_params(seed=5, gen=0, flips=6, min_size=0, self_bit=1, keep=(128, 192, 224, 256), V=3, redraw=5):
    p = abi.PopulationParams()
    p.seed, p.generation, p.flips, p.min_size, p.self_bit = seed, gen, flips, min_size, self_bit
    for j, k in enumerate(keep):
        p.keep_p256[j] = k
    p.value_range, p.redraw_p256 = V, redraw
    return p


def _bits(ho, n):
    return np.unpackbits(ho.view(np.uint8), bitorder="little").reshape(ho.shape[:-1] + (-1,))[..., :n]


@pytest.mark.parametrize("alg,n", [(psync.OTR(), 64), (psync.BenOr(), 70)], ids=["otr-n64", "benor-n70"])
def test_population_fresh_properties(alg, n):
    P, R = 400, 6
    min_size = n // 2 + 1 if alg.alg_id == abi.PSG_ALG_BENOR else 0
    with psync.GpuRound(alg, n, R, batch_capacity=P) as g:
        g._ctx.population_fresh(10, P, _pop_params(min_size=min_size))
        ho, init = g._ctx.population_read(np.arange(P))
    b = _bits(ho, n)
    assert (b[:, :, np.arange(n), np.arange(n)] == 1).all()                 # self bit
    W = (n + 63) // 64
    tail = _bits(ho, 64 * W)[..., n:]
    assert not tail.any()                                                  # no pid >= n
    sizes = b.sum(-1)
    assert (sizes >= min_size).all()
    assert (sizes[3::4] == n).all()                                        # keep 256/256: everyone
    if min_size == 0:
        off = b[0::4].sum() - P // 4 * R * n                               # keep 128/256, self bits aside
        assert abs(off / (P // 4 * R * n * (n - 1)) - 0.5) < 0.02
    if alg.alg_id == abi.PSG_ALG_BENOR:
        assert set(np.unique(init)) <= {0, 1}
    else:
        assert init.min() >= 1 and init.max() <= 3 and len(np.unique(init)) == 3


def test_population_next_ops_and_determinism(oracle_mod):
    n, R, P = 32, 5, 64
    flips = 7
    outs = []
    for _ in range(2):  # same parameters -> same populations (a pure function of them)
        with psync.GpuRound(psync.OTR(), n, R, batch_capacity=P, value_range=3) as g:
            ctx = g._ctx
            ctx.population_fresh(0, P, _pop_params(flips=flips))
            ho0, in0 = ctx.population_read(np.arange(P))
            parent = np.array([5] * 10 + [3] * 30 + [0] * (P - 40), np.uint32)
            op = np.array([0] * 10 + [1] * 30 + [2] * (P - 40), np.uint8)
            ctx.population_next(parent, op, _pop_params(gen=1, flips=flips))
            ho1, in1 = ctx.population_read(np.arange(P))
            _, pi = ctx.run_batch_np(0, P)
        outs.append((ho0, in0, ho1, in1, pi))
        # copies are exact, mutants differ from the parent in at most `flips` links
        assert (ho1[:10] == ho0[5]).all() and (in1[:10] == in0[5]).all()
        diff = (_bits(ho1[10:40], n) != _bits(ho0[3][None], n)).sum((1, 2, 3))
        assert (diff <= flips).all() and (diff > 0).any()
        assert (in1[10:40] != in0[3]).mean() < 0.2
        assert (_bits(ho1, n)[:, :, np.arange(n), np.arange(n)] == 1).all()
        # the kernels run exactly the loaded population (oracle under the read-back sets)
        _, opi, _, _, _ = oracle_mod.run_schedule(g.cfg, 0, P, ho1, None, in1, per_instance=True)
        assert [int(x["digest"]) for x in pi] == [x.digest for x in opi]
    a, b = outs
    assert all((x == y).all() for x, y in zip(a[:4], b[:4]))


def test_population_argument_errors():
    with psync.GpuRound(psync.OTR(), 16, 4, batch_capacity=8) as g:
        ctx = g._ctx
        with pytest.raises(lib.PsgError):
            ctx.population_next(np.zeros(8, np.uint32), np.zeros(8, np.uint8), _pop_params())  # nothing loaded
        ctx.population_fresh(0, 8, _pop_params())
        with pytest.raises(lib.PsgError):
            ctx.population_next(np.full(8, 9, np.uint32), np.ones(8, np.uint8), _pop_params())  # parent >= 8
        with pytest.raises(lib.PsgError):
            ctx.population_next(np.zeros(8, np.uint32), np.full(8, 3, np.uint8), _pop_params())  # bad op
        with pytest.raises(lib.PsgError):
            ctx.population_fresh(0, 9, _pop_params())  # > batch_capacity
        with pytest.raises(lib.PsgError):
            ctx.population_read(np.array([8], np.uint32))
    with psync.GpuRound(psync.EpsilonConsensus(), 8, 4, batch_capacity=8) as g:
        with pytest.raises(lib.PsgError):
            g._ctx.population_fresh(0, 8, _pop_params())


def test_device_and_host_search_paths_agree_on_outcome():
    """The device-population search and the host one both find the OTR mutant."""
    for dp in (True, False):
        with A.Adversary(psync.OTR(variant=1), 16, 8, targets=["Agreement"], population=2048, values=2, seed=3,
                         device_pop=dp) as adv:
            assert adv.device_population() == dp
            res = adv.search(generations=40, want=1)
        assert res.counterexamples and res.counterexamples[0].violated == ["Agreement"]
