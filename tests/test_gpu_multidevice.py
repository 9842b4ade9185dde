"""Multi-device contexts (psg_config.n_devices, SURVEY §8b "multi-GPU runs inside one
context, with one host thread per device"). The leased box has one GPU, so the
device list is [0, 0]: two per-device contexts on the same card, each with its own
stream, buffers and host thread. A multi-device run must equal the single-device
run bit for bit: summaries (every counter but kernel_ns), per-instance summaries,
decisions, fetched records, explicit schedules and Spec programs.
"""
import numpy as np
import pytest

from round_amd import abi, psync
from round_amd.lib import PsgError

pytestmark = pytest.mark.gpu


def _sum(s):
    return abi.summary_to_list(s)[:-1]


def _pi(res):
    return [(s.digest, tuple(s.first_fail), s.term_round, s.n_decided) for s in res.per_instance]


CASES = [
    ("otr-n64", psync.OTR(), 64, 20_001, dict(value_range=64, seed=2)),
    ("lv-n64", psync.LastVoting(), 64, 5_003, dict(seed=11)),
    ("floodmin-n256", psync.FloodMin(8), 256, 1_001, dict(seed=17)),
    ("benor-n128", psync.BenOr(), 128, 2_000, dict(seed=25)),
    ("kset-n256", psync.KSetAgreement(2), 256, 97, dict(seed=21)),
]


@pytest.mark.parametrize("cid,alg,n,count,kw", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]], ids=["x2", "x3"])
def test_multi_equals_single(cid, alg, n, count, kw, devices):
    begin = 123_456
    with psync.GpuRound(alg, n, batch_capacity=count, **kw) as one:
        r1 = one.run(begin, count, per_instance=True)
        d1 = one.decisions()
        f1 = one.fetch([begin, begin + count // 2, begin + count - 1, 7])
    with psync.GpuRound(alg, n, batch_capacity=count, devices=devices, **kw) as many:
        r2 = many.run(begin, count, per_instance=True)
        d2 = many.decisions()
        f2 = many.fetch([begin, begin + count // 2, begin + count - 1, 7])
    assert _sum(r2.summary) == _sum(r1.summary)
    assert _pi(r2) == _pi(r1)
    assert d2 == d1
    assert [(s.digest, s.term_round) for s in f2[0]] == [(s.digest, s.term_round) for s in f1[0]]
    assert [(r.decision, r.decision_round, r.halt_round, r.final_x) for r in f2[1]] == \
           [(r.decision, r.decision_round, r.halt_round, r.final_x) for r in f1[1]]


def test_multi_host_inputs_and_fetch():
    """Staged host inputs are split by slice; fetch routes each id to its slice's device."""
    n, count, begin = 64, 3001, 40
    rng = np.random.default_rng(3)
    init = rng.integers(1, 6, size=(count, n), dtype=np.int32)
    ids = [begin, begin + 1, begin + 1499, begin + 1500, begin + 1501, begin + count - 1]
    out = []
    for devices in (None, [0, 0]):
        with psync.GpuRound(psync.OTR(), n, seed=31, batch_capacity=count, devices=devices) as g:
            g.load_inputs(begin, count, init)
            r = g.run(begin, count, per_instance=True)
            f = g.fetch(ids)
            out.append((_sum(r.summary), _pi(r), [s.digest for s in f[0]]))
    assert out[0] == out[1]


def test_multi_epsilon_f64():
    n, count = 64, 1001
    alg = psync.EpsilonConsensus(5, 1e-6)
    res = []
    for devices in (None, [0, 0]):
        with psync.GpuRound(alg, n, seed=62, batch_capacity=count, devices=devices) as g:
            r = g.run(5, count, per_instance=True)
            dec, dr = g.decisions()
            res.append((_sum(r.summary), _pi(r), [float(x).hex() for x in dec], list(dr)))
    assert res[0] == res[1]


def test_multi_explicit_schedule_and_spec():
    """Explicit schedules are split like the batch; Spec programs run per device."""
    from round_amd import formula
    n, count, begin = 64, 1000, 500
    with psync.GpuRound(psync.OTR(), n, seed=5, value_range=4, batch_capacity=count) as g:
        ho, crash = g.materialize_schedule(begin, count)
    ho = ho.copy()
    ho[:, 3, :, 0] &= np.uint64(0x00FF00FF00FF00FF)  # a non-seeded round
    prog = formula.compile_spec(formula.otr_spec(), abi.PSG_ALG_OTR)
    out = []
    for devices in (None, [0, 0]):
        with psync.GpuRound(psync.OTR(), n, seed=5, value_range=4, batch_capacity=count, devices=devices) as g:
            ho2, _ = g.materialize_schedule(begin, count)
            g.load_schedule(begin, count, ho, crash)
            r = g.run(begin, count, per_instance=True)
            f = g.fetch([begin + 3, begin + 999, begin + 500])
            sp = g.run_spec(begin, count, prog, per_instance=True)
            out.append((ho2.tobytes(), _sum(r.summary), _pi(r), [s.digest for s in f[0]],
                        _sum(sp.summary), [tuple(s.first_fail) for s in sp.per_instance]))
    assert out[0] == out[1]
    # under a loaded schedule a multi-device run covers exactly its range
    with psync.GpuRound(psync.OTR(), n, seed=5, value_range=4, batch_capacity=count, devices=[0, 0]) as g:
        g.load_schedule(begin, count, ho, crash)
        with pytest.raises(PsgError):
            g.run(begin, count - 1)


def test_multi_population_refused():
    with psync.GpuRound(psync.OTR(), 16, batch_capacity=64, devices=[0, 0]) as g:
        p = abi.PopulationParams()
        p.seed, p.min_size, p.value_range = 1, 0, 3
        with pytest.raises(PsgError):
            g._ctx.population_fresh(0, 64, p)


def test_spec_program_algorithm_mismatch():
    """A Spec program compiled for OTR is refused by a LastVoting context, by the program's
    alg field (psync and the C ABI) and by the fused module's own psg_spec_alg."""
    from round_amd import formula
    fused = formula.compile_native(formula.otr_spec(), abi.PSG_ALG_OTR, fused=True, n=64)
    with psync.GpuRound(psync.LastVoting(), 64, seed=1, batch_capacity=64) as g:
        with pytest.raises(ValueError):
            g.run_spec(0, 64, fused)
        with pytest.raises(PsgError) as e:
            g._ctx.run_batch_spec(0, 64, fused, False)
        assert e.value.rc == abi.PSG_EINVAL
        fused.alg = 0  # unbound program: the module's psg_spec_alg still refuses it
        with pytest.raises(PsgError) as e:
            g._ctx.run_batch_spec(0, 64, fused, False)
        assert e.value.rc == abi.PSG_EINVAL
    # the same program runs on an OTR context
    with psync.GpuRound(psync.OTR(), 64, seed=1, batch_capacity=64) as g:
        fused.alg = abi.PSG_ALG_OTR
        g.run_spec(0, 64, fused)


@pytest.mark.parametrize("alg,n,kw", [(psync.OTR(), 64, dict(value_range=64, seed=2)),
                                      (psync.EpsilonConsensus(5, 1e-6), 64, dict(seed=62))],
                         ids=["otr", "epsilon-f64"])
def test_multi_small_batch_after_large(alg, n, kw):
    """a batch smaller than the device list leaves some device an empty
    slice; its decisions from an earlier, larger batch must not be copied (the host buffer
    is sized from the new count). Large batch, then 1 instance, then 0, on [0, 0]."""
    big, begin = 1000, 77
    with psync.GpuRound(alg, n, batch_capacity=big, **kw) as one:
        one.run(begin, 1)
        d_one = one.decisions()
    with psync.GpuRound(alg, n, batch_capacity=big, devices=[0, 0], **kw) as many:
        many.run(begin, big)
        assert many._ctx.last_batch_count() == big
        many.run(begin, 1)
        assert many._ctx.last_batch_count() == 1
        dec, dr = many.decisions()
        assert len(dec) == n and len(dr) == n
        assert [float(x).hex() for x in dec] == [float(x).hex() for x in d_one[0]] and dr == d_one[1]
        many.run(begin, 0)
        assert many._ctx.last_batch_count() == 0
        assert many.decisions() == ([], [])
