"""GPU: compiled Spec programs (psg_run_batch_spec, psg_spec_vm.hip).

1. The reference Specs compiled from the Python DSL and evaluated on the device —
   by the bytecode interpreter and as native lowered wave code (compile_native) —
   give exactly the per-instance results of the hand-lowered kernels (same run:
   digests, first failing check point per slot, termination).
2. Custom specs: both device paths over the device trace == CPU interpreter over
   the oracle trace, bit for bit, incl. n > 64 (lane quantifiers in 64-pid passes).
"""
import pytest

from round_amd import abi, formula as F, psync

import spec_cases

pytestmark = pytest.mark.gpu
H = psync.HOSchedule

REF = [
    ("otr-n64", psync.OTR(), 64, 600, dict(value_range=8, seed=3)),
    ("otr-mutant-n8", psync.OTR(variant=1), 8, 2000, dict(schedule=H(drop_log2=1, good_round=0.0), seed=4)),
    ("otr-n100-W2", psync.OTR(), 100, 100, dict(value_range=4, seed=5)),
    ("otr2-n64", psync.OTR2(), 64, 500, dict(value_range=4, seed=6)),
    ("lv-n16-loss", psync.LastVoting(), 16, 500, dict(value_range=3, seed=7, schedule=H(
        drop_log2=1, good_round=0.0, crash_fmax=7))),
    ("lv-mutant-n6", psync.LastVoting(variant=1), 6, 1500, dict(value_range=5, seed=8)),
    ("lv-n64", psync.LastVoting(), 64, 200, dict(seed=9, rounds=12)),
    ("benor-n8", psync.BenOr(), 8, 1500, dict(seed=10)),
    ("benor-n128-W2", psync.BenOr(), 128, 40, dict(seed=11, rounds=16)),
]


def _rows(pi, k):
    return [(tuple(s.first_fail)[:k], s.term_round) for s in pi]


def _prog(spec, alg_id, mode, n=None):
    if mode == "fused":  # the round kernel instantiated with the Spec as its hook: no trace
        return F.compile_native(spec, alg_id, fused=True, n=n)
    return F.compile_native(spec, alg_id) if mode == "native" else F.compile_spec(spec, alg_id)


@pytest.mark.parametrize("mode", ["vm", "native", "fused"])
@pytest.mark.parametrize("cid,alg,n,count,kw", REF, ids=[c[0] for c in REF])
def test_reference_spec_program_matches_builtin_checks(cid, alg, n, count, kw, mode):
    prog = _prog(F.REFERENCE_SPECS[alg.alg_id](), alg.alg_id, mode, n)
    k = len(prog.slot_names)
    with psync.GpuRound(alg, n, batch_capacity=count, **kw) as gr:
        built = gr.run(0, count, per_instance=True)
        spec = gr.run_spec(0, count, prog, per_instance=True)
    assert _rows(spec.per_instance, k) == _rows(built.per_instance, k)
    assert [s.digest for s in spec.per_instance] == [s.digest for s in built.per_instance]
    assert list(spec.summary.fail_count)[:k] == list(built.summary.fail_count)[:k]
    assert spec.summary.digest == built.summary.digest


@pytest.mark.parametrize("mode", ["vm", "native", "fused"])
@pytest.mark.parametrize("cid,alg,n,kw,mk", spec_cases.CUSTOM, ids=[c[0] for c in spec_cases.CUSTOM])
def test_custom_spec_matches_cpu_interpreter(cid, alg, n, kw, mk, oracle_mod, mode):
    prog = _prog(mk(), alg.alg_id, mode, n)
    count = 300 if n <= 16 else 60
    with psync.GpuRound(alg, n, batch_capacity=count, seed=19, **kw) as gr:
        res = gr.run_spec(100, count, prog, per_instance=True)
    cfg = gr.cfg
    tr = oracle_mod.trace(cfg, 100, count)
    ff, tm = oracle_mod.vm_run(prog, tr, count, n, cfg.rounds)
    k = len(prog.slot_names)
    got = _rows(res.per_instance, k)
    assert got == [(tuple(f), t) for f, t in zip(ff, tm)]
    # counters agree with the per-instance view
    for s in range(k):
        assert res.summary.fail_count[s] == sum(1 for f in ff if f[s] != abi.PSG_NEVER)


def test_spec_program_chunking_and_staged_inputs(oracle_mod, monkeypatch):
    """Host-supplied inputs + a batch spanning several trace chunks (1 MiB budget)."""
    n, count = 16, 3000  # 2880 B of trace per instance: 365 instances per chunk
    monkeypatch.setenv("PSG_SPEC_TRACE_MB", "1")
    init = [[(i + 3 * p) % 5 + 1 for p in range(n)] for i in range(count)]
    prog = F.compile_spec(spec_cases.uniform_agreement(), abi.PSG_ALG_FLOODMIN)
    with psync.GpuRound(psync.FloodMin(2), n, seed=23, value_range=8, batch_capacity=count) as gr:
        gr.load_inputs(0, count, init)
        res = gr.run_spec(0, count, prog, per_instance=True)
        built = gr.run(0, count, per_instance=True)
    assert res.summary.instances == count
    assert [s.digest for s in res.per_instance] == [s.digest for s in built.per_instance]
    cfg = gr.cfg
    tr = oracle_mod.trace(cfg, 0, count, init=init)
    ff, tm = oracle_mod.vm_run(prog, tr, count, n, cfg.rounds)
    assert _rows(res.per_instance, len(prog.slot_names)) == [(tuple(f), t) for f, t in zip(ff, tm)]


def test_bad_program_is_rejected():
    from round_amd.lib import PsgError
    prog = F.compile_spec(spec_cases.uniform_agreement(), abi.PSG_ALG_FLOODMIN)
    prog.code[0] = 0x7F  # unknown opcode
    with psync.GpuRound(psync.FloodMin(2), 8, batch_capacity=4) as gr:
        with pytest.raises(PsgError):
            gr.run_spec(0, 4, prog)
