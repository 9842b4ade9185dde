"""Generic Spec programs (round_amd/formula.py -> include/psg.h bytecode), CPU side.

1. The reference Specs restated in the Python DSL, compiled and run by the CPU
   interpreter (oracle_vm_run) over oracle traces, reproduce the oracle's own
   checker (hand-lowered == Formula-tree interpreter) per instance.
2. Custom specs: compiled program == direct recursive evaluation with a
   brute-forced V.exists domain (tests/formula_ref.py).
3. Compiler errors for shapes the finitization cannot cover exactly.
"""
import pytest

from round_amd import abi, formula as F, psync

import formula_ref
import spec_cases

H = psync.HOSchedule


@pytest.mark.parametrize("alg,n,kw", [
    (psync.OTR(), 8, {}),
    (psync.OTR(), 16, dict(value_range=3, schedule=H(drop_log2=1))),
    (psync.OTR(variant=1), 8, dict(schedule=H(drop_log2=1, good_round=0.0))),
    (psync.OTR2(), 10, {}),
    (psync.LastVoting(), 8, dict(value_range=3, schedule=H(drop_log2=1, good_round=0.0, crash_fmax=3))),
    (psync.LastVoting(variant=1), 6, dict(value_range=5)),
    (psync.BenOr(), 8, {}),
    (psync.BenOr(variant=1), 6, {}),
], ids=lambda v: getattr(v, "class_name", None) or None)
def test_reference_specs_compile_to_the_oracle_checker(alg, n, kw, oracle_mod):
    cfg = psync.make_config(alg, n, seed=13, **kw)
    prog = F.compile_spec(F.REFERENCE_SPECS[alg.alg_id](), alg.alg_id)
    assert prog.slot_names == abi.CHECK_NAMES[alg.alg_id]
    cnt = 200
    tr = oracle_mod.trace(cfg, 0, cnt)
    ff, tm = oracle_mod.vm_run(prog, tr, cnt, n, cfg.rounds)
    _, pi, _ = oracle_mod.run(cfg, 0, cnt, per_instance=True, threads=8)
    k = len(prog.slot_names)
    for i in range(cnt):
        assert ff[i] == list(pi[i].first_fail)[:k] and tm[i] == pi[i].term_round, i


@pytest.mark.parametrize("cid,alg,n,kw,mk", [c for c in spec_cases.CUSTOM if c[2] <= 16],
                         ids=[c[0] for c in spec_cases.CUSTOM if c[2] <= 16])
def test_custom_specs_match_direct_evaluation(cid, alg, n, kw, mk, oracle_mod):
    cfg = psync.make_config(alg, n, seed=17, **kw)
    spec = mk()
    prog = F.compile_spec(spec, alg.alg_id)
    # the direct evaluation brute-forces nested V.exists domains in Python: fewer instances for the
    # larger / nested cases keeps the CPU suite within minutes
    cnt = 12 if n <= 12 and not cid.startswith("lv") else 4
    tr = oracle_mod.trace(cfg, 0, cnt)
    ff, tm = oracle_mod.vm_run(prog, tr, cnt, n, cfg.rounds)
    rf, rt = formula_ref.evaluate(spec, tr, cnt, n, cfg.rounds)
    assert ff == rf and tm == rt


REWRITE_CASES = [(f"ref-{a}", alg, n, kw, F.REFERENCE_SPECS[a]) for a, alg, n, kw in [
    (abi.PSG_ALG_OTR, psync.OTR(), 16, dict(value_range=3, schedule=H(drop_log2=1))),
    (abi.PSG_ALG_OTR2, psync.OTR2(), 10, {}),
    (abi.PSG_ALG_LAST_VOTING, psync.LastVoting(), 16, dict(value_range=3, schedule=H(
        drop_log2=1, good_round=0.0, crash_fmax=7))),
    (abi.PSG_ALG_LAST_VOTING, psync.LastVoting(variant=1), 6, dict(value_range=5)),
    (abi.PSG_ALG_BENOR, psync.BenOr(), 8, {})]] + [c for c in spec_cases.CUSTOM if c[2] <= 16]


def _rewritten(spec, alg_id):
    """The Spec after the library generator's rewrites (psg_spec_rewrite_text), back in the DSL."""
    from round_amd import lib
    return F.from_text(lib.spec_rewrite_text(F.to_text(spec), alg_id))


@pytest.mark.parametrize("cid,alg,n,kw,mk", REWRITE_CASES, ids=[c[0] for c in REWRITE_CASES])
def test_native_rewrites_are_exact(cid, alg, n, kw, mk, oracle_mod):
    """The rewrites of the native lowering (psg_spec_gen.cpp: conjuncts free of a bound
    variable hoisted out of V.exists / P.exists / P.forall, split foralls) give the same
    results as the Spec as written, under the CPU interpreter, check point by check point."""
    cfg = psync.make_config(alg, n, seed=29, **kw)
    spec = mk()
    cnt = 300
    tr = oracle_mod.trace(cfg, 0, cnt)
    f1, t1 = oracle_mod.vm_run(F.compile_spec(spec, alg.alg_id), tr, cnt, n, cfg.rounds)
    f2, t2 = oracle_mod.vm_run(F.compile_spec(_rewritten(spec, alg.alg_id), alg.alg_id), tr, cnt, n, cfg.rounds)
    assert f1 == f2 and t1 == t2


def test_rewrites_shapes():
    """The hoisting shapes: V.exists(v => A && B(v)) -> A && V.exists(v => B(v)) for
    a cross-lane A (LastVoting's `ts == r/4 ==> coord.commit`), and P.exists(j => P.forall(i =>
    i.decided && i.decision == init(j.x))) -> P.forall(i => i.decided) && P.exists(j => ...)."""
    P, V, init = F.P, F.V, F.init
    c = F.coord
    spec = F.Spec(properties=[
        ("A", V.exists(lambda v: P.forall(lambda i: (i.ts == F.r // 4).implies(F.Field(F.FIELD_COMMIT, c))
                                          & i.decided.implies(i.decision == v)))),
        ("B", P.exists(lambda j: P.forall(lambda i: i.decided & (i.decision == init(j.x)))))])
    rw = _rewritten(spec, abi.PSG_ALG_LAST_VOTING)
    a, b = [f for _, f in rw.properties]
    assert isinstance(a, F.Bin) and a.op == "AND"
    assert isinstance(a.x, F.Quant) and a.x.kind == "forall"   # the coord.commit implication, out of V.exists
    assert isinstance(a.y, F.Quant) and a.y.kind == "vint"
    assert isinstance(b, F.Bin) and b.op == "AND"
    assert isinstance(b.x, F.Quant) and b.x.kind == "forall"   # P.forall(i => i.decided), hoisted
    assert isinstance(b.y, F.Quant) and b.y.kind == "exists"


def test_custom_specs_find_violations(oracle_mod):
    """A false property is reported at the first check point it fails."""
    spec = F.Spec(properties=[("NobodyDecides", F.P.forall(lambda i: ~i.decided))])
    cfg = psync.make_config(psync.FloodMin(1), 6, seed=3, value_range=5)
    prog = F.compile_spec(spec, abi.PSG_ALG_FLOODMIN)
    tr = oracle_mod.trace(cfg, 0, 10)
    ff, _ = oracle_mod.vm_run(prog, tr, 10, 6, cfg.rounds)
    assert all(f == [3] for f in ff)  # FloodMin(f=1) decides in round k = 2 (first r > f): check point 3


def test_compiler_rejects_inexact_witness_shapes():
    P, V = F.P, F.V
    with pytest.raises(F.FormulaError):  # v used in arithmetic
        F.compile_spec(F.Spec([V.exists(lambda v: P.forall(lambda i: i.x + 1 == v * 2))]))
    with pytest.raises(F.FormulaError):  # field of the wrong algorithm
        F.compile_spec(F.Spec([P.forall(lambda i: i.ts >= 0)]), abi.PSG_ALG_OTR)
    with pytest.raises(F.FormulaError):  # Python boolean operators on formulas
        F.compile_spec(F.Spec([P.forall(lambda i: i.decided and i.x > 0)]))


def test_program_layout():
    prog = F.compile_spec(F.otr_spec(), abi.PSG_ALG_OTR)
    assert prog.term_entry >= 0 and prog.n_vars <= 16
    assert prog.slot_flags == [0, 0, 0, 0, 0, 0, 0, F.SPEC_RELATIONAL]
    assert all(prog.code[e - 1] & 0xFF == 0 or e == 0 for e in prog.slot_entry)  # each root follows a HALT


@pytest.mark.parametrize("name", ["otr", "otr2", "lv", "benor", "custom", "termcse"])
def test_native_lowering_builds(name):
    """compile_native (the library's generator + hiprtc) builds a gfx950 module (no GPU needed)."""
    specs = {"otr": (F.otr_spec, abi.PSG_ALG_OTR), "otr2": (F.otr2_spec, abi.PSG_ALG_OTR2),
             "lv": (F.lv_spec, abi.PSG_ALG_LAST_VOTING), "benor": (F.benor_spec, abi.PSG_ALG_BENOR),
             "custom": (spec_cases.lv_custom, abi.PSG_ALG_LAST_VOTING),
             "termcse": (spec_cases.term_shared_shapes, abi.PSG_ALG_OTR)}
    mk, alg = specs[name]
    prog = F.compile_native(mk(), alg)
    import os
    assert os.path.getsize(prog.module_path) > 1000


@pytest.mark.parametrize("alg", sorted(F.FUSED_KERNELS), ids=lambda a: abi.CHECK_NAMES and str(a))
def test_fused_lowering_builds(alg):
    """compile_native(fused=True): each integer-state round kernel instantiated with a
    generated Spec hook compiles for gfx950 (both HO-set sources, one wave count)."""
    spec = F.REFERENCE_SPECS[alg]() if alg in F.REFERENCE_SPECS else spec_cases.uniform_agreement()
    prog = F.compile_native(spec, alg, fused=True, n=64)
    import os
    assert os.path.getsize(prog.module_path) > 1000
    from round_amd import lib
    src = lib.spec_native_source(F.to_text(spec), alg, True, 64)  # what the module was built from
    assert f"psg_fused_a{alg}_w1" in src and f"psg_fused_x_a{alg}_w1" in src
    assert f"psg_spec_alg = {alg};" in src and prog.alg == alg


def test_lowering_shapes_in_source():
    """The shape analyses of the generator, read off the source it emits: a nested process
    quantifier whose body reads its variable only through fields walks the distinct field
    tuples (quant_tup), guarded by the implication's conjuncts that read only that process
    (tup_uniform_g), unguarded otherwise; the symmetric-check-point lowering (spec::uniform)
    goes with the "nosym" option."""
    from round_amd import lib
    P = F.P

    def src(f, **kw):
        return lib.spec_native_source(F.to_text(F.Spec(properties=[("X", f)])), abi.PSG_ALG_OTR, **kw)
    guarded = src(P.exists(lambda i: P.forall(lambda j: (j.decided & (j.x > 0)).implies(j.decision == i.x))))
    assert "quant_tup" in guarded and "tup_uniform_g" in guarded
    plain = src(P.exists(lambda i: P.forall(lambda j: j.decided & (j.decision == i.x))))
    assert "quant_tup" in plain and "tup_uniform_g" not in plain and "tup_uniform<" in plain
    assert "spec::uniform<" in plain and "spec::uniform<" not in src(
        P.exists(lambda i: P.forall(lambda j: j.decided & (j.decision == i.x))), options=["nosym"])
    # V.exists finitization: order comparisons on the breakpoints, == / != on the candidates plus
    # one outside value, a pinned variable at its pin (exactness: test_gpu_spec, all three modes)
    V = F.V
    assert "spec::exists_int_bp<" in src(V.exists(lambda v: P.forall(lambda i: i.x <= v)))
    assert "spec::exists_int_eq<" in src(V.exists(lambda v: P.forall(lambda i: i.x == v)))
    assert "spec::exists_int_pin<" in src(V.exists(lambda v: P.forall(lambda i: i.decided.implies(i.decision == v))))
