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
    cnt = 12
    tr = oracle_mod.trace(cfg, 0, cnt)
    ff, tm = oracle_mod.vm_run(prog, tr, cnt, n, cfg.rounds)
    rf, rt = formula_ref.evaluate(spec, tr, cnt, n, cfg.rounds)
    assert ff == rf and tm == rt


def _breakpoint_domain(q, st, env):
    """The native lowering's candidates for an order-compared V.exists (exists_int_bp):
    each source's values shifted by its breakpoint offsets, plus Int.MaxValue."""
    if F._eq_only(q):
        return st.dom
    exprs, fsets = F._Compiler().witnesses(q)
    sh = F._breakpoint_shifts(q, exprs, fsets)
    vals = [[formula_ref.ev(t, st, env)] for t in exprs]
    vals += [[st.field(f, tag, p) for p in range(st.n)] for f, tag in fsets]
    dom = {formula_ref.INT_MAX}
    for vs, m in zip(vals, sh):
        for v in vs:
            dom |= {formula_ref._wrap(v + d) for d in (-1, 0, 1) if (m >> (d + 1)) & 1}
    return sorted(dom)


@pytest.mark.parametrize("cid,alg,n,kw,mk", [c for c in spec_cases.CUSTOM if c[2] <= 16] + [
    ("lv-ref", psync.LastVoting(), 8, dict(value_range=3, schedule=H(drop_log2=1, good_round=0.0, crash_fmax=3)),
     F.lv_spec)], ids=[c[0] for c in spec_cases.CUSTOM if c[2] <= 16] + ["lv-ref"])
def test_breakpoint_finitization_is_exact(cid, alg, n, kw, mk, oracle_mod, monkeypatch):
    """V.exists over Int decided on the breakpoint candidates (native exists_int_bp) equals
    the brute-forced domain, check point by check point."""
    cfg = psync.make_config(alg, n, seed=23, **kw)
    spec = mk()
    cnt = 8
    tr = oracle_mod.trace(cfg, 0, cnt)
    want = formula_ref.evaluate(spec, tr, cnt, n, cfg.rounds)
    monkeypatch.setattr(formula_ref, "VINT_DOMAIN", _breakpoint_domain)
    assert formula_ref.evaluate(spec, tr, cnt, n, cfg.rounds) == want


def _rewritten(spec):
    """The Spec with every formula passed through the native lowering's V.exists rewrites."""
    memo = {}
    g = F._rinv_guard(spec)
    invs = [F._rewrite_vint(inv if g is None else (inv & g), memo) for inv in spec.invariants]
    props = [(name, F._rewrite_vint(f, memo)) for name, f in spec.properties]
    sp = None if spec.safety_predicate is None else F._rewrite_vint(spec.safety_predicate, memo)
    plain = [inv if g is None else (inv & g) for inv in spec.invariants]
    return (F.Spec(plain, [], spec.properties, spec.safety_predicate, phase_length=spec.phase_length),
            F.Spec(invs, [], props, sp, phase_length=spec.phase_length))


REWRITE_CASES = [(f"ref-{a}", alg, n, kw, F.REFERENCE_SPECS[a]) for a, alg, n, kw in [
    (abi.PSG_ALG_OTR, psync.OTR(), 16, dict(value_range=3, schedule=H(drop_log2=1))),
    (abi.PSG_ALG_OTR2, psync.OTR2(), 10, {}),
    (abi.PSG_ALG_LAST_VOTING, psync.LastVoting(), 16, dict(value_range=3, schedule=H(
        drop_log2=1, good_round=0.0, crash_fmax=7))),
    (abi.PSG_ALG_LAST_VOTING, psync.LastVoting(variant=1), 6, dict(value_range=5)),
    (abi.PSG_ALG_BENOR, psync.BenOr(), 8, {})]] + [c for c in spec_cases.CUSTOM if c[2] <= 16]


@pytest.mark.parametrize("swap", [False, True], ids=["hoist", "swap+hoist"])
@pytest.mark.parametrize("cid,alg,n,kw,mk", REWRITE_CASES, ids=[c[0] for c in REWRITE_CASES])
def test_native_rewrites_are_exact(cid, alg, n, kw, mk, oracle_mod, swap, monkeypatch):
    """The V.exists rewrites of the native lowering (swap to put the pinned variable
    innermost, hoist conjuncts free of the variable) give the same results as the
    Spec as written, under the CPU interpreter, check point by check point."""
    monkeypatch.setattr(F, "SWAP_VINT", swap)
    cfg = psync.make_config(alg, n, seed=29, **kw)
    orig, rw = _rewritten(mk())
    cnt = 300
    tr = oracle_mod.trace(cfg, 0, cnt)
    f1, t1 = oracle_mod.vm_run(F.compile_spec(orig, alg.alg_id), tr, cnt, n, cfg.rounds)
    f2, t2 = oracle_mod.vm_run(F.compile_spec(rw, alg.alg_id), tr, cnt, n, cfg.rounds)
    assert f1 == f2 and t1 == t2


def test_rewrites_shapes():
    """LastVoting's majority clause: the pinned value variable moves innermost and the
    conjuncts free of it are hoisted out (the lowering then takes one candidate)."""
    spec = F.lv_spec()
    F.SWAP_VINT = True
    try:
        mb = F._rewrite_vint(spec.invariants[0])
    finally:
        F.SWAP_VINT = False
    vints = [x for x in F._walk(mb) if isinstance(x, F.Quant) and x.kind == "vint"]
    assert len(vints) == 2
    outer, inner = vints
    assert F._pins(inner.body, inner.var.uid) is not None  # v, pinned by x / decision / vote
    assert F._pins(outer.body, outer.var.uid) is None       # t


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
    """codegen_hip output compiles for gfx950 (hipcc --genco; no GPU needed)."""
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
    src = F._fused_source(alg, [1]) + F.codegen_hip(spec, alg)[0]  # what the module was built from
    assert f"psg_fused_a{alg}_w1" in src and f"psg_fused_x_a{alg}_w1" in src
    assert f"psg_spec_alg = {alg};" in src and prog.alg == alg


def test_symmetric_and_guard_classification():
    """The shape analyses behind the symmetric-check-point lowering (_symmetric: a process
    variable read only through current / old fields) and the guarded distinct-state walk
    (_tuple_guard: the conjuncts that read only the quantified process)."""
    P, init, old = F.P, F.init, F.old

    def q(mk):
        e = mk()
        assert isinstance(e, F.Quant)
        return e
    assert F._symmetric(q(lambda: P.forall(lambda i: i.decided.implies(i.decision == old(i.decision)))))
    assert not F._symmetric(q(lambda: P.forall(lambda i: i.x == init(i.x))))  # reads init
    A = P.filter(lambda i: i.decided)
    assert not F._symmetric(q(lambda: P.forall(lambda i: A.contains(i))))  # used as a pid
    # forall(j => A(j) ==> B): the conjuncts of A reading only j
    g = F._tuple_guard(q(lambda: P.forall(lambda j: (j.decided & (j.x > 0)).implies(j.decision == 3))))
    assert len(g) == 2
    outer = F.Var("proc")
    g = F._tuple_guard(q(lambda: P.forall(lambda j: (outer.decided & j.decided).implies(j.decision == outer.x))))
    assert len(g) == 1  # outer.decided reads another process
    assert F._tuple_guard(q(lambda: P.exists(lambda j: j.decided & (j.decision == outer.x)))) != []
    assert F._tuple_guard(q(lambda: P.forall(lambda j: j.decided & (j.decision == 1)))) == []  # not an implication
