"""Formula text: the JVM plugin's way in for generic Specs.

integration/scala/GpuSpec.scala writes a psync.Spec as the S-expression text of the
reference's own Formula trees (Binding ForAll / Exists / Comprehension, Application,
Variable, Literal — psync/formula/Formula.scala), and psg_spec_from_text (host C++
in libpsg, round_amd/csrc/psg_spec_text.cpp) compiles it to the psg_spec_program
bytecode. These CPU tests check that compiler against the Python one
(round_amd/formula.py compile_spec) word for word, on the reference Specs, the custom
Specs of the GPU suites and hand-written texts in the shapes FormulaExtractor
produces (flattened multi-variable binders, n-ary And, `val A = ...` lets), and run
the compiled programs through the CPU interpreter against the oracle's checker.
"""
import pytest

from round_amd import abi, formula as F, lib, psync

import spec_cases

P, V, n, r, init = F.P, F.V, F.n, F.r, F.init


def _same(a, b):
    assert (a.code, a.slot_entry, a.slot_flags, a.term_entry, a.n_vars, a.slot_names) == \
           (b.code, b.slot_entry, b.slot_flags, b.term_entry, b.n_vars, b.slot_names)


@pytest.mark.parametrize("alg", sorted(F.REFERENCE_SPECS))
def test_reference_specs_compile_identically(alg):
    spec = F.REFERENCE_SPECS[alg]()
    text = F.to_text(spec)
    want = F.compile_spec(spec, alg)
    got = lib.spec_from_text(text, alg)
    _same(got, want)
    assert got.alg == alg
    _same(F.compile_spec(F.from_text(text), alg), want)


@pytest.mark.parametrize("cid,alg,nn,kw,mk", spec_cases.CUSTOM, ids=[c[0] for c in spec_cases.CUSTOM])
def test_custom_specs_compile_identically(cid, alg, nn, kw, mk):
    spec = mk()
    _same(lib.spec_from_text(F.to_text(spec), alg.alg_id), F.compile_spec(spec, alg.alg_id))


# hand-written texts in FormulaExtractor's shapes, each with its DSL equivalent
LV_MAJORITY_LET = """
(Spec (phase 1)
  (invariants
    (Exists ((v Int) (t Int))
      (Exists ((A Set))
        (App And (App Eq (Var A) (Comprehension ((i pid)) (App Geq (App ts (Var i)) (Var t))))
                 (App Gt (App Cardinality (Var A)) (App Divides (Var n) (Lit 2)))
                 (App Gt (Var r) (Lit 0))
                 (App Leq (Var t) (App Divides (Var r) (Lit 4)))
                 (ForAll ((i pid)) (App Implies (App In (Var i) (Var A)) (App Eq (App x (Var i)) (Var v)))))))))
"""


def _lv_majority_dsl():
    def body(v, t):
        A = P.filter(lambda i: i.ts >= t)
        return (A.size > n // 2) & (r > 0) & (t <= r // 4) & P.forall(lambda i: A.contains(i).implies(i.x == v))
    return F.Spec([V.exists(lambda v: V.exists(lambda t: body(v, t)))])


AGREEMENT_FLAT = """
(Spec (phase 1) (invariants)
  (properties
    (prop "Agreement" (ForAll ((i pid) (j pid))
        (App Implies (App And (App decided (Var i)) (App decided (Var j)))
                     (App Eq (App decision (Var i)) (App decision (Var j))))))
    (prop "Irrevocability" (ForAll ((i pid))
        (App Implies (App __old__decided (Var i))
                     (App And (App decided (Var i)) (App Eq (App __old__decision (Var i)) (App decision (Var i)))))))
    (prop "Termination" (ForAll ((i pid)) (App decided (Var i))))))
"""


def _agreement_dsl():
    return F.Spec(properties=[
        ("Agreement", P.forall(lambda i: P.forall(lambda j: (i.decided & j.decided).implies(
            i.decision == j.decision)))),
        ("Irrevocability", P.forall(lambda i: F.old(i.decided).implies(
            i.decided & (F.old(i.decision) == i.decision)))),
        ("Termination", P.forall(lambda i: i.decided)),
    ])


NARY_AND = """
(Spec (phase 1)
  (invariants (ForAll ((i pid)) (App And (App Not (App decided (Var i))) (App Geq (App x (Var i)) (Lit 1))
                                         (App Leq (App x (Var i)) (Lit 100000)) (Lit true))))
  (safetyPredicate (ForAll ((p pid)) (App Gt (App Cardinality (App HO (Var p))) (App Divides (Var n) (Lit 2))))))
"""


def _nary_dsl():
    return F.Spec([P.forall(lambda i: (~i.decided & (i.x >= 1)) & (i.x <= 100000) & F.true)],
                  safety_predicate=P.forall(lambda p: p.HO.size > n // 2))


@pytest.mark.parametrize("text,mk,alg", [
    (LV_MAJORITY_LET, _lv_majority_dsl, abi.PSG_ALG_LAST_VOTING),
    (AGREEMENT_FLAT, _agreement_dsl, abi.PSG_ALG_OTR),
    (NARY_AND, _nary_dsl, abi.PSG_ALG_BENOR),
], ids=["let", "flat-binders", "nary-and"])
def test_extractor_shapes(text, mk, alg):
    want = F.compile_spec(mk(), alg)
    _same(lib.spec_from_text(text, alg), want)
    _same(F.compile_spec(F.from_text(text), alg), want)


@pytest.mark.parametrize("text,msg", [
    ("(Spec (invariants (ForAll ((v Int)) (App Gt (Var v) (Lit 0)))))", "ForAll over Int"),
    ("(Spec (invariants (ForAll ((i pid)) (App x (Var j)))))", "unbound variable j"),
    ("(Spec (invariants (ForAll ((i pid)) (App frob (Var i)))))", "unknown symbol frob"),
    ("(Spec (invariants (Exists ((v Int)) (App Gt (App Times (Var v) (Lit 2)) (Lit 3)))))", "only appear directly"),
    ("(Spec (invariants (ForAll ((i pid)) (App ts (Var i)))))", "not part of this algorithm"),
    ("(Spec (invariants (ForAll ((i pid)) (App decided (Var i)))", "missing [)]"),
    ("(Spec (invariants))", "at least one"),
])
def test_rejected_texts(text, msg):
    with pytest.raises(F.FormulaError, match=msg):
        lib.spec_from_text(text, abi.PSG_ALG_OTR)
    with pytest.raises(F.FormulaError):
        F.compile_spec(F.from_text(text), abi.PSG_ALG_OTR)


@pytest.mark.parametrize("alg,nn,kw", [
    (psync.OTR(), 8, {}),
    (psync.LastVoting(), 8, dict(value_range=3, schedule=psync.HOSchedule(drop_log2=1, good_round=0.0,
                                                                          crash_fmax=3))),
    (psync.BenOr(), 8, {}),
], ids=lambda v: getattr(v, "class_name", None) or None)
def test_text_programs_reproduce_the_oracle_checker(alg, nn, kw, oracle_mod):
    """The C-compiled reference Spec, run by the CPU interpreter over oracle traces, gives
    the oracle checker's first failing check points and termination rounds."""
    cfg = psync.make_config(alg, nn, seed=13, **kw)
    prog = lib.spec_from_text(F.to_text(F.REFERENCE_SPECS[alg.alg_id]()), alg.alg_id)
    cnt = 150
    tr = oracle_mod.trace(cfg, 0, cnt)
    ff, tm = oracle_mod.vm_run(prog, tr, cnt, nn, cfg.rounds)
    _, pi, _ = oracle_mod.run(cfg, 0, cnt, per_instance=True, threads=8)
    k = len(prog.slot_names)
    for i in range(cnt):
        assert ff[i] == list(pi[i].first_fail)[:k] and tm[i] == pi[i].term_round, i


def test_names_buffer_too_small_is_an_error():
    """slot names are never silently truncated (they must line up with slot_entry)."""
    import ctypes as C
    L = lib.load()
    text = F.to_text(F.otr_spec())
    cp, err = abi.SpecProgram(), C.create_string_buffer(512)
    small = C.create_string_buffer(8)
    rc = L.psg_spec_from_text(text.encode(), abi.PSG_ALG_OTR, C.byref(cp), small, len(small), err, len(err))
    assert rc == abi.PSG_ERANGE and "bytes needed" in err.value.decode()
    assert cp.n_words == 0 and not cp.code  # nothing allocated on the error path
    need = int(err.value.decode().split(":")[1].split()[0])
    exact = C.create_string_buffer(need)
    assert L.psg_spec_from_text(text.encode(), abi.PSG_ALG_OTR, C.byref(cp), exact, need, err, len(err)) == 0
    assert exact.value.decode().split("\n")[0] == "Safety"
    L.psg_spec_release(C.byref(cp))


def test_deep_nesting_is_refused_not_a_crash():
    """text nested past 512 forms gets PSG_EINVAL instead of overflowing the stack."""
    deep = "(Spec (invariants " + "(Not " * 100000 + "true" + ")" * 100000 + "))"
    with pytest.raises(F.FormulaError, match="nesting deeper than 512"):
        lib.spec_from_text(deep, abi.PSG_ALG_OTR)


def test_wide_conjunction_is_shallow_not_a_crash():
    """a 100k-conjunct (App And ...) folds into a tree of depth 32 + log2(arity)
    instead of a 100k-deep chain, so the lowering and the native generator do not overflow the
    stack (run on a 1 MB thread, the JVM's default stack size); <= 32 arguments keep the DSL's
    left-deep shape."""
    import threading
    atoms = " ".join("(App Leq (App x (Var i)) (Lit %d))" % j for j in range(100000))
    wide = "(Spec (invariants (ForAll ((i pid)) (App And " + atoms + "))))"
    out = {}

    def run():
        out["prog"] = lib.spec_from_text(wide, abi.PSG_ALG_OTR)
        few = " ".join("(App Leq (App x (Var i)) (Lit %d))" % j for j in range(2000))
        out["src"] = lib.spec_native_source(wide.replace(atoms, few), abi.PSG_ALG_OTR)

    old = threading.stack_size(1 << 20)
    try:
        th = threading.Thread(target=run)
        th.start()
        th.join()
    finally:
        threading.stack_size(old)
    assert out["prog"].slot_names[0] == "Safety" and "struct GenSpec" in out["src"]
