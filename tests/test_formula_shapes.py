"""formula.py's quantifier lowering vs the reference's own extractor tests.

src/test/scala/psync/macros/FormulaExtractorSuite.scala:42-56 pins how the Scala
macro turns Set operations into Formula trees:

  s.forall(_ > 2)  -> ForAll(List(v), Implies(In(v, s), Gt(v, 2)))
  s.exists(_ <= 2) -> Exists(List(v), And(In(v, s), Leq(v, 2)))
  s.filter(_ <= 2) -> Comprehension(List(v), And(In(v, s), Leq(v, 2)))
  s.count(_ <= 2)  -> Cardinality(Comprehension(List(v), And(In(v, s), Leq(v, 2))))

with one bound variable shared by the binder and every occurrence. The DSL's
`P.filter(...)` sets (Comprehension) offer the same four operations; this test
checks (1) the trees they build have exactly those shapes and (2) their compiled
programs, run by the CPU interpreter over oracle traces, agree with the Scala Set
semantics evaluated directly in Python (s.forall(p) = every member satisfies p,
...), and with the independent recursive evaluator (tests/formula_ref.py).
"""
import pytest

from round_amd import abi, formula as F, psync

import formula_ref

P = F.P


def _big(i):  # the set s of the suite, over processes: s = P.filter(i => i.x > 1)
    return i.x > 1


S = P.filter(_big)


def _is_in(e, var):
    return isinstance(e, F.Contains) and e.comp is S and e.e is var


def test_forall_shape():
    q = S.forall(lambda v: v.x > 2)
    assert isinstance(q, F.Quant) and q.kind == "forall"
    assert isinstance(q.body, F.Bin) and q.body.op == "IMPL"
    assert _is_in(q.body.x, q.var)
    assert isinstance(q.body.y, F.Bin) and q.body.y.op == "GT" and q.body.y.x.proc is q.var


def test_exists_shape():
    q = S.exists(lambda v: v.x <= 2)
    assert isinstance(q, F.Quant) and q.kind == "exists"
    assert isinstance(q.body, F.Bin) and q.body.op == "AND"
    assert _is_in(q.body.x, q.var)
    assert q.body.y.op == "LE" and q.body.y.x.proc is q.var


def test_filter_and_count_shape():
    c = S.filter(lambda v: v.x <= 2)
    assert isinstance(c, F.Comprehension)
    assert c.body.op == "AND" and _is_in(c.body.x, c.var) and c.body.y.x.proc is c.var
    k = S.count(lambda v: v.x <= 2)
    assert isinstance(k, F.Quant) and k.kind == "count"  # Cardinality(Comprehension(...))
    assert k.body.op == "AND" and _is_in(k.body.x, k.var)


def _scala(tr, n, R, inst, c):
    """The four operations with Scala Set semantics on check point c of an instance."""
    base = inst * (R + 1) * 9 * n + c * 9 * n
    x = [tr[base + p] for p in range(n)]
    s = [p for p in range(n) if x[p] > 1]
    return (all(x[v] > 2 for v in s), any(x[v] <= 2 for v in s), len([v for v in s if x[v] <= 2]))


@pytest.mark.parametrize("alg,n,kw", [(psync.FloodMin(2), 9, dict(value_range=4)),
                                      (psync.OTR(), 12, dict(value_range=3)),
                                      (psync.LastVoting(), 7, dict(value_range=4))])
def test_set_operations_evaluate_like_scala(alg, n, kw, oracle_mod):
    spec = F.Spec(properties=[
        ("Forall", S.forall(lambda v: v.x > 2)),
        ("Exists", S.exists(lambda v: v.x <= 2)),
        ("Count0", S.count(lambda v: v.x <= 2) == 0),
        ("Count1", S.filter(lambda v: v.x <= 2).size == 1),
    ])
    cfg = psync.make_config(alg, n, seed=21, **kw)
    prog = F.compile_spec(spec, alg.alg_id)
    cnt, R = 40, cfg.rounds
    tr = oracle_mod.trace(cfg, 0, cnt)
    ff, _ = oracle_mod.vm_run(prog, tr, cnt, n, R)
    rf, _ = formula_ref.evaluate(spec, tr, cnt, n, R)
    assert ff == rf
    seen = [set(), set(), set()]
    for i in range(cnt):
        want = [abi.PSG_NEVER] * 4
        for c in range(R + 1):
            fa, ex, k = _scala(tr, n, R, i, c)
            seen[0].add(fa), seen[1].add(ex), seen[2].add(k)
            for slot, ok in enumerate((fa, ex, k == 0, k == 1)):
                if not ok and want[slot] == abi.PSG_NEVER:
                    want[slot] = c
        assert ff[i] == want, i
    assert seen[0] == {True, False} and seen[1] == {True, False} and len(seen[2]) > 1
