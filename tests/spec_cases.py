"""Custom Spec programs shared by the CPU (test_formula.py) and GPU (test_gpu_spec.py) tests."""
from round_amd import formula as F, psync

P, V, VB, n, r, init, old = F.P, F.V, F.VB, F.n, F.r, F.init, F.old
H = psync.HOSchedule


def uniform_agreement():
    return F.Spec(properties=[
        ("Termination", P.forall(lambda i: i.decided)),
        ("UniformAgreement", P.forall(lambda i: P.forall(lambda j: (i.decided & j.decided).implies(
            i.decision == j.decision)))),
        ("XNonIncreasing", P.forall(lambda i: i.x <= old(i.x))),
        ("XInitial", P.forall(lambda i: P.exists(lambda j: i.x == init(j.x)))),
    ])


def at_most_two_decisions():
    """|{decisions}| <= 2 as two nested V.exists over Int."""
    return F.Spec(properties=[
        ("TwoSet", V.exists(lambda v1: V.exists(lambda v2: P.forall(lambda i: i.decided.implies(
            (i.decision == v1) | (i.decision == v2)))))),
        ("DecidedCount", P.filter(lambda i: i.decided).size <= n),
    ])


def lv_custom():
    return F.Spec(
        invariants=[P.forall(lambda i: i.commit.implies(P.exists(lambda j: j.x == i.vote)))],
        properties=[
            ("TsBound", P.forall(lambda i: i.ts <= r // 4)),
            ("PhaseEnd", ((r % 4) == 0).implies(P.forall(lambda i: ~i.ready))),
            ("WitnessExpr", V.exists(lambda v: (v == r // 4 + 1) & (v > 0))),
            ("CoordVote", F.coord.commit.implies(P.exists(lambda j: j.x == F.coord.vote) | (r >= 0))),
        ])


def benor_custom():
    return F.Spec(
        properties=[
            ("MajorityHO", P.forall(lambda p: p.HO.size > n // 2)),
            ("VoteIsX", P.forall(lambda i: i.vote.isDefined.implies(
                VB.exists(lambda b: (i.vote == F.Some(b)) & (P.filter(lambda j: j.x == b).size >= 0))))),
            ("Termination", P.forall(lambda i: i.decided)),
        ])


def witness_shapes():
    """V.exists shapes the native lowering specializes: a count guard with a
    non-majority threshold (enumeration filtered by count), a guard whose runtime
    threshold is < 1 (general finitization), equality-only variables (one value
    outside the candidates), and a guard under a lane quantifier."""
    return F.Spec(properties=[
        ("GuardLow", V.exists(lambda v: (P.filter(lambda i: i.x == v).size >= 2)
                              & P.exists(lambda j: j.decided & (j.decision == v)))),
        ("GuardVacuous", V.exists(lambda v: (P.filter(lambda i: i.x == v).size > n - 1000)
                                  & P.forall(lambda j: j.decided.implies(j.decision == v)))),
        ("EqFresh", V.exists(lambda v: P.forall(lambda i: i.decided.implies(i.decision != v)))),
        ("EqNone", V.exists(lambda v: P.forall(lambda i: (i.x == v) | (i.decision != v)))),
        ("GuardInLane", P.forall(lambda i: i.decided.implies(V.exists(lambda v: (
            n // 2 < P.filter(lambda j: j.x == v).size) & (i.decision == v))))),
        ("GuardEqN", V.exists(lambda v: (P.filter(lambda i: old(i.x) == v).size == n) & (r > 0))),
        # three init-membership sets: two LDS sets, the third falls back to the tuple loop
        ("Members", P.forall(lambda i: P.exists(lambda j: init(j.x) == i.x)
                             & P.exists(lambda j: init(j.decided) == i.decided)
                             & P.exists(lambda j: i.decision == init(j.decision)))),
        ("MemberUniform", P.exists(lambda j: init(j.x) == r + 1)),
    ])


def set_operations():
    """Set forall / exists / filter / count of a comprehension, lowered like
    FormulaExtractorSuite.scala:42-56 (tests/test_formula_shapes.py)."""
    S = P.filter(lambda i: i.x > 1)
    return F.Spec(properties=[
        ("SetForall", S.forall(lambda v: v.x > 2)),
        ("SetExists", S.exists(lambda v: v.x <= 2)),
        ("SetCount", S.count(lambda v: v.x <= 2) <= n // 2),
        ("SetFilter", S.filter(lambda v: v.decided).size == P.filter(lambda v: v.decided & (v.x > 1)).size),
    ])


def pin_shapes():
    """V.exists shapes with equality pins (a P.forall conjunct `cond ==> term == v` leaves one
    candidate once some process has cond): conditional and unconditional pins, several pins,
    v-free conjuncts hoisted out, two nested V.exists swapped so the pinned one is innermost
    (LastVoting's majority shape), both nested variables pinned, pins on old state."""
    return F.Spec(properties=[
        ("PinSwap", V.exists(lambda v: V.exists(lambda t: (P.filter(lambda i: i.x >= t).size > n // 2)
                                                 & P.forall(lambda i: (i.x >= t).implies(i.x == v)
                                                            & i.decided.implies(i.decision == v))))),
        ("PinPlain", V.exists(lambda v: P.forall(lambda i: i.x == v))),
        ("PinTwo", V.exists(lambda v: P.forall(lambda i: i.decided.implies(i.decision == v)
                                               & (i.x > 2).implies(i.x == v)) & (v > 0))),
        ("PinHoist", V.exists(lambda v: (r > 1) & P.forall(lambda i: i.decided.implies(i.decision == v))
                              & (P.filter(lambda i: i.x == v).size >= 1))),
        ("PinNested", V.exists(lambda v: V.exists(lambda w: P.forall(lambda i: i.decided.implies(i.decision == v))
                                                  & P.forall(lambda j: (j.x > v).implies(j.x == w))))),
        ("PinOld", V.exists(lambda v: P.forall(lambda i: old(i.decided).implies(old(i.decision) == v)))),
    ])


def order_shapes():
    """V.exists over Int with order comparisons (the native lowering's breakpoint
    finitization, spec::exists_int_bp: one candidate per breakpoint, not v-1, v, v+1)."""
    return F.Spec(properties=[
        ("OrdMajority", V.exists(lambda t: (P.filter(lambda i: i.x >= t).size > n // 2) & (t > r // 4))),
        ("OrdBetween", V.exists(lambda t: (t > r) & (t < r + 2))),
        ("OrdAbove", V.exists(lambda t: P.forall(lambda i: i.x < t) & (t <= 6 - r))),
        ("OrdTop", V.exists(lambda t: P.forall(lambda i: i.x < t) & (t > r + 5))),
        ("OrdNe", V.exists(lambda t: (t != r) & (t >= r) & (t <= r + 1))),
        ("OrdMix", V.exists(lambda t: (t > 1) & P.exists(lambda i: i.x == t)
                            & P.forall(lambda i: i.decided.implies(i.decision >= t)))),
        ("OrdOld", V.exists(lambda t: P.forall(lambda i: old(i.x) <= t) & (t < r))),
    ])


def symmetric_shapes():
    """Shapes of the symmetric-check-point lowering (spec::uniform: every process holds the
    same current / old fields): counts of symmetric bodies, old fields, a process used as a
    pid (Contains) or read through init (not symmetric), quantifiers nested in both orders,
    coord's fields, and pins / count guards decided by process 0's value."""
    A = P.filter(lambda i: i.decided)
    return F.Spec(properties=[
        ("SymCount", P.filter(lambda i: i.x == old(i.x)).size >= n // 2),
        ("SymInitLe", P.forall(lambda i: P.exists(lambda j: init(j.x) <= i.x))),
        ("SymPid", P.forall(lambda i: A.contains(i).implies(i.decision == i.x))),
        ("SymNested", P.exists(lambda i: P.forall(lambda j: (j.x == i.x) | (init(j.x) > i.x)))),
        ("SymCountEq", P.forall(lambda i: P.filter(lambda j: j.x == i.x).size == n)),
        ("SymCoord", P.forall(lambda i: i.x >= F.coord.x) | (r > 100)),
        ("SymPinGuard", V.exists(lambda v: (P.filter(lambda i: i.x == v).size > n // 2)
                                 & P.forall(lambda i: i.decided.implies(i.decision == v)))),
        ("SymMember", P.forall(lambda i: i.decided.implies(P.exists(lambda j: init(j.x) == i.decision)))),
    ])


def guard_shapes():
    """Guarded distinct-state quantifiers (spec::quant_tup_gc): nested forall(j => A(j) ==> B),
    exists / count(j => A(j) && B) with A on j's current / old fields, several guard conjuncts,
    a guard no process meets (the quantifier's identity) and a guard mixed with the outer
    variable (only j's conjuncts guard)."""
    return F.Spec(properties=[
        ("GForall", P.forall(lambda i: P.forall(lambda j: (j.decided & (j.x > 0) & i.decided).implies(
            j.decision == i.decision)))),
        ("GExists", P.forall(lambda i: P.exists(lambda j: j.decided & (j.decision == i.x)) | ~i.decided)),
        ("GCount", P.forall(lambda i: (P.filter(lambda j: j.decided & (j.decision == i.decision)).size >= 1)
                            | ~i.decided)),
        ("GEmpty", P.forall(lambda i: P.forall(lambda j: (j.x < -5).implies(j.decision == i.x + 7)))),
        ("GEmptyCount", P.exists(lambda i: P.filter(lambda j: (j.x < -5) & (j.x == i.x)).size == 0)),
        ("GOld", P.exists(lambda i: P.forall(lambda j: old(j.decided).implies(j.decided & (j.x >= i.x - 100))))),
    ])


def split_shapes():
    """Split foralls and hoisted conjuncts (formula._split_forall / _proc_step / _vint_step):
    a conjunct free of the outer variable leaves a process quantifier (exists and forall, the
    inner variable then bound twice, once by the hoisted lane-level forall and once by the walk
    left inside), a cross-lane conjunct (coord's field, a nested count) leaves V.exists, and the
    split under an implication / disjunction (no hoisting there)."""
    c = F.coord
    cdec = F.Field(F.FIELD_DECIDED, c)
    return F.Spec(properties=[
        ("SplitExists", P.exists(lambda j: P.forall(lambda i: i.decided & (i.decision >= j.x - 1))) | (r < 3)),
        ("SplitForall", P.forall(lambda j: P.forall(lambda i: (i.x >= -100) & (i.x != j.x + 100)))),
        ("SplitMixed", P.exists(lambda j: (r > 0) & P.forall(lambda i: cdec.implies(i.decided)
                                                             & i.decided.implies(i.decision <= j.x + 2)))
         | (r < 4)),
        ("SplitCount", P.exists(lambda j: P.forall(lambda i: (P.filter(lambda k: k.x == i.x).size >= 1)
                                                   & (i.x >= j.x - 1)))),
        ("SplitVint", V.exists(lambda v: P.forall(lambda i: cdec.implies(i.decided)
                                                  & i.decided.implies(i.decision == v))) | (r < 5)),
        ("SplitVint2", V.exists(lambda v: V.exists(lambda t: (P.filter(lambda i: i.x >= t).size > n // 2)
                                                   & P.forall(lambda i: (i.x >= t).implies(i.x == v)
                                                              & (c.x >= -100)))) | (r < 2)),
        ("SplitUnder", P.forall(lambda j: j.decided.implies(P.exists(lambda i: i.decided & (i.decision == j.decision))))),
    ])


def term_shared_shapes():
    """Termination repeating a closed subformula that two other slots share (so
    fail() hoists it as cse0 / ucse0). term() is a separate function: it must lower the
    subformula itself instead of naming fail()'s local."""
    return F.Spec(properties=[
        ("Termination", P.forall(lambda i: i.decided)),
        ("AllOrNone", P.forall(lambda i: i.decided) | (n == 0)),
        ("AllOrOne", P.forall(lambda i: i.decided) | (n == 1)),
    ])


# (id, algorithm, n, make_config kwargs, spec factory)
CUSTOM = [
    ("fm-n12", psync.FloodMin(2), 12, dict(value_range=8, schedule=H(drop_log2=0, good_round=0.0, crash_fmax=3)),
     uniform_agreement),
    ("fm-n100", psync.FloodMin(2), 100, dict(value_range=8, schedule=H(drop_log2=0, good_round=0.0, crash_fmax=3)),
     uniform_agreement),
    ("kses-n16", psync.KSetEarlyStopping(4, 2), 16, dict(value_range=6), at_most_two_decisions),
    ("kses-n70", psync.KSetEarlyStopping(4, 2), 70, dict(value_range=6), at_most_two_decisions),
    ("kset-n16", psync.KSetAgreement(2), 16, dict(value_range=6), at_most_two_decisions),
    ("lv-n8", psync.LastVoting(), 8, dict(value_range=4, schedule=H(drop_log2=1, good_round=0.0, crash_fmax=3)),
     lv_custom),
    ("slv-n16", psync.ShortLastVoting(), 16, dict(value_range=4), uniform_agreement),
    ("benor-n8", psync.BenOr(), 8, {}, benor_custom),
    ("otr2-n12", psync.OTR2(), 12, dict(value_range=4), uniform_agreement),
    ("otr-n16-shapes", psync.OTR(), 16, dict(value_range=3), witness_shapes),
    ("otr2-n100-shapes", psync.OTR2(), 100, dict(value_range=3), witness_shapes),
    ("otr-n12-sets", psync.OTR(), 12, dict(value_range=3), set_operations),
    ("fm-n70-sets", psync.FloodMin(2), 70, dict(value_range=4, schedule=H(drop_log2=0, good_round=0.0,
                                                                            crash_fmax=3)), set_operations),
    ("fm-n8-shapes", psync.FloodMin(2), 8, dict(value_range=3, schedule=H(drop_log2=0, good_round=0.0,
                                                                           crash_fmax=3)), witness_shapes),
    ("otr-n16-pins", psync.OTR(), 16, dict(value_range=3), pin_shapes),
    ("otr2-n100-pins", psync.OTR2(), 100, dict(value_range=4), pin_shapes),
    ("fm-n8-pins", psync.FloodMin(2), 8, dict(value_range=3, schedule=H(drop_log2=0, good_round=0.0,
                                                                         crash_fmax=3)), pin_shapes),
    ("lv-n8-pins", psync.LastVoting(), 8, dict(value_range=3), pin_shapes),
    ("otr-n16-order", psync.OTR(), 16, dict(value_range=3), order_shapes),
    ("lv-n8-order", psync.LastVoting(), 8, dict(value_range=3, schedule=H(drop_log2=1, good_round=0.0)),
     order_shapes),
    # symmetric check points: n = 1 (every state), one initial value (from round 0), mixed
    ("otr-n1-sym", psync.OTR(), 1, dict(value_range=3), symmetric_shapes),
    ("otr-n16-v1-sym", psync.OTR(), 16, dict(value_range=1), symmetric_shapes),
    ("otr-n16-sym", psync.OTR(), 16, dict(value_range=3), symmetric_shapes),
    ("otr2-n100-v1-sym", psync.OTR2(), 100, dict(value_range=1), symmetric_shapes),
    ("lv-n8-v1-sym", psync.LastVoting(), 8, dict(value_range=1), lv_custom),
    ("fm-n8-sym", psync.FloodMin(2), 8, dict(value_range=2, schedule=H(drop_log2=0, good_round=0.0,
                                                                        crash_fmax=3)), symmetric_shapes),
    # guarded tuple quantifiers: crashed / undecided processes outside the guard set
    ("otr-n16-guard", psync.OTR(), 16, dict(value_range=3), guard_shapes),
    ("fm-n12-guard", psync.FloodMin(2), 12, dict(value_range=4, schedule=H(drop_log2=0, good_round=0.0,
                                                                            crash_fmax=3)), guard_shapes),
    ("lv-n8-guard", psync.LastVoting(), 8, dict(value_range=3, schedule=H(drop_log2=1, good_round=0.0,
                                                                           crash_fmax=3)), guard_shapes),
    ("otr2-n100-guard", psync.OTR2(), 100, dict(value_range=3), guard_shapes),
    # split foralls / hoisted conjuncts
    ("otr-n16-split", psync.OTR(), 16, dict(value_range=3), split_shapes),
    ("fm-n12-split", psync.FloodMin(2), 12, dict(value_range=4, schedule=H(drop_log2=0, good_round=0.0,
                                                                            crash_fmax=3)), split_shapes),
    ("lv-n8-split", psync.LastVoting(), 8, dict(value_range=3, schedule=H(drop_log2=1, good_round=0.0,
                                                                           crash_fmax=3)), split_shapes),
    ("fm-n100-split", psync.FloodMin(2), 100, dict(value_range=4, schedule=H(drop_log2=0, good_round=0.0,
                                                                              crash_fmax=3)), split_shapes),
    # Termination sharing a subformula hoisted in fail()
    ("otr-n16-termcse", psync.OTR(), 16, dict(value_range=3), term_shared_shapes),
    ("fm-n12-termcse", psync.FloodMin(2), 12, dict(value_range=4, schedule=H(drop_log2=0, good_round=0.0,
                                                                              crash_fmax=3)), term_shared_shapes),
]
