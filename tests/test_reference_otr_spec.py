"""Pin of the Spec evaluator (the checker's slot verdicts) against the reference's own
OTR and LastVoting formulas.

`src/test/scala/psync/logic/OtrExample.scala:32-59` states OTR's properties and
invariants as Formulas over `data`, `decided` (pre-state), `data1`, `decided1`
(post-state) and `data0` (initial values):

  agreement (32)           forall i,j. decided(i) && decided(j) ==> data(i) == data(j)
  integrity (33)           forall i. decided(i) ==> decided1(i) && data(i) == data1(i)
  termination (34)         forall i. decided(i)
  validity (35)            forall i. exists j. data(i) == data0(j)
  invariantAgreement (41)  (forall i. !decided(i)) || exists v, A. A == {i. data(i) == v}
                             && |A| > 2n/3 && forall i. decided(i) ==> data(i) == v
  invariantProgress1 (50)  exists v, A. A == {i. data(i) == v} && |A| == n
                             && forall i. decided(i) ==> data(i) == v
  invariantProgress2 (56)  exists v. forall i. decided(i) && data(i) == v
  magicRound (98)          exists A. |A| > 2n/3 && forall i. ho(i) == A

and the suite's verification conditions (109-212, five of them `ignore`d there because
z3 is slow) relate them. `OtrExample`'s one variable `data` is the process's value and,
once it decided, its decision; on the OTR of `example/Otr.scala` (x, decided, decision)
the model's `data(i)` is therefore `decided ? decision : x` (the same mapping
tests/test_reference_lv.py uses for `LvExample.scala`, where round4 writes `data1`
where the code writes `decision`). `data0(j)` is `init(j.x)`.

Every check point of oracle runs (n = 4 ... 64, with and without self delivery, with
the real `afterDecision = 2` exit and without exits, reference OTR and the build's
mutant) is evaluated with those formulas, transcribed literally below (V finitized
exactly: every v the formulas can witness is some data(i)), and compared with the
checker's slot verdicts at that check point (`oracle.trace_checks`, hand-lowered
evaluator == Formula interpreter, spec_mode 2). Relations asserted, each a theorem
about the formulas under the mapping (no algorithm property needed):

  Agreement slot      <=>  agreement
  Irrevocability slot <=>  integrity(pre = previous check point, post = this one)
  Integrity slot      <=>  agreement && (forall i. decided(i) ==> exists j. data(i) == data0(j))
  Validity slot       <=>  forall i. decided(i) ==> exists j. data(i) == data0(j)
  Termination         <=>  termination
  Invariant0 slot      ==>  invariantAgreement && validity[data := x]
  Invariant1 slot      ==>  invariantProgress1 && validity[data := x]
  Invariant2 slot     <=>  invariantProgress2 && validity
  Safety slot         <=>  Invariant0 || Invariant1 || Invariant2

and, wherever every decided process holds x == decision (the reachable states of the
reference OTR, asserted there), Invariant0 / Invariant1 are EQUIVALENT to their
model side. The model's own VCs are checked concretely on the reference OTR's
transitions (OtrExample.scala:109-212, incl. the ignored "invariant is inductive",
"1st / 2nd magic round", "invariant 1 is inductive"). Teeth: a checker mutant that
reports any one slot as holding everywhere (or failing everywhere) breaks its
relation on these runs.

LastVoting (`LvExample.scala:59-63` properties, `invariant1` 221-238) is pinned the
same way against the LastVoting checker's slots: Agreement / Irrevocability /
Integrity / Validity / Termination equivalences, and Invariant0 (safetyInv,
`LastVoting.scala:44`) ==> invariant1 with the model's phase `r` = the Spec's r/4.

The GPU's checker equals the oracle's per instance (first failing check point of
every slot: test_gpu_parity.py, test_gpu_sampled.py); the GPU test at the end pins
the GPU's first failing check points directly to the formulas above on the
states of the same instances (digests equal).
"""
import numpy as np
import pytest

from round_amd import abi, psync

NF = 9
X, DECIDED, DECISION, TS, READY, COMMIT, VOTE = 0, 1, 2, 3, 4, 5, 6
SAFETY, INV0, INV1, INV2, AGREEMENT, VALIDITY, INTEGRITY, IRREVOCABILITY = range(8)
TERM = 15


# ------------------------------------------------------------------ the reference formulas
# Arrays are [..., n] over pids (leading axes: instance, check point). Every formula returns
# a bool array over the leading axes.

def agreement(data, decided):
    """OtrExample.scala:32 / LvExample.scala:60: forall i,j. decided(i) && decided(j) ==> data(i) == data(j)."""
    eq = data[..., :, None] == data[..., None, :]
    both = decided[..., :, None] & decided[..., None, :]
    return (~both | eq).all(axis=(-1, -2))


def integrity(data, decided, data1, decided1):
    """OtrExample.scala:33 / LvExample.scala:61: forall i. decided(i) ==> decided1(i) && data(i) == data1(i)."""
    return (~decided | (decided1 & (data == data1))).all(-1)


def termination(decided):
    """OtrExample.scala:34: forall i. decided(i)."""
    return decided.all(-1)


def validity(data, data0):
    """OtrExample.scala:35: forall i. exists j. data(i) == data0(j)."""
    return (data[..., :, None] == data0[..., None, :]).any(-1).all(-1)


def _by_value(data):
    """E[..., v, i] = data(i) == v for the candidate values v = data(0..n-1): every v an
    existential over V can witness in the formulas below (their A = {i. data(i) == v} is
    non-empty, or every data(i) equals v)."""
    return data[..., None, :] == data[..., :, None]


def invariant_agreement(data, decided, n):
    """OtrExample.scala:41-48."""
    E = _by_value(data)
    card = E.sum(-1)
    dec_v = (~decided[..., None, :] | E).all(-1)           # forall i. decided(i) ==> data(i) == v
    return (~decided).all(-1) | ((card > (2 * n) // 3) & dec_v).any(-1)


def invariant_progress1(data, decided, n):
    """OtrExample.scala:50-54."""
    E = _by_value(data)
    dec_v = (~decided[..., None, :] | E).all(-1)
    return ((E.sum(-1) == n) & dec_v).any(-1)


def invariant_progress2(data, decided):
    """OtrExample.scala:56-57: exists v. forall i. decided(i) && data(i) == v."""
    E = _by_value(data)
    return (decided[..., None, :] & E).all(-1).any(-1)


def magic_round(ho_sets, n):
    """OtrExample.scala:98-101: exists A. |A| > 2n/3 && forall i. ho(i) == A (ho_sets: [..., n] masks)."""
    same = (ho_sets == ho_sets[..., :1]).all(-1)
    size = np.array([bin(int(m)).count("1") for m in ho_sets[..., 0].ravel()]).reshape(ho_sets.shape[:-1])
    return same & (size > (2 * n) // 3)


def model_view(tr):
    """(data, decided, x, data0) of traces [..., R+1, F, n]: data = decision once decided, else x."""
    x = tr[..., X, :].astype(np.int64)
    decided = tr[..., DECIDED, :] != 0
    data = np.where(decided, tr[..., DECISION, :].astype(np.int64), x)
    data0 = x[..., :1, :]  # init(j.x): x at check point 0, broadcast over check points
    return data, decided, x, data0


def _holds(bits, slot):
    return (bits >> slot) & 1 == 1


def otr_relations(tr, bits, n):
    """Every relation of the module docstring at every check point; returns the count of
    check points where a relation fails, per relation (all zero = pinned)."""
    data, decided, x, data0 = model_view(tr)
    data0 = np.broadcast_to(data0, data.shape)
    dec_valid = (~decided | (data[..., :, None] == data0[..., None, :]).any(-1)).all(-1)
    agr = agreement(data, decided)
    integ = np.ones(agr.shape, bool)
    integ[:, 1:] = integrity(data[:, :-1], decided[:, :-1], data[:, 1:], decided[:, 1:])
    validx = validity(x, data0)
    ia, p1, p2 = invariant_agreement(data, decided, n), invariant_progress1(data, decided, n), \
        invariant_progress2(data, decided)
    consistent = (~decided | (x == data)).all(-1)  # decided ==> x == decision
    s = {k: _holds(bits, v) for k, v in dict(safety=SAFETY, inv0=INV0, inv1=INV1, inv2=INV2, agr=AGREEMENT,
                                               val=VALIDITY, integ=INTEGRITY, irr=IRREVOCABILITY, term=TERM).items()}
    fails = {
        "Agreement<=>agreement": s["agr"] != agr,
        "Irrevocability<=>integrity": s["irr"] != integ,
        "Integrity<=>agreement&&validity(decided)": s["integ"] != (agr & dec_valid),
        "Validity<=>validity(decided)": s["val"] != dec_valid,
        "Termination<=>termination": s["term"] != termination(decided),
        "Invariant0==>invariantAgreement&&validity[x]": s["inv0"] & ~(ia & validx),
        "Invariant1==>invariantProgress1&&validity[x]": s["inv1"] & ~(p1 & validx),
        "Invariant2<=>invariantProgress2&&validity": s["inv2"] != (p2 & validity(data, data0)),
        "Safety<=>Inv0||Inv1||Inv2": s["safety"] != (s["inv0"] | s["inv1"] | s["inv2"]),
        "consistent==>(Invariant0<=>model)": consistent & (s["inv0"] != (ia & validx)),
        "consistent==>(Invariant1<=>model)": consistent & (s["inv1"] != (p1 & validx)),
    }
    return {k: int(v.sum()) for k, v in fails.items()}, dict(agr=agr, integ=integ, ia=ia, p1=p1, p2=p2,
                                                           validx=validx, consistent=consistent, data=data,
                                                           decided=decided, data0=data0)


# (n, drop_log2, good-round probability, self delivery, afterDecision (None = no exit), variant, V)
CASES = [
    (4, 2, 0.3, True, 2, 0, 3), (4, 1, 0.2, False, 2, 0, 3), (4, 1, 0.2, True, None, 0, 3),
    (7, 2, 0.25, True, 2, 0, 3), (7, 1, 0.3, False, None, 0, 2),
    (16, 3, 0.25, False, 2, 0, 3), (16, 1, 0.1, True, 2, 0, 2), (16, 2, 0.3, True, None, 0, 3),
    (64, 3, 0.25, True, 2, 0, 3), (64, 2, 0.4, False, 2, 0, 2), (64, 3, 0.25, True, None, 0, 64),
    # the build's mutant (variant 1: decide threshold n/2): states that violate the
    # model (at n = 64 random schedules almost never reach one; the adversary search does)
    (6, 1, 0.1, True, 2, 1, 2), (7, 2, 0.1, False, 2, 1, 2), (7, 1, 0.1, True, 2, 1, 3), (16, 2, 0.1, True, 2, 1, 2),
]
R = 10


def _run(oracle_mod, n, drop, good, self_bit, after, variant, count=None, V=3):
    count = count or (300 if n <= 16 else 80)
    alg = psync.OTR(afterDecision=after if after is not None else R + 2, variant=variant)
    cfg = psync.make_config(alg, n, R, seed=131 + n + 7 * variant, value_range=V,
                            schedule=psync.HOSchedule(drop_log2=drop, good_round=good, self_bit=self_bit))
    tr, bits = oracle_mod.trace_checks(cfg, 0, count, threads=8, spec_mode=2)
    return cfg, tr, bits


@pytest.mark.parametrize("n,drop,good,self_bit,after,variant,V", CASES,
                         ids=[f"n{c[0]}-d{c[1]}-s{int(c[3])}-{'exit' if c[4] else 'noexit'}-v{c[5]}-V{c[6]}"
                              for c in CASES])
def test_otr_checker_matches_reference_formulas(n, drop, good, self_bit, after, variant, V, oracle_mod):
    cfg, tr, bits = _run(oracle_mod, n, drop, good, self_bit, after, variant, V=V)
    fails, m = otr_relations(tr, bits, n)
    assert all(v == 0 for v in fails.values()), fails
    if variant == 0:
        # reachable states of the reference OTR: decided ==> x == decision (the model's single
        # `data` is sound), and the model's invariant holds everywhere
        assert m["consistent"].all()
        assert m["ia"].all() and m["agr"].all()
    else:
        # the mutant really leaves the model: these runs exercise the relations on violations
        assert (~m["ia"]).any() and (~_holds(bits, INV0)).any()


@pytest.mark.parametrize("n,drop,good,self_bit", [(4, 1, 0.3, True), (7, 2, 0.3, False), (16, 1, 0.3, False),
                                                  (64, 2, 0.4, False)])
def test_otr_model_vcs_hold_on_transitions(n, drop, good, self_bit, oracle_mod):
    """OtrExample.scala:109-212 on concrete transitions of the reference OTR (no exit, as in
    the model): each `assertUnsat(List(hyps..., Not(goal)))` becomes hyps ==> goal on every
    (pre, post) pair the oracle executes; magicRound reads the round's HO sets."""
    cfg, tr, bits = _run(oracle_mod, n, drop, good, self_bit, None, 0)
    _, m = otr_relations(tr, bits, n)
    ho, _ = oracle_mod.materialize_schedule(cfg, 0, tr.shape[0])
    magic = magic_round(ho[..., 0].astype(np.uint64), n)              # [count, R]
    ia, p1, p2, agr, integ = m["ia"], m["p1"], m["p2"], m["agr"], m["integ"]
    data, decided, data0 = m["data"], m["decided"], m["data0"]
    val = validity(data, data0)
    pre, post = slice(None, -1), slice(1, None)
    assert ia[:, 0].all()                                              # initial state implies invariant (109)
    assert (~ia | agr).all()                                           # invariant implies agreement (114)
    assert (~p2 | termination(decided)).all()                          # invariant implies termination (119)
    assert val[:, 0].all()                                             # validity holds initially (124)
    assert (~ia[:, pre] | ia[:, post]).all()                           # invariant is inductive (146, ignored)
    assert (~(ia[:, pre] & magic) | p1[:, post]).all()                 # 1st magic round (155, ignored)
    assert (~p1[:, pre] | p1[:, post]).all()                           # invariant 1 is inductive (165, ignored)
    assert (~(p1[:, pre] & magic) | p2[:, post]).all()                 # 2nd magic round (174, ignored)
    assert (~p2[:, pre] | p2[:, post]).all()                           # invariant 2 is inductive (184)
    assert (~(ia[:, pre] & ia[:, post]) | integ[:, post]).all()        # integrity (193)
    assert (~(ia[:, pre] & ia[:, post] & val[:, pre]) | val[:, post]).all()  # validity is inductive (203)
    # the magic-round VCs were exercised, not vacuous
    assert (ia[:, pre] & magic).sum() > 0 and (p1[:, pre] & magic).sum() > 0


@pytest.mark.parametrize("slot,name", [(SAFETY, "Safety<=>Inv0||Inv1||Inv2"), (INV0, None), (INV1, None),
                                       (INV2, "Invariant2<=>invariantProgress2&&validity"),
                                       (AGREEMENT, "Agreement<=>agreement"),
                                       (VALIDITY, "Validity<=>validity(decided)"),
                                       (INTEGRITY, "Integrity<=>agreement&&validity(decided)"),
                                       (IRREVOCABILITY, "Irrevocability<=>integrity"),
                                       (TERM, "Termination<=>termination")])
def test_checker_mutants_are_caught(slot, name, oracle_mod):
    """Teeth: a checker that reports one slot as always holding, or as always failing, breaks
    that slot's relation on the mutant-algorithm runs (for Invariant0/1 the always-holding
    mutant breaks the implication; the always-failing one the equivalence on consistent states)."""
    runs = [_run(oracle_mod, 7, 2, 0.1, False, 2, 1, V=2), _run(oracle_mod, 6, 1, 0.1, True, 2, 1, V=2),
            _run(oracle_mod, 16, 2, 0.1, True, 2, 1, V=2), _run(oracle_mod, 16, 2, 0.3, True, 2, 0)]
    caught = {"always": False, "never": False}
    for cfg, tr, bits in runs:
        for kind, forced in (("always", bits | np.uint16(1 << slot)), ("never", bits & np.uint16(~(1 << slot) & 0xFFFF))):
            fails, _ = otr_relations(tr, forced, cfg.n)
            if name is not None:
                caught[kind] |= fails[name] > 0
            else:
                rel = "Invariant0" if slot == INV0 else "Invariant1"
                imp = [k for k in fails if k.startswith(rel + "==>")][0]
                eqv = [k for k in fails if k.startswith("consistent==>(" + rel)][0]
                caught[kind] |= (fails[imp] if kind == "always" else fails[eqv]) > 0
    if slot == VALIDITY:
        # OTR only ever decides a value it received, i.e. an initial value: Validity holds on every
        # reachable state, of the mutant too, so a checker that always says "holds" is
        # indistinguishable on executions; the model side agrees that it holds everywhere
        for cfg, tr, bits in runs:
            data, decided, _, data0 = model_view(tr)
            assert validity(data, np.broadcast_to(data0, data.shape)).all()
        assert caught["never"], caught
        return
    assert caught["always"] and caught["never"], caught


# ------------------------------------------------------------------ LastVoting (LvExample.scala)

def lv_invariant1(tr, n):
    """LvExample.scala:221-238 at every check point c (model phase r = c / 4, the Spec's
    r/4; coord(i) = r % n), data = decision once decided else x, V and t finitized exactly
    (v: data values of A, a non-empty majority; t: the timestamps, A changes only there)."""
    count, C = tr.shape[0], tr.shape[1]
    out = np.zeros((count, C), bool)
    for i in range(count):
        data0 = set(int(v) for v in tr[i, 0, X])
        for c in range(C):
            s = tr[i, c]
            dec = s[DECIDED] != 0
            data = np.where(dec, s[DECISION], s[X]).astype(np.int64)
            ts, ready, commit, vote = s[TS].astype(np.int64), s[READY] != 0, s[COMMIT] != 0, s[VOTE].astype(np.int64)
            r = c // 4
            co = r % n
            no_dec = bool((~dec & ~ready).all())
            maj = False
            if not no_dec:
                for t in sorted(set(ts.tolist())):
                    if t > r:
                        continue
                    A = t <= ts
                    if not n < 2 * int(A.sum()):
                        continue
                    for v in set(data[A].tolist()):
                        ok = ((~A | (data == v)) & (~dec | (data == v)) & (~commit | (vote == v)) &
                              (~ready | (vote == v)) & ((ts != r) | bool(commit[co])))
                        if ok.all():
                            maj = True
                            break
                    if maj:
                        break
            out[i, c] = (no_dec or maj) and all(int(v) in data0 for v in data)
    return out


LV_CASES = [(4, 300, psync.HOSchedule(drop_log2=2, good_round=0.0), 3, 0),
            (7, 300, psync.HOSchedule(drop_log2=2, good_round=0.0, self_bit=False), 3, 0),
            (16, 150, psync.HOSchedule(drop_log2=3, good_round=0.0, crash_fmax=7), 5, 0),
            (64, 40, psync.HOSchedule(drop_log2=2, good_round=0.0, crash_fmax=20), 6, 0),
            (6, 300, psync.HOSchedule(drop_log2=1, good_round=0.0), 5, 1)]


@pytest.mark.parametrize("n,count,sched,V,variant", LV_CASES, ids=[f"n{c[0]}-v{c[4]}" for c in LV_CASES])
def test_lv_checker_matches_reference_formulas(n, count, sched, V, variant, oracle_mod):
    Rl = 16
    cfg = psync.make_config(psync.LastVoting(variant=variant), n, Rl, seed=700 + n, value_range=V, schedule=sched)
    tr, bits = oracle_mod.trace_checks(cfg, 0, count, threads=8, spec_mode=2)
    data, decided, x, data0 = model_view(tr)
    data0 = np.broadcast_to(data0, data.shape)
    dec_valid = (~decided | (data[..., :, None] == data0[..., None, :]).any(-1)).all(-1)
    agr = agreement(data, decided)
    integ = np.ones(agr.shape, bool)
    integ[:, 1:] = integrity(data[:, :-1], decided[:, :-1], data[:, 1:], decided[:, 1:])
    inv1 = lv_invariant1(tr, n)
    # LastVoting's slots: Safety, Invariant0 (safetyInv), Invariant1, Agreement, Validity, Integrity, Irrevocability
    names = psync.LastVoting().check_names
    sl = {nm: _holds(bits, k) for k, nm in enumerate(names)}
    assert (sl["Agreement"] == agr).all()
    assert (sl["Irrevocability"] == integ).all()
    assert (sl["Validity"] == dec_valid).all()
    assert (sl["Integrity"] == (agr & dec_valid)).all()
    assert (_holds(bits, TERM) == termination(decided)).all()
    assert (~sl["Invariant0"] | inv1).all(), np.argwhere(sl["Invariant0"] & ~inv1)[:5]
    # Invariant1 (LastVoting.scala:51) = exists j. forall i. decided(i) && decision(i) == init(j.x)
    assert (sl["Invariant1"] == (invariant_progress2(data, decided) & validity(data, data0))).all()
    if variant == 0:
        assert inv1.all() and sl["Invariant0"].all()
    else:
        assert (~sl["Safety"]).any()  # the mutant's violations are in these runs


# ------------------------------------------------------------------ the GPU checker, directly

@pytest.mark.gpu
@pytest.mark.parametrize("n,variant,drop,V", [(16, 0, 2, 3), (7, 1, 2, 2), (16, 1, 2, 2), (64, 0, 2, 3), (64, 0, 3, 64)])
def test_gpu_first_fail_matches_reference_formulas(n, variant, drop, V, oracle_mod):
    """The GPU's first failing check point of every exactly-determined slot equals the first
    check point where the reference formula fails, on the states of the same instances
    (trace from the oracle; the GPU's per-instance digests equal the oracle's)."""
    count = 400
    alg = psync.OTR(variant=variant)
    cfg, tr, bits = _run(oracle_mod, n, drop, 0.2, True, 2, variant, count=count, V=V)
    data, decided, x, data0 = model_view(tr)
    data0 = np.broadcast_to(data0, data.shape)
    dec_valid = (~decided | (data[..., :, None] == data0[..., None, :]).any(-1)).all(-1)
    agr = agreement(data, decided)
    integ = np.ones(agr.shape, bool)
    integ[:, 1:] = integrity(data[:, :-1], decided[:, :-1], data[:, 1:], decided[:, 1:])
    model = {AGREEMENT: agr, IRREVOCABILITY: integ, VALIDITY: dec_valid, INTEGRITY: agr & dec_valid,
             INV2: invariant_progress2(data, decided) & validity(data, data0)}

    def first_false(a):
        return np.where(a.all(-1), 255, np.argmin(a, axis=-1))

    with psync.GpuRound(alg, n, rounds=R, seed=cfg.seed, value_range=V, batch_capacity=count,
                        schedule=psync.HOSchedule(drop_log2=drop, good_round=0.2)) as g:
        assert g.cfg.seed == cfg.seed and g.cfg.param == cfg.param
        res = g.run(0, count, per_instance=True)
    ff = np.array([list(s.first_fail) for s in res.per_instance])
    term = np.array([s.term_round for s in res.per_instance])
    for slot, a in model.items():
        assert (ff[:, slot] == first_false(a)).all(), (slot, np.argwhere(ff[:, slot] != first_false(a))[:5])
    t = termination(decided)
    assert (term == np.where(t.any(-1), np.argmax(t, axis=-1), 255)).all()
    osum, opi, _ = oracle_mod.run(cfg, 0, count, per_instance=True, threads=8)
    assert [s.digest for s in res.per_instance] == [s.digest for s in opi]  # the same executions
    if variant:
        assert (ff[:, AGREEMENT] != 255).any() and (ff[:, IRREVOCABILITY] != 255).any()
