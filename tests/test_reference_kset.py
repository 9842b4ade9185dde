"""KSetAgreement's decider adoption, pinned to the reference's own expression.

`example/KSetAgreement.scala:47` is `val content = mailbox.map{ case (k,v) => v }` with
`v: (Boolean, Map[ProcessID,Int])`. The function returns a pair, so Scala 2.13 resolves
`map` to `MapOps.map[K2,V2]` and `content` is a `Map[Boolean, Map[ProcessID,Int]]` built by
inserting the messages in the mailbox's iteration order: a later decider overwrites the
value of key `true`. `content.find(_._1).get._2` (:53) is therefore the `t` of the LAST
decider in Map iteration order (insertion order = ascending pid for <= 4 entries, Map1..Map4;
CHAMP order for >= 5).

This file restates the algorithm independently in pure Python (a dict built exactly like
`content`, `_py_champ` for the Map order) and checks the C++ oracle against it: two
hand-built known-answer schedules (n = 5 insertion order, n = 8 CHAMP order) where a
non-decider hears two deciders holding different `t`, and random explicit schedules. The
GPU tests run the same schedules through `psg_load_schedule` and compare with the oracle.
"""
import numpy as np
import pytest

from round_amd import abi, psync
from test_oracle_kat import _py_champ

NEVER = abi.PSG_NEVER


def _map_order(keys, tiebreak):
    keys = sorted(keys)  # the HO harness inserts senders in ascending pid
    if tiebreak == abi.PSG_TIE_MIN_PID or len(keys) <= 4:
        return keys
    return _py_champ(keys)


def py_kset(n, k, init, ho, tiebreak=abi.PSG_TIE_CHAMP, adopt="last"):
    """Literal restatement of KSetProcess (KSetAgreement.scala:21-63) under explicit HO sets
    ho[r][p] (bit q: p hears q). Returns [(decision, decision_round, halt_round)] per p.
    adopt="first" is the mutant (find on an Iterable instead of the collapsed Map)."""
    t = [{p: init[p]} for p in range(n)]  # Map(id -> io.initialValue)
    decider = [False] * n
    halted = [False] * n
    rec = [[0, -1, -1] for _ in range(n)]
    for r in range(len(ho)):
        pre = [(decider[q], dict(t[q])) for q in range(n)]  # broadcast(decider -> t)
        alive = [not h for h in halted]
        for p in range(n):
            if halted[p]:
                continue
            senders = [q for q in range(n) if alive[q] and (ho[r][p] >> q) & 1]
            mailbox = [(q, pre[q]) for q in _map_order(senders, tiebreak)]
            if adopt == "last":
                content = {}
                for _, v in mailbox:  # mailbox.map{ case (k,v) => v }: Map[Boolean, ...]
                    content[v[0]] = v[1]
                found = content.get(True)
            else:
                found = next((v[1] for _, v in mailbox if v[0]), None)
            if decider[p]:
                v = min(t[p].values())  # pick(t)
                rec[p] = [v, r, r]
                halted[p] = True  # exitAtEndOfRound
            elif found is not None:  # content.exists(_._1)
                decider[p] = True
                t[p] = dict(found)
            else:
                same = sum(1 for _, v in mailbox if v[1] == t[p])
                if same > n - k:
                    decider[p] = True
                else:
                    for _, v in mailbox:
                        t[p] = {**t[p], **v[1]}  # t ++ v
    return [tuple(x) for x in rec]


def _kat_n5():
    """n = 5, k = 4 (same.size > 1). Round 0: {0,1} and {2,3} merge pairwise, p4 alone.
    Round 1: the pairs hear themselves again: p0..p3 become deciders with t = {0,1} / {2,3}.
    Round 2: p4 hears {0, 2, 4} (3 entries: insertion order 0, 2, 4) -> content(true) is
    p2's t = {2,3}; p0..p3 decide and exit. Round 3: p4 decides min(30, 40) = 30 (the first
    decider's t would give 10)."""
    n, k = 5, 4
    init = [10, 20, 30, 40, 50]
    r0 = [0b00011, 0b00011, 0b01100, 0b01100, 0b10000]
    r2 = [0b00011, 0b00011, 0b01100, 0b01100, 0b10101]
    return n, k, init, [r0, r0, r2, r2]


def _kat_n8():
    """n = 8, k = 7. Rounds 0-1: pairs {0,1} {2,3} {4,5} become deciders; p6, p7 alone.
    Round 2: p7 hears {1,3,5,6,7}: CHAMP order 5, 1, 6, 7, 3, so the last decider is p3
    (t = {2,3}); the first is p5 and the largest pid is p5 (t = {4,5}). Round 3: p7 decides 30
    and exits; p6 hears {6,7} and adopts t7. Round 4: p6 decides 30."""
    n, k = 8, 7
    init = [10, 20, 30, 40, 50, 60, 70, 80]
    pairs = [0b11, 0b11, 0b1100, 0b1100, 0b110000, 0b110000, 1 << 6, 1 << 7]
    r2 = pairs[:7] + [0b11101010]
    r3 = [0] * 6 + [0b11000000, 1 << 7]
    r4 = [0] * 6 + [1 << 6, 0]
    return n, k, init, [pairs, pairs, r2, r3, r4]


def _oracle_recs(oracle_mod, n, k, init, ho, tiebreak):
    cfg = psync.make_config(psync.KSetAgreement(k), n, rounds=len(ho), value_range=100, tiebreak=tiebreak)
    s, rec, _ = oracle_mod.run_explicit(cfg, init, ho)
    return [(r.decision if r.decision_round != NEVER and r.decision_round >= 0 else 0,
             r.decision_round if r.decision_round != NEVER else -1,
             r.halt_round if r.halt_round != NEVER else -1) for r in rec], s


def test_champ_order_of_kat_mailbox():
    assert _py_champ([1, 3, 5, 6, 7]) == [5, 1, 6, 7, 3]


@pytest.mark.parametrize("kat,expect_last,expect_first", [
    (_kat_n5, 30, 10),
    (_kat_n8, 30, 50),
])
def test_kset_adopts_last_decider(oracle_mod, kat, expect_last, expect_first):
    n, k, init, ho = kat()
    want = py_kset(n, k, init, ho)
    mutant = py_kset(n, k, init, ho, adopt="first")
    last = n - 1
    assert want[last][0] == expect_last and mutant[last][0] == expect_first
    got, s = _oracle_recs(oracle_mod, n, k, init, ho, abi.PSG_TIE_CHAMP)
    assert got == want
    assert got != mutant  # the KAT discriminates the two readings


def test_kset_min_pid_mode_adopts_largest_decider(oracle_mod):
    """PSG_TIE_MIN_PID = ascending-pid order at every size: the last decider is the largest pid."""
    n, k, init, ho = _kat_n8()
    want = py_kset(n, k, init, ho, tiebreak=abi.PSG_TIE_MIN_PID)
    assert want[7][0] == 50
    got, _ = _oracle_recs(oracle_mod, n, k, init, ho, abi.PSG_TIE_MIN_PID)
    assert got == want


def _random_case(rng, n):
    """Sparse, clustered HO sets: many deciders holding different t early on."""
    R = int(rng.integers(3, 8))
    k = int(rng.integers(max(1, n - 3), n))  # same.size > n - k: a low bar, early deciders
    init = [int(v) for v in rng.integers(1, 1000, n)]
    cluster = rng.integers(0, max(2, n // 3), n)  # rounds 0-1: clusters agree among themselves
    ho = []
    for r in range(R):
        row = []
        for p in range(n):
            m = 1 << p
            for q in range(n):
                pr = (0.9 if cluster[q] == cluster[p] else 0.03) if r < 2 else 0.5
                if rng.random() < pr:
                    m |= 1 << q
            row.append(m)
        ho.append(row)
    return k, init, ho


@pytest.mark.parametrize("tiebreak", [abi.PSG_TIE_CHAMP, abi.PSG_TIE_MIN_PID])
def test_oracle_equals_python_restatement_random(oracle_mod, tiebreak):
    rng = np.random.default_rng(47)
    divergent = 0
    for case in range(120):
        n = int(rng.integers(3, 14))
        k, init, ho = _random_case(rng, n)
        want = py_kset(n, k, init, ho, tiebreak=tiebreak)
        got, _ = _oracle_recs(oracle_mod, n, k, init, ho, tiebreak)
        assert got == want, f"case {case}: n={n} k={k}"
        divergent += want != py_kset(n, k, init, ho, tiebreak=tiebreak, adopt="first")
    assert divergent >= 15  # the random cases exercise the adoption rule, not just the merge


# ------------------------------------------------------------------------------------ GPU
def _gpu_run(n, k, inits, hos, tiebreak, R):
    I = len(inits)
    W = (n + 63) // 64
    ho = np.zeros((I, R, n, W), np.uint64)
    for i, h in enumerate(hos):
        for r in range(R):
            for p in range(n):
                for w in range(W):
                    ho[i, r, p, w] = (int(h[r][p]) >> (64 * w)) & ((1 << 64) - 1)
    init = np.array(inits, np.int32)
    with psync.GpuRound(psync.KSetAgreement(k), n, R, seed=3, value_range=1000, batch_capacity=I,
                        tiebreak=tiebreak) as g:
        ctx = g._ctx
        ctx.load_inputs(0, I, init)
        ctx.load_schedule(0, I, ho, None)
        s, pi = ctx.run_batch_np(0, I)
        dec, dr = ctx.copy_decisions_np()
    return dec, dr, ho, init, g.cfg


@pytest.mark.gpu
@pytest.mark.parametrize("tiebreak", [abi.PSG_TIE_CHAMP, abi.PSG_TIE_MIN_PID])
@pytest.mark.parametrize("kat", [_kat_n5, _kat_n8])
def test_gpu_kset_kat(kat, tiebreak):
    n, k, init, ho = kat()
    want = py_kset(n, k, init, ho, tiebreak=tiebreak)
    dec, dr, *_ = _gpu_run(n, k, [init], [ho], tiebreak, len(ho))
    assert [int(x) for x in dr[0]] == [w[1] if w[1] >= 0 else abi.PSG_NEVER for w in want] or \
        [int(x) for x in dr[0]] == [w[1] for w in want]
    assert [int(dec[0][p]) for p in range(n) if want[p][1] >= 0] == [w[0] for w in want if w[1] >= 0]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [12, 40, 64, 100])
def test_gpu_kset_random_adoption(oracle_mod, n):
    """Random sparse explicit schedules (many deciders with different t) at n = 12 ... 100:
    GPU == oracle per instance, and the Python restatement agrees where it runs (n <= 64)."""
    rng = np.random.default_rng(n)
    I, R = 64, 6
    k = max(1, n - 3)
    hos, inits = [], []
    for _ in range(I):
        _, init, ho = _random_case(rng, n)
        ho = [row for row in ho[:R]] + [[(1 << n) - 1] * n] * max(0, R - len(ho))
        hos.append(ho[:R])
        inits.append(init)
    dec, dr, ho_arr, init_arr, cfg = _gpu_run(n, k, inits, hos, abi.PSG_TIE_CHAMP, R)
    osum, opi, orec, _, _ = oracle_mod.run_schedule(cfg, 0, I, ho_arr, None, init_arr, per_instance=True,
                                                     records=True)
    ord_ = np.array([(r.decision, r.decision_round) for r in orec]).reshape(I, n, 2)
    assert (dr == ord_[:, :, 1]).all()
    assert (dec == ord_[:, :, 0]).all()
