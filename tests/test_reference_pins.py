"""The last reference-held pins of the path (VERDICT r3 "Next round" #2), each with a mutant
that breaks it.

1. `example/Otr2.scala:32-36` — the `ensuring` post-condition of `mmor`:
       mailbox.forall{ (k, v2) => count(v1) > count(v2) || v1 <= v2 }
   checked by the oracle on every mmor it executes (OTR and OTR2 share the round;
   `oracle_mmor_ensuring_stats`), and on the GPU's own OTR2 results: the same explicit
   schedule run for R = 1 .. K rounds gives, through `psg_fetch_instances`, every process's x
   after each round, and each adopted x is checked against the mailbox it was computed from.
2. `src/test/scala/psync/logic/OtrExampleNoMailbox.scala` — OTR with `twoThird(ho(i))` in
   place of the mailbox (`tr` 81-98), its invariants (44-61) and every VC of the file (the
   `ignore`d ones included) evaluated concretely on every round the oracle executes.
3. `src/test/scala/psync/logic/LvExampleNoMailbox.scala` — LastVoting's four rounds over HO
   sets (`round1` .. `round4`, 99-185), `invariant1` / `1c` / `1d` (195-297) and the `maxTS`
   lemma (334-345), on every LastVoting round the oracle executes. The model's `ho(i)` is the
   set of processes i received from (KeySet(mailbox(i)) of LvExample.scala), so a directed
   send that was not made is not heard.
4. `src/test/scala/psync/utils/LongBitSetTests.scala:7-38` — get / set / clear / size of the
   reference's 64-bit heard-from set, restated against the device HO word `Mask<W>`
   (`psg_selftest_bitset`; index mod 64, mod 64W for W words).
"""
import numpy as np
import pytest

from round_amd import abi, psync
import test_reference_lv as LVX
from test_reference_tr import _mmor

NF = 9
X, DECIDED = 0, 1
H = psync.HOSchedule


# ----------------------------------------------------------------------------- 1. Otr2 ensuring
def ensuring(mailbox_vals, v1):
    """Otr2.scala:33-35, literally."""
    cnt = lambda v: sum(1 for v3 in mailbox_vals if v3 == v)  # noqa: E731
    return all(cnt(v1) > cnt(v2) or v1 <= v2 for v2 in mailbox_vals)


@pytest.fixture
def mmor_check(oracle_mod):
    """The oracle's ensuring check is off by default (the CPU baseline times the round alone)."""
    L = oracle_mod.lib()
    L.oracle_set_mmor_check(1)
    yield
    L.oracle_set_mmor_check(0)


def _stats(oracle_mod, reset=False):
    import ctypes as C
    L = oracle_mod.lib()
    calls, fails = C.c_uint64(), C.c_uint64()
    L.oracle_mmor_ensuring_stats(C.byref(calls), C.byref(fails), 1 if reset else 0)
    return calls.value, fails.value


@pytest.mark.parametrize("alg", [psync.OTR(), psync.OTR2()], ids=["otr", "otr2"])
def test_oracle_mmor_satisfies_otr2_ensuring(oracle_mod, mmor_check, alg):
    _stats(oracle_mod, reset=True)
    for n, V, seed in ((4, 3, 1), (16, 4, 2), (64, 64, 3), (64, 2, 4)):
        cfg = psync.make_config(alg, n, 10, seed=seed, value_range=V)
        oracle_mod.run(cfg, 0, 300 if n <= 16 else 60, threads=8)
    calls, fails = _stats(oracle_mod, reset=True)
    assert calls > 10000 and fails == 0, (calls, fails)


def test_ensuring_catches_a_mutant_mmor(oracle_mod, mmor_check):
    """Variant 2 (an oracle-only mutant: mmor ties go to the LARGER value) violates it."""
    _stats(oracle_mod, reset=True)
    cfg = psync.make_config(psync.OTR2(variant=2), 16, 10, seed=5, value_range=4)
    oracle_mod.run(cfg, 0, 300, threads=8)
    calls, fails = _stats(oracle_mod, reset=True)
    assert calls > 0 and fails > 0
    assert not ensuring([1, 1, 2, 2], 2) and ensuring([1, 1, 2, 2], 1) and ensuring([3, 3, 3, 1], 3)


def test_ensuring_check_is_off_by_default(oracle_mod):
    """Without the pin tests' switch the oracle runs mmor alone (what cpu_baseline times)."""
    _stats(oracle_mod, reset=True)
    oracle_mod.run(psync.make_config(psync.OTR(), 16, 10, seed=2, value_range=4), 0, 50, threads=2)
    assert _stats(oracle_mod, reset=True) == (0, 0)


@pytest.mark.gpu
def test_gpu_otr2_adoptions_satisfy_ensuring():
    """The GPU's own OTR2 results: x after every round (runs truncated at R = 1 .. K of one
    explicit schedule, read back by psg_fetch_instances); each x adopted from a mailbox of
    more than 2n/3 messages satisfies Otr2.scala:32-36 against that mailbox."""
    n, I, K = 16, 64, 6
    rng = np.random.default_rng(17)
    ho = np.zeros((I, K, n, 1), np.uint64)
    for i in range(I):
        for k in range(K):
            for p in range(n):
                m = 1 << p
                for q in range(n):
                    if rng.random() < 0.8:
                        m |= 1 << q
                ho[i, k, p, 0] = m
    init = rng.integers(1, 4, (I, n)).astype(np.int32)
    xs = [init]
    alg = psync.OTR2(afterDecision=K + 2)  # nobody halts: every process sends every round
    for R in range(1, K + 1):
        with psync.GpuRound(alg, n, R, seed=3, value_range=3, batch_capacity=I) as g:
            g.load_inputs(0, I, init)
            g.load_schedule(0, I, np.ascontiguousarray(ho[:, :R]))
            g.run(0, I)
            _, rec = g._ctx.fetch_np(np.arange(I, dtype=np.uint64))
        xs.append(np.array(rec["final_x"], dtype=np.int64))
    checked = 0
    for i in range(I):
        for k in range(K):
            for p in range(n):
                mb = [int(xs[k][i, q]) for q in range(n) if (int(ho[i, k, p, 0]) >> q) & 1]
                if len(mb) > 2 * n // 3:
                    v1 = int(xs[k + 1][i, p])
                    assert ensuring(mb, v1), (i, k, p, mb, v1)
                    assert v1 == _mmor(mb)  # and OtrExample.scala:67-75's defs
                    checked += 1
    assert checked > 1000


# ----------------------------------------------------------------------------- 2. OtrExampleNoMailbox
def _otr_nm(n):
    tt = (2 * n) // 3

    def value_is(ho_i, data, f):
        return [j for j in ho_i if data[j] == f]

    def tr(data, decided, ho, data1, decided1):
        """OtrExampleNoMailbox.scala:81-98 (mmor by defs 70-79)."""
        for i in range(n):
            if len(ho[i]) > tt:
                m = _mmor([data[j] for j in ho[i]])
                want = True if len(value_is(ho[i], data, m)) > tt else decided[i]
                if data1[i] != m or decided1[i] != want:
                    return f"p{i}"
            elif decided1[i] != decided[i] or data1[i] != data[i]:
                return f"p{i}: frame"
        return None

    def inv_agreement(data, decided):  # 44-51
        if not any(decided):
            return True
        return any(sum(1 for i in range(n) if data[i] == v) > tt and
                   all(not decided[i] or data[i] == v for i in range(n)) for v in set(data))

    def inv_progress1(data, decided):  # 53-57
        return any(sum(1 for i in range(n) if data[i] == v) == n and
                   all(not decided[i] or data[i] == v for i in range(n)) for v in set(data))

    def inv_progress2(data, decided):  # 59-60
        return any(all(decided[i] and data[i] == v for i in range(n)) for v in set(data))

    def magic(ho):  # 100-103
        return all(h == ho[0] for h in ho) and len(ho[0]) > tt

    return tr, inv_agreement, inv_progress1, inv_progress2, magic


OTR_CASES = [(4, 2, 0.3, True), (7, 2, 0.25, True), (16, 3, 0.25, False), (16, 1, 0.1, True), (64, 3, 0.25, True)]


def _otr_run(oracle_mod, alg, n, drop, good, self_bit, count, R=10, seed=41):
    cfg = psync.make_config(alg, n, R, seed=seed + n, value_range=3,
                            schedule=H(drop_log2=drop, good_round=good, self_bit=self_bit))
    tr = np.frombuffer(oracle_mod.trace(cfg, 0, count, threads=8), dtype=np.int32).reshape(count, R + 1, NF, n)
    ho, _ = oracle_mod.materialize_schedule(cfg, 0, count)
    return tr, ho


@pytest.mark.parametrize("n,drop,good,self_bit", OTR_CASES, ids=[f"n{c[0]}-d{c[1]}-s{int(c[3])}" for c in OTR_CASES])
def test_oracle_rounds_satisfy_otr_nomailbox_model(oracle_mod, n, drop, good, self_bit):
    R = 10
    count = 200 if n <= 16 else 40
    trace, ho = _otr_run(oracle_mod, psync.OTR(afterDecision=R + 2), n, drop, good, self_bit, count, R)
    tr, inv_ag, inv_p1, inv_p2, magic = _otr_nm(n)
    used = dict.fromkeys(["p1", "p2", "magic1", "magic2", "mmor_lemma", "integrity", "decided"], 0)
    for i in range(count):
        data0 = set(int(v) for v in trace[i, 0, X])
        s0 = (list(trace[i, 0, X]), [bool(v) for v in trace[i, 0, DECIDED]])
        assert not any(s0[1]) and inv_ag(*s0)              # initial state implies invariant
        for k in range(R):
            pre = (list(trace[i, k, X]), [bool(v) for v in trace[i, k, DECIDED]])
            post = (list(trace[i, k + 1, X]), [bool(v) for v in trace[i, k + 1, DECIDED]])
            sets = [{q for q in range(n) if (int(ho[i, k, p, q >> 6]) >> (q & 63)) & 1} for p in range(n)]
            err = tr(pre[0], pre[1], sets, post[0], post[1])
            assert err is None, f"instance {i} round {k}: tr {err}"
            a0, a1 = inv_ag(*pre), inv_ag(*post)
            assert not a0 or a1                                 # invariant is inductive (ignored VC)
            if a1:                                              # invariant implies agreement
                assert len({post[0][j] for j in range(n) if post[1][j]}) <= 1
            if inv_p1(*pre):                                    # invariant 1 is inductive (ignored VC)
                used["p1"] += 1
                assert inv_p1(*post)
            if inv_p2(*pre):                                    # invariant 2 is inductive; => termination
                used["p2"] += 1
                assert inv_p2(*post) and all(pre[1])
            if magic(sets) and a0:                              # 1st magic round (ignored VC)
                used["magic1"] += 1
                assert inv_p1(*post)
            if magic(sets) and inv_p1(*pre):                    # 2nd magic round
                used["magic2"] += 1
                assert inv_p2(*post)
            if a0 and a1:                                       # integrity; validity is inductive
                used["integrity"] += any(pre[1])
                assert all(not pre[1][j] or (post[1][j] and pre[0][j] == post[0][j]) for j in range(n))
                assert all(v in data0 for v in post[0])
            for v in set(pre[0]):                               # "mmor unsat" (the lemma)
                if sum(1 for j in range(n) if pre[0][j] == v) > (2 * n) // 3 and \
                        all(len(s) > (2 * n) // 3 for s in sets):
                    used["mmor_lemma"] += 1
                    assert all(x == v for x in post[0])
        used["decided"] += sum(post[1])
    assert used["integrity"] > 0 and used["mmor_lemma"] > 0 and used["p1"] > 0, used


def test_otr_nomailbox_model_has_teeth(oracle_mod):
    """The n/2-threshold mutant (variant 1) breaks tr's twoThird(ho(i)) guard."""
    n, R, count = 7, 8, 200
    trace, ho = _otr_run(oracle_mod, psync.OTR(afterDecision=R + 2, variant=1), n, 1, 0.0, True, count, R)
    tr = _otr_nm(n)[0]
    broken = 0
    for i in range(count):
        for k in range(R):
            sets = [{q for q in range(n) if (int(ho[i, k, p, 0]) >> q) & 1} for p in range(n)]
            broken += tr(list(trace[i, k, X]), [bool(v) for v in trace[i, k, DECIDED]], sets,
                         list(trace[i, k + 1, X]), [bool(v) for v in trace[i, k + 1, DECIDED]]) is not None
    assert broken > 0


# ----------------------------------------------------------------------------- 3. LvExampleNoMailbox
def _heard(n, k, pre, sets):
    """ho(i) of the model in round k (slot k % 4): the processes i received from."""
    co = (k // 4) % n
    slot = k % 4
    out = [set() for _ in range(n)]
    for i in range(n):
        if slot == 0 and i == co:      # everyone sends (x, ts) to the coordinator
            out[i] = set(sets[i])
        elif slot == 1:                # the coordinator broadcasts its vote if commit
            out[i] = {co} if pre["commit"][co] and co in sets[i] else set()
        elif slot == 2 and i == co:    # those with ts == r send x to the coordinator
            out[i] = {j for j in sets[i] if pre["ts"][j] == k // 4}
        elif slot == 3:                # the coordinator broadcasts if ready
            out[i] = {co} if pre["ready"][co] and co in sets[i] else set()
    return out


def _lv_rounds_nm(n, k, pre, post, ho):
    """LvExampleNoMailbox.scala:99-185 over ho = _heard(...); the k == 0 coordinator shortcut of
    LastVoting.scala:127-129 (commit on any non-empty mailbox) is allowed, as in
    test_reference_lv.py."""
    r, co, slot = k // 4, (k // 4) % n, k % 4
    maj = lambda s: n < 2 * len(s)  # noqa: E731  majorityS
    if slot == 0:  # round1: maxTSdef (75-96), then / else branches, frame
        for i in range(n):
            if i == co and (maj(ho[i]) or (k == 0 and ho[i])):
                box = {j: (pre["data"][j], pre["ts"][j]) for j in ho[i]}
                if not (post["commit"][i] and LVX._maxts_ok(box, post["vote"][i])):
                    return f"round1: coordinator p{i}"
            elif post["commit"][i]:
                return f"round1: p{i} commit1"
        return LVX._frame(pre, post, ("decided", "data", "ready", "ts"), n)
    if slot == 1:  # round2
        for i in range(n):
            if co in ho[i]:
                if post["data"][i] != pre["vote"][co] or post["ts"][i] != r:
                    return f"round2: p{i}"
            elif post["data"][i] != pre["data"][i] or post["ts"][i] != pre["ts"][i]:
                return f"round2: p{i} frame"
        return LVX._frame(pre, post, ("decided", "ready", "commit", "vote"), n)
    if slot == 2:  # round3
        for i in range(n):
            if post["ready"][i] != (i == co and maj(ho[i])):
                return f"round3: p{i} ready1"
        return LVX._frame(pre, post, ("decided", "data", "commit", "vote", "ts"), n)
    for i in range(n):  # round4
        if co in ho[i]:
            if post["data"][i] != pre["vote"][co] or not post["decided"][i]:
                return f"round4: p{i}"
        elif post["data"][i] != pre["data"][i] or post["decided"][i] != pre["decided"][i]:
            return f"round4: p{i} frame"
        if post["commit"][i] or post["ready"][i]:
            return f"round4: p{i} reset"
    return LVX._frame(pre, post, ("vote", "ts"), n)


def _invariant1c(n, r, s, data0):
    """LvExampleNoMailbox.scala:255-274: invariant1 without the coordinator conjunct."""
    ok = all(not s["decided"][i] and not s["ready"][i] for i in range(n))
    for t in sorted(set(s["ts"])):
        if ok or t > r:
            continue
        A = [i for i in range(n) if t <= s["ts"][i]]
        if n < 2 * len(A):
            for v in set(s["data"][i] for i in A):
                if all((i not in A or s["data"][i] == v) and (not s["decided"][i] or s["data"][i] == v) and
                       (not s["commit"][i] or s["vote"][i] == v) and (not s["ready"][i] or s["vote"][i] == v)
                       for i in range(n)):
                    ok = True
    return ok and all(s["data"][i] in data0 for i in range(n))


def _maxts_lemma(n, pre, post, co, ho_co):
    """LvExampleNoMailbox.scala:334-345: maxTSdef, A = {i : t <= ts(i)} a majority holding v,
    a majority HO at the coordinator  =>  maxTS == v (here: the coordinator's vote1)."""
    if not n < 2 * len(ho_co):
        return 0
    used = 0
    for t in set(pre["ts"]):
        A = [i for i in range(n) if t <= pre["ts"][i]]
        vals = {pre["data"][i] for i in A}
        if n < 2 * len(A) and len(vals) == 1:
            used += 1
            assert post["vote"][co] == next(iter(vals)), (t, vals, post["vote"][co])
    return used


def _lv_transitions(oracle_mod, alg, n, count, sched, tb, V, R=24, seed=700):
    cfg = psync.make_config(alg, n, R, seed=seed + n, value_range=V, schedule=sched, tiebreak=tb)
    tr = np.frombuffer(oracle_mod.trace(cfg, 0, count, threads=8), dtype=np.int32).reshape(count, R + 1, NF, n)
    ho, _ = oracle_mod.materialize_schedule(cfg, 0, count)
    W = (n + 63) // 64
    for inst in range(count):
        states = [LVX._state(tr[inst, c], n) for c in range(R + 1)]
        for k in range(R):
            pre = states[k]
            sets = []
            for p in range(n):
                if pre["decided"][p]:  # LastVoting decides and exits in the same round
                    sets.append(set())
                    continue
                m = [int(ho[inst, k, p, w]) for w in range(W)]
                sets.append({q for q in range(n) if (m[q >> 6] >> (q & 63)) & 1 and not pre["decided"][q]})
            yield inst, k, states, sets


@pytest.mark.parametrize("n,count,sched,tb,V", LVX.CASES, ids=[f"n{c[0]}-{i}" for i, c in enumerate(LVX.CASES)])
def test_oracle_rounds_satisfy_lv_nomailbox_model(oracle_mod, n, count, sched, tb, V):
    used = {"maxts": 0, "rounds": 0}
    for inst, k, states, sets in _lv_transitions(oracle_mod, psync.LastVoting(), n, count, sched, tb, V):
        pre, post = states[k], states[k + 1]
        data0 = set(states[0]["data"])
        if k == 0:  # initial state implies invariant; validity holds initially
            assert LVX._invariant1(n, 0, pre, data0) and _invariant1c(n, 0, pre, data0)
        ho = _heard(n, k, pre, sets)
        err = _lv_rounds_nm(n, k, pre, post, ho)
        assert err is None, f"instance {inst} round {k}: {err}"
        rr = (k + 1) // 4
        # invariant 1 is inductive at round 1 .. 4 (the ignored VCs), and 1c (1d = 1 with the
        # comprehension variable renamed); invariant implies agreement
        if LVX._invariant1(n, k // 4, pre, data0):
            assert LVX._invariant1(n, rr, post, data0), f"instance {inst}: invariant1 not inductive at {k}"
        assert _invariant1c(n, rr, post, data0)
        assert LVX._agreement(n, post)
        if k % 4 == 0:
            co = (k // 4) % n
            used["maxts"] += _maxts_lemma(n, pre, post, co, ho[co])
        used["rounds"] += 1
    assert used["maxts"] > 0, used


def test_lv_nomailbox_model_has_teeth(oracle_mod):
    """LastVoting's R2 quorum-0 mutant (variant 1) sets ready without a majority: round3 breaks."""
    broken = 0
    for inst, k, states, sets in _lv_transitions(oracle_mod, psync.LastVoting(variant=1), 6, 150, H(), 0, 5, R=16):
        if k % 4 == 2:
            broken += _lv_rounds_nm(6, k, states[k], states[k + 1], _heard(6, k, states[k], sets)) is not None
    assert broken > 0


# ----------------------------------------------------------------------------- 4. LongBitSetTests
class PyLongBitSet:
    """psync/utils/LongBitSet.scala:5-33 restated (the CPU side of the check)."""

    def __init__(self, store=0, wrap=True):
        self.store, self.wrap = store & ((1 << 64) - 1), wrap

    def _b(self, pos):
        return 1 << (pos & 63) if self.wrap else (1 << pos if 0 <= pos < 64 else 0)

    def run(self, ops):
        out = []
        for op, pos in ops:
            if op == "empty":
                self.store = 0
            elif op == "full":
                self.store = (1 << 64) - 1
            elif op == "set":
                self.store |= self._b(pos)
            elif op == "clear":
                self.store &= ~self._b(pos)
            elif op == "flip":
                self.store ^= self._b(pos)
            elif op == "get":
                out.append(1 if self.store & self._b(pos) else 0)
            else:
                out.append(bin(self.store).count("1"))
        return out


def long_bitset_suite(run, size=64):
    """LongBitSetTests.scala:7-38 as a list of (ops, expected results); `run` executes ops.
    size = the set's index range (64 for LongBitSet and Mask<1>; 64W for Mask<W>)."""
    fails = []

    def check(ops, want, what):
        got = run(ops)
        if got != want:
            fails.append((what, got[:8], want[:8]))

    # "full/empty" (9-14)
    check([("empty", 0)] + [("get", i) for i in range(size)], [0] * size, "empty.get")
    check([("full", 0)] + [("get", i) for i in range(size)], [1] * size, "full.get")
    # "set" (16-23) and "clear" (25-32): one batch per i
    for i in range(size):
        check([("empty", 0), ("set", i)] + [("get", j) for j in range(size)],
              [1 if j == i else 0 for j in range(size)], f"set({i})")
        check([("full", 0), ("clear", i)] + [("get", j) for j in range(size)],
              [0 if j == i else 1 for j in range(size)], f"clear({i})")
    # "size" (34-38): indices wrap modulo the set's range
    check([("empty", 0), ("size", 0), ("full", 0), ("size", 0)], [0, size], "size empty/full")
    check([("empty", 0), ("set", 1), ("set", size // 2), ("set", size), ("size", 0)], [3], "set(64) wraps to 0")
    check([("empty", 0), ("set", 1), ("set", size // 2), ("set", size + 1), ("size", 0)], [2], "set(65) wraps to 1")
    return fails


def test_long_bitset_suite_pins_the_restatement():
    assert long_bitset_suite(lambda ops: PyLongBitSet().run(ops)) == []
    # the mutant without the mod-64 index (an out-of-range index ignored) fails "size"
    bad = long_bitset_suite(lambda ops: PyLongBitSet(wrap=False).run(ops))
    assert [w for w, _, _ in bad] == ["set(64) wraps to 0"]


@pytest.mark.gpu
@pytest.mark.parametrize("W", [1, 2, 3, 4])
def test_gpu_mask_passes_long_bitset_tests(W):
    from round_amd import lib
    assert long_bitset_suite(lambda ops: lib.selftest_bitset(ops, W), size=64 * W) == []
    # flip (LongBitSet.scala:9): involution, and equal to set / clear on the bit
    assert lib.selftest_bitset([("empty", 0), ("flip", 5), ("get", 5), ("flip", 5), ("get", 5), ("size", 0)], W) \
        == [1, 0, 0]
    # negative positions wrap modulo 64W on the signed value (Java's `1L << -1` is bit 63 for W = 1)
    size = 64 * W
    assert lib.selftest_bitset([("empty", 0), ("set", -1), ("get", size - 1), ("set", -size - 2),
                                ("get", size - 2), ("size", 0)], W) == [1, 1, 2]
