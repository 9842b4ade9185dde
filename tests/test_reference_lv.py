"""Pin of the LastVoting rounds against the reference's own formal model.

src/test/scala/psync/logic/LvExample.scala (the VMCAI-paper model of LastVoting the
reference's logic tests use) states the four rounds of a phase as relations over
the pre-state (data, timeStamp, vote, commit, ready, decided), the HO sets and the
post-state (the primed symbols), and gives the phase's invariant:

  maxTSdef (78-97): a non-empty map B's maxTS(B) is the value of some entry j such
                    that every entry i has that value or ts(i) <= ts(j);
  round1  (100-127): mailbox(j) defined at i iff j == coord(i) and i in ho(j), holding
                    (data(i), timeStamp(i)); the coordinator with a majority mailbox
                    (n < 2 |mailbox|) sets vote1 = maxTS(mailbox) and commit1; every
                    other process has not commit1; data, decided, ready, ts framed;
  round2  (130-156): mailbox(j) defined at i iff i == coord(i), commit(i), i in ho(j);
                    receivers of the coordinator take data1 = its vote, ts1 = r;
                    others keep data, ts; decided, ready, commit, vote framed;
  round3  (159-181): mailbox(j) = {i : j == coord(i), ts(i) == r, i in ho(j)};
                    ready1(i) == (i == coord(i) and n < 2 |mailbox(i)|); rest framed;
  round4  (184-213): KeySet(mailbox(i)) = {j : j == coord(j), ready(j), j in ho(i)};
                    receivers of the coordinator take data1 = its vote and decided1;
                    everyone commit1 = ready1 = false; vote, ts framed; r < r1;
  invariant1 (221-238) and the properties agreement / integrity / validity (60-63).

This test transcribes those relations literally (below) and evaluates them on every
round the oracle executes (the GPU matches the oracle bit for bit:
test_gpu_parity.py / test_gpu_sampled.py), for n = 4 ... 64, with and without
crashes and losses, under both Scala-Map tie-break modes. Mapping of the model's
symbols onto LastVoting.scala's state (LastVoting.scala:80-212):

  * `r` of the model is the phase: r = k / 4 in round k, and `coord(i) = r % n`
    (LastVoting.scala:95);
  * `data(i)` is the decision once the process decided, else x: round4 writes the
    coordinator's vote into data1 where the code writes `decision`
    (LastVoting.scala:196-202; x is left unchanged there);
  * the model has no exit: a process that decided has halted (it decides and exits
    in the same round), so it neither sends nor receives; its HO set is taken as
    empty and it is removed from the others' HO sets (the HO-model encoding of a
    halted process);
  * LastVoting.scala:127-129 lets the coordinator of round 0 also commit on any
    non-empty mailbox (`r == 0 && mailbox.size > 0`), a case outside round1's
    majority condition: at k = 0 the test checks round1 with that disjunct added,
    and counts how often it applied.
"""
import numpy as np
import pytest

from round_amd import abi, psync

NF = 9
X, DECIDED, DECISION, TS, READY, COMMIT, VOTE = 0, 1, 2, 3, 4, 5, 6


def _maxts_ok(box, val):
    """maxTSdef (LvExample.scala:78-97) for one non-empty map box = {pid: (value, ts)}."""
    return any(box[j][0] == val and all(box[i][0] == val or box[i][1] <= box[j][1] for i in box) for j in box)


def _state(row, n):
    d = {f: [int(v) for v in row[f]] for f in (X, DECIDED, DECISION, TS, READY, COMMIT, VOTE)}
    return {
        "data": [d[DECISION][i] if d[DECIDED][i] else d[X][i] for i in range(n)],
        "decided": [bool(v) for v in d[DECIDED]],
        "ts": d[TS], "ready": [bool(v) for v in d[READY]], "commit": [bool(v) for v in d[COMMIT]],
        "vote": d[VOTE],
    }


def _frame(pre, post, names, n):
    for f in names:
        for i in range(n):
            if pre[f][i] != post[f][i]:
                return f"frame {f} of p{i}: {pre[f][i]} -> {post[f][i]}"
    return None


def _round1(n, r, k, pre, post, ho):
    """LvExample.scala:100-127 (+ LastVoting.scala:127-129 at k == 0, flagged)."""
    co = r % n
    used_r0 = False
    mb = {i: (pre["data"][i], pre["ts"][i]) for i in range(n) if i in ho[co]}  # mailbox1(coord)
    for i in range(n):
        majority = i == co and n < 2 * len(mb)
        r0 = i == co and k == 0 and len(mb) > 0 and not majority
        if majority or r0:
            used_r0 |= r0
            if not (post["commit"][i] and _maxts_ok(mb, post["vote"][i])):
                return f"coordinator p{i}: vote1 {post['vote'][i]} / commit1 {post['commit'][i]} vs maxTS", used_r0
        elif post["commit"][i]:
            return f"p{i}: commit1 without a majority at the coordinator", used_r0
    return _frame(pre, post, ("decided", "data", "ready", "ts"), n), used_r0


def _round2(n, r, pre, post, ho):
    """LvExample.scala:130-156."""
    co = r % n
    for i in range(n):
        if pre["commit"][co] and co in ho[i]:  # IsDefinedAt(mailbox2(i), coord(i))
            if post["data"][i] != pre["vote"][co] or post["ts"][i] != r:
                return f"p{i}: data1/ts1 {post['data'][i]}/{post['ts'][i]} != vote {pre['vote'][co]}/{r}"
        elif post["data"][i] != pre["data"][i] or post["ts"][i] != pre["ts"][i]:
            return f"p{i}: data/ts changed without the coordinator's vote"
    return _frame(pre, post, ("decided", "ready", "commit", "vote"), n)


def _round3(n, r, pre, post, ho):
    """LvExample.scala:159-181."""
    co = r % n
    for i in range(n):
        mb = [j for j in range(n) if i == co and pre["ts"][j] == r and j in ho[i]]
        if post["ready"][i] != (i == co and n < 2 * len(mb)):
            return f"p{i}: ready1 {post['ready'][i]} with |mailbox3| {len(mb)}"
    return _frame(pre, post, ("decided", "data", "commit", "vote", "ts"), n)


def _round4(n, r, pre, post, ho):
    """LvExample.scala:184-213."""
    co = r % n
    for i in range(n):
        if pre["ready"][co] and co in ho[i]:  # coord(i) in KeySet(mailbox4(i))
            if post["data"][i] != pre["vote"][co] or not post["decided"][i]:
                return f"p{i}: data1 {post['data'][i]} / decided1 after the coordinator's vote {pre['vote'][co]}"
        elif post["data"][i] != pre["data"][i] or post["decided"][i] != pre["decided"][i]:
            return f"p{i}: data/decided changed without the coordinator's vote"
        if post["commit"][i] or post["ready"][i]:
            return f"p{i}: commit1/ready1 not reset"
    return _frame(pre, post, ("vote", "ts"), n)


def _invariant1(n, r, s, data0):
    """LvExample.scala:221-238, V and the phase type finitized exactly: v ranges over the
    data values (A is a non-empty majority), t over the timestamps (A = {i : t <= ts(i)}
    only changes at a timestamp, and every ts <= r)."""
    co = r % n
    no_dec = all(not s["decided"][i] and not s["ready"][i] for i in range(n))
    maj = False
    if not no_dec:
        for t in sorted(set(s["ts"])):
            if t > r:
                continue
            A = [i for i in range(n) if t <= s["ts"][i]]
            if not n < 2 * len(A):
                continue
            for v in set(s["data"][i] for i in A):
                if all((i not in A or s["data"][i] == v) and (not s["decided"][i] or s["data"][i] == v) and
                       (not s["commit"][i] or s["vote"][i] == v) and (not s["ready"][i] or s["vote"][i] == v) and
                       (s["ts"][i] != r or s["commit"][co]) for i in range(n)):
                    maj = True
                    break
            if maj:
                break
    valid = all(s["data"][i] in data0 for i in range(n))
    return (no_dec or maj) and valid


def _agreement(n, s):
    """LvExample.scala:60."""
    return len({s["data"][i] for i in range(n) if s["decided"][i]}) <= 1


# (n, count, schedule, tiebreak, value_range)
H = psync.HOSchedule
CASES = [
    (4, 300, H(drop_log2=2, good_round=0.0), abi.PSG_TIE_CHAMP, 3),
    (5, 300, H(drop_log2=1, good_round=0.0, crash_fmax=2), abi.PSG_TIE_CHAMP, 4),
    (7, 300, H(drop_log2=2, good_round=0.0, self_bit=False), abi.PSG_TIE_CHAMP, 3),
    (16, 200, H(drop_log2=3, good_round=0.0, crash_fmax=7), abi.PSG_TIE_CHAMP, 5),
    (16, 200, H(drop_log2=1, good_round=0.0), abi.PSG_TIE_MIN_PID, 5),
    (64, 60, H(drop_log2=4, good_round=0.0, crash_fmax=31), abi.PSG_TIE_CHAMP, 32767),
    (64, 60, H(drop_log2=2, good_round=0.0), abi.PSG_TIE_CHAMP, 3),
    (64, 60, H(drop_log2=2, good_round=0.0, crash_fmax=20), abi.PSG_TIE_MIN_PID, 6),
]


@pytest.mark.parametrize("n,count,sched,tb,V", CASES,
                         ids=[f"n{c[0]}-{i}" for i, c in enumerate(CASES)])
def test_oracle_rounds_satisfy_lv_model(n, count, sched, tb, V, oracle_mod):
    R = 24
    cfg = psync.make_config(psync.LastVoting(), n, R, seed=900 + n, value_range=V, schedule=sched, tiebreak=tb)
    tr = np.frombuffer(oracle_mod.trace(cfg, 0, count, threads=8), dtype=np.int32).reshape(count, R + 1, NF, n)
    ho, _ = oracle_mod.materialize_schedule(cfg, 0, count)
    W = (n + 63) // 64
    stats = {"rounds": 0, "r0_shortcut": 0, "decisions": 0, "commits": 0}
    for inst in range(count):
        states = [_state(tr[inst, c], n) for c in range(R + 1)]
        data0 = set(states[0]["data"])
        assert _invariant1(n, 0, states[0], data0)
        for k in range(R):
            pre, post, r = states[k], states[k + 1], k // 4
            halted = [pre["decided"][i] for i in range(n)]  # LV decides and exits in the same round
            sets = []
            for p in range(n):
                if halted[p]:
                    sets.append(set())
                    continue
                m = [int(ho[inst, k, p, w]) for w in range(W)]
                sets.append({q for q in range(n) if (m[q >> 6] >> (q & 63)) & 1 and not halted[q]})
            if k % 4 == 0:
                err, r0 = _round1(n, r, k, pre, post, sets)
                stats["r0_shortcut"] += r0
            elif k % 4 == 1:
                err = _round2(n, r, pre, post, sets)
            elif k % 4 == 2:
                err = _round3(n, r, pre, post, sets)
            else:
                err = _round4(n, r, pre, post, sets)
            assert err is None, f"instance {inst} round {k} (LvExample round{k % 4 + 1}): {err}"
            # integrity (LvExample.scala:61) on every transition
            assert all(not pre["decided"][i] or (post["decided"][i] and pre["data"][i] == post["data"][i])
                       for i in range(n)), (inst, k)
            rr = (k + 1) // 4  # the phase of the post-state (round4 moves r to r + 1)
            assert _invariant1(n, rr, post, data0), f"instance {inst}: invariant1 false after round {k}"
            assert _agreement(n, post), (inst, k)
            stats["rounds"] += 1
            stats["commits"] += sum(post["commit"]) if k % 4 == 0 else 0
        stats["decisions"] += sum(states[R]["decided"])
    assert stats["rounds"] == count * R
    assert stats["decisions"] > 0 and stats["commits"] > 0, stats


def test_mutant_breaks_the_model(oracle_mod):
    """The test has teeth: the build's LastVoting mutation (variant 1, R2 quorum 0,
    DESIGN §2) sets ready without a majority, which round3 of the model forbids."""
    n, R, count = 6, 16, 200
    cfg = psync.make_config(psync.LastVoting(variant=1), n, R, seed=15, value_range=5)
    tr = np.frombuffer(oracle_mod.trace(cfg, 0, count, threads=8), dtype=np.int32).reshape(count, R + 1, NF, n)
    ho, _ = oracle_mod.materialize_schedule(cfg, 0, count)
    broken = 0
    for inst in range(count):
        for k in range(2, R, 4):
            pre, post = _state(tr[inst, k], n), _state(tr[inst, k + 1], n)
            halted = pre["decided"]
            sets = [set() if halted[p] else {q for q in range(n) if (int(ho[inst, k, p, 0]) >> q) & 1 and not halted[q]}
                    for p in range(n)]
            broken += _round3(n, k // 4, pre, post, sets) is not None
    assert broken > 0
