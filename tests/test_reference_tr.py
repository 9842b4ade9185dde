"""Pin of the OTR round against the reference's own formal transition relation.

src/test/scala/psync/logic/OtrExample.scala (the VMCAI-paper model the
reference's logic tests use) states the OTR round as a formula over the
pre-state (data, decided), the HO sets and the post-state (data1, decided1):

  defs (67-75): mmor(i) occurs in mailbox(i), has maximal multiplicity, and is
                the smallest (Leq) among the values of that multiplicity;
  tr   (77-96): KeySet(mailbox(i)) == ho(i), mailbox(i)(j) == data(j);
                |mailbox(i)| > 2n/3  ==>  data1(i) == mmor(i) and
                    decided1(i) == (|valueIs(mmor(i))| > 2n/3 ? True : decided(i));
                otherwise data1(i) == data(i) and decided1(i) == decided(i);
  magicRound (98-101): exists A. |A| > 2n/3 and forall i. ho(i) == A.

This test evaluates that relation, transcribed literally below, on every
round executed by the oracle (which the GPU matches bit for bit,
test_gpu_parity.py / test_gpu_schedule.py). The model has no exit, so the
instances run with afterDecision > R (nobody halts; every process sends every
round, as in the model). HO sets are the exported schedule of the same
instances (psg_materialize_schedule's CPU restatement). Also pinned: after a
magicRound every process holds the same data (the progress lemma the
reference proves from the model, OtrExample.scala:121-140 "mmor unsat").
"""
import numpy as np
import pytest

from round_amd import psync

NF = 9  # trace fields (include/psg.h enum psg_field)
X, DECIDED = 0, 1


def _mmor(mailbox_vals):
    """OtrExample.scala:67-75 defs, literally: the value with card >= 1 whose card is
    maximal and which is Leq every other value of maximal card."""
    best = None
    for v in set(mailbox_vals):
        c = mailbox_vals.count(v)
        if c < 1:
            continue
        ok = all(mailbox_vals.count(p) <= c for p in set(mailbox_vals))
        ok = ok and all(v <= p for p in set(mailbox_vals) if mailbox_vals.count(p) == c)
        if ok:
            assert best is None, "defs determine mmor uniquely"
            best = v
    return best


def _tr(n, data, decided, ho, data1, decided1):
    """OtrExample.scala:77-96 for one round (lists indexed by pid; ho[i] = set of pids)."""
    two_third = (2 * n) // 3
    for i in range(n):
        mailbox = {j: data[j] for j in ho[i]}              # KeySet == ho(i), LookUp == data(j)
        if len(mailbox) > two_third:                        # twoThirdMap(mailbox(i))
            m = _mmor(list(mailbox.values()))
            if data1[i] != m:
                return f"p{i}: data1 {data1[i]} != mmor {m}"
            a = [j for j in mailbox if mailbox[j] == m]     # valueIs(mmor(i))
            want = True if len(a) > two_third else decided[i]
            if decided1[i] != want:
                return f"p{i}: decided1 {decided1[i]} != {want}"
        else:
            if decided1[i] != decided[i] or data1[i] != data[i]:
                return f"p{i}: frame violated"
    return None


# (n, drop_log2, good-round probability, self delivery); pure HO (no self bit) makes
# the seeded good rounds literal magic rounds (with self delivery only s = all is one)
CASES = [(4, 2, 0.3, True), (4, 1, 0.2, False), (7, 2, 0.25, True), (16, 3, 0.25, False), (16, 1, 0.1, True),
         (64, 3, 0.25, True), (64, 2, 0.4, False)]


@pytest.mark.parametrize("n,drop,good,self_bit", CASES, ids=[f"n{c[0]}-d{c[1]}-g{c[2]}-s{int(c[3])}" for c in CASES])
def test_oracle_rounds_satisfy_reference_tr(n, drop, good, self_bit, oracle_mod):
    R = 10
    count = 300 if n <= 16 else 60
    alg = psync.OTR(afterDecision=R + 2)  # no exit within R rounds: the model has none
    cfg = psync.make_config(alg, n, R, seed=31 + n, value_range=3,
                            schedule=psync.HOSchedule(drop_log2=drop, good_round=good, self_bit=self_bit))
    tr = np.frombuffer(oracle_mod.trace(cfg, 0, count, threads=8), dtype=np.int32).reshape(count, R + 1, NF, n)
    ho, _ = oracle_mod.materialize_schedule(cfg, 0, count)
    rounds_checked = magic = 0
    for i in range(count):
        for k in range(R):
            sets = [{q for q in range(n) if (int(ho[i, k, p, q >> 6]) >> (q & 63)) & 1} for p in range(n)]
            pre, post = tr[i, k], tr[i, k + 1]
            err = _tr(n, list(pre[X]), [bool(v) for v in pre[DECIDED]], sets, list(post[X]),
                      [bool(v) for v in post[DECIDED]])
            assert err is None, f"instance {i} round {k}: {err}"
            rounds_checked += 1
            # magicRound (OtrExample.scala:98-101) => one common data value afterwards
            if all(s == sets[0] for s in sets) and len(sets[0]) > (2 * n) // 3:
                magic += 1
                assert len(set(post[X])) == 1, f"instance {i} round {k}: magic round left {set(post[X])}"
    assert rounds_checked == count * R
    assert magic > 0 or self_bit
