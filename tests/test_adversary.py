"""CPU tests of explicit schedules, the adversary search and record files
(SURVEY §8f rank 4): schedule predicates against brute force, the oracle's
explicit-schedule path against its seeded path, the search / shrink logic with
the oracle as evaluator, and the .psgr format (Python writer, C reader)."""
import os
import subprocess

import numpy as np
import pytest

from round_amd import abi, adversary as A, psync, records, schedules as S

from oracle_eval import OracleEvaluator

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sets(ho, n):
    I, R = ho.shape[:2]
    return [[[frozenset(q for q in range(n) if (int(ho[i, k, p, q >> 6]) >> (q & 63)) & 1) for p in range(n)]
             for k in range(R)] for i in range(I)]


@pytest.mark.parametrize("n", [5, 64, 70])
def test_predicates_match_brute_force(n):
    rng = np.random.default_rng(n)
    I, R = 6, 5
    ho = S.random_omission(rng, I, R, n, 0.8)
    sets = _sets(ho, n)
    assert all(p in sets[i][k][p] for i in range(I) for k in range(R) for p in range(n))  # self bit
    S.force_good_round(ho, rng, n, np.array([0, 1, 1]), np.array([2, 0, 3]))
    S.force_good_round(ho, rng, n, np.array([2]), np.array([1]), self_bit=True)
    S.force_coord_hears_all(ho[3:5], n, [0, 1, 4])
    sets = _sets(ho, n)
    gm = S.good_round(ho, n)
    mj = S.ho_majority(ho, n)
    ch = S.coord_hears_all(ho, n)
    for i in range(I):
        for k in range(R):
            ss = sets[i][k]
            assert gm[i, k] == (all(s == ss[0] for s in ss) and len(ss[0]) > 2 * n // 3)
            assert mj[i, k] == all(len(s) > n // 2 for s in ss)
            c = (k // 4) % n
            assert ch[i, k] == (len(ss[c]) == n)
            assert all(q < n for s in ss for q in s)
    assert gm[0, 2] and gm[1, 0] and gm[1, 3] and gm[2, 1] and ch[3:5, [0, 1]].all()
    assert all(len(s) == n for s in sets[2][1])  # self_bit: the common set is everyone


def test_crash_genome_is_crash_stop():
    rng = np.random.default_rng(1)
    n, R, I = 70, 6, 50
    crash, partial = S.random_crash(rng, I, R, n, 4, p_partial=(0.1, 0.9))
    ho = S.crash_to_ho(crash, partial, R, n)
    assert S.crash_consistent(ho, crash, n, 4).all()
    assert ((crash >= 0).sum(1) <= 4).all()
    ho[0, 0, 0, 0] ^= np.uint64(2) if crash[0, 1] < 0 else np.uint64(0)
    if crash[0, 1] < 0:
        assert not S.crash_consistent(ho, crash, n, 4)[0]


def test_repair_and_random_bits():
    rng = np.random.default_rng(2)
    x = S.random_bits(rng, (4000,), 0.3)
    assert abs(np.bitwise_count(x).sum() / (4000 * 64) - 0.3) < 0.01
    ho = S.random_omission(rng, 10, 4, 100, 0.2)
    S.repair_min_size(ho, rng, 100, 51)
    assert S.ho_majority(ho, 100).all()


ALGS = [(psync.OTR(), 64), (psync.LastVoting(), 64), (psync.FloodMin(f=3), 130), (psync.KSetAgreement(k=2), 100),
        (psync.BenOr(), 128), (psync.OTR2(), 17), (psync.ShortLastVoting(), 64),
        (psync.KSetEarlyStopping(t=3, k=2), 70), (psync.EpsilonConsensus(f=2, epsilon=1e-3), 40)]


@pytest.mark.parametrize("alg,n", ALGS, ids=[type(a).__name__ for a, _ in ALGS])
def test_oracle_explicit_replay_equals_seeded(alg, n, oracle_mod):
    cfg = psync.make_config(alg, n, seed=7)
    cnt = 30
    ho, cr = oracle_mod.materialize_schedule(cfg, 100, cnt)
    a = (oracle_mod.run_real if alg.real else oracle_mod.run)(cfg, 100, cnt, per_instance=True)
    b = oracle_mod.run_schedule(cfg, 100, cnt, ho, cr, per_instance=True)
    assert a[0].digest == b[0].digest
    for x, y in zip(a[1], b[1]):
        assert x.digest == y.digest and bytes(x.first_fail) == bytes(y.first_fail) and x.term_round == y.term_round
    # the materialized sets are the oracle's per-(instance, round, process) HO masks
    if n <= 64:
        for k in (0, cfg.rounds - 1):
            assert int(ho[3, k, 5, 0]) == oracle_mod.ho_mask(cfg, 103, k, 5)


SEARCH = [
    (psync.OTR(variant=1), 8, 6, ["Agreement"]),
    (psync.LastVoting(variant=1), 6, 12, ["Agreement"]),
    (psync.FloodMin(f=2, variant=1), 8, 4, None),
    (psync.EpsilonConsensus(f=1, epsilon=1e-3, variant=1), 8, 6, None),
]


@pytest.mark.parametrize("alg,n,R,targets", SEARCH, ids=[type(a).__name__ for a, *_ in SEARCH])
def test_search_finds_mutant_violation_and_shrinks(alg, n, R, targets, oracle_mod):
    ev = OracleEvaluator(alg, n, R)
    adv = A.Adversary(alg, n, R, targets=targets, population=1024, evaluator=ev, seed=5)
    res = adv.search(generations=60, want=1)
    assert res.counterexamples
    c = res.counterexamples[0]
    # the shrunk schedule still violates (re-run on the oracle) ...
    e = ev(c.inst_id, c.ho[None], None if c.crash is None else c.crash[None], c.init[None])
    bad, first = adv._violations(e)
    assert bad[0] and first[0] == c.check_point
    # ... and no single omitted link of the omission family can be restored
    if adv.model.family == "omission":
        cands = []
        for k in range(R):
            for p in range(n):
                for q in range(n):
                    if not (int(c.ho[k, p, q >> 6]) >> (q & 63)) & 1:
                        h = c.ho.copy()
                        h[k, p, q >> 6] |= np.uint64(1 << (q & 63))
                        cands.append(h)
        if cands:
            hh = np.stack(cands)
            e = ev(c.inst_id, hh, None, np.repeat(c.init[None], len(cands), 0))
            assert not adv._violations(e)[0].any()
    assert "violated" in A.describe(c, n)


@pytest.mark.parametrize("alg,n,R", [(psync.OTR(), 8, 6), (psync.LastVoting(), 6, 12), (psync.FloodMin(f=2), 8, 4),
                                     (psync.BenOr(), 8, 12)], ids=["otr", "lv", "floodmin", "benor"])
def test_search_reference_algorithms_hold(alg, n, R):
    adv = A.Adversary(alg, n, R, population=512, evaluator=OracleEvaluator(alg, n, R), seed=6)
    res = adv.search(generations=20, want=1, shrink=False)
    assert not res.counterexamples
    assert res.schedules_evaluated == 20 * 512


def test_liveness_two_good_rounds_terminate():
    alg, n, R = psync.OTR(), 8, 6
    adv = A.Adversary(alg, n, R, mode="liveness", live_at=[0, 1], population=512,
                      evaluator=OracleEvaluator(alg, n, R), seed=7)
    res = adv.search(generations=5, want=1, shrink=False)
    assert not res.counterexamples


def test_adversary_argument_errors():
    ev = OracleEvaluator(psync.OTR(), 4, 3)
    with pytest.raises(ValueError):
        A.Adversary(psync.OTR(), 4, 3, targets=["Nope"], evaluator=ev)
    with pytest.raises(ValueError):
        A.Adversary(psync.FloodMin(2), 4, 3, mode="liveness", evaluator=ev)
    with pytest.raises(ValueError):
        A.Adversary(psync.OTR(), 4, 3, mode="bogus", evaluator=ev)


def _sample_records(real=False):
    rng = np.random.default_rng(4)
    alg = psync.EpsilonConsensus(f=1) if real else psync.LastVoting()
    n, R, k = 70, 5, 3
    cfg = psync.make_config(alg, n, R, seed=3)
    summ = np.zeros(k, records.SUMMARY_DTYPE)
    summ["digest"] = [1, 2 ** 63 + 5, 7]
    summ["first_fail"][:, :] = 255
    summ["first_fail"][1, 3] = 4
    summ["term_round"] = [2, 255, 5]
    proc = np.zeros((k, n), records.PROCESS_DTYPE)
    proc["decision"] = rng.integers(0, 100, (k, n))
    init = rng.random((k, n)) if real else rng.integers(1, 9, (k, n), dtype=np.int32)
    return records.Records(cfg=cfg, slot_names=alg.check_names, ids=np.array([5, 6, 90], np.uint64), summary=summ,
                           init=init, ho=S.random_omission(rng, k, R, n, 0.5), crash=np.full((k, n), -1, np.int32),
                           process=proc, meta={"why": "test", "list": [1, 2]}, class_name=alg.class_name)


@pytest.mark.parametrize("real", [False, True])
def test_records_round_trip(tmp_path, real):
    rec = _sample_records(real)
    path = str(tmp_path / "r.psgr")
    records.write(path, rec)
    for mm in (True, False):
        b = records.read(path, mmap=mm)
        assert b.count == 3 and b.n == 70 and b.rounds == 5 and b.class_name == rec.class_name
        assert b.slot_names == rec.slot_names and b.meta == rec.meta
        assert (b.ids == rec.ids).all() and (b.summary == rec.summary).all() and (b.ho == rec.ho).all()
        assert (b.init == rec.init).all() and b.init.dtype == (np.float64 if real else np.int32)
        assert (b.process == rec.process).all() and (b.crash == rec.crash).all()
        assert bytes(b.cfg) == bytes(rec.cfg)
    assert os.path.getsize(path) % records.ALIGN == 0


def test_records_rejects_garbage(tmp_path):
    p = tmp_path / "bad.psgr"
    p.write_bytes(b"NOTAREC!" + bytes(4000))
    with pytest.raises(ValueError):
        records.read(str(p))
    p.write_bytes(b"PSGREC")
    with pytest.raises(ValueError):
        records.read(str(p))


C_READER = r"""
#include <stdio.h>
#include <stdlib.h>
#include "psg_records.h"
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  psg_rec_header h;
  if (fread(&h, sizeof h, 1, f) != 1) return 3;
  if (psg_rec_check_header(&h)) return 4;
  const psg_rec_section* s = psg_rec_find(&h, PSG_REC_SUMMARY);
  const psg_rec_section* ho = psg_rec_find(&h, PSG_REC_HO);
  const psg_rec_section* ids = psg_rec_find(&h, PSG_REC_IDS);
  if (!s || !ho || !ids) return 5;
  psg_instance_summary* sum = malloc(s->nbytes);
  uint64_t* id = malloc(ids->nbytes);
  fseek(f, (long)s->offset, SEEK_SET);
  if (fread(sum, 1, s->nbytes, f) != s->nbytes) return 6;
  fseek(f, (long)ids->offset, SEEK_SET);
  if (fread(id, 1, ids->nbytes, f) != ids->nbytes) return 7;
  printf("%s n=%d R=%d count=%llu slots=%u first=%s hdr=%u\n", h.class_name, h.cfg.n, h.cfg.rounds,
         (unsigned long long)h.count, h.n_slots, h.slot_names[0], h.header_bytes);
  for (uint64_t i = 0; i < h.count; ++i)
    printf("%llu %llu %u %u\n", (unsigned long long)id[i], (unsigned long long)sum[i].digest,
           sum[i].first_fail[3], sum[i].term_round);
  printf("ho %llu\n", (unsigned long long)ho->nbytes);
  return 0;
}
"""


def test_records_readable_from_c(tmp_path):
    """include/psg_records.h is all a C (or JNI) reader needs."""
    rec = _sample_records()
    path = str(tmp_path / "r.psgr")
    records.write(path, rec)
    src = tmp_path / "reader.c"
    src.write_text(C_READER)
    exe = str(tmp_path / "reader")
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                           "-o", exe])
    out = subprocess.check_output([exe, path]).decode().split("\n")
    assert out[0] == f"example.LastVoting n=70 R=5 count=3 slots=7 first=Safety hdr={records.C.sizeof(records.Header)}"
    assert out[1:4] == ["5 1 255 2", f"6 {2 ** 63 + 5} 4 255", "90 7 255 5"]
    assert out[4] == f"ho {3 * 5 * 70 * 2 * 8}"
