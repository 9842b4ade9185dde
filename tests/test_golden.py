"""Golden fixtures (tests/golden/*.json, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every fixture bit for bit.
GPU: the HIP path reproduces every fixture bit for bit (through the C ABI).
"""
import glob
import json
import math
import os

import pytest

from round_amd import abi, psync

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(HERE, "*.json")))
NAMES = [os.path.basename(f)[:-5] for f in FILES]


def load(name):
    with open(os.path.join(HERE, name + ".json")) as f:
        return json.load(f)


def to_cfg(d):
    c = abi.Config()
    for k, v in d.items():
        if k != "sched":
            setattr(c, k, v)
    for k, v in d["sched"].items():
        setattr(c.sched, k, v)
    c.abi_version = abi.PSG_ABI_VERSION  # fields added by later ABI versions default to 0
    return c


def rows(per_inst):
    return [["%016x" % s.digest, list(s.first_fail)[: s.n_checks], s.term_round, s.n_decided] for s in per_inst]


def summary_view(s, nck, R):
    return {
        "process_rounds": s.process_rounds,
        "fail_count": list(s.fail_count)[:nck],
        "decided_processes": s.decided_processes,
        "digest": "%016x" % (s.digest & ((1 << 64) - 1)),
        "term_hist": list(s.term_hist)[: R + 2],
    }


# EpsilonConsensus Doubles: the GPU matches the oracle bit for bit except where
# libm log() differs by an ulp (SURVEY §8c "stated absolute tolerance")
F64_ABS_TOL = 1e-12


def _same_f64(got, want, tol=0.0):
    for g, w in zip(got, want):
        for a, b in zip(g, w):
            if math.isnan(a) and math.isnan(b):
                continue
            if not abs(a - b) <= tol:
                return False
    return len(got) == len(want)


def test_fixtures_exist():
    assert len(FILES) >= 10
    for f in FILES:
        assert os.path.getsize(f) < 200_000


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_fixture(name, oracle_mod):
    fx = load(name)
    cfg = to_cfg(fx["config"])
    if cfg.alg == abi.PSG_ALG_EPSILON:
        s, pi, rec, dec, fxv = oracle_mod.run_real(cfg, fx["inst_begin"], fx["count"], per_instance=True,
                                                   records=True, threads=8)
        n = cfg.n
        for inst, want in fx["records_f64"].items():
            i = int(inst) - fx["inst_begin"]
            got = [[dec[i * n + p], fxv[i * n + p]] for p in range(n)]
            assert _same_f64(got, want)
    else:
        s, pi, rec = oracle_mod.run(cfg, fx["inst_begin"], fx["count"], per_instance=True, records=True,
                                    threads=8)
    nck = len(fx["summary"]["fail_count"])
    assert summary_view(s, nck, cfg.rounds) == fx["summary"]
    assert rows(pi) == fx["instances"]
    n = cfg.n
    for inst, want in fx["records"].items():
        i = int(inst) - fx["inst_begin"]
        assert [[r.decision, r.decision_round, r.halt_round, r.final_x] for r in rec[i * n:(i + 1) * n]] == want


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_fixture(name):
    from round_amd import lib
    fx = load(name)
    cfg = to_cfg(fx["config"])
    cfg.batch_capacity = max(fx["count"], 16)
    ctx = lib.Context(cfg)
    try:
        s, pi = ctx.run_batch(fx["inst_begin"], fx["count"], per_instance=True)
        if cfg.alg == abi.PSG_ALG_EPSILON:
            sums, recs, dec, fxv = ctx.fetch_real([int(k) for k in fx["records"]])
            n = cfg.n
            for j, want in enumerate(fx["records_f64"].values()):
                got = [[dec[j * n + p], fxv[j * n + p]] for p in range(n)]
                assert _same_f64(got, want, F64_ABS_TOL)
        else:
            sums, recs = ctx.fetch([int(k) for k in fx["records"]])
    finally:
        ctx.close()
    nck = len(fx["summary"]["fail_count"])
    assert summary_view(s, nck, cfg.rounds) == fx["summary"]
    assert rows(pi) == fx["instances"]
    n = cfg.n
    for j, (inst, want) in enumerate(fx["records"].items()):
        assert [[r.decision, r.decision_round, r.halt_round, r.final_x] for r in recs[j * n:(j + 1) * n]] == want
