#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the CPU oracle.

The reference (Scala) cannot run here and ships no vectors for this path, so
these fixtures are oracle outputs (the oracle itself is pinned by
tests/test_oracle_kat.py). They freeze the semantics: tests/test_golden.py
re-checks the oracle against them on CPU and the HIP path on the GPU.

Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from round_amd import abi, psync  # noqa: E402

H = psync.HOSchedule

# name -> (algorithm, n, instances, make_config kwargs); rows of BASELINE.json configs at reduced I
FIXTURES = {
    "c1_otr_n4": (psync.OTR(), 4, 1000, dict(rounds=10, value_range=4, seed=1)),
    "c2_otr_n64_V2": (psync.OTR(), 64, 200, dict(value_range=2, seed=2)),
    "c2_otr_n64_V4": (psync.OTR(), 64, 200, dict(value_range=4, seed=2)),
    "c2_otr_n64_V64": (psync.OTR(), 64, 200, dict(value_range=64, seed=2)),
    "c3_lv_n64_crash": (psync.LastVoting(), 64, 200, dict(seed=3)),
    "c4_floodmin_n256_f0": (psync.FloodMin(0), 256, 24, dict(seed=4)),
    "c4_floodmin_n256_f2": (psync.FloodMin(2), 256, 24, dict(seed=4)),
    "c4_floodmin_n256_f8": (psync.FloodMin(8), 256, 24, dict(seed=4)),
    "c4_floodmin_n256_f64": (psync.FloodMin(64), 256, 12, dict(seed=4)),
    "c4_kset_n256_k2": (psync.KSetAgreement(2), 256, 12, dict(seed=4)),
    "c4_kset_n256_k2_f4": (psync.KSetAgreement(2), 256, 8, dict(seed=4, schedule=H(drop_log2=0, good_round=0.0,
                                                                                      crash_fmax=4))),
    "c5_benor_n128": (psync.BenOr(), 128, 100, dict(seed=5)),
    # second-wave algorithms
    "w2_otr2_n64_V4": (psync.OTR2(), 64, 200, dict(value_range=4, seed=6)),
    "w2_slv_n64": (psync.ShortLastVoting(), 64, 200, dict(seed=7)),
    "w2_slv_n16_loss": (psync.ShortLastVoting(), 16, 400, dict(value_range=5, seed=7, schedule=H(
        drop_log2=1, good_round=0.0, crash_fmax=7))),
    "w2_kset_es_n64_t8_k2": (psync.KSetEarlyStopping(8, 2), 64, 200, dict(seed=8)),
    "w2_epsilon_n7_f1": (psync.EpsilonConsensus(1, 0.1), 7, 300, dict(seed=9)),
    "w2_epsilon_n64_f5": (psync.EpsilonConsensus(5, 1e-6), 64, 100, dict(seed=9)),
}

BEGIN = 12345
N_RECORDS = 3


def config_dict(cfg):
    # the device list (n_devices / devices) is run plumbing, not part of a fixture
    d = {f: getattr(cfg, f) for f, _ in abi.Config._fields_ if f not in ("sched", "n_devices", "devices")}
    d["sched"] = {f: getattr(cfg.sched, f) for f, _ in abi.Schedule._fields_}
    return d


def config_from_dict(d):
    c = abi.Config()
    for k, v in d.items():
        if k != "sched":
            setattr(c, k, v)
    for k, v in d["sched"].items():
        setattr(c.sched, k, v)
    return c


def inst_row(s):
    return ["%016x" % s.digest, list(s.first_fail)[: s.n_checks], s.term_round, s.n_decided]


def make(name):
    alg, n, count, kw = FIXTURES[name]
    cfg = psync.make_config(alg, n, batch_capacity=count, **kw)
    extra = {}
    if alg.real:
        s, pi, rec, dec, fx = oracle.run_real(cfg, BEGIN, count, per_instance=True, records=True, threads=8)
        # Double decision / final x (JSON floats round-trip exactly)
        extra["records_f64"] = {str(BEGIN + i): [[dec[i * n + p], fx[i * n + p]] for p in range(n)]
                                for i in range(N_RECORDS)}
    else:
        s, pi, rec = oracle.run(cfg, BEGIN, count, per_instance=True, records=True, threads=8)
    return dict(extra, **{
        "name": name,
        "class": alg.class_name,
        "config": config_dict(cfg),
        "inst_begin": BEGIN,
        "count": count,
        "summary": {
            "process_rounds": s.process_rounds,
            "fail_count": list(s.fail_count)[: len(abi.CHECK_NAMES[alg.alg_id])],
            "decided_processes": s.decided_processes,
            "digest": "%016x" % (s.digest & ((1 << 64) - 1)),
            "term_hist": list(s.term_hist)[: cfg.rounds + 2],
        },
        "instances": [inst_row(x) for x in pi],
        "records": {str(BEGIN + i): [[r.decision, r.decision_round, r.halt_round, r.final_x]
                                     for r in rec[i * n:(i + 1) * n]] for i in range(N_RECORDS)},
    })


def main(names=None):
    oracle.build()
    for name in names or FIXTURES:
        fx = make(name)
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(fx, f, separators=(",", ":"))
        print(name, fx["summary"]["fail_count"])


if __name__ == "__main__":
    main(sys.argv[1:])
