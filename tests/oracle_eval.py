"""CPU evaluator for round_amd.adversary (TEST INFRASTRUCTURE ONLY): runs explicit
schedules on the oracle so the search / shrink logic is testable without a GPU.
The product search uses GpuEvaluator (the HIP library); this is the checker."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import oracle as oracle_mod  # noqa: E402

from round_amd import psync, records  # noqa: E402
from round_amd.adversary import Eval  # noqa: E402


def summaries_np(pi):
    out = np.zeros(len(pi), records.SUMMARY_DTYPE)
    for i, s in enumerate(pi):
        out[i]["digest"] = s.digest
        out[i]["first_fail"] = list(s.first_fail)
        out[i]["term_round"] = s.term_round
        out[i]["n_checks"] = s.n_checks
        out[i]["n_decided"] = s.n_decided
    return out


class OracleEvaluator:
    def __init__(self, alg, n, rounds, value_range=3, seed=1, threads=8):
        self.cfg = psync.make_config(alg, n, rounds, seed=seed, value_range=value_range)
        self.real = alg.real
        self.threads = threads

    def __call__(self, inst_begin, ho, crash, init):
        I, n = ho.shape[0], self.cfg.n
        summ, pi, recs, dec, fx = oracle_mod.run_schedule(self.cfg, inst_begin, I, ho, crash, init,
                                                          per_instance=True, records=True, threads=self.threads)
        r = np.array([(x.decision, x.decision_round) for x in recs], np.int64).reshape(I, n, 2)
        decision = dec.reshape(I, n) if self.real else r[:, :, 0].astype(np.int32)
        return Eval(summaries_np(pi), decision, r[:, :, 1].astype(np.int32))
