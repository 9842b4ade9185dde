#!/usr/bin/env python3
"""Adversary-search throughput: explicit schedules evaluated
per second by round_amd.adversary on one MI355X, host generation included, and
the time to the first counterexample for mutated algorithms.

Rows (one JSON line each, then a JSON list in --out):
  * reference OTR n=64 R=20, safety search, 2^15 schedules per generation: no
    counterexample expected; reports schedules/s and the GPU share of the time;
  * mutants (OTR, LastVoting, FloodMin, BenOr): generations / seconds / schedules
    to the first counterexample and the shrunk counterexample's size.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from round_amd import adversary as A, psync  # noqa: E402


def row(name, alg, n, R, targets=None, population=4096, generations=10, want=1, stop=True, values=3):
    t0 = time.perf_counter()
    with A.Adversary(alg, n, R, targets=targets, population=population, values=values, seed=7) as adv:
        res = adv.search(generations=generations, want=want if stop else 10 ** 9, shrink=stop)
    out = {"row": name, "class": alg.class_name, "variant": alg.variant, "n": n, "rounds": R,
           "population": population, "generations": res.generations,
           "schedules": res.schedules_evaluated, "seconds": round(res.seconds, 3),
           "schedules_per_s": round(res.schedules_per_second, 1),
           "checked_process_rounds_per_s": round(res.schedules_per_second * n * R, 1),
           "gpu_seconds": round(res.gpu_seconds, 3), "found": len(res.counterexamples),
           "wall_s": round(time.perf_counter() - t0, 3)}
    if res.counterexamples:
        c = res.counterexamples[0]
        out.update(violated=c.violated, check_point=c.check_point, omitted_links=int(c.omitted_links))
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--population", type=int, default=32768)
    ap.add_argument("--generations", type=int, default=8)
    a = ap.parse_args()
    rows = [row("ref_otr_n64", psync.OTR(), 64, 20, population=a.population, generations=a.generations,
                stop=False, values=3)]
    rows.append(row("mut_otr_n64_safety", psync.OTR(variant=1), 64, 8, ["Safety"], population=4096, generations=60))
    rows.append(row("mut_otr_n16_agreement", psync.OTR(variant=1), 16, 8, ["Agreement"], population=4096,
                    generations=60, values=2))
    rows.append(row("mut_lv_n8_agreement", psync.LastVoting(variant=1), 8, 12, ["Agreement"], population=4096,
                    generations=60))
    rows.append(row("mut_floodmin_n8", psync.FloodMin(2, variant=1), 8, 4, population=4096, generations=60))
    rows.append(row("mut_benor_n8", psync.BenOr(variant=1), 8, 12, population=4096, generations=60, values=2))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
