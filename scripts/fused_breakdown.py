#!/usr/bin/env python3
"""Cost of each part of a fused Spec: the OTR headline workload (n=64, V=64, R=20) run with
fused modules that evaluate one formula of OTR.spec at a time (plus an empty Spec: the
round kernel alone), kernel time per launch. Compile here (native modules are cached under
build/spec and travel with the tree), run on the GPU box.

usage: fused_breakdown.py [--compile-only] [--instances N] [--alg otr|lv] [--nosym] [--nosplit]
(--nosym: modules without the symmetric-check-point lowering, formula.SYMMETRIC_LOWERING)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from round_amd import abi, formula, psync  # noqa: E402
from round_amd import formula as F  # noqa: E402
from round_amd.formula import P, Spec, init, old, true  # noqa: E402


def otr_variants():
    full = formula.otr_spec()
    props = dict(full.properties)
    v = {"rounds_only": Spec(properties=[("T", true)]), "full": full}
    for i, f in enumerate(full.invariants):
        v[f"inv{i}"] = Spec([f])
    for name, f in full.properties:
        v[name] = Spec([true] if name == "Termination" else [], properties=[(name, f)])
    v["keep_init"] = Spec([P.forall(lambda i: P.exists(lambda j1: i.x == init(j1.x)))])
    del props
    return v


def lv_variants():
    full = formula.lv_spec()
    v = {"rounds_only": Spec(properties=[("T", true)], phase_length=4), "full": full}
    for i, f in enumerate(full.invariants):
        v[f"inv{i}"] = Spec([f], phase_length=4)
    v["rinv_only"] = Spec([true], full.round_invariants, phase_length=4)
    for name, f in full.properties:
        v[name] = Spec([true] if name == "Termination" else [], properties=[(name, f)], phase_length=4)
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compile-only", action="store_true")
    ap.add_argument("--instances", type=int, default=2_500_000)
    ap.add_argument("--alg", default="otr")
    ap.add_argument("--nosym", action="store_true")
    ap.add_argument("--nosplit", action="store_true", help="modules without formula.SPLIT_FORALL")
    ap.add_argument("--timers", action="store_true",
                    help="profiling modules (-DPSG_PHASE_TIMERS=1) of the full Spec and the round kernel alone; "
                         "run with PSG_LIB=round_amd/libpsg_timers.so PSG_PHASE_TIMERS=1")
    args = ap.parse_args()
    F.SYMMETRIC_LOWERING = not args.nosym
    F.SPLIT_FORALL = not args.nosplit
    if args.alg == "otr":
        alg, aid, kw, variants = psync.OTR(), abi.PSG_ALG_OTR, dict(value_range=64), otr_variants()
    else:
        alg, aid, kw, variants = psync.LastVoting(), abi.PSG_ALG_LAST_VOTING, {}, lv_variants()
    if args.timers:
        variants = {k: v for k, v in variants.items() if k in ("full", "rounds_only")}
    defs = ("PSG_PHASE_TIMERS=1",) if args.timers else ()
    progs = {k: formula.compile_native(s, aid, fused=True, n=64, defines=defs) for k, s in variants.items()}
    if args.compile_only:
        print("compiled", len(progs))
        return
    I = args.instances
    with psync.GpuRound(alg, 64, seed=7, batch_capacity=I, **kw) as g:
        g.load_inputs(0, I)
        g.run(0, I)  # warm up the built-in kernel
        base = [g.run(0, I).summary.kernel_ns for _ in range(2)]
        print(json.dumps({"variant": "built-in", "kernel_ms": min(base) / 1e6}), flush=True)
        for k, p in progs.items():
            g.run_spec(0, I, p)
            t = [g.run_spec(0, I, p).summary.kernel_ns for _ in range(2)]
            print(json.dumps({"variant": k, "symmetric": not args.nosym, "split": not args.nosplit, "kernel_ms": min(t) / 1e6}), flush=True)


if __name__ == "__main__":
    main()
