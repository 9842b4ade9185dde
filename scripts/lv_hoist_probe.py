#!/usr/bin/env python3
"""Experiment: LastVoting's majority clause with its own-lane pin conjuncts (decided ==>
decision == v, commit / ready ==> vote == v) computed once per value candidate, per lane,
before the walk over the round candidates t (a hand edit of the generated source), against the
generator's output. Fused modules, 2.5e6 instances. usage: lv_hoist_probe.py [--compile-only]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from round_amd import abi, formula, psync  # noqa: E402

ATOMS = [f"(int32_t)(((x.own(0, {c})) == 0) | (((int32_t)((x.own(0, {t})) == (v4))) != 0))"
         for c, t in ((1, 2), (5, 6), (4, 6))]
HEAD = "[&](int32_t v4) -> int32_t { return ([&]() -> int32_t { "
B_DEF = "".join(f"const int32_t hB{k}_ = {a}; " for k, a in enumerate(ATOMS))


def patched():
    orig = formula.codegen_hip

    def gen(spec, alg=None):
        src, prog = orig(spec, alg)
        assert src.count(HEAD) == 2 and all(src.count(a) == 2 for a in ATOMS)
        for k, a in enumerate(ATOMS):
            src = src.replace(a, f"hB{k}_")
        src = src.replace(HEAD, HEAD + B_DEF)
        return src, prog
    return gen


def main():
    full = formula.lv_spec()
    mods = {"generated": formula.compile_native(full, abi.PSG_ALG_LAST_VOTING, fused=True, n=64)}
    formula.codegen_hip = patched()
    mods["hoisted_pins"] = formula.compile_native(full, abi.PSG_ALG_LAST_VOTING, fused=True, n=64)
    if "--compile-only" in sys.argv:
        print("compiled", len(mods))
        return
    I = 2_500_000
    with psync.GpuRound(psync.LastVoting(), 64, seed=7, batch_capacity=I) as g:
        g.load_inputs(0, I)
        base = g.run(0, I)
        want = base.summary
        for _ in range(2):
            for k, p in mods.items():
                r = g.run_spec(0, I, p)
                print(json.dumps({"variant": k, "kernel_ms": r.summary.kernel_ns / 1e6}), flush=True)


if __name__ == "__main__":
    main()
