"""Probe: headline OTR kernel time vs R (rounds after every process halted are
check-only rounds: the state is frozen, the Spec is still evaluated), to price
a check-only round against an executed round. Usage: python scripts/probe_rounds.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from round_amd import psync  # noqa: E402

I = 10_000_000
out = {}
for R in (5, 10, 20, 40, 80):
    with psync.GpuRound(psync.OTR(), 64, R, seed=2, value_range=64, batch_capacity=I) as g:
        g.load_inputs(0, I)
        g.run(0, I)
        ks = [g.run(0, I).summary.kernel_ns / 1e6 for _ in range(3)]
        h = g.run(0, I).summary.term_hist
    out[R] = min(ks)
    print(f"R={R}: kernel {min(ks):.2f} ms; terminated by check point 4: {sum(h[:5]) / I:.4f}", flush=True)
print(json.dumps(out))
