#!/usr/bin/env python3
"""Run otr_kernel<1> at several round counts (same instances) for a PMC split of
per-round costs: instances halt by round ~3, so R=40 vs R=20 isolates the cost
of a check point on a frozen state, R=4 vs R=2 the cost of a live round."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa
from round_amd import psync
I = int(os.environ.get("PROBE_I", "2000000"))
res = []
for V in (64, 2):
    for R in (1, 2, 4, 20, 40):
        with psync.GpuRound(psync.OTR(), 64, rounds=R, value_range=V, seed=2, batch_capacity=I) as g:
            g.load_inputs(0, I)
            s = g.run(0, I).summary
            res.append({"V": V, "R": R, "kernel_ms": s.kernel_ns / 1e6})
print(json.dumps(res))
