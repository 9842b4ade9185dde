import os, sys
sys.path.insert(0, os.getcwd())
from round_amd import psync
I = 10_000_000
for V in (64, 2):
    with psync.GpuRound(psync.OTR(), 64, 20, seed=2, value_range=V, batch_capacity=I) as g:
        g.load_inputs(0, I)
        g.run(0, I)
        r = g.run(0, I)
        print("V", V, "kernel ms", r.summary.kernel_ns / 1e6, flush=True)
