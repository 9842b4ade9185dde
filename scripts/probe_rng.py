"""Probe: kernel time of the headline OTR launch vs the number of Philox calls per
process-round (drop_log2 d needs W*d words = ceil(d/2) calls), to price the RNG.
Usage: python scripts/probe_rng.py [instances]   (PSG_LIB selects an A/B build)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from round_amd import lib, psync  # noqa: E402

I = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
out = {"lib": lib.LIB_PATH}
for d in (3, 0, 2, 4, 5, 6):
    with psync.GpuRound(psync.OTR(), 64, 20, seed=2, value_range=64, batch_capacity=I,
                        schedule=psync.HOSchedule(drop_log2=d, good_round=0.25)) as g:
        g.load_inputs(0, I)
        g.run(0, I)
        ks = []
        for _ in range(3):
            r = g.run(0, I)
            ks.append(r.summary.kernel_ns / 1e6)
    out[f"drop{d}"] = min(ks)
    print(f"drop_log2={d}: kernel {min(ks):.2f} ms", flush=True)
print(json.dumps(out))
