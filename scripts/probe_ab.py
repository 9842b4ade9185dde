"""A/B probe of the headline launch (OTR n=64, 1e7 instances, R=20, V=64 and V=2):
min kernel ms over 5 launches for the library PSG_LIB points at (default: in-tree)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from round_amd import lib, psync  # noqa: E402

I = 10_000_000
for V in (64, 2):
    with psync.GpuRound(psync.OTR(), 64, 20, seed=2, value_range=V, batch_capacity=I) as g:
        g.load_inputs(0, I)
        g.run(0, I)
        ks = [g.run(0, I).summary.kernel_ns / 1e6 for _ in range(5)]
        d = g.run(0, I).summary.digest
    print(f"{os.path.basename(os.path.dirname(os.path.dirname(lib.LIB_PATH)))} V={V}: {min(ks):.2f} ms digest {d}",
          flush=True)
