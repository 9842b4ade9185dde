"""A/B probe of the headline launch (OTR n=64, 1e7 instances, R=20, V=64 and V=2; arg lv: C3 LastVoting;
kset: the C4 KSet rows at f = 0, 1, 8, 16, 64; fm, kses, benor, slv, eps: the C4 / C5 / W2 rows):
min kernel ms over 5 launches for the library PSG_LIB points at (default: in-tree). A second
argument keeps only the row whose label ends with it (e.g. `kset f=64`, for a profile)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from round_amd import lib, psync  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "otr"
if which == "otr":
    runs = [(psync.OTR(), 10_000_000, dict(value_range=V), f"V={V}") for V in (64, 2)]
elif which == "kset":  # C4 KSet rows (bench_configs.py): n=256, k=2, 2e5 instances, R=16, crash-stop f
    runs = [(psync.KSetAgreement(2), 200_000, dict(schedule=psync.HOSchedule(drop_log2=0, good_round=0.0,
                                                                              crash_fmax=f)), f"KSet f={f}")
            for f in (0, 1, 8, 16, 64)]
elif which == "fm":  # C4 FloodMin rows (bench_configs.py): n=256, 1e6 instances, default schedule, R = f + 2
    runs = [(psync.FloodMin(f), 1_000_000, {}, f"FloodMin f={f}") for f in (0, 8, 64)]
elif which == "kses":  # W2 KSetEarlyStopping: n=256, t=64, k=2, 1e6 instances, default rounds / schedule
    runs = [(psync.KSetEarlyStopping(64, 2), 1_000_000, {}, "KSetES W2")]
elif which == "benor":  # C5: BenOr n=128, 1e6 instances, R=64
    runs = [(psync.BenOr(), 1_000_000, {}, "BenOr C5")]
elif which == "slv":  # W2 ShortLastVoting: n=64, 1.25e7 instances, default rounds / schedule
    runs = [(psync.ShortLastVoting(), 12_500_000, {}, "SLV W2")]
elif which == "eps":  # W2 EpsilonConsensus: n=64, f=5, 1e6 instances, default rounds / schedule
    runs = [(psync.EpsilonConsensus(5, 1e-6), 1_000_000, {}, "Epsilon W2")]
else:  # BASELINE C3 shard: LastVoting n=64, 1.25e7 instances, crash-stop
    runs = [(psync.LastVoting(), 12_500_000, {}, "LV C3")]
only = sys.argv[2] if len(sys.argv) > 2 else None  # optional: run only the row whose label ends with this
for alg, I, kw, label in runs:
    if only and not label.endswith(only):
        continue
    n, R = {"kset": (256, 16), "fm": (256, None), "kses": (256, None), "benor": (128, 64), "slv": (64, None), "eps": (64, None)}.get(
        which, (64, 20))  # None: the algorithm's default rounds
    with psync.GpuRound(alg, n, R, seed=2, batch_capacity=I, **kw) as g:
        g.load_inputs(0, I)
        g.run(0, I)
        ks = [g.run(0, I).summary.kernel_ns / 1e6 for _ in range(5)]
        d = g.run(0, I).summary.digest
    print(f"{os.path.basename(os.path.dirname(os.path.dirname(lib.LIB_PATH)))} {label}: {min(ks):.2f} ms digest {d}",
          flush=True)
