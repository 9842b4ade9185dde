"""Phase-timer probe (profiling build: PSG_LIB=round_amd/libpsg_timers.so PSG_PHASE_TIMERS=1).

  python3 scripts/probe_phases.py [otr|lv|fm|kset|benor]   # otr: headline launch at V=64 and V=2;
                                                    # lv: BASELINE C3 shard; fm / kset: C4 rows
"""
import os
import sys

sys.path.insert(0, os.getcwd())
from round_amd import psync  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "otr"
if which == "otr":
    runs = [(psync.OTR(), 64, 20, 10_000_000, dict(value_range=V), f"V {V}") for V in (64, 2)]
elif which == "lv":
    runs = [(psync.LastVoting(), 64, 20, 12_500_000, {}, "C3")]
elif which == "benor":
    runs = [(psync.BenOr(), 128, 64, 1_000_000, {}, "C5 BenOr")]
elif which == "fm":
    runs = [(psync.FloodMin(f), 256, f + 2, 1_000_000, {}, f"FloodMin f={f}") for f in (0, 8)]
elif which == "kset4":  # the C4 KSet rows' schedule (bench_configs.py)
    runs = [(psync.KSetAgreement(2), 256, 16, 200_000,
             dict(schedule=psync.HOSchedule(drop_log2=0, good_round=0.0, crash_fmax=f)), f"KSet C4 f={f}")
            for f in (0, 1, 32, 64)]
else:
    runs = [(psync.KSetAgreement(2), 256, 16, 200_000, {}, "KSet k=2")]
for alg, n, R, I, kw, label in runs:
    with psync.GpuRound(alg, n, R, seed=2, batch_capacity=I, **kw) as g:
        g.load_inputs(0, I)
        g.run(0, I)
        r = g.run(0, I)
        print(label, "kernel ms", r.summary.kernel_ns / 1e6, flush=True)
