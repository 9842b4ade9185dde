"""Phase timers of the fused OTR / LastVoting modules (profiling builds: PSG_LIB=round_amd/timers.so
PSG_PHASE_TIMERS=1; the module compiled with generator option DPSG_PHASE_TIMERS=1)."""
import os
import sys

sys.path.insert(0, os.getcwd())
from round_amd import abi, formula as F, lib, psync  # noqa: E402

I = int(os.environ.get("PSG_PROBE_I", "2500000"))
for which in sys.argv[1:] or ["otr", "lv"]:
    if which == "otr":
        alg, spec, kw = psync.OTR(), F.otr_spec(), dict(value_range=64)
    else:
        alg, spec, kw = psync.LastVoting(), F.lv_spec(), {}
    prog = lib.spec_compile_native(F.to_text(spec), alg.alg_id, True, 64, options=["DPSG_PHASE_TIMERS=1"])
    with psync.GpuRound(alg, 64, seed=7, batch_capacity=I, **kw) as g:
        g.load_inputs(0, I)
        print(which, "built-in", flush=True)
        g.run(0, I)
        print(which, "fused", flush=True)
        r = g.run_spec(0, I, prog)
        print(which, "fused kernel ms", r.summary.kernel_ns / 1e6, flush=True)
