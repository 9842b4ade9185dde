"""Fused-module A/B (probe): the G1 fused row's workload (OTR n=64 V=64, or LastVoting n=64) at
PSG_PROBE_I instances with the library-compiled module and with code objects given on the
command line. python3 scripts/probe_fused.py otr|lv a.co b.co ..."""
import os
import sys

sys.path.insert(0, os.getcwd())
from round_amd import abi, formula as F, lib, psync  # noqa: E402

which = sys.argv[1]
I = int(os.environ.get("PSG_PROBE_I", "2500000"))
if which == "otr":
    alg, spec, kw = psync.OTR(), F.otr_spec(), dict(value_range=64)
else:
    alg, spec, kw = psync.LastVoting(), F.lv_spec(), {}
prog = lib.spec_compile_native(F.to_text(spec), alg.alg_id, True, 64)
paths = [("hiprtc", prog.module_path)] + [(os.path.basename(p), p) for p in sys.argv[2:]]
with psync.GpuRound(alg, 64, seed=7, batch_capacity=I, **kw) as g:
    g.load_inputs(0, I)
    g.run(0, I)
    print(f"built-in: {min(g.run(0, I).summary.kernel_ns for _ in range(3)) / 1e6:.2f} ms", flush=True)
    for rep in range(2):
        for name, p in paths:
            prog.module_path = p
            g.run_spec(0, I, prog)
            ks = [g.run_spec(0, I, prog).summary.kernel_ns / 1e6 for _ in range(3)]
            print(f"{name}: {min(ks):.2f} ms", flush=True)
