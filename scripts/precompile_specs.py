#!/usr/bin/env python3
"""Compile every native / fused Spec module the GPU tests, bench_configs.py and
scripts/fused_breakdown.py load (formula.compile_native, cached by source hash under
build/spec), in parallel, so GPU calls do not spend box time in hipcc.

usage: precompile_specs.py [-j JOBS]
"""
import argparse
import os
import sys
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def jobs():
    from round_amd import abi, formula as F
    import spec_cases
    import test_gpu_spec as T
    out = []
    for _, alg, n, _, _ in T.REF:
        out.append(("ref", alg.alg_id, False, None))
        out.append(("ref", alg.alg_id, True, n))
    for cid, alg, n, _, _ in spec_cases.CUSTOM:
        out.append((cid, alg.alg_id, False, None))
        out.append((cid, alg.alg_id, True, n))
    for alg in F.FUSED_KERNELS:
        out.append(("fusedbuild", alg, True, 64))
    for a in (abi.PSG_ALG_OTR, abi.PSG_ALG_OTR2, abi.PSG_ALG_LAST_VOTING, abi.PSG_ALG_BENOR):
        out.append(("ref", a, False, None))
    out.append(("lv_custom", abi.PSG_ALG_LAST_VOTING, False, None))
    out.append(("ref", abi.PSG_ALG_OTR, True, 64))
    out.append(("ref", abi.PSG_ALG_LAST_VOTING, True, 64))
    # the Formula-text route (psg_spec_compile_native: the library's own generator + hiprtc),
    # tests/test_spec_native_text.py, tests/test_jni_shim.py and the G1 *_text rows
    for a, n in ((abi.PSG_ALG_OTR, 64), (abi.PSG_ALG_LAST_VOTING, 64), (abi.PSG_ALG_OTR2, 100),
                 (abi.PSG_ALG_BENOR, 128)):
        out.append(("text", a, True, n))
    return sorted(set(out), key=str)


def build(job):
    from round_amd import formula as F
    import spec_cases
    kind, alg, fused, n = job
    if kind == "text":  # compiled in-process by libpsg (hiprtc), as the JVM plugin would
        from round_amd import lib
        return os.path.basename(lib.spec_compile_native(F.to_text(F.REFERENCE_SPECS[alg]()), alg, fused, n).module_path)
    if kind in ("ref", "fusedbuild"):
        spec = F.REFERENCE_SPECS[alg]() if alg in F.REFERENCE_SPECS else spec_cases.uniform_agreement()
    elif kind == "lv_custom":
        spec = spec_cases.lv_custom()
    else:
        spec = dict((c[0], c[4]) for c in spec_cases.CUSTOM)[kind]()
    p = F.compile_native(spec, alg, fused=fused, n=n)
    return os.path.basename(p.module_path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=6)
    args = ap.parse_args()
    js = jobs()
    with ProcessPoolExecutor(args.j) as ex:
        for j, m in zip(js, ex.map(build, js)):
            print(j, m, flush=True)
    import subprocess
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "fused_breakdown.py"), "--compile-only"], check=True)
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "fused_breakdown.py"), "--compile-only",
                    "--alg", "lv"], check=True)


if __name__ == "__main__":
    main()
