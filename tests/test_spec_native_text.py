"""Native Spec lowering from Formula text through the C ABI (psg_spec_compile_native).

The JVM plugin hands a psync.Spec to the library as Formula text (integration/scala/
GpuSpec.scala). psg_spec_from_text compiles it to bytecode; psg_spec_compile_native also
lowers it to native gfx950 code in-process (round_amd/csrc/psg_spec_gen.cpp, compiled with
hiprtc). It is the only generator: formula.compile_native writes a DSL Spec as Formula text and
calls it, so the DSL and the JVM routes build the same module. CPU tests: every
reference and custom Spec of the GPU suites and the FormulaExtractor-shaped texts lower, native
and fused; the DSL -> text -> DSL round trip lowers to the same source; a hiprtc compile yields a gfx950 code
object whose program equals psg_spec_from_text's. GPU tests: the library-compiled fused module's
results equal the built-in checker's, word for word.
"""
import ctypes as C
import os

import pytest

from round_amd import abi, formula as F, lib, psync

import spec_cases
import test_spec_text as TT

CASES = [(f"ref-{a}", a, 64, lambda a=a: F.to_text(F.REFERENCE_SPECS[a]())) for a in sorted(F.REFERENCE_SPECS)]
CASES += [(c[0], c[1].alg_id, c[2], lambda mk=c[4]: F.to_text(mk())) for c in spec_cases.CUSTOM]
CASES += [("let", abi.PSG_ALG_LAST_VOTING, 8, lambda: TT.LV_MAJORITY_LET),
          ("flat-binders", abi.PSG_ALG_OTR, 8, lambda: TT.AGREEMENT_FLAT),
          ("nary-and", abi.PSG_ALG_BENOR, 8, lambda: TT.NARY_AND)]


@pytest.mark.parametrize("cid,alg,n,text", CASES, ids=[c[0] for c in CASES])
def test_native_source_generates(cid, alg, n, text):
    """Every Spec lowers (native and fused), the fused module holds the algorithm's kernels
    for n's wave count, and the DSL route reaches the same generator with the same text."""
    t = text()
    for fused in (False, True):
        if fused and alg not in F.FUSED_KERNELS:
            continue
        src = lib.spec_native_source(t, alg, fused, n)
        assert "struct GenSpec" in src and f"psg_spec_alg = {alg};" in src, (cid, fused)
        if fused:
            W = (n + 63) // 64
            assert f"psg_fused_a{alg}_w{W}(" in src and f"psg_fused_x_a{alg}_w{W}(" in src
    assert lib.spec_native_source(F.to_text(F.from_text(t)), alg) == lib.spec_native_source(t, alg)


def test_generator_options():
    """Generator options (psg.h psg_spec_set_options / PSG_SPEC_OPTIONS): nosym drops the symmetric-check-point lowering, nosplit the
    split foralls, D<NAME>=<VALUE> adds a #define; the default source has neither change."""
    t = F.to_text(F.otr_spec())
    base = lib.spec_native_source(t, abi.PSG_ALG_OTR)
    assert "spec::uniform<" in base and "spec::uniform<" not in lib.spec_native_source(t, abi.PSG_ALG_OTR,
                                                                                      options=["nosym"])
    assert lib.spec_native_source(t, abi.PSG_ALG_OTR, options=["DPSG_PHASE_TIMERS=1"]).startswith(
        "#define PSG_PHASE_TIMERS 1\n")
    lv = F.to_text(F.lv_spec())
    assert lib.spec_native_source(lv, abi.PSG_ALG_LAST_VOTING) != lib.spec_native_source(
        lv, abi.PSG_ALG_LAST_VOTING, options=["nosplit"])
    with pytest.raises(F.FormulaError, match="invalid generator options"):
        lib.spec_native_source(t, abi.PSG_ALG_OTR, options=["bogus"])
    assert "PSG_SPEC_OPTIONS" not in os.environ


def test_generator_options_are_per_thread():
    """8 threads lower concurrently, each with its own options (psg_spec_set_options is
    thread-local): every result equals the single-threaded result for those options."""
    import threading
    t_otr, t_lv = F.to_text(F.otr_spec()), F.to_text(F.lv_spec())
    jobs = [(lib.spec_native_source, t_otr, abi.PSG_ALG_OTR, ()),
            (lib.spec_native_source, t_otr, abi.PSG_ALG_OTR, ("nosym",)),
            (lib.spec_native_source, t_lv, abi.PSG_ALG_LAST_VOTING, ("nosplit",)),
            (lib.spec_native_source, t_otr, abi.PSG_ALG_OTR, ("DPSG_PHASE_TIMERS=1",)),
            (lib.spec_rewrite_text, t_lv, abi.PSG_ALG_LAST_VOTING, ()),
            (lib.spec_rewrite_text, t_lv, abi.PSG_ALG_LAST_VOTING, ("nosplit",)),
            (lib.spec_native_source, t_lv, abi.PSG_ALG_LAST_VOTING, ("nosym", "DPSG_QUEUE_CHUNK=3")),
            (lib.spec_rewrite_text, t_otr, abi.PSG_ALG_OTR, ("nosplit",))]
    want = [fn(t, alg, options=o) for fn, t, alg, o in jobs]
    got = [[] for _ in jobs]
    errors = []

    def worker(i):
        fn, t, alg, o = jobs[i]
        try:
            for _ in range(12):
                got[i].append(fn(t, alg, options=o))
        except Exception as e:  # noqa: BLE001 — reported below
            errors.append((i, e))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(jobs))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for i in range(len(jobs)):
        assert all(g == want[i] for g in got[i]), i
    # the options differ in effect, so a leak between threads would have shown
    assert want[0] != want[1] and want[4] != want[5] and want[3].startswith("#define PSG_PHASE_TIMERS 1\n")


def test_nested_options_restore_the_outer_ones():
    """_SpecOptions restores the thread's previous options on exit: an inner call
    with its own options leaves the outer call's options in force."""
    t = F.to_text(F.otr_spec())
    want = lib.spec_native_source(t, abi.PSG_ALG_OTR, options=["nosym"])
    with lib._SpecOptions(["nosym"]):
        lib.spec_native_source(t, abi.PSG_ALG_OTR, options=["DPSG_PHASE_TIMERS=1"])
        # the outer options are back: a call with no options of its own sees nosym
        n = C.c_size_t(0)
        err = C.create_string_buffer(512)
        L = lib.load()
        assert L.psg_spec_native_source(t.encode(), abi.PSG_ALG_OTR, 0, 0, None, C.byref(n), err, 512) == abi.PSG_ERANGE
        buf = C.create_string_buffer(n.value)
        assert L.psg_spec_native_source(t.encode(), abi.PSG_ALG_OTR, 0, 0, buf, C.byref(n), err, 512) == abi.PSG_OK
        assert buf.value.decode() == want
    assert "spec::uniform<" in lib.spec_native_source(t, abi.PSG_ALG_OTR)
    with pytest.raises(F.FormulaError):
        with lib._SpecOptions(["nosym"]):
            lib.spec_native_source(t, abi.PSG_ALG_OTR, options=["bogus"])


def test_probe_switches_rejected():
    """A define naming a probe-build switch (PSG_AB*) never reaches a product module: from the
    per-thread setter and from the environment alike the entry points return PSG_EINVAL."""
    import subprocess
    import sys
    t = F.to_text(F.otr_spec())
    with pytest.raises(F.FormulaError, match="invalid generator options"):
        lib.spec_native_source(t, abi.PSG_ALG_OTR, options=["DPSG_ABL_NOCHECK=1"])
    L = lib.load()
    assert L.psg_spec_set_options(b"DPSG_AB_NO_CW=1") == abi.PSG_EINVAL
    assert L.psg_spec_set_options(b"D=1") == abi.PSG_EINVAL
    # allow-list and integer values only: no result-changing define, no source text
    assert L.psg_spec_set_options(b"DPSG_MAX_CHECKS=3") == abi.PSG_EINVAL
    assert L.psg_spec_set_options(b"DPSG_FUSED_MODULE=1") == abi.PSG_EINVAL
    assert L.psg_spec_set_options(b"DPSG_OTR_WPE=4\nint x;") == abi.PSG_EINVAL
    assert L.psg_spec_set_options(b"DPSG_OTR_WPE=a") == abi.PSG_EINVAL
    assert L.psg_spec_set_options(b"DPSG_OTR_WPE=-3") == abi.PSG_OK
    assert L.psg_spec_set_options(b"DPSG_QUEUE_CHUNK=8,nosym") == abi.PSG_OK
    assert L.psg_spec_set_options(None) == abi.PSG_OK
    # through the environment (the JVM route): a child process, rc of psg_spec_native_source
    code = ("import ctypes as C, sys; sys.path.insert(0, %r); from round_amd import lib, formula as F, abi; "
            "L = lib.load(); n = C.c_size_t(0); err = C.create_string_buffer(512); "
            "rc = L.psg_spec_native_source(F.to_text(F.otr_spec()).encode(), abi.PSG_ALG_OTR, 0, 0, None, "
            "C.byref(n), err, 512); print(rc, err.value.decode())") % os.path.dirname(os.path.dirname(
                os.path.abspath(__file__)))
    env = dict(os.environ, PSG_SPEC_OPTIONS="DPSG_ABL_NOCHECK=1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    rc, _, msg = out.stdout.strip().partition(" ")
    assert int(rc) == abi.PSG_EINVAL and "probe build" in msg, out


def test_native_source_rejects_like_the_bytecode_compiler():
    with pytest.raises(F.FormulaError, match="ForAll over Int"):
        lib.spec_native_source("(Spec (invariants (ForAll ((v Int)) (App Gt (Var v) (Lit 0)))))", abi.PSG_ALG_OTR)
    with pytest.raises(F.FormulaError, match="no integer state"):
        lib.spec_native_source(F.to_text(F.otr_spec()), abi.PSG_ALG_EPSILON, True, 64)


def test_hiprtc_compile_on_the_host(tmp_path):
    """In-process compile (no GPU): a gfx950 code object in the given cache, the program of
    psg_spec_from_text, the cached object reused by a second call."""
    text = F.to_text(F.otr_spec())
    prog = lib.spec_compile_native(text, abi.PSG_ALG_OTR, True, 64, cache_dir=str(tmp_path))
    assert prog.module_path.startswith(str(tmp_path)) and os.path.getsize(prog.module_path) > 10_000
    with open(prog.module_path, "rb") as f:
        assert f.read(4) == b"\x7fELF"
    TT._same(prog, lib.spec_from_text(text, abi.PSG_ALG_OTR))
    mtime = os.path.getmtime(prog.module_path)
    again = lib.spec_compile_native(text, abi.PSG_ALG_OTR, True, 64, cache_dir=str(tmp_path))
    assert again.module_path == prog.module_path and os.path.getmtime(again.module_path) == mtime
    # formula.compile_native is this route: the DSL Spec finds this very file
    assert F.compile_native(F.from_text(text), abi.PSG_ALG_OTR, fused=True, n=64,
                            cache_dir=str(tmp_path)).module_path == prog.module_path


@pytest.mark.gpu
@pytest.mark.parametrize("alg,mk,n,count,kw", [
    (psync.OTR(), F.otr_spec, 64, 20_000, dict(value_range=64, seed=2)),
    (psync.LastVoting(), F.lv_spec, 64, 5_000, dict(seed=7)),
    (psync.OTR2(), F.otr2_spec, 100, 2_000, dict(value_range=4, seed=3)),
    (psync.BenOr(), F.benor_spec, 128, 2_000, dict(seed=5)),
], ids=["otr", "lv", "otr2-n100", "benor-n128"])
def test_text_fused_module_equals_builtin_and_python(alg, mk, n, count, kw):
    """The Spec given as text, lowered and compiled by the library (hiprtc; built into the
    default cache by __graft_entry__.build(), scripts/precompile_specs.py), run fused: every
    counter and per-instance result equals the built-in checker's and the DSL route's
    (formula.compile_native), word for word."""
    text = F.to_text(mk())
    prog_c = lib.spec_compile_native(text, alg.alg_id, True, n)
    prog_py = F.compile_native(mk(), alg.alg_id, fused=True, n=n)
    with psync.GpuRound(alg, n, batch_capacity=count, **kw) as g:
        builtin = g.run(0, count, per_instance=True)
        rc = g.run_spec(0, count, prog_c, per_instance=True)
        rp = g.run_spec(0, count, prog_py, per_instance=True)
    key = lambda r: (abi.summary_to_list(r.summary)[:-1],
                     [(s.digest, tuple(s.first_fail), s.term_round) for s in r.per_instance])
    assert key(rc) == key(rp)
    assert key(rc) == key(builtin)


_TOOLCHAIN_PROBE = r"""
import hashlib, os, sys
if sys.argv[1] == "torch":
    import torch  # noqa: F401  (the process now holds torch's bundled HIP libraries)
sys.path.insert(0, sys.argv[3])
from round_amd import lib, formula as F, abi
p = lib.spec_compile_native(F.to_text(F.otr_spec()), abi.PSG_ALG_OTR, False, 0, cache_dir=sys.argv[2])
maps = open('/proc/self/maps').read()
comgr = sorted(set(l.split()[-1] for l in maps.splitlines() if 'amd_comgr' in l))
print(os.path.basename(p.module_path), hashlib.sha256(open(p.module_path, 'rb').read()).hexdigest(), '|'.join(comgr))
"""


def test_module_toolchain_independent_of_torch(tmp_path):
    """A module compiled in a process that imported torch first (which binds torch's bundled
    ROCm 7.0 hiprtc / comgr under the same sonames) is the module a plain process compiles: the
    generator loads the image's comgr and hiprtc into a namespace of their own (psg_spec_gen.cpp
    rtc_api). Round 5's one-process config run had loaded a torch-compiled fused LastVoting
    module with 416 B of scratch, 3.4x slower."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for mode in ("plain", "torch"):
        r = subprocess.run([sys.executable, "-c", _TOOLCHAIN_PROBE, mode, str(tmp_path / mode), root],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        out[mode] = r.stdout.split()
    assert out["plain"][:2] == out["torch"][:2]  # same cache key, same code object bytes
    assert any(p.startswith("/opt/rocm") for p in out["torch"][2].split("|")), out["torch"]


def test_fused_lastvoting_defaults_to_no_symmetric_lowering():
    """Fused LastVoting modules drop the symmetric-check-point lowering by default (measured faster,
    psg_spec_gen.cpp module_source); "sym" brings it back, "nosym" is the default's own source; the
    non-fused LastVoting module and fused OTR keep it."""
    t = F.to_text(F.lv_spec())
    fused = lib.spec_native_source(t, abi.PSG_ALG_LAST_VOTING, fused=True, n=64)
    assert "spec::uniform<" not in fused
    assert fused == lib.spec_native_source(t, abi.PSG_ALG_LAST_VOTING, fused=True, n=64, options=["nosym"])
    assert "spec::uniform<" in lib.spec_native_source(t, abi.PSG_ALG_LAST_VOTING, fused=True, n=64, options=["sym"])
    assert "spec::uniform<" in lib.spec_native_source(t, abi.PSG_ALG_LAST_VOTING)
    assert "spec::uniform<" in lib.spec_native_source(F.to_text(F.otr_spec()), abi.PSG_ALG_OTR, fused=True, n=64)
