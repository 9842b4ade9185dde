"""ctypes binding of the CPU oracle (oracle/psg_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py. The product path (round_amd/) never imports it.
"""
import ctypes as C
import os
import subprocess

from round_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
SRC = os.path.join(HERE, "psg_oracle.cpp")

SPEC_DIRECT, SPEC_INTERP, SPEC_BOTH = 0, 1, 2


def build(force=False):
    """Compile the oracle with g++ (recipe also in oracle/Makefile)."""
    if not force and os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= max(
            os.path.getmtime(SRC), os.path.getmtime(os.path.join(HERE, "..", "include", "psg.h"))):
        return LIB_PATH
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_run.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_int32), C.POINTER(abi.Summary),
                                 C.POINTER(abi.InstanceSummary), C.POINTER(abi.ProcessRecord),
                                 C.c_int32, C.c_int32]
        L.oracle_run.restype = C.c_int
        L.oracle_run_explicit.argtypes = [C.POINTER(abi.Config), C.POINTER(C.c_int32), C.POINTER(C.c_uint64),
                                          C.POINTER(abi.InstanceSummary), C.POINTER(abi.ProcessRecord),
                                          C.POINTER(C.c_int64), C.c_int32]
        L.oracle_run_explicit.restype = C.c_int
        L.oracle_run_real.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_double), C.POINTER(abi.Summary),
                                      C.POINTER(abi.InstanceSummary), C.POINTER(abi.ProcessRecord),
                                      C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int32]
        L.oracle_run_real.restype = C.c_int
        L.oracle_run_explicit_real.argtypes = [C.POINTER(abi.Config), C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                               C.POINTER(abi.InstanceSummary), C.POINTER(abi.ProcessRecord),
                                               C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.oracle_run_explicit_real.restype = C.c_int
        L.oracle_trace.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_uint64, C.POINTER(C.c_int32),
                                   C.POINTER(C.c_int32), C.c_int32]
        L.oracle_trace.restype = C.c_int
        L.oracle_trace_checks.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_uint64, C.POINTER(C.c_int32),
                                          C.POINTER(C.c_int32), C.POINTER(C.c_uint16), C.c_int32, C.c_int32]
        L.oracle_trace_checks.restype = C.c_int
        L.oracle_vm_run.argtypes = [C.POINTER(abi.SpecProgram), C.POINTER(C.c_int32), C.c_uint64, C.c_int32,
                                    C.c_int32, C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]
        L.oracle_vm_run.restype = C.c_int
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_philox.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.oracle_java_first_boolean.argtypes = [C.c_int64]
        L.oracle_java_first_boolean.restype = C.c_int
        L.oracle_scala_improve.argtypes = [C.c_uint32]
        L.oracle_scala_improve.restype = C.c_uint32
        L.oracle_scala_map_order.argtypes = [C.POINTER(C.c_int32), C.c_int32, C.c_int32, C.POINTER(C.c_int32)]
        L.oracle_ho_mask.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_int32, C.c_int32]
        L.oracle_ho_mask.restype = C.c_uint64
        L.oracle_init_value.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_int32]
        L.oracle_init_value.restype = C.c_int32
        L.oracle_crash_round.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_int32]
        L.oracle_crash_round.restype = C.c_int32
        L.oracle_run_schedule.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.POINTER(abi.Summary),
                                          C.POINTER(abi.InstanceSummary), C.POINTER(abi.ProcessRecord),
                                          C.c_void_p, C.c_void_p, C.c_int32]
        L.oracle_run_schedule.restype = C.c_int
        L.oracle_materialize_schedule.argtypes = [C.POINTER(abi.Config), C.c_uint64, C.c_uint64, C.c_void_p,
                                                  C.c_void_p]
        L.oracle_materialize_schedule.restype = C.c_int
        _lib = L
    return _lib


class OracleError(RuntimeError):
    pass


def _check(rc):
    if rc != 0:
        raise OracleError(f"oracle rc={rc}: {lib().oracle_last_error().decode()}")


def run(cfg, inst_begin=0, count=1, ids=None, init=None, per_instance=False, records=False,
        threads=1, spec_mode=SPEC_DIRECT):
    """Run instances on the CPU oracle. Returns (Summary, [InstanceSummary], [ProcessRecord])."""
    L = lib()
    if ids is not None:
        count = len(ids)
        ids_arr = (C.c_uint64 * count)(*ids)
    else:
        ids_arr = None
    init_arr = None
    if init is not None:
        flat = [int(v) for row in init for v in row]
        init_arr = (C.c_int32 * len(flat))(*flat)
    summ = abi.Summary()
    pi = (abi.InstanceSummary * count)() if per_instance else None
    rec = (abi.ProcessRecord * (count * cfg.n))() if records else None
    rc = L.oracle_run(C.byref(cfg), inst_begin, count, ids_arr, init_arr, C.byref(summ), pi, rec,
                      threads, spec_mode)
    _check(rc)
    return summ, (list(pi) if pi is not None else None), (list(rec) if rec is not None else None)


def run_real(cfg, inst_begin=0, count=1, ids=None, init=None, per_instance=False, records=False, threads=1):
    """Real-valued algorithm (EpsilonConsensus) on the CPU oracle.

    Returns (Summary, [InstanceSummary], [ProcessRecord], decisions, final_x) where the
    last two are flat [count*n] Double lists (None unless records=True)."""
    L = lib()
    if ids is not None:
        count = len(ids)
        ids_arr = (C.c_uint64 * count)(*ids)
    else:
        ids_arr = None
    init_arr = None
    if init is not None:
        flat = [float(v) for row in init for v in row]
        init_arr = (C.c_double * len(flat))(*flat)
    summ = abi.Summary()
    pi = (abi.InstanceSummary * count)() if per_instance else None
    cells = count * cfg.n
    rec = (abi.ProcessRecord * cells)() if records else None
    dec = (C.c_double * cells)() if records else None
    fx = (C.c_double * cells)() if records else None
    rc = L.oracle_run_real(C.byref(cfg), inst_begin, count, ids_arr, init_arr, C.byref(summ), pi, rec, dec, fx,
                           threads)
    _check(rc)
    return (summ, (list(pi) if pi is not None else None), (list(rec) if rec is not None else None),
            (list(dec) if dec is not None else None), (list(fx) if fx is not None else None))


def run_explicit_real(cfg, init, ho):
    """One real-valued instance with an explicit HO schedule ho[k][p] (n <= 64).
    Returns (InstanceSummary, [ProcessRecord], decisions, final_x)."""
    L = lib()
    n = cfg.n
    if len(ho) != cfg.rounds or any(len(row) != n for row in ho):
        raise ValueError("ho must be [rounds][n]")
    flat = [m & ((1 << 64) - 1) for row in ho for m in row]
    ho_arr = (C.c_uint64 * len(flat))(*flat)
    init_arr = (C.c_double * n)(*[float(v) for v in init])
    s = abi.InstanceSummary()
    rec = (abi.ProcessRecord * n)()
    dec = (C.c_double * n)()
    fx = (C.c_double * n)()
    _check(L.oracle_run_explicit_real(C.byref(cfg), init_arr, ho_arr, C.byref(s), rec, dec, fx))
    return s, list(rec), list(dec), list(fx)


def run_explicit(cfg, init, ho, spec_mode=SPEC_BOTH):
    """One instance with an explicit HO schedule ho[k][p] (bit q: p hears q), n <= 64.

    Returns (InstanceSummary, [ProcessRecord], trace) with trace[c] = (x[], decided[]).
    """
    L = lib()
    n, R = cfg.n, cfg.rounds
    init_arr = (C.c_int32 * n)(*init)
    flat = [int(ho[k][p]) for k in range(R) for p in range(n)]
    ho_arr = (C.c_uint64 * len(flat))(*flat)
    s = abi.InstanceSummary()
    rec = (abi.ProcessRecord * n)()
    tr = (C.c_int64 * ((R + 1) * 2 * n))()
    _check(L.oracle_run_explicit(C.byref(cfg), init_arr, ho_arr, C.byref(s), rec, tr, spec_mode))
    trace = []
    for c in range(R + 1):
        base = c * 2 * n
        trace.append(([tr[base + p] for p in range(n)], [tr[base + n + p] for p in range(n)]))
    return s, list(rec), trace


def philox(ctr, key):
    L = lib()
    a = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    L.oracle_philox(a, k, o)
    return list(o)


def java_first_boolean(seed):
    return bool(lib().oracle_java_first_boolean(seed))


def scala_improve(h):
    return lib().oracle_scala_improve(h & 0xFFFFFFFF)


def scala_map_order(keys, tiebreak=abi.PSG_TIE_CHAMP):
    m = len(keys)
    a = (C.c_int32 * m)(*keys)
    o = (C.c_int32 * m)()
    lib().oracle_scala_map_order(a, m, tiebreak, o)
    return list(o)


def ho_mask(cfg, inst, k, p):
    return lib().oracle_ho_mask(C.byref(cfg), inst, k, p)


def init_value(cfg, inst, p):
    return lib().oracle_init_value(C.byref(cfg), inst, p)


def crash_round(cfg, inst, p):
    return lib().oracle_crash_round(C.byref(cfg), inst, p)


NFIELDS = 9


def trace(cfg, inst_begin, count, init=None, threads=8):
    """Per-check-point process states of each instance, the layout psg_run_batch_spec
    traces on the device: flat int32 [count][R+1][9][n] (Option None = INT32_MIN).
    init: optional [count][n] initial values (else seeded)."""
    per = (cfg.rounds + 1) * NFIELDS * cfg.n
    out = (C.c_int32 * (count * per))()
    init_arr = None
    if init is not None:
        flat = [int(v) for row in init for v in row]
        init_arr = (C.c_int32 * len(flat))(*flat)
    _check(lib().oracle_trace(C.byref(cfg), inst_begin, count, init_arr, out, threads))
    return out


def trace_checks(cfg, inst_begin, count, init=None, threads=8, spec_mode=2):
    """(trace, bits): the states of trace() as numpy int32 [count][R+1][9][n] and the
    checker's verdict per check point, uint16 [count][R+1] (bit s = slot s holds, bit 15 =
    Termination holds). spec_mode 0 hand-lowered, 1 Formula interpreter, 2 both (required
    equal)."""
    import numpy as np
    R, n = cfg.rounds, cfg.n
    tr = np.zeros((count, R + 1, NFIELDS, n), np.int32)
    bits = np.zeros((count, R + 1), np.uint16)
    init_arr = None
    if init is not None:
        init_arr = np.ascontiguousarray(init, np.int32)
    _check(lib().oracle_trace_checks(C.byref(cfg), inst_begin, count,
                                     init_arr.ctypes.data_as(C.POINTER(C.c_int32)) if init_arr is not None else None,
                                     tr.ctypes.data_as(C.POINTER(C.c_int32)),
                                     bits.ctypes.data_as(C.POINTER(C.c_uint16)), threads, spec_mode))
    return tr, bits


def vm_run(program, tr, count, n, rounds):
    """Evaluate a compiled Spec (round_amd.formula.Program) on traces with the CPU
    interpreter: returns ([first_fail per slot] per instance, [term_round])."""
    cp = program.to_c()
    ff = (C.c_uint8 * (count * abi.PSG_MAX_CHECKS))()
    tm = (C.c_uint8 * count)()
    _check(lib().oracle_vm_run(C.byref(cp), tr, count, n, rounds, ff, tm))
    k = len(program.slot_entry)
    return [list(ff[i * abi.PSG_MAX_CHECKS:i * abi.PSG_MAX_CHECKS + k]) for i in range(count)], list(tm)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def run_schedule(cfg, inst_begin, count, ho, crash=None, init=None, per_instance=False, records=False,
                 threads=8):
    """Instances under an explicit schedule (psg_load_schedule semantics).

    ho: uint64 [count][R][n][W]; crash: int32 [count][n] or None; init: [count][n]
    int32 (Doubles for EpsilonConsensus) or None = seeded. Returns (Summary,
    [InstanceSummary], [ProcessRecord], decisions, final_x) — the last two only for
    real-valued algorithms with records=True."""
    import numpy as np
    real = cfg.alg == abi.PSG_ALG_EPSILON
    W = (cfg.n + 63) // 64
    ho = np.ascontiguousarray(ho, dtype=np.uint64).reshape(count, cfg.rounds, cfg.n, W)
    cr = None if crash is None else np.ascontiguousarray(crash, dtype=np.int32).reshape(count, cfg.n)
    ini = None
    if init is not None:
        ini = np.ascontiguousarray(init, dtype=np.float64 if real else np.int32).reshape(count, cfg.n)
    summ = abi.Summary()
    pi = (abi.InstanceSummary * count)() if per_instance else None
    cells = count * cfg.n
    rec = (abi.ProcessRecord * cells)() if records else None
    dec = np.zeros(cells, np.float64) if (records and real) else None
    fx = np.zeros(cells, np.float64) if (records and real) else None
    rc = lib().oracle_run_schedule(C.byref(cfg), inst_begin, count, None if real else _ptr(ini),
                                   _ptr(ini) if real else None, _ptr(ho), _ptr(cr), C.byref(summ), pi, rec,
                                   _ptr(dec), _ptr(fx), threads)
    _check(rc)
    return (summ, (list(pi) if pi is not None else None), (list(rec) if rec is not None else None), dec, fx)


def materialize_schedule(cfg, inst_begin, count):
    """The seeded schedule in the explicit layout: (ho uint64 [count][R][n][W], crash int32 [count][n])."""
    import numpy as np
    W = (cfg.n + 63) // 64
    ho = np.zeros((count, cfg.rounds, cfg.n, W), np.uint64)
    cr = np.zeros((count, cfg.n), np.int32)
    _check(lib().oracle_materialize_schedule(C.byref(cfg), inst_begin, count, _ptr(ho), _ptr(cr)))
    return ho, cr
