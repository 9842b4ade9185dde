"""ctypes binding of round_amd/libpsg.so (the HIP product library, include/psg.h).

There is no CPU fallback: if the library is missing or no HIP device is
present, construction raises. The library is built in-tree by
`make -C round_amd/csrc` (or __graft_entry__.build()).

Note on the HIP runtime: libpsg.so links libamdhip64.so.7. When the process
also uses PyTorch (bench.py: torch.distributed over RCCL), import torch BEFORE
this module so that the dynamic linker binds libpsg.so to the HIP runtime
torch already loaded (same SONAME), keeping one HIP runtime per process.
"""
import ctypes as C
import os
import threading
import sys

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PSG_LIB") or os.path.join(HERE, "libpsg.so")  # PSG_LIB: A/B builds

EXPORTED_SYMBOLS = [
    "psg_config_default", "psg_check_count", "psg_check_name", "psg_alg_from_class",
    "psg_create", "psg_load_inputs", "psg_run_batch", "psg_copy_decisions", "psg_last_batch_count",
    "psg_fetch_instances", "psg_last_error", "psg_destroy", "psg_create_error",
    "psg_selftest_map_head", "psg_load_inputs_f64", "psg_copy_decisions_f64", "psg_fetch_instances_f64",
    "psg_run_batch_spec", "psg_load_schedule", "psg_clear_schedule", "psg_materialize_schedule",
    "psg_population_fresh", "psg_population_next", "psg_population_read", "psg_spec_from_text", "psg_spec_release",
    "psg_spec_compile_native", "psg_spec_native_source", "psg_selftest_bitset", "psg_spec_rewrite_text",
    "psg_spec_set_options",
]


class PsgError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"psg error {rc}: {msg}")
        self.rc = rc


_lib = None


def load():
    """Load libpsg.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PsgError(abi.PSG_ENODEV, f"{LIB_PATH} not built (run make -C round_amd/csrc)")
    L = C.CDLL(LIB_PATH)
    L.psg_config_default.argtypes = [C.POINTER(abi.Config), C.c_int32, C.c_int32]
    L.psg_check_count.argtypes = [C.c_int32]
    L.psg_check_name.argtypes = [C.c_int32, C.c_int32]
    L.psg_check_name.restype = C.c_char_p
    L.psg_alg_from_class.argtypes = [C.c_char_p]
    L.psg_create.argtypes = [C.POINTER(C.c_void_p), C.POINTER(abi.Config)]
    L.psg_load_inputs.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_int32)]
    L.psg_run_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(abi.Summary),
                                C.POINTER(abi.InstanceSummary)]
    L.psg_copy_decisions.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    L.psg_last_batch_count.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.psg_fetch_instances.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t,
                                      C.POINTER(abi.InstanceSummary), C.POINTER(abi.ProcessRecord)]
    L.psg_last_error.argtypes = [C.c_void_p]
    L.psg_last_error.restype = C.c_char_p
    L.psg_destroy.argtypes = [C.c_void_p]
    L.psg_destroy.restype = None
    L.psg_create_error.restype = C.c_char_p
    L.psg_load_inputs_f64.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_double)]
    L.psg_copy_decisions_f64.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int32)]
    L.psg_fetch_instances_f64.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t,
                                          C.POINTER(abi.InstanceSummary), C.POINTER(abi.ProcessRecord),
                                          C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.psg_run_batch_spec.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(abi.SpecProgram),
                                     C.POINTER(abi.Summary), C.POINTER(abi.InstanceSummary)]
    L.psg_load_schedule.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]
    L.psg_clear_schedule.argtypes = [C.c_void_p]
    L.psg_materialize_schedule.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]
    L.psg_population_fresh.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(abi.PopulationParams)]
    L.psg_population_next.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(abi.PopulationParams)]
    L.psg_population_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
    L.psg_spec_from_text.argtypes = [C.c_char_p, C.c_int32, C.POINTER(abi.SpecProgram), C.c_char_p, C.c_size_t,
                                     C.c_char_p, C.c_size_t]
    try:  # (A/B builds of older kernels, PSG_LIB, may predate these; test_abi checks the in-tree library)
        L.psg_spec_compile_native.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_int32, C.c_char_p,
                                              C.POINTER(abi.SpecProgram), C.c_char_p, C.c_size_t, C.c_char_p,
                                              C.c_size_t]
        L.psg_spec_native_source.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_int32, C.c_char_p,
                                             C.POINTER(C.c_size_t), C.c_char_p, C.c_size_t]
        L.psg_spec_rewrite_text.argtypes = [C.c_char_p, C.c_int32, C.c_char_p, C.POINTER(C.c_size_t), C.c_char_p,
                                            C.c_size_t]
        L.psg_selftest_bitset.argtypes = [C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                          C.POINTER(C.c_int32), C.c_int32]
        L.psg_spec_set_options.argtypes = [C.c_char_p]
    except AttributeError:
        pass
    L.psg_spec_release.argtypes = [C.POINTER(abi.SpecProgram)]
    L.psg_spec_release.restype = None
    L.psg_selftest_map_head.argtypes = [C.c_int32, C.POINTER(C.c_uint64), C.c_int32, C.c_int32,
                                        C.POINTER(C.c_int32)]
    _lib = L
    return L


class Context:
    """One psg_ctx: one HIP device, or several (cfg.n_devices, one host thread per device)."""

    def __init__(self, cfg: abi.Config):
        L = load()
        self.cfg = cfg
        h = C.c_void_p()
        rc = L.psg_create(C.byref(h), C.byref(cfg))
        if rc != 0:
            raise PsgError(rc, L.psg_create_error().decode())
        self._h = h

    def _check(self, rc):
        if rc != 0:
            raise PsgError(rc, load().psg_last_error(self._h).decode())

    @property
    def real(self):
        return self.cfg.alg == abi.PSG_ALG_EPSILON

    def load_inputs(self, inst_begin, count, init=None):
        arr = None
        if init is not None and hasattr(init, "dtype"):  # numpy fast path
            import numpy as np
            a = np.ascontiguousarray(init, dtype=np.float64 if self.real else np.int32)
            if a.size != count * self.cfg.n:
                raise ValueError("init must be [count][n]")
            fn = load().psg_load_inputs_f64 if self.real else load().psg_load_inputs
            ptr = a.ctypes.data_as(C.POINTER(C.c_double if self.real else C.c_int32))
            self._check(fn(self._h, inst_begin, count, ptr))
            return
        if init is not None:
            if self.real:
                flat = [float(v) for row in init for v in row]
            else:
                flat = [int(v) for row in init for v in row]
            if len(flat) != count * self.cfg.n:
                raise ValueError("init must be [count][n]")
            arr = ((C.c_double if self.real else C.c_int32) * len(flat))(*flat)
        if self.real:
            self._check(load().psg_load_inputs_f64(self._h, inst_begin, count, arr))
        else:
            self._check(load().psg_load_inputs(self._h, inst_begin, count, arr))

    def run_batch(self, inst_begin, count, per_instance=False):
        s = abi.Summary()
        pi = (abi.InstanceSummary * count)() if per_instance else None
        self._check(load().psg_run_batch(self._h, inst_begin, count, C.byref(s), pi))
        return s, (list(pi) if pi is not None else None)

    def run_batch_np(self, inst_begin, count):
        """psg_run_batch with the per-instance summaries as a numpy structured array
        (round_amd.records.SUMMARY_DTYPE)."""
        import numpy as np
        from .records import SUMMARY_DTYPE
        s = abi.Summary()
        pi = np.zeros(count, SUMMARY_DTYPE)
        ptr = pi.ctypes.data_as(C.POINTER(abi.InstanceSummary))
        self._check(load().psg_run_batch(self._h, inst_begin, count, C.byref(s), ptr))
        return s, pi

    def last_batch_count(self) -> int:
        """Instances of the last batch, the library's own record (psg_last_batch_count)."""
        k = C.c_uint64()
        self._check(load().psg_last_batch_count(self._h, C.byref(k)))
        return int(k.value)

    def copy_decisions_np(self):
        """(decision, decision_round) of the last batch as numpy [count][n] arrays."""
        import numpy as np
        shape = (self.last_batch_count(), self.cfg.n)
        dr = np.zeros(shape, np.int32)
        pdr = dr.ctypes.data_as(C.POINTER(C.c_int32))
        if self.real:
            dec = np.zeros(shape, np.float64)
            self._check(load().psg_copy_decisions_f64(self._h, dec.ctypes.data_as(C.POINTER(C.c_double)), pdr))
        else:
            dec = np.zeros(shape, np.int32)
            self._check(load().psg_copy_decisions(self._h, dec.ctypes.data_as(C.POINTER(C.c_int32)), pdr))
        return dec, dr

    def fetch_np(self, ids):
        """psg_fetch_instances into numpy: (SUMMARY_DTYPE [k], PROCESS_DTYPE [k][n])."""
        import numpy as np
        from .records import PROCESS_DTYPE, SUMMARY_DTYPE
        ids = np.ascontiguousarray(ids, np.uint64)
        k = int(ids.shape[0])
        sums = np.zeros(k, SUMMARY_DTYPE)
        recs = np.zeros((k, self.cfg.n), PROCESS_DTYPE)
        self._check(load().psg_fetch_instances(self._h, ids.ctypes.data_as(C.POINTER(C.c_uint64)), k,
                                               sums.ctypes.data_as(C.POINTER(abi.InstanceSummary)),
                                               recs.ctypes.data_as(C.POINTER(abi.ProcessRecord))))
        return sums, recs

    def run_batch_spec(self, inst_begin, count, program, per_instance=False):
        """psg_run_batch_spec with a compiled Spec (round_amd.formula.Program)."""
        s = abi.Summary()
        pi = (abi.InstanceSummary * count)() if per_instance else None
        cp = program.to_c()
        self._check(load().psg_run_batch_spec(self._h, inst_begin, count, C.byref(cp), C.byref(s), pi))
        return s, (list(pi) if pi is not None else None)

    def copy_decisions(self):
        """(decision, decision_round) of the last batch, [count*n] each (Double decisions
        for real-valued algorithms)."""
        cells = self.last_batch_count() * self.cfg.n
        dr = (C.c_int32 * cells)()
        if self.real:
            dec = (C.c_double * cells)()
            self._check(load().psg_copy_decisions_f64(self._h, dec, dr))
        else:
            dec = (C.c_int32 * cells)()
            self._check(load().psg_copy_decisions(self._h, dec, dr))
        return list(dec), list(dr)

    def fetch(self, ids):
        k = len(ids)
        arr = (C.c_uint64 * k)(*ids)
        sums = (abi.InstanceSummary * k)()
        recs = (abi.ProcessRecord * (k * self.cfg.n))()
        self._check(load().psg_fetch_instances(self._h, arr, k, sums, recs))
        return list(sums), list(recs)

    def fetch_real(self, ids):
        """fetch() plus the Double decision and final x of every process ([k*n] each)."""
        k = len(ids)
        arr = (C.c_uint64 * k)(*ids)
        sums = (abi.InstanceSummary * k)()
        recs = (abi.ProcessRecord * (k * self.cfg.n))()
        dec = (C.c_double * (k * self.cfg.n))()
        fx = (C.c_double * (k * self.cfg.n))()
        self._check(load().psg_fetch_instances_f64(self._h, arr, k, sums, recs, dec, fx))
        return list(sums), list(recs), list(dec), list(fx)

    def load_schedule(self, inst_begin, count, ho, crash=None):
        """psg_load_schedule: ho uint64 [count][R][n][W], crash int32 [count][n] or None."""
        import numpy as np
        W = (self.cfg.n + 63) // 64
        ho = np.ascontiguousarray(ho, dtype=np.uint64)
        if ho.size != count * self.cfg.rounds * self.cfg.n * W:
            raise ValueError("ho must be [count][rounds][n][W] uint64")
        cr = None
        if crash is not None:
            cr = np.ascontiguousarray(crash, dtype=np.int32)
            if cr.size != count * self.cfg.n:
                raise ValueError("crash must be [count][n] int32")
        self._check(load().psg_load_schedule(self._h, inst_begin, count, ho.ctypes.data_as(C.c_void_p),
                                             None if cr is None else cr.ctypes.data_as(C.c_void_p)))

    def clear_schedule(self):
        self._check(load().psg_clear_schedule(self._h))

    def materialize_schedule(self, inst_begin, count):
        """The seeded schedule: (ho uint64 [count][R][n][W], crash int32 [count][n])."""
        import numpy as np
        W = (self.cfg.n + 63) // 64
        ho = np.zeros((count, self.cfg.rounds, self.cfg.n, W), np.uint64)
        cr = np.zeros((count, self.cfg.n), np.int32)
        self._check(load().psg_materialize_schedule(self._h, inst_begin, count, ho.ctypes.data_as(C.c_void_p),
                                                    cr.ctypes.data_as(C.c_void_p)))
        return ho, cr

    def population_fresh(self, inst_begin, count, params):
        """psg_population_fresh: a random population of explicit schedules + inputs, on the device."""
        self._check(load().psg_population_fresh(self._h, inst_begin, count, C.byref(params)))

    def population_next(self, parent, op, params):
        """psg_population_next: slot i <- copy (op 0) / mutant (1) of slot parent[i], or fresh (2)."""
        import numpy as np
        parent = np.ascontiguousarray(parent, np.uint32)
        op = np.ascontiguousarray(op, np.uint8)
        if parent.shape != op.shape:
            raise ValueError("parent and op must have one entry per slot")
        self._check(load().psg_population_next(self._h, parent.ctypes.data_as(C.c_void_p),
                                               op.ctypes.data_as(C.c_void_p), C.byref(params)))

    def population_read(self, rows):
        """Slots `rows` of the loaded population: (ho uint64 [k][R][n][W], init int32 [k][n])."""
        import numpy as np
        rows = np.ascontiguousarray(rows, np.uint32)
        k = int(rows.shape[0])
        W = (self.cfg.n + 63) // 64
        ho = np.zeros((k, self.cfg.rounds, self.cfg.n, W), np.uint64)
        init = np.zeros((k, self.cfg.n), np.int32)
        self._check(load().psg_population_read(self._h, rows.ctypes.data_as(C.c_void_p), k,
                                               ho.ctypes.data_as(C.c_void_p), init.ctypes.data_as(C.c_void_p)))
        return ho, init

    def close(self):
        if getattr(self, "_h", None):
            load().psg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def check_names(alg):
    L = load()
    return [L.psg_check_name(alg, i).decode() for i in range(L.psg_check_count(alg))]


def loaded_path():
    """Absolute path of the loaded libpsg.so (for diagnostics)."""
    load()
    with open("/proc/self/maps") as f:
        for line in f:
            if line.rstrip().endswith("libpsg.so"):
                return line.split()[-1]
    return None


if __name__ == "__main__":  # pragma: no cover
    print(loaded_path(), file=sys.stderr)


def selftest_map_head(sets, tiebreak=abi.PSG_TIE_CHAMP, device=0):
    """First pid of each 64-bit pid set in Scala Map order, computed on the GPU
    (test hook for the per-receiver mailbox.head helper)."""
    L = load()
    k = len(sets)
    arr = (C.c_uint64 * max(1, k))(*[s & ((1 << 64) - 1) for s in sets])
    out = (C.c_int32 * max(1, k))()
    rc = L.psg_selftest_map_head(device, arr, k, tiebreak, out)
    if rc != 0:
        raise PsgError(rc, "psg_selftest_map_head failed")
    return list(out)[:k]


BITSET_OPS = {"empty": 0, "full": 1, "set": 2, "clear": 3, "flip": 4, "get": 5, "size": 6}


def selftest_bitset(ops, W=1, device=0):
    """Run [(op, pos)] (BITSET_OPS names) on one Mask<W> on the GPU; the get / size results
    in order (test hook: psync.utils.LongBitSet's operations on the device HO word)."""
    L = load()
    flat = []
    n_out = 0
    for op, pos in ops:
        flat += [BITSET_OPS[op], int(pos)]
        n_out += op in ("get", "size")
    arr = (C.c_int32 * max(1, len(flat)))(*flat)
    out = (C.c_int32 * max(1, n_out))()
    rc = L.psg_selftest_bitset(device, W, arr, len(ops), out, n_out)
    if rc != 0:
        raise PsgError(rc, "psg_selftest_bitset failed")
    return list(out)[:n_out]


def spec_from_text(text, alg=0):
    """psg_spec_from_text (host code, no GPU): Formula text -> formula.Program (bytecode).
    Raises formula.FormulaError with the library's message on a rejected text."""
    from . import formula
    L = load()
    cp = abi.SpecProgram()
    err = C.create_string_buffer(1024)
    size = 4096
    while True:  # PSG_ERANGE: the slot names need a larger buffer (never truncated)
        names = C.create_string_buffer(size)
        rc = L.psg_spec_from_text(text.encode(), int(alg), C.byref(cp), names, len(names), err, len(err))
        if rc != abi.PSG_ERANGE or size >= 1 << 24:
            break
        size *= 4
    if rc != 0:
        raise formula.FormulaError(err.value.decode() or f"psg_spec_from_text rc={rc}")
    try:
        code = [cp.code[k] for k in range(cp.n_words)]
        entry = [cp.slot_entry[k] for k in range(cp.n_slots)]
        flags = [cp.slot_flags[k] for k in range(cp.n_slots)]
        prog = formula.Program(code, entry, flags, cp.term_entry, cp.n_vars, names.value.decode().split("\n"), None)
        prog.alg = cp.alg
        return prog
    finally:
        L.psg_spec_release(C.byref(cp))


_spec_opts = threading.local()  # the option string this thread last set through _SpecOptions


class _SpecOptions:
    """The generator's options (psg.h psg_spec_set_options) on the calling thread for the
    duration of one call; the environment is not touched, so threads never share them. On exit
    the thread's previous options are restored (nested calls keep the outer ones); None (the
    library falls back to PSG_SPEC_OPTIONS) only when nothing was set before."""

    def __init__(self, options):
        self.options = ",".join(options)

    def __enter__(self):
        from . import formula
        self.prev = getattr(_spec_opts, "value", None)
        if load().psg_spec_set_options(self.options.encode()) != 0:
            load().psg_spec_set_options(None if self.prev is None else self.prev.encode())
            raise formula.FormulaError(f"invalid generator options {self.options!r}")
        _spec_opts.value = self.options

    def __exit__(self, *exc):
        load().psg_spec_set_options(None if self.prev is None else self.prev.encode())
        _spec_opts.value = self.prev


def spec_compile_native(text, alg=0, fused=False, n=0, cache_dir=None, options=()):
    """psg_spec_compile_native (host code, hiprtc, no GPU needed): Formula text -> a
    formula.Program whose module_path is the natively lowered (fused: with the round kernel)
    code object, compiled in-process by the library. options: generator options (psg.h
    PSG_SPEC_OPTIONS: "nosym", "nosplit", "D<NAME>=<VALUE>")."""
    from . import formula
    L = load()
    cp = abi.SpecProgram()
    err = C.create_string_buffer(8192)
    names = C.create_string_buffer(1 << 16)
    with _SpecOptions(options):
        rc = L.psg_spec_compile_native(text.encode(), int(alg), 1 if fused else 0, int(n),
                                       cache_dir.encode() if cache_dir else None, C.byref(cp), names, len(names),
                                       err, len(err))
    if rc != 0:
        raise formula.FormulaError(err.value.decode() or f"psg_spec_compile_native rc={rc}")
    try:
        code = [cp.code[k] for k in range(cp.n_words)]
        entry = [cp.slot_entry[k] for k in range(cp.n_slots)]
        flags = [cp.slot_flags[k] for k in range(cp.n_slots)]
        prog = formula.Program(code, entry, flags, cp.term_entry, cp.n_vars, names.value.decode().split("\n"), None)
        prog.alg = cp.alg
        prog.module_path = cp.module_path.decode()
        return prog
    finally:
        path = cp.module_path
        L.psg_spec_release(C.byref(cp))
        del path


def _text_call(fn, name, options, *args):
    """A psg.h entry point with the (out, *out_len, err, err_len) buffer contract -> str."""
    from . import formula
    err = C.create_string_buffer(8192)
    size = C.c_size_t(0)
    with _SpecOptions(options):
        rc = fn(*args, None, C.byref(size), err, len(err))
        if rc not in (0, abi.PSG_ERANGE):
            raise formula.FormulaError(err.value.decode() or f"{name} rc={rc}")
        buf = C.create_string_buffer(size.value)
        rc = fn(*args, buf, C.byref(size), err, len(err))
    if rc != 0:
        raise formula.FormulaError(err.value.decode() or f"{name} rc={rc}")
    return buf.value.decode()


def spec_native_source(text, alg=0, fused=False, n=0, options=()):
    """psg_spec_native_source: the HIP source psg_spec_compile_native compiles (no compile)."""
    L = load()
    return _text_call(L.psg_spec_native_source, "psg_spec_native_source", options, text.encode(), int(alg),
                      1 if fused else 0, int(n))


def spec_rewrite_text(text, alg=0, options=()):
    """psg_spec_rewrite_text: the Spec after the native lowering's exact rewrites, as Formula text."""
    L = load()
    return _text_call(L.psg_spec_rewrite_text, "psg_spec_rewrite_text", options, text.encode(), int(alg))
