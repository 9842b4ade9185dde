"""The JNI shim (integration/jni/psg_jni.c) without a JVM.

The image has no JDK, so the shim is built against integration/jni/jni_min/jni.h (the
JNI types and the JNIEnv functions it calls, declaration only) and, for execution,
linked with tests/jni/fake_jni.c, a JNIEnv in C over plain heap objects
(tests/jni/Makefile -> tests/jni/libpsg_jni_test.so). CPU tests: it compiles with
-Wall -Werror; every `@native def` of integration/scala/GpuRound.scala has a C entry
point with the JNI-mangled name and matching parameter types; short Java arrays are
refused with IllegalArgumentException before any element is touched; compileSpec
returns what psg_spec_from_text compiles. The GPU test drives a whole batch through
the shim and compares it with the Python binding of the same C ABI.
"""
import ctypes as C
import os
import re
import subprocess

import pytest

from round_amd import abi, formula as F, lib, psync

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "integration", "jni", "psg_jni.c")
SCALA = os.path.join(ROOT, "integration", "scala", "GpuRound.scala")
SO = os.path.join(ROOT, "tests", "jni", "libpsg_jni_test.so")
FJ_INT, FJ_LONG, FJ_BYTE, FJ_DOUBLE = 1, 2, 3, 4

SCALA_TO_JNI = {"Int": "jint", "Long": "jlong", "Double": "jdouble", "Boolean": "jboolean", "String": "jstring",
                "Array[Int]": "jintArray", "Array[Long]": "jlongArray", "Array[Byte]": "jbyteArray",
                "Array[Double]": "jdoubleArray", "Unit": "void"}


def test_shim_compiles_warning_free():
    subprocess.check_call(["gcc", "-fsyntax-only", "-std=c99", "-Wall", "-Wextra", "-Werror",
                           "-I", os.path.join(ROOT, "integration", "jni", "jni_min"),
                           "-I", os.path.join(ROOT, "include"), SHIM])


def _scala_natives():
    src = open(SCALA).read()
    body = src[src.index("object GpuRoundNative"):src.index("/** HO schedule")]
    out = {}
    for m in re.finditer(r"@native def (\w+)\(([^)]*)\):\s*([\w\[\]]+)", body, re.S):
        params = [p.split(":")[1].strip() for p in m.group(2).replace("\n", " ").split(",") if p.strip()]
        out[m.group(1)] = (params, m.group(3))
    return out


def _c_entries():
    src = open(SHIM).read()
    out = {}
    for m in re.finditer(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+Java_psync_gpu_GpuRoundNative_00024_(\w+)\(([^)]*)\)",
                         src, re.S):
        params = [" ".join(p.split()[:-1]) for p in m.group(3).replace("\n", " ").split(",")]
        out[m.group(2)] = (params[2:], m.group(1))  # drop JNIEnv*, jobject self
    return out


def test_every_native_method_has_a_matching_entry_point():
    """JNI name mangling of `object GpuRoundNative` (GpuRoundNative$ -> _00024) and the
    parameter / return types of each @native def."""
    scala, c = _scala_natives(), _c_entries()
    assert set(scala) == set(c), (set(scala) ^ set(c))
    for name, (params, ret) in scala.items():
        cparams, cret = c[name]
        assert [SCALA_TO_JNI[p] for p in params] == cparams, name
        assert SCALA_TO_JNI[ret] == cret, name
    nm = subprocess.check_output(["nm", "-D", "--defined-only", SO]).decode()
    for name in scala:
        assert f"Java_psync_gpu_GpuRoundNative_00024_{name}" in nm


class Shim:
    def __init__(self):
        self.L = C.CDLL(SO)
        L = self.L
        L.fj_env.restype = C.c_void_p
        L.fj_new.restype = C.c_void_p
        L.fj_new.argtypes = [C.c_int, C.c_int]
        L.fj_string.restype = C.c_void_p
        L.fj_string.argtypes = [C.c_char_p]
        L.fj_data.restype = C.c_void_p
        L.fj_data.argtypes = [C.c_void_p]
        L.fj_len.argtypes = [C.c_void_p]
        L.fj_free.argtypes = [C.c_void_p]
        L.fj_fake_ctx.restype = C.c_void_p
        L.fj_fake_ctx.argtypes = [C.c_int, C.c_int]
        self.env = L.fj_env()

    def fn(self, name, restype, *argtypes):
        f = getattr(self.L, "Java_psync_gpu_GpuRoundNative_00024_" + name)
        f.restype = restype
        f.argtypes = [C.c_void_p, C.c_void_p] + list(argtypes)
        return lambda *a: f(self.env, None, *a)

    def array(self, kind, values):
        o = self.L.fj_new(kind, len(values))
        ct = {FJ_INT: C.c_int32, FJ_LONG: C.c_int64, FJ_BYTE: C.c_int8, FJ_DOUBLE: C.c_double}[kind]
        buf = (ct * max(1, len(values))).from_address(self.L.fj_data(o))
        for k, v in enumerate(values):
            buf[k] = v
        return o

    def values(self, kind, o):
        ct = {FJ_INT: C.c_int32, FJ_LONG: C.c_int64, FJ_BYTE: C.c_uint8, FJ_DOUBLE: C.c_double}[kind]
        n = self.L.fj_len(o)
        return list((ct * max(1, n)).from_address(self.L.fj_data(o)))[:n]

    def exception(self):
        cls, msg = C.create_string_buffer(256), C.create_string_buffer(1024)
        return (cls.value.decode(), msg.value.decode()) if self.L.fj_take_exception(cls, 256, msg, 1024) else None


@pytest.fixture(scope="module")
def shim():
    if not os.path.exists(SO):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(SO)])
    return Shim()


def test_short_arrays_are_refused(shim):
    """ADVICE: the shim checks every Java array's length before taking its elements."""
    h = shim.L.fj_fake_ctx(64, 20)  # n = 64, R = 20; no psg context behind it
    load = shim.fn("loadInputs", None, C.c_int64, C.c_int64, C.c_int64, C.c_void_p)
    load(h, 0, 10, shim.array(FJ_INT, [1] * (10 * 64 - 1)))
    exc = shim.exception()
    assert exc[0] == "java/lang/IllegalArgumentException" and "639 elements, 640 needed" in exc[1]
    load(h, 0, 10, shim.array(FJ_INT, [1] * (10 * 64)))  # long enough: reaches the C ABI (null context)
    exc = shim.exception()
    assert exc[0] == "java/lang/IllegalArgumentException" and exc[1].startswith("psg error -22")
    sched = shim.fn("loadSchedule", None, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p)
    sched(h, 0, 2, shim.array(FJ_LONG, [0] * (2 * 20 * 64 - 1)), None)
    assert "2559 elements, 2560 needed" in shim.exception()[1]
    sched(h, 0, 2, shim.array(FJ_LONG, [0] * (2 * 20 * 64)), shim.array(FJ_INT, [0] * 127))
    assert "crash has 127 elements, 128 needed" in shim.exception()[1]
    # copyDecisions sizes its check from the library's own last batch (psg_last_batch_count):
    # with no context behind the handle that is 0 cells, and the C ABI refuses the null context
    copy = shim.fn("copyDecisions", None, C.c_int64, C.c_void_p, C.c_void_p)
    copy(h, shim.array(FJ_INT, []), None)
    assert shim.exception()[1].startswith("psg error -22")
    fetch = shim.fn("fetch", None, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p)
    fetch(h, shim.array(FJ_LONG, [1, 2]), shim.array(FJ_BYTE, [0] * 48), shim.array(FJ_INT, [0] * (2 * 64 * 4 - 1)))
    assert "records has 511 elements, 512 needed" in shim.exception()[1]
    fetch(h, shim.array(FJ_LONG, [1, 2]), shim.array(FJ_BYTE, [0] * 47), shim.array(FJ_INT, [0] * 512))
    assert "sums has 47 elements, 48 needed" in shim.exception()[1]
    run = shim.fn("runBatch", C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p)
    assert run(h, 0, 4, shim.array(FJ_BYTE, [0] * 95)) is None
    assert "perInstance has 95 elements, 96 needed" in shim.exception()[1]
    assert run(h, -1, 4, None) is None
    assert "begin / count" in shim.exception()[1]
    assert shim.L.fj_take_oob() == 0


def test_compile_spec_through_the_shim(shim):
    comp = shim.fn("compileSpec", C.c_void_p, C.c_void_p, C.c_int32)
    names = shim.fn("compileSpecNames", C.c_void_p, C.c_void_p, C.c_int32)
    for alg, mk in F.REFERENCE_SPECS.items():
        text = F.to_text(mk())
        packed = shim.values(FJ_INT, comp(shim.L.fj_string(text.encode()), alg))
        want = lib.spec_from_text(text, alg)
        ns, nw = packed[0], packed[1]
        assert (packed[2], packed[3]) == (want.term_entry, want.n_vars)
        assert packed[4:4 + nw] == want.code
        assert packed[4 + nw:4 + nw + ns] == want.slot_entry and packed[4 + nw + ns:] == want.slot_flags
        nm = names(shim.L.fj_string(text.encode()), alg)
        assert C.string_at(shim.L.fj_data(nm)).decode().split("\n") == want.slot_names
    assert comp(shim.L.fj_string(b"(Spec (invariants (App frob (Lit 1))))"), 1) is None
    exc = shim.exception()
    assert exc[0] == "java/lang/IllegalArgumentException" and "unknown symbol frob" in exc[1]


def test_create_without_a_device_throws(shim):
    """Without a GPU (this container) create() throws instead of returning a handle."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    create = shim.fn("create", C.c_int64, *([C.c_int32] * 3 + [C.c_int64] + [C.c_int32] * 3 + [C.c_double] +
                                            [C.c_int32] * 3 + [C.c_int64] + [C.c_int32] * 5 + [C.c_uint8, C.c_void_p]))
    h = create(1, 64, 20, 2, 64, 2, 0, 0.0, 0, 0, 0, 100, 3, 1 << 30, -1, -1, -1, 1, None)
    assert h == 0
    exc = shim.exception()
    assert exc is not None and "psg error" in exc[1]


@pytest.mark.gpu
def test_batch_through_the_shim_equals_the_python_binding(shim):
    """create / loadInputs / runBatch / copyDecisions / fetch / runBatchSpec / destroy through
    the JNI entry points, against psync.GpuRound on the same configuration."""
    n, R, count, begin, V = 64, 20, 3000, 777, 64
    create = shim.fn("create", C.c_int64, *([C.c_int32] * 3 + [C.c_int64] + [C.c_int32] * 3 + [C.c_double] +
                                            [C.c_int32] * 3 + [C.c_int64] + [C.c_int32] * 5 + [C.c_uint8, C.c_void_p]))
    for devices in (None, [0, 0]):
        dev = None if devices is None else shim.array(FJ_INT, devices)
        h = create(abi.PSG_ALG_OTR, n, R, 2, V, 2, 0, 0.0, 0, 0, 0, count, 3, 1 << 30, -1, -1, -1, 1, dev)
        assert h != 0, shim.exception()
        load = shim.fn("loadInputs", None, C.c_int64, C.c_int64, C.c_int64, C.c_void_p)
        load(h, begin, count, None)
        pi = shim.L.fj_new(FJ_BYTE, count * 24)
        run = shim.fn("runBatch", C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p)
        summ = shim.values(FJ_LONG, run(h, begin, count, pi))
        dec, drd = shim.L.fj_new(FJ_INT, count * n), shim.L.fj_new(FJ_INT, count * n)
        shim.fn("copyDecisions", None, C.c_int64, C.c_void_p, C.c_void_p)(h, dec, drd)
        ids = [begin, begin + 1234, begin + count - 1]
        fs, fr = shim.L.fj_new(FJ_BYTE, 3 * 24), shim.L.fj_new(FJ_INT, 3 * n * 4)
        shim.fn("fetch", None, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p)(h, shim.array(FJ_LONG, ids), fs, fr)
        text = F.to_text(F.otr_spec())
        packed = shim.values(FJ_INT, shim.fn("compileSpec", C.c_void_p, C.c_void_p, C.c_int32)(
            shim.L.fj_string(text.encode()), abi.PSG_ALG_OTR))
        ns, nw = packed[0], packed[1]
        rbs = shim.fn("runBatchSpec", C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                      C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p)
        ssum = shim.values(FJ_LONG, rbs(h, begin, count, shim.array(FJ_INT, packed[4:4 + nw]),
                                        shim.array(FJ_INT, packed[4 + nw:4 + nw + ns]),
                                        shim.array(FJ_INT, packed[4 + nw + ns:]), packed[2], packed[3],
                                        abi.PSG_ALG_OTR, None, None))
        # after an empty batch the last batch holds 0 instances (an empty Java array
        # is enough and nothing is written past it); a batch of 1 on a two-device list leaves
        # one device with an empty slice, whose stale size must not be copied
        run(h, begin, 0, None)
        copy = shim.fn("copyDecisions", None, C.c_int64, C.c_void_p, C.c_void_p)
        copy(h, shim.L.fj_new(FJ_INT, 0), shim.L.fj_new(FJ_INT, 0))
        assert shim.exception() is None and shim.L.fj_take_oob() == 0
        one, one_r = shim.L.fj_new(FJ_INT, n), shim.L.fj_new(FJ_INT, n)
        run(h, begin, 1, None)
        copy(h, one, one_r)
        assert shim.exception() is None and shim.L.fj_take_oob() == 0
        assert shim.values(FJ_INT, one) == shim.values(FJ_INT, dec)[:n]
        assert shim.values(FJ_INT, one_r) == shim.values(FJ_INT, drd)[:n]
        shim.fn("destroy", None, C.c_int64)(h)
        assert shim.exception() is None and shim.L.fj_take_oob() == 0
        with psync.GpuRound(psync.OTR(), n, rounds=R, seed=2, value_range=V, batch_capacity=count) as g:
            g.load_inputs(begin, count)
            r = g.run(begin, count, per_instance=True)
            d, dr = g.decisions()
            s2, rec2 = g.fetch(ids)
            sp = g.run_spec(begin, count, F.compile_spec(F.otr_spec(), abi.PSG_ALG_OTR))
        assert summ[:-1] == abi.summary_to_list(r.summary)[:-1]
        assert bytes(shim.values(FJ_BYTE, pi)) == b"".join(bytes(s) for s in r.per_instance)
        assert shim.values(FJ_INT, dec) == list(d) and shim.values(FJ_INT, drd) == list(dr)
        assert bytes(shim.values(FJ_BYTE, fs)) == b"".join(bytes(s) for s in s2)
        assert shim.values(FJ_INT, fr) == [v for x in rec2 for v in (x.decision, x.decision_round, x.halt_round,
                                                                         x.final_x)]
        assert ssum[:-1] == abi.summary_to_list(sp.summary)[:-1]


@pytest.mark.gpu
def test_native_spec_through_the_shim(shim):
    """compileSpecNative (psg_spec_compile_native) + runBatchSpec with its module: the fused
    text-lowered OTR Spec gives the built-in checker's counters (the JVM's fast route)."""
    n, R, count, V = 64, 20, 4000, 64
    create = shim.fn("create", C.c_int64, *([C.c_int32] * 3 + [C.c_int64] + [C.c_int32] * 3 + [C.c_double] +
                                            [C.c_int32] * 3 + [C.c_int64] + [C.c_int32] * 5 + [C.c_uint8, C.c_void_p]))
    h = create(abi.PSG_ALG_OTR, n, R, 2, V, 2, 0, 0.0, 0, 0, 0, count, 3, 1 << 30, -1, -1, -1, 1, None)
    assert h != 0, shim.exception()
    text = shim.L.fj_string(F.to_text(F.otr_spec()).encode())
    packed = shim.values(FJ_INT, shim.fn("compileSpec", C.c_void_p, C.c_void_p, C.c_int32)(text, abi.PSG_ALG_OTR))
    path = shim.fn("compileSpecNative", C.c_void_p, C.c_void_p, C.c_int32, C.c_uint8, C.c_int32)(
        text, abi.PSG_ALG_OTR, 1, n)
    assert path and shim.exception() is None
    ns, nw = packed[0], packed[1]
    rbs = shim.fn("runBatchSpec", C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                  C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p)
    ssum = shim.values(FJ_LONG, rbs(h, 0, count, shim.array(FJ_INT, packed[4:4 + nw]),
                                    shim.array(FJ_INT, packed[4 + nw:4 + nw + ns]),
                                    shim.array(FJ_INT, packed[4 + nw + ns:]), packed[2], packed[3],
                                    abi.PSG_ALG_OTR, path, None))
    summ = shim.values(FJ_LONG, shim.fn("runBatch", C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p)(
        h, 0, count, None))
    shim.fn("destroy", None, C.c_int64)(h)
    assert shim.exception() is None and shim.L.fj_take_oob() == 0
    assert ssum[:-1] == summ[:-1]
