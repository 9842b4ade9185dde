"""The C-ABI library: loads without a GPU, exports every symbol include/psg.h
declares, and its struct layouts match the ctypes mirror (checked by compiling a
C probe against the header). No compute calls here (no GPU in CI)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from round_amd import abi, lib, psync

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "psg.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(psg_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = lib.load()
    names = header_functions()
    assert set(names) == set(lib.EXPORTED_SYMBOLS)
    out = subprocess.check_output(["nm", "-D", "--defined-only", lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert hasattr(L, n)


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "psg.h"
#define P(T, F) printf(#T "." #F " %zu\n", offsetof(T, F));
int main(void) {
  printf("psg_schedule %zu\n", sizeof(psg_schedule));
  printf("psg_config %zu\n", sizeof(psg_config));
  printf("psg_summary %zu\n", sizeof(psg_summary));
  printf("psg_instance_summary %zu\n", sizeof(psg_instance_summary));
  printf("psg_process_record %zu\n", sizeof(psg_process_record));
  P(psg_config, seed) P(psg_config, value_range) P(psg_config, batch_capacity) P(psg_config, sched)
  P(psg_config, param2) P(psg_config, real_param)
  P(psg_summary, fail_count) P(psg_summary, decided_processes) P(psg_summary, term_hist) P(psg_summary, kernel_ns)
  P(psg_instance_summary, first_fail) P(psg_instance_summary, term_round) P(psg_instance_summary, n_decided)
  P(psg_schedule, crash_fmax) P(psg_schedule, self_bit)
  printf("psg_population_params %zu\n", sizeof(psg_population_params));
  P(psg_population_params, flips) P(psg_population_params, keep_p256) P(psg_population_params, redraw_p256)
  return 0;
}
"""


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)], text=True).splitlines())
    want = {
        "psg_schedule": C.sizeof(abi.Schedule),
        "psg_config": C.sizeof(abi.Config),
        "psg_summary": C.sizeof(abi.Summary),
        "psg_instance_summary": C.sizeof(abi.InstanceSummary),
        "psg_process_record": C.sizeof(abi.ProcessRecord),
        "psg_config.seed": abi.Config.seed.offset,
        "psg_config.value_range": abi.Config.value_range.offset,
        "psg_config.batch_capacity": abi.Config.batch_capacity.offset,
        "psg_config.sched": abi.Config.sched.offset,
        "psg_config.param2": abi.Config.param2.offset,
        "psg_config.real_param": abi.Config.real_param.offset,
        "psg_summary.fail_count": abi.Summary.fail_count.offset,
        "psg_summary.decided_processes": abi.Summary.decided_processes.offset,
        "psg_summary.term_hist": abi.Summary.term_hist.offset,
        "psg_summary.kernel_ns": abi.Summary.kernel_ns.offset,
        "psg_instance_summary.first_fail": abi.InstanceSummary.first_fail.offset,
        "psg_instance_summary.term_round": abi.InstanceSummary.term_round.offset,
        "psg_instance_summary.n_decided": abi.InstanceSummary.n_decided.offset,
        "psg_schedule.crash_fmax": abi.Schedule.crash_fmax.offset,
        "psg_schedule.self_bit": abi.Schedule.self_bit.offset,
        "psg_population_params": C.sizeof(abi.PopulationParams),
        "psg_population_params.flips": abi.PopulationParams.flips.offset,
        "psg_population_params.keep_p256": abi.PopulationParams.keep_p256.offset,
        "psg_population_params.redraw_p256": abi.PopulationParams.redraw_p256.offset,
    }
    assert {k: int(v) for k, v in got.items()} == want


def test_header_constants_match_mirror():
    txt = open(HEADER).read()
    for name in ["PSG_ALG_OTR", "PSG_ALG_LAST_VOTING", "PSG_ALG_FLOODMIN", "PSG_ALG_KSET", "PSG_ALG_BENOR"]:
        m = re.search(name + r"\s*=\s*(\d+)", txt)
        assert int(m.group(1)) == getattr(abi, name)
    for name in ["PSG_MAX_N", "PSG_MAX_ROUNDS", "PSG_MAX_CHECKS", "PSG_EINVAL", "PSG_ENODEV", "PSG_ERANGE"]:
        m = re.search(r"#define " + name + r"\s+\(?(-?\d+)", txt)
        assert int(m.group(1)) == getattr(abi, name), name


def test_check_names_and_class_mapping():
    L = lib.load()
    for alg, names in abi.CHECK_NAMES.items():
        assert lib.check_names(alg) == names
        assert L.psg_check_name(alg, len(names)) is None
    for cls, alg in abi.CLASS_TO_ALG.items():
        assert L.psg_alg_from_class(cls.encode()) == alg
        assert psync.ALGORITHMS[cls].alg_id == alg
    assert L.psg_alg_from_class(b"example.Nope") == abi.PSG_EINVAL


def test_config_default_matches_host_mirror():
    L = lib.load()
    for cls, A in psync.ALGORITHMS.items():
        alg = A()
        n = 64
        c = abi.Config()
        assert L.psg_config_default(C.byref(c), alg.alg_id, n) == 0
        h = psync.make_config(alg, n)
        for f in ["abi_version", "alg", "n", "rounds", "value_range", "param", "tiebreak"]:
            assert getattr(c, f) == getattr(h, f), (cls, f)
        for f in ["drop_log2", "good_p32", "good_min", "crash_fmax", "ho_min", "self_bit"]:
            assert getattr(c.sched, f) == getattr(h.sched, f), (cls, f)


@pytest.mark.parametrize("field,value", [("n", 0), ("n", 257), ("rounds", 0), ("rounds", 251),
                                          ("alg", 9), ("abi_version", 7), ("tiebreak", 5)])
def test_create_rejects_invalid_config(field, value):
    L = lib.load()
    cfg = psync.make_config(psync.OTR(), 8)
    setattr(cfg, field, value)
    h = C.c_void_p()
    assert L.psg_create(C.byref(h), C.byref(cfg)) == abi.PSG_EINVAL
    assert h.value is None
    assert L.psg_create_error()


def test_create_without_device_fails_loudly():
    """No CPU fallback: without a HIP device psg_create reports ENODEV (on a GPU box it succeeds)."""
    L = lib.load()
    cfg = psync.make_config(psync.OTR(), 8, batch_capacity=16)
    h = C.c_void_p()
    rc = L.psg_create(C.byref(h), C.byref(cfg))
    if rc == 0:
        L.psg_destroy(h)
    else:
        assert rc == abi.PSG_ENODEV
        with pytest.raises(lib.PsgError):
            psync.GpuRound(psync.OTR(), 8)


def test_null_arguments():
    L = lib.load()
    assert L.psg_create(None, None) == abi.PSG_EINVAL
    assert L.psg_run_batch(None, 0, 1, None, None) == abi.PSG_EINVAL
    assert L.psg_fetch_instances(None, None, 0, None, None) == abi.PSG_EINVAL
    L.psg_destroy(None)
