"""On-disk result records (".psgr", include/psg_records.h): writer and reader.

A record file holds, for `count` instances, any of: global ids, per-instance
summaries (psg_instance_summary), initial values, the explicit HO schedule and
crash rounds that replay them (psg_load_schedule layout), per-process records
and a JSON provenance blob. The adversary search (round_amd/adversary.py)
writes its counterexamples in this format; `replay()` re-executes a file's
instances on the GPU and compares the outcome with what the file recorded.

Reference counterpart: none — the reference reports results through
`ConsensusIO.decide` callbacks (e.g. example/Otr.scala:68-70) and logs
(psync/runtime/InstanceHandler.scala:248-257).
"""
import ctypes as C
import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import abi

MAGIC = b"PSGREC\r\n"
VERSION = 2  # 2: psg_config of ABI 4 (device list)
ALIGN = 64
MAX_SECTIONS = 16
NAME_BYTES = 24

IDS, SUMMARY, INIT_I32, INIT_F64, HO, CRASH, PROCESS, DECISION_F64, META = range(1, 10)
_KIND_NAMES = {IDS: "ids", SUMMARY: "summary", INIT_I32: "init", INIT_F64: "init", HO: "ho", CRASH: "crash",
               PROCESS: "process", DECISION_F64: "decision_f64", META: "meta"}

# numpy views of the psg.h structs
SUMMARY_DTYPE = np.dtype([("digest", "<u8"), ("first_fail", "u1", (abi.PSG_MAX_CHECKS,)), ("term_round", "u1"),
                          ("n_checks", "u1"), ("n_decided", "<u2")])
PROCESS_DTYPE = np.dtype([("decision", "<i4"), ("decision_round", "<i4"), ("halt_round", "<i4"),
                          ("final_x", "<i4")])
assert SUMMARY_DTYPE.itemsize == C.sizeof(abi.InstanceSummary) == 24
assert PROCESS_DTYPE.itemsize == C.sizeof(abi.ProcessRecord) == 16


class Section(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("elem_bytes", C.c_uint32), ("offset", C.c_uint64), ("nbytes", C.c_uint64)]


class Header(C.Structure):
    _fields_ = [
        ("magic", C.c_char * 8),
        ("version", C.c_uint32),
        ("header_bytes", C.c_uint32),
        ("cfg", abi.Config),
        ("count", C.c_uint64),
        ("n_sections", C.c_uint32),
        ("n_slots", C.c_uint32),
        ("slot_names", (C.c_char * NAME_BYTES) * abi.PSG_MAX_CHECKS),
        ("class_name", C.c_char * 64),
        ("sections", Section * MAX_SECTIONS),
    ]


@dataclass
class Records:
    """Contents of a .psgr file (arrays are None when the section is absent)."""
    cfg: abi.Config
    slot_names: List[str]
    ids: np.ndarray
    summary: Optional[np.ndarray] = None   # SUMMARY_DTYPE [count]
    init: Optional[np.ndarray] = None      # int32 or float64 [count][n]
    ho: Optional[np.ndarray] = None        # uint64 [count][R][n][W]
    crash: Optional[np.ndarray] = None     # int32 [count][n]
    process: Optional[np.ndarray] = None   # PROCESS_DTYPE [count][n]
    decision_f64: Optional[np.ndarray] = None
    meta: Dict = field(default_factory=dict)
    class_name: str = ""

    @property
    def count(self):
        return int(self.ids.shape[0])

    @property
    def n(self):
        return int(self.cfg.n)

    @property
    def rounds(self):
        return int(self.cfg.rounds)

    @property
    def W(self):
        return (self.n + 63) // 64


def _align(x):
    return (x + ALIGN - 1) // ALIGN * ALIGN


def write(path, rec: Records):
    """Write `rec` to `path` (include/psg_records.h layout)."""
    count, n, R, W = rec.count, rec.n, rec.rounds, rec.W
    payloads = [(IDS, 8, np.ascontiguousarray(rec.ids, "<u8").reshape(count))]
    if rec.summary is not None:
        payloads.append((SUMMARY, 24, np.ascontiguousarray(rec.summary, SUMMARY_DTYPE).reshape(count)))
    if rec.init is not None:
        real = np.asarray(rec.init).dtype.kind == "f"
        payloads.append((INIT_F64 if real else INIT_I32, 8 if real else 4,
                         np.ascontiguousarray(rec.init, "<f8" if real else "<i4").reshape(count, n)))
    if rec.ho is not None:
        payloads.append((HO, 8, np.ascontiguousarray(rec.ho, "<u8").reshape(count, R, n, W)))
    if rec.crash is not None:
        payloads.append((CRASH, 4, np.ascontiguousarray(rec.crash, "<i4").reshape(count, n)))
    if rec.process is not None:
        payloads.append((PROCESS, 16, np.ascontiguousarray(rec.process, PROCESS_DTYPE).reshape(count, n)))
    if rec.decision_f64 is not None:
        payloads.append((DECISION_F64, 8, np.ascontiguousarray(rec.decision_f64, "<f8").reshape(count, n)))
    meta = json.dumps(rec.meta or {}, sort_keys=True).encode()
    payloads.append((META, 1, np.frombuffer(meta, np.uint8)))
    if len(payloads) > MAX_SECTIONS:
        raise ValueError("too many sections")
    h = Header()
    h.magic = MAGIC
    h.version = VERSION
    h.header_bytes = C.sizeof(Header)
    h.cfg = rec.cfg
    h.count = count
    h.n_sections = len(payloads)
    if len(rec.slot_names) > abi.PSG_MAX_CHECKS:
        raise ValueError("more than PSG_MAX_CHECKS slots")
    h.n_slots = len(rec.slot_names)
    for i, s in enumerate(rec.slot_names):
        h.slot_names[i].value = s.encode()[:NAME_BYTES - 1]
    h.class_name = rec.class_name.encode()[:63]
    off = _align(C.sizeof(Header))
    for i, (kind, eb, arr) in enumerate(payloads):
        h.sections[i].kind, h.sections[i].elem_bytes = kind, eb
        h.sections[i].offset, h.sections[i].nbytes = off, arr.nbytes
        off = _align(off + arr.nbytes)
    with open(path, "wb") as f:
        f.write(bytes(h))
        for i, (_, _, arr) in enumerate(payloads):
            f.seek(h.sections[i].offset)
            f.write(arr.tobytes())
        f.truncate(off)


def read(path, mmap=True) -> Records:
    """Read a .psgr file; array sections are memory-mapped (read-only) when mmap=True."""
    with open(path, "rb") as f:
        raw = f.read(C.sizeof(Header))
    if len(raw) < C.sizeof(Header):
        raise ValueError(f"{path}: truncated header")
    h = Header.from_buffer_copy(raw)
    if raw[:8] != MAGIC:
        raise ValueError(f"{path}: not a .psgr file")
    if h.version != VERSION or h.header_bytes != C.sizeof(Header):
        raise ValueError(f"{path}: unsupported version {h.version} / header {h.header_bytes} bytes")
    if h.n_sections > MAX_SECTIONS or h.n_slots > abi.PSG_MAX_CHECKS:
        raise ValueError(f"{path}: corrupt header")
    cfg = abi.Config()
    C.memmove(C.byref(cfg), C.byref(h.cfg), C.sizeof(abi.Config))
    count, n, R = int(h.count), int(cfg.n), int(cfg.rounds)
    W = (n + 63) // 64
    shapes = {IDS: ("<u8", (count,)), SUMMARY: (SUMMARY_DTYPE, (count,)), INIT_I32: ("<i4", (count, n)),
              INIT_F64: ("<f8", (count, n)), HO: ("<u8", (count, R, n, W)), CRASH: ("<i4", (count, n)),
              PROCESS: (PROCESS_DTYPE, (count, n)), DECISION_F64: ("<f8", (count, n))}
    out = {}
    meta = {}
    for i in range(h.n_sections):
        s = h.sections[i]
        if s.kind == META:
            with open(path, "rb") as f:
                f.seek(s.offset)
                meta = json.loads(f.read(s.nbytes).decode() or "{}")
            continue
        if s.kind not in shapes:
            continue  # unknown section kinds are skipped (forward compatibility)
        dt, shape = shapes[s.kind]
        dt = np.dtype(dt)
        if int(np.prod(shape)) * dt.itemsize != s.nbytes:
            raise ValueError(f"{path}: section {s.kind} has {s.nbytes} bytes, expected shape {shape}")
        if mmap and s.nbytes:
            arr = np.memmap(path, dtype=dt, mode="r", offset=s.offset, shape=shape)
        else:
            with open(path, "rb") as f:
                f.seek(s.offset)
                arr = np.frombuffer(f.read(s.nbytes), dtype=dt).reshape(shape)
        out[_KIND_NAMES[s.kind]] = arr
    if "ids" not in out:
        raise ValueError(f"{path}: no IDS section")
    names = [h.slot_names[i].value.decode() for i in range(h.n_slots)]
    return Records(cfg=cfg, slot_names=names, meta=meta, class_name=h.class_name.decode(), **out)


def replay(path_or_records, device=0, compare=True):
    """Re-execute the instances of a record file on the GPU with their recorded
    inputs and schedule (seeded when the file holds none) and return the fresh
    per-instance summaries (SUMMARY_DTYPE). With compare=True, raise if any
    recorded summary differs (digest, first failing check points, termination)."""
    from . import lib
    rec = read(path_or_records) if isinstance(path_or_records, str) else path_or_records
    cfg = abi.Config()
    C.memmove(C.byref(cfg), C.byref(rec.cfg), C.sizeof(abi.Config))
    cfg.device = device
    cfg.n_devices = 0  # replay on the one given device, whatever the recording context drove
    ids = np.asarray(rec.ids, np.uint64)
    # contiguous id ranges replay as batches; the file's rows are in id order per range
    out = np.zeros(rec.count, SUMMARY_DTYPE)
    starts = [0] + [i for i in range(1, rec.count) if ids[i] != ids[i - 1] + 1] + [rec.count]
    cfg.batch_capacity = max(1, max(b - a for a, b in zip(starts, starts[1:])) if rec.count else 1)
    ctx = lib.Context(cfg)
    try:
        for a, b in zip(starts, starts[1:]):
            if b <= a:
                continue
            begin = int(ids[a])
            if rec.init is not None:
                ctx.load_inputs(begin, b - a, np.asarray(rec.init[a:b]))
            if rec.ho is not None:
                ctx.load_schedule(begin, b - a, np.asarray(rec.ho[a:b]),
                                  None if rec.crash is None else np.asarray(rec.crash[a:b]))
            else:
                ctx.clear_schedule()
            _, pi = ctx.run_batch_np(begin, b - a)
            out[a:b] = pi
    finally:
        ctx.close()
    if compare and rec.summary is not None:
        want = np.asarray(rec.summary)
        k = len(rec.slot_names)
        bad = np.nonzero((want["digest"] != out["digest"]) | (want["term_round"] != out["term_round"]) |
                         (want["first_fail"][:, :k] != out["first_fail"][:, :k]).any(1))[0]
        if len(bad):
            raise AssertionError(f"replay differs from the record for {len(bad)} instance(s), first id "
                                 f"{int(ids[bad[0]])}")
    return out
