"""ctypes mirror of include/psg.h (struct layouts and constants only).

Shared by the product binding (round_amd.lib) and by the test-side oracle
binding (oracle/oracle.py): both libraries speak the same C structs.
"""
import ctypes as C

PSG_ABI_VERSION = 4

PSG_ALG_OTR = 1
PSG_ALG_LAST_VOTING = 2
PSG_ALG_FLOODMIN = 3
PSG_ALG_KSET = 4
PSG_ALG_BENOR = 5
PSG_ALG_OTR2 = 6
PSG_ALG_SLV = 7
PSG_ALG_KSET_ES = 8
PSG_ALG_EPSILON = 9

PSG_TIE_CHAMP = 0
PSG_TIE_MIN_PID = 1

PSG_OK = 0
PSG_EINVAL = -22
PSG_ENOMEM = -12
PSG_ENODEV = -19
PSG_EIO = -5
PSG_ERANGE = -34

PSG_MAX_N = 256
PSG_MAX_ROUNDS = 250
PSG_MAX_CHECKS = 12
PSG_NEVER = 0xFF
PSG_MAX_DEVICES = 16

# Reference class name -> alg id ("Algorithm ids are keyed on the
# reference class name").
CLASS_TO_ALG = {
    "example.OTR": PSG_ALG_OTR,
    "example.LastVoting": PSG_ALG_LAST_VOTING,
    "example.FloodMin": PSG_ALG_FLOODMIN,
    "example.KSetAgreement": PSG_ALG_KSET,
    "example.BenOr": PSG_ALG_BENOR,
    "example.OTR2": PSG_ALG_OTR2,
    "example.ShortLastVoting": PSG_ALG_SLV,
    "example.KSetEarlyStopping": PSG_ALG_KSET_ES,
    "example.EpsilonConsensus": PSG_ALG_EPSILON,
}

# Check-slot names per algorithm (psg_check_name). Slot 0 of OTR/LV/BenOr is
# "Safety": at least one invariant holds (psync/verification/Verifier.scala:234-275).
CHECK_NAMES = {
    PSG_ALG_OTR: ["Safety", "Invariant0", "Invariant1", "Invariant2",
                  "Agreement", "Validity", "Integrity", "Irrevocability"],
    PSG_ALG_LAST_VOTING: ["Safety", "Invariant0", "Invariant1",
                          "Agreement", "Validity", "Integrity", "Irrevocability"],
    PSG_ALG_BENOR: ["Safety", "Invariant0", "Agreement", "Irrevocability", "SafetyPredicate"],
    PSG_ALG_FLOODMIN: ["KAgreement", "KValidity"],
    PSG_ALG_KSET: ["KAgreement", "KValidity"],
    PSG_ALG_OTR2: ["Safety", "Invariant0", "Invariant1", "Invariant2",
                   "Agreement", "Validity", "Integrity", "Irrevocability"],
    PSG_ALG_SLV: ["KAgreement", "KValidity"],
    PSG_ALG_KSET_ES: ["KAgreement", "KValidity"],
    PSG_ALG_EPSILON: ["EpsAgreement", "EpsValidity", "SafetyPredicate"],
}
# Slots whose falsity is a violation (invariant slots are informational: an
# individual invariant of a sequence legitimately fails before/after its phase;
# "SafetyPredicate" records when the environment left the Spec's assumption,
# psync/Specs.scala:9, evaluated on the effective heard-of sets).
VIOLATION_SLOTS = {
    PSG_ALG_OTR: [0, 4, 5, 6, 7],
    PSG_ALG_LAST_VOTING: [0, 3, 4, 5, 6],
    PSG_ALG_BENOR: [0, 2, 3],
    PSG_ALG_FLOODMIN: [0, 1],
    PSG_ALG_KSET: [0, 1],
    PSG_ALG_OTR2: [0, 4, 5, 6, 7],
    PSG_ALG_SLV: [0, 1],
    PSG_ALG_KSET_ES: [0, 1],
    PSG_ALG_EPSILON: [0, 1],
}


class Schedule(C.Structure):
    _fields_ = [
        ("drop_log2", C.c_uint32),
        ("good_p32", C.c_uint32),
        ("good_min", C.c_int32),
        ("crash_fmax", C.c_int32),
        ("ho_min", C.c_int32),
        ("self_bit", C.c_uint32),
    ]


class Config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("alg", C.c_int32),
        ("n", C.c_int32),
        ("rounds", C.c_int32),
        ("seed", C.c_uint64),
        ("value_range", C.c_int32),
        ("param", C.c_int32),
        ("tiebreak", C.c_int32),
        ("device", C.c_int32),
        ("variant", C.c_int32),
        ("batch_capacity", C.c_uint64),
        ("sched", Schedule),
        ("param2", C.c_int32),
        ("reserved", C.c_int32),
        ("real_param", C.c_double),
        ("n_devices", C.c_int32),
        ("devices", C.c_int32 * PSG_MAX_DEVICES),
    ]


class Summary(C.Structure):
    _fields_ = [
        ("instances", C.c_int64),
        ("process_rounds", C.c_int64),
        ("active_process_rounds", C.c_int64),
        ("live_instance_rounds", C.c_int64),
        ("fail_count", C.c_int64 * PSG_MAX_CHECKS),
        ("decided_processes", C.c_int64),
        ("digest", C.c_int64),
        ("term_hist", C.c_int64 * (PSG_MAX_ROUNDS + 2)),
        ("kernel_ns", C.c_int64),
    ]


class InstanceSummary(C.Structure):
    _fields_ = [
        ("digest", C.c_uint64),
        ("first_fail", C.c_uint8 * PSG_MAX_CHECKS),
        ("term_round", C.c_uint8),
        ("n_checks", C.c_uint8),
        ("n_decided", C.c_uint16),
    ]


class ProcessRecord(C.Structure):
    _fields_ = [
        ("decision", C.c_int32),
        ("decision_round", C.c_int32),
        ("halt_round", C.c_int32),
        ("final_x", C.c_int32),
    ]


assert C.sizeof(InstanceSummary) == 24
assert C.sizeof(ProcessRecord) == 16

# Fields of Summary that are summed across ranks (everything but kernel_ns).
SUMMARY_SUM_FIELDS = 4 + PSG_MAX_CHECKS + 2 + (PSG_MAX_ROUNDS + 2)


def summary_to_list(s):
    """Summary -> flat list of int64 in struct order (kernel_ns last)."""
    out = [s.instances, s.process_rounds, s.active_process_rounds, s.live_instance_rounds]
    out += list(s.fail_count)
    out += [s.decided_processes, s.digest]
    out += list(s.term_hist)
    out.append(s.kernel_ns)
    return out


def summary_from_list(vals):
    s = Summary()
    it = iter(vals)
    s.instances = next(it)
    s.process_rounds = next(it)
    s.active_process_rounds = next(it)
    s.live_instance_rounds = next(it)
    for i in range(PSG_MAX_CHECKS):
        s.fail_count[i] = next(it)
    s.decided_processes = next(it)
    d = next(it)
    s.digest = ((d + (1 << 63)) % (1 << 64)) - (1 << 63)
    for i in range(PSG_MAX_ROUNDS + 2):
        s.term_hist[i] = next(it)
    s.kernel_ns = next(it)
    return s


def summary_dict(s, alg, rounds):
    """Readable view of a Summary."""
    names = CHECK_NAMES[alg]
    return {
        "instances": s.instances,
        "process_rounds": s.process_rounds,
        "active_process_rounds": s.active_process_rounds,
        "live_instance_rounds": s.live_instance_rounds,
        "fail_count": {names[i]: s.fail_count[i] for i in range(len(names))},
        "decided_processes": s.decided_processes,
        "digest": s.digest & ((1 << 64) - 1),
        "term_hist": [s.term_hist[i] for i in range(rounds + 2)],
        "kernel_ns": s.kernel_ns,
    }


class SpecProgram(C.Structure):
    """psg_spec_program (include/psg.h): a compiled Spec (round_amd/formula.py)."""
    _fields_ = [
        ("n_slots", C.c_int32),
        ("n_words", C.c_int32),
        ("code", C.POINTER(C.c_int32)),
        ("slot_entry", C.POINTER(C.c_int32)),
        ("slot_flags", C.POINTER(C.c_int32)),
        ("term_entry", C.c_int32),
        ("n_vars", C.c_int32),
        ("module_path", C.c_char_p),
        ("alg", C.c_int32),
    ]


class PopulationParams(C.Structure):
    """psg_population_params (include/psg.h): device-side search populations."""
    _fields_ = [
        ("seed", C.c_uint64),
        ("generation", C.c_uint32),
        ("flips", C.c_uint32),
        ("min_size", C.c_int32),
        ("self_bit", C.c_uint32),
        ("keep_p256", C.c_uint32 * 4),
        ("value_range", C.c_int32),
        ("redraw_p256", C.c_uint32),
    ]
