"""Host-side mirror of the reference's plugin interface for the HO round path.

The reference user writes `class OTR(rt, timeout, afterDecision) extends
Algorithm[ConsensusIO[Int], OtrProcess]` (example/Otr.scala:89) and runs it by
`alg.startInstance(id, io)` (psync/Algorithm.scala:36-42) over the netty
runtime chosen by `Runtime.apply` (psync/runtime/Runtime.scala:167-177). Here
the same algorithm classes (same names, same constructor parameters) are
descriptors handed to `GpuRound`, which executes millions of instances in
lockstep on an MI355X through the C ABI of include/psg.h.

Error behaviour mirrors the reference: misuse raises (the reference's
`Logger.logAndThrow`, psync/runtime/InstanceHandler.scala:346, 351; JVM
`assert`s, e.g. InstanceHandler.scala:116), nothing is silently ignored, and a
missing HIP library is a hard error (no CPU fallback).
"""
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

from . import abi


@dataclass
class HOSchedule:
    """Seeded adversarial HO schedule (faults are HO sets, psync/Process.scala:14).

    drop_log2   0 = no benign loss; k > 0: each non-self link lost w.p. 2**-k.
    good_round  probability that a round is "good" (every HO(p) = one common s,
                |s| > good_min; OTR's livenessPredicate, example/Otr.scala:96).
    crash_fmax  None = no crashes; else f ~ U{0..crash_fmax} processes crash
                (permanent send omission from a uniform crash round).
    ho_min      None; else |HO(p)| <= ho_min is raised to all processes
                (BenOr safetyPredicate |HO(p)| > n/2, example/BenOr.scala:92).
    self_bit    the runtime always delivers a process's message to itself
                (psync/Round.scala:114-116); False = pure HO.
    """
    drop_log2: int = 3
    good_round: float = 0.25
    good_min: Optional[int] = None
    crash_fmax: Optional[int] = None
    ho_min: Optional[int] = None
    self_bit: bool = True

    def to_c(self):
        s = abi.Schedule()
        s.drop_log2 = int(self.drop_log2)
        s.good_p32 = min(int(round(self.good_round * 2 ** 32)), 2 ** 32 - 1)
        s.good_min = -1 if self.good_min is None else int(self.good_min)
        s.crash_fmax = -1 if self.crash_fmax is None else int(self.crash_fmax)
        s.ho_min = -1 if self.ho_min is None else int(self.ho_min)
        s.self_bit = 1 if self.self_bit else 0
        return s


class Algorithm:
    """Descriptor of a reference algorithm class (psync/Algorithm.scala:13-31)."""
    class_name = ""
    alg_id = 0
    phase_length = 1  # rounds.length (psync/Process.scala:28)
    real = False  # Double-valued (RealConsensusIO) algorithm
    epsilon = 0.0

    def __init__(self, param=0, variant=0, param2=0):
        self.param = int(param)
        self.param2 = int(param2)
        self.variant = int(variant)

    def default_schedule(self, n):
        return HOSchedule()

    def default_rounds(self, n):
        return 20

    def default_value_range(self, n):
        return 4

    @property
    def check_names(self) -> List[str]:
        return abi.CHECK_NAMES[self.alg_id]

    @property
    def violation_slots(self) -> List[int]:
        return abi.VIOLATION_SLOTS[self.alg_id]


class OTR(Algorithm):
    """example.OTR(rt, timeout, afterDecision = 2) — example/Otr.scala:89."""
    class_name = "example.OTR"
    alg_id = abi.PSG_ALG_OTR

    def __init__(self, afterDecision=2, variant=0):
        super().__init__(afterDecision, variant)


class LastVoting(Algorithm):
    """example.LastVoting(rt, timeout, progress = Quorum) — example/LastVoting.scala:11."""
    class_name = "example.LastVoting"
    alg_id = abi.PSG_ALG_LAST_VOTING
    phase_length = 4

    def default_schedule(self, n):
        return HOSchedule(drop_log2=4, good_round=0.0, crash_fmax=(n - 1) // 2)

    def default_value_range(self, n):
        return 2 ** 15 - 1  # values must be nonzero (asserts at LastVoting.scala:134, 156, 198)


class FloodMin(Algorithm):
    """example.FloodMin(rt, f, timeout) — example/FloodMin.scala:38."""
    class_name = "example.FloodMin"
    alg_id = abi.PSG_ALG_FLOODMIN

    def __init__(self, f=2, variant=0):
        super().__init__(f, variant)

    def default_schedule(self, n):
        return HOSchedule(drop_log2=0, good_round=0.0, crash_fmax=self.param)

    def default_rounds(self, n):
        return self.param + 2  # decides in round f+1 (first r > f)

    def default_value_range(self, n):
        return 1_000_000


class KSetAgreement(Algorithm):
    """example.KSetAgreement(rt, k, timeout) — example/KSetAgreement.scala:70-87."""
    class_name = "example.KSetAgreement"
    alg_id = abi.PSG_ALG_KSET

    def __init__(self, k=2, variant=0):
        super().__init__(k, variant)

    def default_schedule(self, n):
        return HOSchedule(drop_log2=0, good_round=0.0, crash_fmax=self.param - 1)  # f < k

    def default_rounds(self, n):
        return 16

    def default_value_range(self, n):
        return 1_000_000


class BenOr(Algorithm):
    """example.BenOr(rt, timeout) — example/BenOr.scala:86-124."""
    class_name = "example.BenOr"
    alg_id = abi.PSG_ALG_BENOR
    phase_length = 2

    def default_schedule(self, n):
        return HOSchedule(drop_log2=2, good_round=0.0, ho_min=n // 2)

    def default_rounds(self, n):
        return 64

    def default_value_range(self, n):
        return 2


class OTR2(Algorithm):
    """example.OTR2(rt, timeout, afterDecision = 2) — example/Otr2.scala:69 (decision: Option[Int])."""
    class_name = "example.OTR2"
    alg_id = abi.PSG_ALG_OTR2

    def __init__(self, afterDecision=2, variant=0):
        super().__init__(afterDecision, variant)


class ShortLastVoting(Algorithm):
    """example.ShortLastVoting(rt, timeout) — example/ShortLastVoting.scala:108 (3-round phase)."""
    class_name = "example.ShortLastVoting"
    alg_id = abi.PSG_ALG_SLV
    phase_length = 3

    def default_schedule(self, n):
        return HOSchedule(drop_log2=4, good_round=0.0, crash_fmax=(n - 1) // 2)

    def default_rounds(self, n):
        return 30

    def default_value_range(self, n):
        return 2 ** 15 - 1


class KSetEarlyStopping(Algorithm):
    """example.KSetEarlyStopping(rt, t, k, timeout) — example/KSetEarlyStopping.scala:47
    (runner defaults t = 2, k = 2, KSetEarlyStopping.scala:63-67)."""
    class_name = "example.KSetEarlyStopping"
    alg_id = abi.PSG_ALG_KSET_ES

    def __init__(self, t=2, k=2, variant=0):
        super().__init__(t, variant, param2=k)

    def default_schedule(self, n):
        return HOSchedule(drop_log2=0, good_round=0.0, crash_fmax=self.param)  # at most t crashes

    def default_rounds(self, n):
        return self.param // self.param2 + 2  # everyone decides once r > t/k

    def default_value_range(self, n):
        return 1_000_000


class EpsilonConsensus(Algorithm):
    """example.EpsilonConsensus(rt, f, epsilon, timeout) — example/Epsilon.scala:72 (Double
    values; runner defaults f = 1, epsilon = 0.1, 7 replicas, Epsilon.scala:83-89)."""
    class_name = "example.EpsilonConsensus"
    alg_id = abi.PSG_ALG_EPSILON
    real = True

    def __init__(self, f=1, epsilon=0.1, variant=0):
        super().__init__(f, variant)
        self.epsilon = float(epsilon)

    def default_schedule(self, n):
        # |mailbox| >= n - f (the commented assert, Epsilon.scala:57): HO(p) := all below that
        return HOSchedule(drop_log2=4, good_round=0.0, ho_min=n - self.param - 1)

    def default_rounds(self, n):
        return 12


ALGORITHMS = {c.class_name: c for c in (OTR, LastVoting, FloodMin, KSetAgreement, BenOr,
                                          OTR2, ShortLastVoting, KSetEarlyStopping, EpsilonConsensus)}


def make_config(alg: Algorithm, n: int, rounds: Optional[int] = None, seed: int = 1,
                schedule: Optional[HOSchedule] = None, value_range: Optional[int] = None,
                tiebreak: int = abi.PSG_TIE_CHAMP, device: int = 0,
                batch_capacity: int = 1 << 20, devices: Optional[Sequence[int]] = None) -> abi.Config:
    """Build a psg_config (the reference's `new OTR(rt, ...)` + RTOptions). `devices`:
    run every batch split over these HIP devices (one host thread each) instead of `device`."""
    if not (1 <= n <= abi.PSG_MAX_N):
        raise ValueError(f"n={n} out of range 1..{abi.PSG_MAX_N}")
    c = abi.Config()
    c.abi_version = abi.PSG_ABI_VERSION
    c.alg = alg.alg_id
    c.n = n
    c.rounds = alg.default_rounds(n) if rounds is None else rounds
    if not (1 <= c.rounds <= abi.PSG_MAX_ROUNDS):
        raise ValueError(f"rounds={c.rounds} out of range")
    c.seed = seed & ((1 << 64) - 1)
    c.value_range = alg.default_value_range(n) if value_range is None else value_range
    c.param = alg.param
    c.param2 = alg.param2
    c.real_param = alg.epsilon
    c.tiebreak = tiebreak
    c.device = device
    c.variant = alg.variant
    c.batch_capacity = batch_capacity
    c.sched = (schedule or alg.default_schedule(n)).to_c()
    if devices:
        if len(devices) > abi.PSG_MAX_DEVICES:
            raise ValueError(f"at most {abi.PSG_MAX_DEVICES} devices per context")
        c.n_devices = len(devices)
        for i, d in enumerate(devices):
            c.devices[i] = int(d)
    return c


@dataclass
class BatchResult:
    """Result of one batch (psg_summary + optional per-instance summaries)."""
    alg: Algorithm
    rounds: int
    summary: abi.Summary
    per_instance: Optional[list] = None

    def as_dict(self):
        return abi.summary_dict(self.summary, self.alg.alg_id, self.rounds)

    def violations(self):
        names = self.alg.check_names
        return {names[i]: self.summary.fail_count[i] for i in self.alg.violation_slots}


class SpecResult:
    """Result of a batch checked against a user Spec: counts per compiled slot."""

    def __init__(self, slot_names, rounds, summary, per_instance=None):
        self.slot_names, self.rounds, self.summary, self.per_instance = slot_names, rounds, summary, per_instance

    def fail_count(self):
        return {name: self.summary.fail_count[i] for i, name in enumerate(self.slot_names)}


class GpuRound:
    """Lockstep HO executor on one MI355X — the drop-in for in-JVM execution.

    `GpuRound(alg, n, ...)` corresponds to choosing a runtime backend
    (psync/runtime/Runtime.scala:167-177) for `alg`; `run(begin, count)` to
    `startInstance` for every id in the range followed by the round loop of
    psync/runtime/InstanceHandler.scala:164-258, with the Spec checked after
    every round.
    """

    def __init__(self, alg: Algorithm, n: int, rounds: Optional[int] = None, seed: int = 1,
                 schedule: Optional[HOSchedule] = None, value_range: Optional[int] = None,
                 tiebreak: int = abi.PSG_TIE_CHAMP, device: int = 0, batch_capacity: int = 1 << 20,
                 devices: Optional[Sequence[int]] = None):
        from . import lib
        self.alg = alg
        self.cfg = make_config(alg, n, rounds, seed, schedule, value_range, tiebreak, device, batch_capacity,
                               devices)
        self._ctx = lib.Context(self.cfg)

    @property
    def n(self):
        return self.cfg.n

    @property
    def rounds(self):
        return self.cfg.rounds

    def load_inputs(self, inst_begin: int, count: int, init: Optional[Sequence[Sequence[int]]] = None):
        self._ctx.load_inputs(inst_begin, count, init)

    def run(self, inst_begin: int, count: int, per_instance: bool = False) -> BatchResult:
        s, pi = self._ctx.run_batch(inst_begin, count, per_instance)
        return BatchResult(self.alg, self.cfg.rounds, s, pi)

    def run_spec(self, inst_begin: int, count: int, spec, per_instance: bool = False):
        """Run with a user Spec (round_amd.formula.Spec or a compiled Program) instead
        of the built-in checks. Returns (BatchResult-like summary, slot names)."""
        from . import formula
        prog = spec if isinstance(spec, formula.Program) else formula.compile_spec(spec, self.alg.alg_id)
        if prog.alg and prog.alg != self.alg.alg_id:
            raise ValueError(f"Spec program was compiled for algorithm {prog.alg}, this GpuRound runs "
                             f"{self.alg.class_name} ({self.alg.alg_id})")
        s, pi = self._ctx.run_batch_spec(inst_begin, count, prog, per_instance)
        return SpecResult(prog.slot_names, self.cfg.rounds, s, pi)

    def load_schedule(self, inst_begin: int, count: int, ho, crash=None):
        """Explicit HO sets for instances [inst_begin, inst_begin+count): uint64
        [count][R][n][W] (psg_load_schedule); crash [count][n] marks crashed processes."""
        self._ctx.load_schedule(inst_begin, count, ho, crash)

    def clear_schedule(self):
        self._ctx.clear_schedule()

    def materialize_schedule(self, inst_begin: int, count: int):
        """The seeded HO sets of instances [inst_begin, inst_begin+count), as data."""
        return self._ctx.materialize_schedule(inst_begin, count)

    def decisions(self):
        return self._ctx.copy_decisions()

    def fetch(self, ids: Sequence[int]):
        return self._ctx.fetch(ids)

    def fetch_real(self, ids: Sequence[int]):
        return self._ctx.fetch_real(ids)

    def close(self):
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
