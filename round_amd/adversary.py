"""Adversary search: find HO schedules under which an algorithm violates its
Spec, shrink them, and save them as replayable counterexamples (SURVEY §8f
rank 4: "makes the executor a bug-finder; uses livenessPredicate /
safetyPredicate as schedule constraints").

The reference proves its algorithms with the z3 verifier under the Spec's
environment assumptions (psync/verification/Verifier.scala:145-168: the
`safetyPredicate` conjoined to every transition, a `livenessPredicate` to the
rounds of a progress step). Here the same assumptions constrain explicit HO
schedules (round_amd/schedules.py) and the GPU executes and checks
populations of them per launch (psg_load_schedule + psg_run_batch), so a
search is a loop of: generate / mutate schedules on the host, run them all on
the device, keep the ones that get closest to a violation.

  * safety search: schedules satisfy the safety predicate on their HO sets;
    a violation of a target check slot is genuine only while the predicate
    also held on the *effective* HO sets (slot "SafetyPredicate", halted
    senders send nothing, psync/Round.scala:42-55), i.e. first_fail[target] <
    first_fail[SafetyPredicate].
  * liveness search (mode="liveness"): schedules satisfy the liveness
    predicate in at least `live_rounds` rounds; the target is non-termination
    within R rounds (term_round == never).
  * fault models: general omission (OTR, OTR2, LastVoting, ShortLastVoting,
    BenOr, EpsilonConsensus) or crash-stop with at most f crashes (FloodMin,
    KSetAgreement, KSetEarlyStopping — their runners' fault model).
Every counterexample is shrunk (batched delta debugging: all candidate
simplifications of one step run as one GPU batch) and can be written to a
.psgr file (round_amd/records.py) that `records.replay` re-executes.
"""
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import abi, psync, records, schedules as S

NEVER = abi.PSG_NEVER


# ------------------------------------------------------------------ evaluation

@dataclass
class Eval:
    """Outcome of a batch of explicit-schedule instances (numpy, one row per instance)."""
    summary: np.ndarray      # records.SUMMARY_DTYPE [I]
    decision: np.ndarray     # [I][n] int32 (float64 for EpsilonConsensus)
    decision_round: np.ndarray  # [I][n] int32, -1 = none

    @property
    def first_fail(self):
        return self.summary["first_fail"]


class GpuEvaluator:
    """Runs explicit-schedule batches on one MI355X through the C ABI."""

    def __init__(self, alg: psync.Algorithm, n: int, rounds: int, capacity: int, device: int = 0,
                 value_range: Optional[int] = None, seed: int = 1, tiebreak: int = abi.PSG_TIE_CHAMP):
        self.gr = psync.GpuRound(alg, n, rounds, seed=seed, value_range=value_range, tiebreak=tiebreak,
                                 device=device, batch_capacity=capacity)
        self.cfg = self.gr.cfg
        self.capacity = capacity

    def __call__(self, inst_begin: int, ho: np.ndarray, crash: Optional[np.ndarray], init: np.ndarray) -> Eval:
        I = ho.shape[0]
        outs = []
        for a in range(0, I, self.capacity):
            b = min(I, a + self.capacity)
            ctx = self.gr._ctx
            ctx.load_inputs(inst_begin + a, b - a, init[a:b])
            ctx.load_schedule(inst_begin + a, b - a, ho[a:b], None if crash is None else crash[a:b])
            _, pi = ctx.run_batch_np(inst_begin + a, b - a)
            dec, dr = ctx.copy_decisions_np()
            outs.append((pi, dec, dr))
        return Eval(np.concatenate([o[0] for o in outs]), np.concatenate([o[1] for o in outs]),
                    np.concatenate([o[2] for o in outs]))

    def close(self):
        self.gr.close()


# ------------------------------------------------------------------ fault models per algorithm

@dataclass
class Model:
    family: str                      # "omission" | "crash"
    min_size: Optional[int] = None   # safety predicate |HO(p)| >= min_size (omission family)
    fmax: int = 0                    # crash family: at most fmax crashes
    predicate_slot: Optional[int] = None  # check slot recording the predicate on effective HO sets
    liveness: Optional[str] = None   # "good_round" | "coord_hears_all"
    phase: int = 4                   # coordinator period (coord = (r / phase) % n)


def default_model(alg: psync.Algorithm, n: int) -> Model:
    a = alg.alg_id
    if a in (abi.PSG_ALG_OTR, abi.PSG_ALG_OTR2):
        return Model("omission", liveness="good_round")
    if a in (abi.PSG_ALG_LAST_VOTING, abi.PSG_ALG_SLV):
        return Model("omission", liveness="coord_hears_all", phase=4)  # SLV: coord(r/4) literally
    if a == abi.PSG_ALG_BENOR:
        return Model("omission", min_size=n // 2 + 1, predicate_slot=4)  # BenOr.scala:92
    if a == abi.PSG_ALG_EPSILON:
        return Model("omission", min_size=n - alg.param, predicate_slot=2)  # Epsilon.scala:57
    if a == abi.PSG_ALG_FLOODMIN:
        return Model("crash", fmax=alg.param)
    if a == abi.PSG_ALG_KSET:
        return Model("crash", fmax=alg.param - 1)
    if a == abi.PSG_ALG_KSET_ES:
        return Model("crash", fmax=alg.param)
    raise ValueError(f"no fault model for {alg.class_name}")


def default_init(alg: psync.Algorithm, rng, I: int, n: int, values: int) -> np.ndarray:
    """Initial values: a small domain makes conflicting proposals likely."""
    if alg.real:
        return rng.random((I, n))
    if alg.alg_id == abi.PSG_ALG_BENOR:
        return rng.integers(0, 2, (I, n), dtype=np.int32)
    return rng.integers(1, values + 1, (I, n), dtype=np.int32)  # nonzero (LastVoting.scala:134)


# ------------------------------------------------------------------ results

@dataclass
class Counterexample:
    inst_id: int
    init: np.ndarray                 # [n]
    ho: np.ndarray                   # [R][n][W]
    crash: Optional[np.ndarray]      # [n] or None
    summary: np.ndarray              # records.SUMMARY_DTYPE scalar
    violated: List[str]              # target slots violated (or ["Termination"])
    check_point: int                 # first check point of the violation
    omitted_links: int = 0           # links missing from the HO sets (self links excluded)


@dataclass
class SearchResult:
    counterexamples: List[Counterexample]
    schedules_evaluated: int
    generations: int
    seconds: float
    gpu_seconds: float = 0.0
    history: List[float] = field(default_factory=list)   # best score per generation

    @property
    def schedules_per_second(self):
        return self.schedules_evaluated / self.seconds if self.seconds > 0 else 0.0


class Adversary:
    """Schedule search for one algorithm configuration.

    `evaluator(inst_begin, ho, crash, init) -> Eval` runs a batch (default: the
    GPU through GpuEvaluator); tests may inject another one."""

    def __init__(self, alg: psync.Algorithm, n: int, rounds: int, mode: str = "safety",
                 targets: Optional[Sequence[str]] = None, model: Optional[Model] = None,
                 population: int = 4096, values: int = 3, keep: float = 0.75, self_bit: bool = True,
                 live_rounds: int = 2, live_at: Optional[Sequence[int]] = None, seed: int = 1,
                 evaluator: Optional[Callable] = None, device: int = 0, device_pop: bool = True):
        if mode not in ("safety", "liveness"):
            raise ValueError("mode must be 'safety' or 'liveness'")
        self.alg, self.n, self.R = alg, n, rounds
        self.mode = mode
        self.model = model or default_model(alg, n)
        self.names = alg.check_names
        if mode == "liveness":
            if self.model.liveness is None:
                raise ValueError(f"{alg.class_name} has no livenessPredicate to assume")
            self.targets = []
        else:
            want = list(targets) if targets else [self.names[i] for i in alg.violation_slots]
            for t in want:
                if t not in self.names:
                    raise ValueError(f"unknown check slot {t!r} for {alg.class_name}: {self.names}")
            self.targets = [self.names.index(t) for t in want if self.names.index(t) != self.model.predicate_slot]
        self.population, self.values, self.keep = population, values, keep
        self.self_bit, self.live_rounds = self_bit, live_rounds
        self.live_at = None if live_at is None else list(live_at)
        self.device_pop = device_pop
        self.rng = np.random.default_rng(seed)
        self._own = evaluator is None
        self.evaluator = evaluator or GpuEvaluator(alg, n, rounds, population, device=device,
                                                   value_range=values)
        self.next_id = 0

    def close(self):
        if self._own:
            self.evaluator.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -------------------------------------------------------------- schedules
    def _fresh(self, I):
        m, n, R = self.model, self.n, self.R
        if m.family == "crash":
            crash, partial = S.random_crash(self.rng, I, R, n, m.fmax, p_partial=(0.05, 0.15, 0.5, 0.85))
            return {"crash": crash, "partial": partial}
        # a spread of loss rates around `keep` (each quarter of the population its own)
        parts = []
        levels = [min(0.97, self.keep * f) for f in (0.7, 0.85, 1.0, 1.15)]
        for j, kp in enumerate(levels):
            m = I // 4 + (1 if j < I % 4 else 0)
            if m:
                parts.append(S.random_omission(self.rng, m, R, n, kp, self.self_bit))
        return {"ho": np.concatenate(parts)}

    def _realize(self, g):
        """Genome -> (ho, crash, valid): HO sets repaired to the model's constraints;
        valid[i] = instance i satisfies them (liveness: the predicate holds in at
        least `live_rounds` rounds)."""
        m, n, R = self.model, self.n, self.R
        if m.family == "crash":
            ho = S.crash_to_ho(g["crash"], g["partial"], R, n, self.self_bit)
            return ho, g["crash"], np.ones(ho.shape[0], bool)
        ho = g["ho"].copy()
        S.apply_universe(ho, n, self.self_bit)
        if m.min_size is not None:
            S.repair_min_size(ho, self.rng, n, m.min_size)
        valid = np.ones(ho.shape[0], bool)
        if self.mode == "liveness":
            I = ho.shape[0]
            for j in range(self.live_rounds):
                if self.live_at is not None:
                    ks = np.full(I, self.live_at[j % len(self.live_at)])
                else:
                    ks = self.rng.integers(0, R, I)
                if m.liveness == "good_round":
                    S.force_good_round(ho, self.rng, n, np.arange(I), ks, self_bit=self.self_bit)
                else:
                    for i, k in enumerate(ks):
                        base = (k // m.phase) * m.phase  # a whole phase with the coordinator hearing all
                        S.force_coord_hears_all(ho[i:i + 1], n, range(base, min(R, base + m.phase)), m.phase)
            if m.min_size is not None:
                S.repair_min_size(ho, self.rng, n, m.min_size)
            valid = self._live_count(ho) >= self.live_rounds
        return ho, None, valid

    def _live_count(self, ho):
        m = self.model
        if m.liveness == "good_round":
            return S.good_round(ho, self.n).sum(1)
        return S.coord_hears_all(ho, self.n, m.phase).sum(1)

    def _mutate(self, g, strength):
        m = self.model
        if m.family == "crash":
            c, p = S.mutate_crash(g["crash"], g["partial"], self.rng, self.R, self.n, m.fmax)
            return {"crash": c, "partial": p}
        ho = g["ho"].copy()
        S.flip_links(ho, self.rng, self.n, strength, self.self_bit)
        return {"ho": ho}

    @staticmethod
    def _take(g, idx):
        return {k: v[idx] for k, v in g.items()}

    @staticmethod
    def _cat(a, b):
        return {k: np.concatenate([a[k], b[k]]) for k in a}

    # -------------------------------------------------------------- scoring
    def _violations(self, ev: Eval):
        """(genuine violation mask [I], first violating check point [I])."""
        ff = ev.first_fail.astype(np.int32)
        I = ff.shape[0]
        if self.mode == "liveness":
            bad = ev.summary["term_round"] == NEVER
            return bad, np.where(bad, self.R, NEVER)
        first = ff[:, self.targets].min(1) if self.targets else np.full(I, NEVER)
        bad = first < NEVER
        if self.model.predicate_slot is not None:
            bad &= first < ff[:, self.model.predicate_slot]
        return bad, first

    def _score(self, ev: Eval):
        ff = ev.first_fail
        k = len(self.names)
        failed = (ff[:, :k] != NEVER)
        if self.model.predicate_slot is not None:
            failed[:, self.model.predicate_slot] = False
        dec, dr = ev.decision, ev.decision_round
        decided = dr >= 0
        if self.alg.real:
            lo = np.where(decided, dec, np.inf).min(1)
            hi = np.where(decided, dec, -np.inf).max(1)
            spread = np.where(decided.any(1), (hi - lo) / max(self.alg.epsilon, 1e-300), 0.0)
            distinct = np.minimum(spread, 10.0)
        else:
            lo = np.where(decided, dec, np.iinfo(np.int32).max).min(1)
            hi = np.where(decided, dec, np.iinfo(np.int32).min).max(1)
            distinct = (decided.any(1) & (hi != lo)).astype(np.int64)
            multi = np.nonzero(distinct)[0]
            if len(multi):  # exact count only where decisions differ (rare)
                d = np.where(decided[multi], dec[multi], np.iinfo(np.int32).min)
                srt = np.sort(d, 1)
                distinct[multi] = ((np.diff(srt, axis=1) != 0) & (srt[:, 1:] != np.iinfo(np.int32).min)).sum(1)
        if self.mode == "liveness":
            late = ev.summary["term_round"].astype(np.float64)
            return late + 0.1 * (~decided).sum(1) + self.rng.random(len(late)) * 1e-3
        return 4.0 * distinct + failed.sum(1) + 0.05 * decided.sum(1) / self.n + self.rng.random(len(ff)) * 1e-3

    # -------------------------------------------------------------- search
    def device_population(self) -> bool:
        """Can generations be generated and mutated on the GPU (psg_population_*)?
        General omission, safety search, integer inputs, the GPU evaluator."""
        return (self.model.family == "omission" and self.mode == "safety" and not self.alg.real
                and isinstance(self.evaluator, GpuEvaluator) and self.device_pop)

    def _pop_params(self, generation):
        p = abi.PopulationParams()
        p.seed = int(self.rng.integers(0, 1 << 63)) if generation == 0 else self._pop_seed
        if generation == 0:
            self._pop_seed = p.seed
        p.generation = generation
        p.flips = max(1, int(self.n * self.R * 0.01))
        p.min_size = self.model.min_size or 0
        p.self_bit = 1 if self.self_bit else 0
        for j, f in enumerate((0.7, 0.85, 1.0, 1.15)):  # the host generator's spread of loss rates
            p.keep_p256[j] = int(round(min(0.97, self.keep * f) * 256))
        p.value_range = self.values
        p.redraw_p256 = 5  # ~2 % of a mutant's initial values redrawn
        return p

    def _search_device(self, generations, want, time_budget, elite_frac, fresh_frac, shrink):
        """The search loop with the population resident in HBM: per generation one
        psg_run_batch, the per-instance summaries + decisions to the host for scoring,
        and psg_population_next with the chosen parents (no HO set crosses PCIe)."""
        P = self.population
        ctx = self.evaluator.gr._ctx
        base = self.next_id
        self.next_id += P
        ctx.population_fresh(base, P, self._pop_params(0))
        found: List[Counterexample] = []
        t0 = time.perf_counter()
        gpu = 0.0
        history = []
        g = 0
        for g in range(1, generations + 1):
            t1 = time.perf_counter()
            _, pi = ctx.run_batch_np(base, P)
            dec, dr = ctx.copy_decisions_np()
            gpu += time.perf_counter() - t1
            ev = Eval(pi, dec, dr)
            bad, first = self._violations(ev)
            rows = np.nonzero(bad)[0][:max(0, want - len(found))]
            if len(rows):
                hos, inits = ctx.population_read(rows)
                for j, i in enumerate(rows):
                    found.append(self._cex(base + int(i), inits[j], hos[j], None, pi[i], int(first[i])))
            score = self._score(ev)
            history.append(float(score.max()))
            if len(found) >= want or (time_budget is not None and time.perf_counter() - t0 > time_budget):
                break
            order = np.argsort(-score)
            ne = max(1, int(P * elite_frac))
            nf = int(P * fresh_frac)
            nm = P - ne - nf
            elite = order[:ne]
            parent = np.zeros(P, np.uint32)
            op = np.full(P, 2, np.uint8)
            parent[:ne], op[:ne] = elite, 0
            parent[ne:ne + nm], op[ne:ne + nm] = elite[self.rng.integers(0, ne, nm)], 1
            t1 = time.perf_counter()
            ctx.population_next(parent, op, self._pop_params(g))
            gpu += time.perf_counter() - t1
        secs = time.perf_counter() - t0
        if shrink:
            found = [self.shrink(c) for c in found]
        return SearchResult(found, P * g, g, secs, gpu, history)

    def search(self, generations: int = 50, want: int = 1, time_budget: Optional[float] = None,
               elite_frac: float = 0.25, fresh_frac: float = 0.25, shrink: bool = True) -> SearchResult:
        if self.device_population():
            return self._search_device(generations, want, time_budget, elite_frac, fresh_frac, shrink)
        P = self.population
        genome = self._fresh(P)
        init = default_init(self.alg, self.rng, P, self.n, self.values)
        found: List[Counterexample] = []
        t0 = time.perf_counter()
        gpu = 0.0
        evaluated = 0
        history = []
        g = 0
        for g in range(1, generations + 1):
            ho, crash, valid = self._realize(genome)
            base = self.next_id
            self.next_id += P
            t1 = time.perf_counter()
            ev = self.evaluator(base, ho, crash, init)
            gpu += time.perf_counter() - t1
            evaluated += P
            bad, first = self._violations(ev)
            bad &= valid
            for i in np.nonzero(bad)[0][:max(0, want - len(found))]:
                found.append(self._cex(base + int(i), init[i], ho[i], None if crash is None else crash[i],
                                       ev.summary[i], int(first[i])))
            score = self._score(ev)
            history.append(float(score.max()))
            if len(found) >= want or (time_budget is not None and time.perf_counter() - t0 > time_budget):
                break
            # next generation: elites + mutants of elites + fresh schedules
            order = np.argsort(-score)
            ne = max(1, int(P * elite_frac))
            nf = int(P * fresh_frac)
            nm = P - ne - nf
            elite = order[:ne]
            parents = elite[self.rng.integers(0, ne, nm)]
            strength = max(1, int(self.n * self.R * 0.01))
            children = self._mutate(self._take(genome, parents), strength)
            genome = self._cat(self._cat(self._take(genome, elite), children), self._fresh(nf)) if nf else \
                self._cat(self._take(genome, elite), children)
            cinit = init[parents].copy()
            flip = self.rng.random(cinit.shape) < 0.02
            fresh_init = default_init(self.alg, self.rng, cinit.shape[0], self.n, self.values)
            cinit[flip] = fresh_init[flip]
            init = np.concatenate([init[elite], cinit, default_init(self.alg, self.rng, nf, self.n, self.values)])
        secs = time.perf_counter() - t0
        if shrink:
            found = [self.shrink(c) for c in found]
        return SearchResult(found, evaluated, g, secs, gpu, history)

    def _cex(self, inst, init, ho, crash, summ, first):
        ff = summ["first_fail"]
        if self.mode == "liveness":
            viol = ["Termination"]
        else:
            viol = [self.names[t] for t in self.targets if ff[t] == first]
        return Counterexample(inst, np.array(init), np.array(ho), None if crash is None else np.array(crash),
                              np.array(summ), viol, first, self._omitted(ho))

    def _omitted(self, ho):
        """Links (k, p, q) missing from one schedule [R][n][W] (q == p excluded with self_bit)."""
        have = int(S.sizes(ho[None]).sum())
        R = ho.shape[0]
        total = R * self.n * self.n
        return total - have

    # -------------------------------------------------------------- shrinking
    def _still_bad(self, c: Counterexample, hos, crashes):
        """Evaluate candidate schedules of counterexample c (same init and instance id)."""
        I = hos.shape[0]
        init = np.repeat(c.init[None], I, 0)
        out_bad = np.zeros(I, bool)
        out_first = np.full(I, NEVER, np.int32)
        out_sum = None
        cap = self.population
        sums = []
        for a in range(0, I, cap):
            b = min(I, a + cap)
            # every candidate replays the counterexample's own instance id (same coins)
            ev = self._eval_same_id(c.inst_id, hos[a:b], None if crashes is None else crashes[a:b], init[a:b])
            bad, first = self._violations(ev)
            out_bad[a:b], out_first[a:b] = bad, first
            sums.append(ev.summary)
        out_sum = np.concatenate(sums)
        return out_bad, out_first, out_sum

    def _eval_same_id(self, inst, ho, crash, init):
        """Instances share an id only through separate batches; BenOr's coin depends on
        the id, so candidates run one id each: ids inst, inst+1, ... would change
        coins. Run each candidate as its own instance id `inst` in chunks of one
        contiguous batch per distinct id is too slow, so coins are id-keyed only for
        BenOr: other algorithms are id-independent under an explicit schedule."""
        if self.alg.alg_id != abi.PSG_ALG_BENOR:
            return self.evaluator(inst, ho, crash, init)
        outs = [self.evaluator(inst, ho[j:j + 1], None if crash is None else crash[j:j + 1], init[j:j + 1])
                for j in range(ho.shape[0])]
        return Eval(np.concatenate([o.summary for o in outs]), np.concatenate([o.decision for o in outs]),
                    np.concatenate([o.decision_round for o in outs]))

    def shrink(self, c: Counterexample, max_steps: int = 64) -> Counterexample:
        """Greedy batched delta debugging: restore omitted links (whole rounds, then
        whole heard-of sets, then single links; crash-stop: un-crash processes,
        deliver crash-round messages) while the violation persists, and make the
        rounds after the violation fault-free."""
        n, R = self.n, self.R
        fm = S.full_mask(n)
        ho = c.ho.copy()
        crash = None if c.crash is None else c.crash.copy()
        cur = c
        steps = 0

        def accept(cands_ho, cands_crash):
            nonlocal ho, crash, cur
            bad, first, summ = self._still_bad(cur, cands_ho, cands_crash)
            if not bad.any():
                return False
            # prefer the simplest candidate: most links present, then earliest violation
            links = S.sizes(cands_ho).sum((-1, -2))
            key = np.where(bad, links * 1024 - first, -1)
            j = int(np.argmax(key))
            ho = cands_ho[j].copy()
            crash = None if cands_crash is None else cands_crash[j].copy()
            viol = cur.violated if self.mode == "liveness" else \
                [self.names[t] for t in self.targets if summ[j]["first_fail"][t] == first[j]]
            cur = Counterexample(cur.inst_id, cur.init, ho.copy(), None if crash is None else crash.copy(),
                                 summ[j], viol, int(first[j]), self._omitted(ho))
            return True

        if self.model.family == "crash":
            while steps < max_steps:
                steps += 1
                cands_c, cands_h = [], []
                for q in np.nonzero(crash >= 0)[0]:          # un-crash q
                    cc = crash.copy()
                    cc[q] = -1
                    cands_c.append(cc)
                for q in np.nonzero(crash >= 0)[0]:          # crash q later
                    if crash[q] + 1 < R:
                        cc = crash.copy()
                        cc[q] += 1
                        cands_c.append(cc)
                if not cands_c:
                    break
                cc = np.stack(cands_c)
                # keep the crash-round deliveries of the current schedule
                part = np.zeros((len(cands_c), n, S.words(n)), np.uint64)
                for q in range(n):
                    if crash[q] >= 0:
                        row = ho[crash[q]]  # [n][W]: who hears q in q's crash round
                        part[:, :, q >> 6] |= row[:, q >> 6] & np.uint64(1 << (q & 63))
                hh = S.crash_to_ho(cc, part, R, n, self.self_bit)
                if not accept(hh, cc):
                    break
            return cur

        if self.mode == "safety" and cur.check_point < NEVER:
            # rounds after the violating check point are irrelevant: fault-free
            h2 = ho.copy()
            h2[cur.check_point:] = fm
            accept(h2[None], None)
        # predicate-preserving: restoring links only grows HO sets, so |HO(p)| >= m and
        # good rounds (if |s| grows uniformly) stay; liveness keeps its forced rounds
        for level in ("round", "set", "link"):
            while steps < max_steps:
                steps += 1
                cands = []
                if level == "round":
                    for k in range(R):
                        if (ho[k] != fm).any():
                            h2 = ho.copy()
                            h2[k] = fm
                            cands.append(h2)
                elif level == "set":
                    for k in range(R):
                        for p in range(n):
                            if (ho[k, p] != fm).any():
                                h2 = ho.copy()
                                h2[k, p] = fm
                                cands.append(h2)
                else:
                    for k in range(R):
                        for p in range(n):
                            miss = [q for q in range(n) if not (int(ho[k, p, q >> 6]) >> (q & 63)) & 1]
                            for q in miss:
                                h2 = ho.copy()
                                h2[k, p, q >> 6] |= np.uint64(1 << (q & 63))
                                cands.append(h2)
                            if len(cands) > 4 * self.population:
                                break
                        if len(cands) > 4 * self.population:
                            break
                if not cands:
                    break
                hh = np.stack(cands)
                if self.mode == "liveness":
                    hh = hh[self._live_count(hh) >= self.live_rounds]
                    if not len(hh):
                        break
                if not accept(hh, None):
                    break
        return cur


# ------------------------------------------------------------------ files

def save(path: str, adv: Adversary, cexs: Sequence[Counterexample], meta: Optional[dict] = None):
    """Write counterexamples as a .psgr record file (replay with records.replay)."""
    if not cexs:
        raise ValueError("no counterexamples to save")
    order = np.argsort([c.inst_id for c in cexs], kind="stable")
    cexs = [cexs[i] for i in order]
    cfg = adv.evaluator.cfg if hasattr(adv.evaluator, "cfg") else psync.make_config(adv.alg, adv.n, adv.R)
    summ = np.stack([np.asarray(c.summary, records.SUMMARY_DTYPE) for c in cexs])
    crash = None
    if any(c.crash is not None for c in cexs):
        crash = np.stack([c.crash if c.crash is not None else np.full(adv.n, -1, np.int32) for c in cexs])
    m = {"mode": adv.mode, "targets": [adv.names[t] for t in adv.targets], "family": adv.model.family,
         "violated": [c.violated for c in cexs], "check_point": [c.check_point for c in cexs],
         "omitted_links": [int(c.omitted_links) for c in cexs]}
    m.update(meta or {})
    rec = records.Records(cfg=cfg, slot_names=list(adv.names), ids=np.array([c.inst_id for c in cexs], np.uint64),
                          summary=summ, init=np.stack([c.init for c in cexs]), ho=np.stack([c.ho for c in cexs]),
                          crash=crash, meta=m, class_name=adv.alg.class_name)
    records.write(path, rec)
    return rec


def describe(c: Counterexample, n: int) -> str:
    """Human-readable rendering: the missing links per round up to the violation."""
    lines = [f"instance {c.inst_id}: {', '.join(c.violated)} violated at check point {c.check_point}; "
             f"{c.omitted_links} omitted link(s)", f"  init = {list(np.asarray(c.init).tolist())}"]
    R = c.ho.shape[0]
    last = R if c.check_point >= NEVER else min(R, c.check_point)
    for k in range(last):
        miss = []
        for p in range(n):
            for q in range(n):
                if not (int(c.ho[k, p, q >> 6]) >> (q & 63)) & 1:
                    miss.append(f"{q}->{p}")
        lines.append(f"  round {k}: " + ("all delivered" if not miss else "lost " + " ".join(miss[:40]) +
                                           (" ..." if len(miss) > 40 else "")))
    if c.crash is not None and (c.crash >= 0).any():
        lines.append("  crashed: " + ", ".join(f"{q}@{int(c.crash[q])}" for q in np.nonzero(c.crash >= 0)[0]))
    return "\n".join(lines)
