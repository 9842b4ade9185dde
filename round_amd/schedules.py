"""Explicit HO schedules as data: generation, the reference's Spec predicates,
repair and mutation (host side, numpy), for psg_load_schedule and the
adversary search.

A schedule batch is `ho`: uint64 [I][R][n][W] (W = ceil(n/64); bit q of word w
of ho[i, k, p] = process 64w+q is in HO(p) in round k) plus `crash`: int32
[I][n] (-1 = correct). Faults are HO sets in the reference
(psync/Process.scala:14: `HO` is the Spec-level heard-of set), so every fault
model below is a family of such arrays.

Predicates restate the Specs' environment assumptions over given HO sets:
  * BenOr `safetyPredicate = P.forall(p => p.HO.size > n/2)` (example/BenOr.scala:92)
  * OTR / OTR2 `livenessPredicate` good round
    `S.exists(s => P.forall(p => p.HO == s && s.size > 2*n/3))` (example/Otr.scala:96-97,
    example/Otr2.scala:74)
  * LastVoting `livenessPredicate`
    `P.exists(p => P.forall(q => p == coord && p.HO.contains(q) && p.HO.size > n/2))`
    (example/LastVoting.scala:20-22): the coordinator of the round hears everyone
  * EpsilonConsensus: |HO(p)| >= n - f (the commented assert `mailbox.size >= n - f`,
    example/Epsilon.scala:57)
  * crash-stop with at most f crashes (FloodMin / KSet / KSetEarlyStopping runners)
The `Verifier` assumes the safety predicate on every transition and a liveness
predicate on the rounds of a progress step (psync/verification/Verifier.scala:
145-168); the search uses them the same way (constraint on the explicit sets).
"""
from typing import Optional

import numpy as np

U64 = np.uint64
ALL = np.uint64(0xFFFFFFFFFFFFFFFF)


def words(n: int) -> int:
    return (n + 63) // 64


def full_mask(n: int) -> np.ndarray:
    """uint64 [W]: the set of all n processes."""
    W = words(n)
    m = np.zeros(W, U64)
    for w in range(W):
        b = min(64, n - 64 * w)
        m[w] = ALL if b == 64 else np.uint64((1 << b) - 1)
    return m


def self_mask(n: int) -> np.ndarray:
    """uint64 [n][W]: row p = {p}."""
    W = words(n)
    m = np.zeros((n, W), U64)
    for p in range(n):
        m[p, p >> 6] = np.uint64(1 << (p & 63))
    return m


def sizes(ho: np.ndarray) -> np.ndarray:
    """|HO(p)| per (instance, round, process): int [I][R][n]."""
    return np.bitwise_count(ho).sum(-1, dtype=np.int32)


def contains(ho: np.ndarray, q: int) -> np.ndarray:
    """q in HO(p) per (instance, round, process): bool [I][R][n]."""
    return ((ho[..., q >> 6] >> U64(q & 63)) & U64(1)).astype(bool)


# ------------------------------------------------------------------ predicates (per instance, per round)

def ho_majority(ho: np.ndarray, n: int) -> np.ndarray:
    """BenOr safetyPredicate per round: forall p. |HO(p)| > n/2 -> bool [I][R]."""
    return (sizes(ho) > n // 2).all(-1)


def ho_at_least(ho: np.ndarray, m: int) -> np.ndarray:
    """forall p. |HO(p)| >= m -> bool [I][R]."""
    return (sizes(ho) >= m).all(-1)


def good_round(ho: np.ndarray, n: int) -> np.ndarray:
    """OTR livenessPredicate per round: exists s. forall p. HO(p) == s && |s| > 2n/3 -> bool [I][R]."""
    same = (ho == ho[:, :, :1, :]).all(-1).all(-1)
    return same & (sizes(ho[:, :, :1, :])[..., 0] > (2 * n) // 3)


def coord_hears_all(ho: np.ndarray, n: int, phase: int = 4) -> np.ndarray:
    """LastVoting livenessPredicate per round k: HO(coord) = all processes with
    coord = (k / phase) % n (example/LastVoting.scala:20-22, 95) -> bool [I][R]."""
    I, R = ho.shape[:2]
    fm = full_mask(n)
    out = np.zeros((I, R), bool)
    for k in range(R):
        c = (k // phase) % n
        out[:, k] = (ho[:, k, c, :] == fm).all(-1)
    return out


def crash_consistent(ho: np.ndarray, crash: np.ndarray, n: int, fmax: int) -> np.ndarray:
    """Crash-stop pattern with at most fmax crashes: correct processes are heard by
    everyone every round, a process crashed at round c is heard by nobody after c
    (any subset in round c), self always heard -> bool [I]."""
    I, R = ho.shape[:2]
    ok = (crash >= 0).sum(-1) <= fmax
    for q in range(n):
        h = contains(ho, q)  # [I][R][n]
        cq = crash[:, q]
        k = np.arange(R)[None, :]
        before = (cq[:, None] < 0) | (k < cq[:, None])  # must be heard by all
        after = (cq[:, None] >= 0) & (k > cq[:, None])  # heard by nobody but itself
        others = np.ones(n, bool)
        others[q] = False
        ok &= ~(before[:, :, None] & ~h).any((1, 2))
        ok &= ~(after[:, :, None] & h & others[None, None, :]).any((1, 2))
    return ok


# ------------------------------------------------------------------ generators

def random_bits(rng: np.random.Generator, shape, density: float, digits: int = 8) -> np.ndarray:
    """uint64 words whose bits are set independently w.p. `density` (rounded to
    `digits` binary digits): x = r_j | x for a 1 digit, r_j & x for a 0 digit,
    from the least significant digit up, with fresh uniform words r_j."""
    q = int(round(min(max(density, 0.0), 1.0) * (1 << digits)))
    if q >= 1 << digits:
        return np.full(shape, ALL, U64)
    if q == 0:
        return np.zeros(shape, U64)
    while q % 2 == 0:  # drop trailing zero digits (they would AND with an all-zero start)
        q //= 2
        digits -= 1
    x = np.zeros(shape, U64)
    for j in range(digits):
        r = rng.integers(0, 1 << 64, size=shape, dtype=U64, endpoint=False)
        x = (r | x) if (q >> j) & 1 else (r & x)
    return x


def apply_universe(ho: np.ndarray, n: int, self_bit: bool) -> np.ndarray:
    """Clear bits >= n; with self_bit add p to HO(p) (psync/Round.scala:114-116)."""
    ho &= full_mask(n)
    if self_bit:
        ho |= self_mask(n)[None, None]
    return ho


def random_omission(rng, I: int, R: int, n: int, keep: float, self_bit: bool = True) -> np.ndarray:
    """General omission: each link delivered w.p. `keep`, independently."""
    ho = random_bits(rng, (I, R, n, words(n)), keep)
    return apply_universe(ho, n, self_bit)


def random_crash(rng, I: int, R: int, n: int, fmax: int, p_partial: float = 0.5):
    """Crash-stop genome: crash [I][n] (<= fmax crashed, uniform crash rounds) and
    partial [I][n][W] (receiver p's share of the crash-round messages)."""
    crash = np.full((I, n), -1, np.int32)
    f = rng.integers(0, fmax + 1, size=I)
    for i in range(I):
        who = rng.permutation(n)[:f[i]]
        crash[i, who] = rng.integers(0, R, size=len(who))
    if np.ndim(p_partial) == 0:
        partial = random_bits(rng, (I, n, words(n)), float(p_partial))
    else:  # one delivery density per instance, drawn from the given levels
        lv = np.asarray(p_partial, float)
        pick = rng.integers(0, len(lv), I)
        partial = np.zeros((I, n, words(n)), U64)
        for j, d in enumerate(lv):
            sel = np.nonzero(pick == j)[0]
            if len(sel):
                partial[sel] = random_bits(rng, (len(sel), n, words(n)), float(d))
    return crash, partial


def crash_to_ho(crash: np.ndarray, partial: np.ndarray, R: int, n: int, self_bit: bool = True) -> np.ndarray:
    """HO sets of a crash-stop genome: q in HO(p, k) iff q correct, or k < crash(q),
    or k == crash(q) and q in partial(p)."""
    I = crash.shape[0]
    W = words(n)
    ho = np.zeros((I, R, n, W), U64)
    bit = np.zeros((n, W), U64)
    for q in range(n):
        bit[q, q >> 6] = np.uint64(1 << (q & 63))
    for k in range(R):
        alive = (crash < 0) | (k < crash)      # [I][n] heard by all
        now = crash == k                        # [I][n] partially heard
        a = (alive[:, :, None] * bit[None]).sum(1, dtype=U64)   # [I][W]
        c = (now[:, :, None] * bit[None]).sum(1, dtype=U64)     # [I][W]
        ho[:, k] = a[:, None, :] | (c[:, None, :] & partial)
    return apply_universe(ho, n, self_bit)


# ------------------------------------------------------------------ repair and mutation

def repair_min_size(ho: np.ndarray, rng, n: int, m: int) -> np.ndarray:
    """Add random senders to every HO(p) with fewer than m members (keeps the
    set's existing members). Used for |HO(p)| > n/2 (m = n/2 + 1) and n - f."""
    fm = full_mask(n)
    for _ in range(64):
        bad = sizes(ho) < m
        if not bad.any():
            return ho
        idx = np.nonzero(bad)
        ho[idx] |= random_bits(rng, (len(idx[0]), ho.shape[-1]), 0.5) & fm
    bad = sizes(ho) < m
    ho[np.nonzero(bad)] = fm
    return ho


def force_good_round(ho: np.ndarray, rng, n: int, inst: np.ndarray, k: np.ndarray, keep: float = 0.9,
                     self_bit: bool = False):
    """Make round k[j] of instance inst[j] a good round (one common set s with |s| > 2n/3).
    With self_bit (p always in HO(p)) the common set must contain everyone: s = all."""
    fm = full_mask(n)
    thr = (2 * n) // 3
    for i, kk in zip(inst, k):
        s = fm.copy() if self_bit else random_bits(rng, (ho.shape[-1],), keep) & fm
        while int(np.bitwise_count(s).sum()) <= thr:
            s |= random_bits(rng, (ho.shape[-1],), 0.5) & fm
        ho[i, kk, :, :] = s
    return ho


def force_coord_hears_all(ho: np.ndarray, n: int, rounds=None, phase: int = 4) -> np.ndarray:
    """HO(coord(k)) := all processes in the given rounds (all rounds by default)."""
    fm = full_mask(n)
    R = ho.shape[1]
    for k in (range(R) if rounds is None else rounds):
        ho[:, k, (k // phase) % n, :] = fm
    return ho


def flip_links(ho: np.ndarray, rng, n: int, per_instance: int, self_bit: bool = True) -> np.ndarray:
    """Flip `per_instance` random links (k, p, q) of every instance (q != p when self_bit)."""
    I, R = ho.shape[:2]
    m = I * per_instance
    ii = np.repeat(np.arange(I), per_instance)
    kk = rng.integers(0, R, m)
    pp = rng.integers(0, n, m)
    qq = rng.integers(0, n, m)
    if self_bit:
        qq = np.where(qq == pp, (qq + 1) % n, qq)
    np.bitwise_xor.at(ho, (ii, kk, pp, qq >> 6), (np.uint64(1) << (qq & 63).astype(U64)))
    return ho


def mutate_crash(crash: np.ndarray, partial: np.ndarray, rng, R: int, n: int, fmax: int, rate: float = 0.3):
    """Crash-stop genome mutation: move / add / remove one crash, flip crash-round deliveries."""
    I = crash.shape[0]
    crash = crash.copy()
    partial = partial.copy()
    for i in range(I):
        u = rng.random()
        crashed = np.nonzero(crash[i] >= 0)[0]
        if u < rate and len(crashed):                       # move a crash round
            q = rng.choice(crashed)
            crash[i, q] = rng.integers(0, R)
        elif u < 2 * rate and len(crashed) < fmax:           # crash one more process
            q = rng.choice(np.nonzero(crash[i] < 0)[0])
            crash[i, q] = rng.integers(0, R)
        elif u < 2.5 * rate and len(crashed):                # un-crash one
            crash[i, rng.choice(crashed)] = -1
        p = rng.integers(0, n)
        q = rng.integers(0, n)
        partial[i, p, q >> 6] ^= np.uint64(1 << (q & 63))
    return crash, partial
