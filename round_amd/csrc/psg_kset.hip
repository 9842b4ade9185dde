// psg_kset.hip — KSetAgreement on gfx950.
//
// Reference: example/KSetAgreement.scala:21-68. The state t: Map[ProcessID,Int]
// only ever holds entries (q -> initialValue_q) (init `Map(id -> v)` at 30,
// merge `a ++ b` at 36-38), so it is exactly a set of origins over the fixed
// initial vector: a W x 64-bit mask per process; `t == t'` is mask equality,
// `t ++ t'` is OR, pick(t) = min of the initial values of the origins (40).
// Payloads (decider, t) are staged in LDS; each process walks the alive senders
// with broadcast LDS reads. `content.find(_._1)` (47-53) takes the LAST decider
// message in Scala Map iteration order (CHAMP for > 4 entries).
// Philox round keys formed per call in this translation unit (packed KSet C4 -3..5 %; the hoisted
// 20-SGPR key schedule spilled here — and won in OTR / LastVoting / FloodMin / BenOr: round-4 A/B)
#ifndef PSG_PHILOX_OPAQUE_KEYS
#define PSG_PHILOX_OPAQUE_KEYS 1
#endif
#include "psg_device.hpp"
#include "psg_kernels.hpp"
#include "psg_packed.hpp"

namespace psg {

template <int W>
struct KsLds {
  static constexpr int G = Geometry<W>::kGroups;
  uint64_t ts[G][64 * W * W];  // staged t masks [pid][word]
  int32_t x0s[G][64 * W];      // initial values (for pick)
  int32_t ds[G][64 * W];       // staged decisions (spec)
};

// pick(t) = t.values.min over the staged initial values. Fast path: if t holds
// an origin of the instance's smallest initial value xmin (Emin = those origins,
// uniform), that is the min; otherwise walk t.
template <int W>
PSG_DEV int32_t kset_pick(const Mask<W>& t, const int32_t* x0s, const Mask<W>& Emin, int32_t xmin) {
  if (many(mand(t, Emin))) return xmin;
  int32_t m = INT32_MAX;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint64_t b = t.w[w];
    while (b) {
      const int q = w * 64 + __builtin_ctzll(b);
      b &= b - 1;
      m = min(m, x0s[q]);
    }
  }
  return m;
}

// t mask of process q from the staged rows: [pid][word] (CS = 0) or [word][pid] with a
// column stride CS (the lane-packed path: lanes store consecutive words, no bank conflicts)
template <int W, int CS = 0>
PSG_DEV Mask<W> load_t(const uint64_t* ts, int q) {
  Mask<W> m;
#pragma unroll
  for (int w = 0; w < W; ++w) m.w[w] = CS ? ts[w * CS + q] : ts[q * W + w];
  return m;
}

// `content.find(_._1).get._2` of receiver p (KSetAgreement.scala:47-53). `content =
// mailbox.map{ case (k,v) => v }` maps to pairs, so it is a Map[Boolean, Map[ProcessID,Int]]
// built in the mailbox's iteration order, each decider message overwriting key `true`: the
// adopted t is the LAST decider message's in Scala Map iteration order — the last pid of cand
// up to 4 mailbox entries (Map1..Map4), under PSG_TIE_MIN_PID, or when the candidates agree
// on t; otherwise the CHAMP order's last (max sort key).
// hol / ncols (optional): the round's holder columns (kset_packed): the candidates' t agree
// iff every column holds all of them or none, so no candidate's t is read.
template <int W, int CS = 0>
PSG_DEV int kset_find(const KArgs& a, const uint64_t* ts, const Mask<W>& M, const Mask<W>& cand,
                      const uint64_t (*hol)[W] = nullptr, int ncols = 0) {
  int qs = mlast(cand);
  if (a.tiebreak == PSG_TIE_CHAMP && mpopc(M) > 4 && mpopc(cand) > 1) {
    bool differ = false;
    if (hol) {
      for (int c = 0; c < ncols; ++c) {
        Mask<W> x;
#pragma unroll
        for (int w = 0; w < W; ++w) x.w[w] = cand.w[w] & hol[c][w];
        differ = differ || (many(x) && !meq(x, cand));
      }
    } else {
      const Mask<W> t0 = load_t<W, CS>(ts, qs);
#pragma unroll
      for (int w = 0; w < W; ++w) {
        uint64_t m = cand.w[w];
        while (m) {
          const int q = w * 64 + __builtin_ctzll(m);
          m &= m - 1;
          if (!meq(load_t<W, CS>(ts, q), t0)) differ = true;
        }
      }
    }
    if (differ) {
      uint64_t best = 0;  // max key; keys of distinct pids differ (>=: the first candidate sets qs)
#pragma unroll
      for (int w = 0; w < W; ++w) {
        uint64_t m = cand.w[w];
        while (m) {
          const int q = w * 64 + __builtin_ctzll(m);
          m &= m - 1;
          const uint32_t hq = scala_improve((uint32_t)q);
          int depth = 0;
#pragma unroll
          for (int v = 0; v < W; ++v) {
            uint64_t mm = M.w[v];
            while (mm) {
              const int f = v * 64 + __builtin_ctzll(mm);
              mm &= mm - 1;
              if (f != q) depth = max(depth, champ_cpl(hq, scala_improve((uint32_t)f)));
            }
          }
          const uint64_t key = champ_key(hq, depth);
          if (key >= best) {
            best = key;
            qs = q;
          }
        }
      }
    }
  }
  return qs;
}

// ---------------------------------------------------------------- lane-packed path (n > 64)
// kset_body's built-in-checker path with one wave per instance and the W processes
// l + 64 j in lane l (psg_packed.hpp): the t masks are staged in this wave's LDS (word-major,
// [word][pid]: each store instruction writes 64 consecutive words, no bank conflicts; the
// pid-major rows measured 47 % of LDS cycles in conflicts) for the uniform class reads and
// the per-lane find; the
// k-agreement check's ballots are wave ballots; no round needs a block barrier.
template <int W>
struct KsPk {
  static constexpr int kClasses = 8;
  int32_t x0s[64 * W];
  static constexpr int kCols = 32;
  uint64_t ct[kClasses][W];  // a round's classes of equal t among the alive senders: their t
  uint64_t ce[kClasses][W];  // ... and their members
  uint64_t hol[kCols][W];    // holders H_o of each varying origin o (column form, below)
};

// The pre-round t staging ([word][pid], 8 KB at W = 4) is needed only in the few rounds before
// every alive t is equal (tuni) — two or three of an instance's rounds — so the block's four
// waves share two buffers (wave w uses buffer w / 2) under an LDS lock instead of owning one
// each: 52 -> 36 KB of LDS per block, four blocks per CU instead of three.
#ifndef PSG_KSET_STAGE_BUFS
#define PSG_KSET_STAGE_BUFS 2  // staging buffers per 4-wave block (wave w uses buffer w * BUFS / 4)
#endif
template <int W>
struct KsStage {
  static constexpr int kWaves = 4;  // kset_packed_kernel: 256-thread blocks, one instance per wave
  static constexpr int kBufs = PSG_KSET_STAGE_BUFS;
  static_assert(kBufs >= 1 && kWaves % kBufs == 0, "every staging buffer is shared by the same number of waves");
  uint64_t ts[kBufs][64 * W * W];
  int lock[kBufs];
  PSG_DEV void init() {
    if (threadIdx.x < kBufs) lock[threadIdx.x] = 0;
  }
  // Wave-uniform spin lock. Deadlock-free because no wave holding a buffer ever waits for another
  // wave: between acquire() and release() only wave-level syncs (lds_sync<1>) may run — a block
  // barrier (__syncthreads) there would wait for a wave spinning here, which never arrives.
  PSG_DEV uint64_t* acquire(int b, int lane) {
    while (true) {
      int got = 0;
      if (lane == 0) got = atomicCAS(&lock[b], 0, 1) == 0 ? 1 : 0;
      if (__builtin_amdgcn_readfirstlane(got)) break;
      __builtin_amdgcn_s_sleep(4);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return ts[b];
  }
  PSG_DEV void release(int b, int lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // this wave's reads of ts done
    if (lane == 0) atomicExch(&lock[b], 0);
  }
};

// Wave AND / OR of a per-lane mask (DPP OR reductions; AND = NOT OR NOT).
template <int W>
PSG_DEV void pk_and_or(const Mask<W>& a, const Mask<W>& o, Mask<W>& all, Mask<W>& any) {
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const uint64_t na = ~a.w[w];
    all.w[w] = ~((uint64_t)wave_or((uint32_t)na) | ((uint64_t)wave_or((uint32_t)(na >> 32)) << 32));
    any.w[w] = (uint64_t)wave_or((uint32_t)o.w[w]) | ((uint64_t)wave_or((uint32_t)(o.w[w] >> 32)) << 32);
  }
}

// Hand-off to the uniform-t tail kernel (HAND, below). Header word of batch row i: bits 0-7 the
// round the tail resumes at, bit 8 its deciders' "pick(t) is not an initial value", bit 9 "the
// instance was finished here", bits 32-63 pick(t) of the common t. Per-lane word: bits 0-7 the
// lane's Checks::ffv, 8-19 the flag word fw (decider bits 0-3, not-initial bits 8-11), 32-63 the
// slots' halt rounds as bytes (0xFF = not halted). Decisions of halted processes in [row][n].
constexpr uint64_t kHandDone = 1ull << 9;

template <int W, bool HAND>
PSG_DEV void kset_packed(const Pk<W>& P, const KArgs& a, uint64_t i, uint64_t inst, KsPk<W>& L, KsStage<W>& S,
                         int sbuf, int32_t* x0lds, BlockCounters* bc, PhaseTimers& pt) {
  const int n = a.n, kk = a.param;
  const int need = a.variant == 1 ? 1 : n - kk;  // same.size > n - k (KSetAgreement.scala:56)
  Sched<W, false> sc;
  sc.setup(a, inst, P.lane, false);
  sc.prep_good(0, P.lane, a.R);
  int32_t cr[W];
  pk_crash_rounds<W>(P, a, inst, cr);
  // A process decides and exits in the same round with decision = pick(t) (KSetAgreement.scala:
  // 48-50): its decide value is `decision`, its decide round is its halt round, and decided =
  // halted (halt_round >= 0) at every check point; decider is bit j of a flag word, with bit
  // 8 + j the decision's "not an initial value" (its X0 probe, taken when it decides). Fewer
  // live registers: 2 waves/SIMD with four 256-bit t masks per lane.
  int32_t x0[W], decision[W], halt_round[W];
  uint32_t fw = 0;
  Mask<W> t[W];
  int32_t xmin_l = INT32_MAX;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    x0[j] = 0;
    if (P.val[j])
      x0[j] = a.init ? init_x(a, i, inst, P.pid(j)) : sc.init_value(P.pid(j), PSG_ALG_KSET);
    L.x0s[P.pid(j)] = x0[j];
    if (P.val[j]) xmin_l = min(xmin_l, x0[j]);
    // t = Map(id -> io.initialValue); decider = false (KSetAgreement.scala:27-31)
    t[j] = mzero<W>();
    if (P.val[j]) t[j].w[j] = 1ull << P.lane;
    decision[j] = 0;
    halt_round[j] = -1;
  }
  X0Set<W> X0;
  pk_x0_build<W>(P, X0, x0lds, x0);  // ends with an LDS fence: x0s visible too
  const int32_t xmin = Grp<1>::dpp_reduce32<false>(xmin_l);
  uint32_t emin[W];
#pragma unroll
  for (int j = 0; j < W; ++j) emin[j] = P.val[j] & eq01(x0[j], xmin);
  const Mask<W> Emin = P.ballot(emin);
  Checks ck;
  ck.reset();
  auto check = [&](int c) {
    uint32_t decided[W], notinit[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      decided[j] = halt_round[j] >= 0 ? 1u : 0u;
      notinit[j] = (fw >> (8 + j)) & 1u;
    }
    pk_kagree_check_m<W>(P, ck, c, kk, decided, decision, cr, notinit);
  };
  check(0);
  pt.mark(0);
  Mask<W> act;
  {
    uint32_t al[W];
#pragma unroll
    for (int j = 0; j < W; ++j) al[j] = P.val[j];
    act = P.ballot(al);
  }
  // tuni: every alive process holds the same t. No round changes that (a merge's union and an
  // adoption are that t again), so from the first round it holds on the staging, the round-0
  // closed form and the classes / columns are skipped: same = |M|, t unchanged.
  bool tuni = false;
  const bool lazy = sc.drop == 0 && sc.ho_min < 0;  // crash-round survival words drawn on demand (below)
  // HAND: the rounds from the first with every alive t equal (or with every process halted) run
  // in kset_tail_kernel, whose live state fits twice the waves per SIMD; this kernel stores the
  // state that kernel needs and leaves the instance.
  auto handoff = [&](int k, int32_t pu, uint32_t punot) {
    uint32_t hr = 0;
#pragma unroll
    for (int j = 0; j < W; ++j) hr |= ((uint32_t)halt_round[j] & 0xFFu) << (8 * j);
    const uint32_t x = ((uint32_t)ck.ffv & 0xFFu) | ((fw & 0xF0Fu) << 8);
    a.hand_meta[i * 64 + (uint64_t)P.lane] = (uint64_t)x | ((uint64_t)hr << 32);
#pragma unroll
    for (int j = 0; j < W; ++j)
      if (P.val[j] && halt_round[j] >= 0) a.hand_dec[i * (uint64_t)a.n + (uint64_t)P.pid(j)] = decision[j];
    if (P.lane == 0) a.hand_hdr[i] = (uint64_t)((uint32_t)k | (punot << 8)) | ((uint64_t)(uint32_t)pu << 32);
    lds_sync<1>();  // x0s reads done before the next instance restages them
    pt.mark(3);
  };
  for (int k = 0; k < a.R; ++k) {
    // Once every process halted the state is frozen; the round has no step to take, but its
    // check point is still evaluated (every counted process-round is checked).
    const bool live = many(act);
    if constexpr (HAND) {
      if (!live) {
        handoff(k, 0, 0u);
        return;
      }
    }
    if (live) {
      Mask<W> goodS;
      const bool good = sc.good_round(k, P.lane, a.R, goodS);
      Mask<W> CB = mzero<W>(), CN = mzero<W>();
      if (sc.crash_on) {
#pragma unroll
        for (int j = 0; j < W; ++j) {
          CB.w[j] = __builtin_amdgcn_ballot_w64((uint32_t)cr[j] < (uint32_t)k);
          CN.w[j] = __builtin_amdgcn_ballot_w64(cr[j] == k);
        }
      }
      uint32_t dw[W];
#pragma unroll
      for (int j = 0; j < W; ++j) dw[j] = (fw >> j) & 1u;
      const Mask<W> Dm = mand(P.ballot(dw), act);  // senders' decider flags (pre-state)
      // round 0 (every alive sender still holds only its own origin): closed form below
      bool closed = false;
      if (!tuni) {
        uint32_t notown[W];
#pragma unroll
        for (int j = 0; j < W; ++j) {
          Mask<W> own = mzero<W>();
          if (P.val[j]) own.w[j] = 1ull << P.lane;
          notown[j] = meq(t[j], own) ? 0u : 1u;
        }
        closed = !many(mand(act, P.ballot(notown)));
      }
      // Every alive sender holding the same t (the common case once round 0 has spread the
      // origins) is one compare per slot against the first alive sender's t (read from its
      // lane) and a ballot; then tuni holds for the rest of the instance.
      if (!tuni && !closed) {
        const int q0 = mfirst(act), j0 = q0 >> 6, l0 = q0 & 63;
        Mask<W> t0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          t0.w[w] = readlane64(t[0].w[w], l0);
#pragma unroll
          for (int j = 1; j < W; ++j)
            if (j0 == j) t0.w[w] = readlane64(t[j].w[w], l0);
        }
        uint32_t dif = 0;
#pragma unroll
        for (int j = 0; j < W; ++j) dif |= (uint32_t)((act.w[j] >> P.lane) & 1ull) & (meq(t[j], t0) ? 0u : 1u);
        tuni = !pk_any(dif);
        if constexpr (HAND) {
          if (tuni) {  // every decision from here on is pick(t0); its X0 probe taken once
            const int32_t pu = kset_pick<W>(t0, L.x0s, Emin, xmin);
            handoff(k, pu, 1u - X0.contains01(pu));
            return;
          }
        }
      }
      // the pre-round t masks staged for the class reads and adoptions ([word][pid])
      const bool staged = !tuni && (!closed || many(Dm));
      uint64_t* ts = nullptr;
      if (staged) {
        ts = S.acquire(sbuf, P.lane);
#pragma unroll
        for (int j = 0; j < W; ++j)
#pragma unroll
          for (int w = 0; w < W; ++w) ts[w * 64 * W + P.pid(j)] = t[j].w[w];
        lds_sync<1>();
      }
      // The classes of equal t among the alive senders (same = mailbox.filter(_._2._2 == t).size,
      // uni = t ++ every received t) are the same for every receiver: found once per round (at
      // most kClasses; the rest, rem, is walked sender by sender), their t and member masks kept
      // in this wave's LDS, each slot's class index in cls (4 bits per slot, 15 = none). So the
      // receivers need only the pre-round staging, not their own pre-round t, and each slot's t
      // is updated in place (no second set of W x W mask words per lane).
      //
      // Column form (the common case, few origins vary): I = the origins every alive sender
      // holds, U = those some alive sender holds, D = U \ I the varying ones. Every alive t is
      // I + (t & D), so for a receiver p (alive, M its senders, all alive)
      //   uni  = t_p + {o in D : M meets H_o}                 H_o = {alive q : o in t_q}
      //   same = |M & Eq_p|,  Eq_p = AND over o in D of (o in t_p ? H_o : not H_o)
      // — |D| column steps per slot instead of a walk over the senders or their classes.
      int ncls = 0, ncols = 0;
      uint32_t cls = 0xFFFFu;
      Mask<W> rem = act, D = mzero<W>();
      const bool cols = !tuni && !closed;
      if (cols) {
        Mask<W> il, ul;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          il.w[w] = ~0ull;
          ul.w[w] = 0ull;
        }
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const bool s = (act.w[j] >> P.lane) & 1ull;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            il.w[w] &= s ? t[j].w[w] : ~0ull;
            ul.w[w] |= s ? t[j].w[w] : 0ull;
          }
        }
        Mask<W> I, U;
        pk_and_or<W>(il, ul, I, U);
        D = mandn(U, I);
        ncols = mpopc(D);
      }
      const bool colform = cols && ncols <= KsPk<W>::kCols;
      if (colform) {
        Mask<W> dd = D;
        for (int c = 0; c < ncols; ++c) {
          const int o = mtake_first(dd);
          uint32_t hb[W];
#pragma unroll
          for (int j = 0; j < W; ++j) hb[j] = mtest(t[j], o) ? 1u : 0u;
          const Mask<W> H = mand(P.ballot(hb), act);
#pragma unroll
          for (int w = 0; w < W; ++w)
            if (P.lane == w) L.hol[c][w] = H.w[w];
        }
        lds_sync<1>();
      } else if (cols) {
        for (; ncls < KsPk<W>::kClasses && many(rem); ++ncls) {
          const Mask<W> tq = load_t<W, 64 * W>(ts, mfirst(rem));
          uint32_t mine[W];
#pragma unroll
          for (int jj = 0; jj < W; ++jj) {
            mine[jj] = meq(t[jj], tq) ? 1u : 0u;
            if (mine[jj] && ((cls >> (4 * jj)) & 15u) == 15u) cls = (cls & ~(15u << (4 * jj))) | ((uint32_t)ncls << (4 * jj));
          }
          const Mask<W> E = mand(P.ballot(mine), rem);
          rem = mandn(rem, E);
          if (P.lane < W) {  // uniform values: lane w stores word w
#pragma unroll
            for (int w = 0; w < W; ++w)
              if (P.lane == w) {
                L.ct[ncls][w] = tq.w[w];
                L.ce[ncls][w] = E.w[w];
              }
          }
        }
        lds_sync<1>();
      }
      pt.mark(1);
      pt.add(0, 1);  // event-count builds: round paths (live, closed, uniform t, columns, classes)
      pt.add(1, closed);
      pt.add(2, tuni);
      pt.add(3, colform);
      pt.add(4, colform ? ncols : 0);
      pt.add(5, cols && !colform);
      pt.add(6, cols && !colform ? mpopc(rem) : 0);
      pt.add(7, many(CN));
      // one slot at a time (its HO set M, its merge or adoption)
      if (!HAND && tuni) {
        // Every sender's t is t_p, so a step reads its mailbox only through hc (some decider
        // heard) and same = |M| > need (KSetAgreement.scala:46-58), and t never changes (a
        // union or an adoption is t_p again). In a crash round (no benign loss, no ho_min) M
        // lies between Mlo (every crashing sender's message lost) and Mhi (all delivered); when
        // both bounds give the same hc and |M| > need for every live slot of the wave, the
        // round's survival words change nothing and are not drawn (each is a pure function of
        // (instance, round, pid): skipping one moves no other draw).
        const bool lazyr = lazy && many(CN);
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const bool halted = halt_round[j] >= 0;
          const uint32_t decider = (fw >> j) & 1u;
          const uint32_t live = P.val[j] & (halted ? 0u : 1u) & (1u - decider);
          uint32_t hc, big;
          bool exact = !lazyr;
          if (lazyr) {
            uint64_t one[W], zero[W];
#pragma unroll
            for (int w = 0; w < W; ++w) {
              one[w] = ~0ull;
              zero[w] = 0ull;
            }
            const Mask<W> Mhi = mand(sc.assemble(P.pid(j), good, goodS, CB, CN, one, one), act);
            const Mask<W> Mlo = mand(sc.assemble(P.pid(j), good, goodS, CB, CN, one, zero), act);
            const uint32_t hlo = many(mand(Mlo, Dm)) ? 1u : 0u, hhi = many(mand(Mhi, Dm)) ? 1u : 0u;
            const uint32_t plo = mpopc(Mlo) > need ? 1u : 0u, phi = mpopc(Mhi) > need ? 1u : 0u;
            hc = hlo;
            big = plo;
            // undetermined: hc open, or no decider heard for sure and |M| > need open
            exact = pk_any(live & ((hlo ^ hhi) | ((1u - hlo) & (plo ^ phi))));
          }
          if (exact) {
            const Mask<W> M = mand(sc.ho(k, P.pid(j), good, goodS, CB, CN), act);
            hc = many(mand(M, Dm)) ? 1u : 0u;
            big = mpopc(M) > need ? 1u : 0u;
          }
          pt.mark(6);  // (profiling builds: t6 = the slots' HO sets)
          if (!halted && decider) {  // decide(pick(t)); exitAtEndOfRound (KSetAgreement.scala:48-50)
            const int32_t v = kset_pick<W>(t[j], L.x0s, Emin, xmin);
            decision[j] = v;
            fw |= (1u - X0.contains01(v)) << (8 + j);
            halt_round[j] = k;
          }
          fw |= (live & (hc | big)) << j;  // adopts, or merges with same > n - k: decider
          pt.mark(2);
        }
      } else {
#pragma unroll
        for (int j = 0; j < W; ++j) {
          uint32_t becomeDec = 0;
          const bool halted = halt_round[j] >= 0;  // before this round (set below when it decides)
          const uint32_t decider = (fw >> j) & 1u;
          const Mask<W> M = mand(sc.ho(k, P.pid(j), good, goodS, CB, CN), act);
          pt.mark(6);
          const uint32_t live = P.val[j] & (halted ? 0u : 1u) & (1u - decider);
          const uint32_t hc = many(mand(M, Dm)) ? 1u : 0u;
          const uint32_t adopt = live & hc, mergep = live & (1u - hc);
          Mask<W> tnew = t[j];
          if (pk_any(mergep)) {
            int same = 0;
            Mask<W> uni = t[j];
            if (closed) {
              same = ((M.w[j] >> P.lane) & 1ull) ? 1 : 0;
              uni = mor(t[j], M);
            } else if (colform) {
              Mask<W> Eq = act, dd = D;
              for (int c = 0; c < ncols; ++c) {
                const int o = mtake_first(dd);
                Mask<W> H;
#pragma unroll
                for (int w = 0; w < W; ++w) H.w[w] = L.hol[c][w];
                const bool hit = many(mand(M, H));
                const uint64_t bit = 1ull << (o & 63);
                const bool mine = mtest(t[j], o);
#pragma unroll
                for (int w = 0; w < W; ++w) {
                  uni.w[w] |= (hit && (o >> 6) == w) ? bit : 0ull;
                  Eq.w[w] &= mine ? H.w[w] : ~H.w[w];
                }
              }
              same = mpopc(mand(M, Eq));
            } else {
              const int mc = (int)((cls >> (4 * j)) & 15u);
              for (int c = 0; c < ncls; ++c) {
                Mask<W> E, tq;
#pragma unroll
                for (int w = 0; w < W; ++w) {
                  E.w[w] = L.ce[c][w];
                  tq.w[w] = L.ct[c][w];
                }
                const Mask<W> ME = mand(M, E);
                if (c == mc) same = mpopc(ME);
                if (many(ME)) uni = mor(uni, tq);
              }
              Mask<W> rr = rem;
              while (many(rr)) {
                const int q = mtake_first(rr);
                const Mask<W> tq = load_t<W, 64 * W>(ts, q);
                if (mtest(M, q)) {
                  same += meq(tq, t[j]) ? 1 : 0;
                  uni = mor(uni, tq);
                }
              }
            }
            if (mergep) {
              if (same > need) becomeDec = 1;
              else tnew = uni;
            }
          }
          if (adopt) {  // t = content.find(_._1).get._2 — last decider message in iteration order
            tnew = load_t<W, 64 * W>(ts, kset_find<W, 64 * W>(a, ts, M, mand(M, Dm), colform ? L.hol : nullptr, ncols));
            becomeDec = 1;
          }
          if (!halted && decider) {  // decide(pick(t)); exitAtEndOfRound (KSetAgreement.scala:48-50)
            const int32_t v = kset_pick<W>(t[j], L.x0s, Emin, xmin);
            decision[j] = v;
            fw |= (1u - X0.contains01(v)) << (8 + j);
            halt_round[j] = k;
          }
          if (!halted) {  // the post-round state of slot j (its pre-round t is in the staging)
            t[j] = tnew;
            fw |= becomeDec << j;
          }
          pt.mark(2);
        }
      }
      if (staged) S.release(sbuf, P.lane);  // all reads of ts (and hol / ct / ce) done
      uint32_t al[W];
#pragma unroll
      for (int j = 0; j < W; ++j) {
        al[j] = P.val[j] & (halt_round[j] >= 0 ? 0u : 1u);
      }
      act = P.ballot(al);
      pt.mark(2);
    }
    check(k + 1);
    pt.mark(live ? 4 : 5);
  }
  int32_t mainx[W];
#pragma unroll
  for (int j = 0; j < W; ++j) mainx[j] = P.val[j] ? kset_pick<W>(t[j], L.x0s, Emin, xmin) : 0;
  pk_finish<W>(P, a, i, ck, 2, decision, halt_round, halt_round, mainx, bc);
  if constexpr (HAND) {
    if (P.lane == 0) a.hand_hdr[i] = kHandDone;
  }
  lds_sync<1>();  // x0s reads done before the next instance restages them
  pt.mark(3);
}

// The uniform-t tail of a handed-off instance (kset_packed<W, true>): every alive process holds
// the same t (or none is alive), so no round changes any t (a union of equal t's and an adoption
// are that t), every decision is pick(t) = pu, and a step reads its mailbox only through hc (some
// decider heard) and |M| > n - k (KSetAgreement.scala:46-58). The lane keeps its slots' decision,
// halt round and crash round and one flag word — no t masks, staging, classes, columns or X0 set —
// so the kernel runs at twice the general kernel's waves per SIMD. Every check point is evaluated.
// LAZY (no benign loss, no ho_min: the C4 schedules): HO(p) = B0 \ CB \ (CN \ survivors_p), plus
// p itself under the runtime's self delivery (Sched::assemble), so the mailboxes are uniform but
// for the self bit and, in a crash round, the crashing senders p hears.
template <int W, bool LAZY>
PSG_DEV void kset_tail(const Pk<W>& P, const KArgs& a, uint64_t i, uint64_t inst, uint64_t h, BlockCounters* bc,
                       PhaseTimers& pt) {
  const int n = a.n, kk = a.param;
  const int need = a.variant == 1 ? 1 : n - kk;  // same.size > n - k (KSetAgreement.scala:56)
  const int k0 = (int)(h & 0xFFu);
  const uint32_t punot = (uint32_t)(h >> 8) & 1u;
  const int32_t pu = (int32_t)(uint32_t)(h >> 32);
  Sched<W, false> sc;
  sc.setup(a, inst, P.lane, false);
  sc.prep_good(k0, P.lane, a.R);
  int32_t cr[W];
  pk_crash_rounds<W>(P, a, inst, cr);
  const uint64_t m = a.hand_meta[i * 64 + (uint64_t)P.lane];
  Checks ck;
  ck.ffv = (int32_t)(m & 0xFFu);
  uint32_t fw = ((uint32_t)m >> 8) & 0xF0Fu;  // decider bit j, not-initial bit 8 + j
  int32_t decision[W], halt_round[W];
  uint32_t al[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const uint32_t b = (uint32_t)(m >> (32 + 8 * j)) & 0xFFu;
    halt_round[j] = b == 0xFFu ? -1 : (int32_t)b;
    decision[j] = 0;
    if (P.val[j] && halt_round[j] >= 0) decision[j] = a.hand_dec[i * (uint64_t)n + (uint64_t)P.pid(j)];
    al[j] = P.val[j] & (halt_round[j] >= 0 ? 0u : 1u);
  }
  Mask<W> act = P.ballot(al);
  auto check = [&](int c) {
    uint32_t decided[W], notinit[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      decided[j] = halt_round[j] >= 0 ? 1u : 0u;
      notinit[j] = (fw >> (8 + j)) & 1u;
    }
    pk_kagree_check_m<W>(P, ck, c, kk, decided, decision, cr, notinit);
  };
  pt.mark(0);
  for (int k = k0; k < a.R; ++k) {
    const bool live = many(act);
    if (live) {
      Mask<W> goodS;
      const bool good = sc.good_round(k, P.lane, a.R, goodS);
      Mask<W> CB = mzero<W>(), CN = mzero<W>();
      if (sc.crash_on) {
#pragma unroll
        for (int j = 0; j < W; ++j) {
          CB.w[j] = __builtin_amdgcn_ballot_w64((uint32_t)cr[j] < (uint32_t)k);
          CN.w[j] = __builtin_amdgcn_ballot_w64(cr[j] == k);
        }
      }
      uint32_t dw[W];
#pragma unroll
      for (int j = 0; j < W; ++j) dw[j] = (fw >> j) & 1u;
      const Mask<W> Dm = mand(P.ballot(dw), act);  // senders' decider flags (pre-state)
      uint32_t hcb = 0, bigb = 0;                   // per slot j: hc (some decider heard), |M| > need
      if constexpr (LAZY) {
        // Ulo (every crashing sender lost) is uniform. In a crash round M lies between Ulo and
        // Uhi = Ulo + CNa: when both bounds give the same hc and |M| > need for every live slot
        // of the wave, the round's survival words change nothing and are not drawn (each is a pure
        // function of (instance, round, pid): skipping one moves no other draw); otherwise the
        // slot draws the survival words of the crashing senders' 64-pid words only (Sched::draw's
        // loss-free crash-round calls).
        const Mask<W> B0 = good ? goodS : sc.full;
        const Mask<W> Ulo = mand(mandn(B0, mor(CB, CN)), act);
        const Mask<W> CNa = mand(mand(B0, CN), act);
        const bool crashr = many(CNa);
        const int plo_u = mpopc(Ulo), phi_u = plo_u + mpopc(CNa);
        const bool hlo_u = many(mand(Ulo, Dm)), hhi_u = hlo_u || many(mand(CNa, Dm));
        const uint32_t selfb = sc.self_bit ? 1u : 0u;
        uint32_t und = 0;
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const uint32_t live_j = P.val[j] & (halt_round[j] >= 0 ? 0u : 1u) & (1u - ((fw >> j) & 1u));
          const uint32_t self = selfb & (uint32_t)(act.w[j] >> P.lane) & 1u;
          const uint32_t sd = self & (uint32_t)(Dm.w[j] >> P.lane);
          const uint32_t inlo = (uint32_t)(Ulo.w[j] >> P.lane) & 1u;
          const uint32_t hlo = (hlo_u ? 1u : 0u) | sd;
          const uint32_t plo = plo_u + (int)(self & (1u - inlo)) > need ? 1u : 0u;
          hcb |= hlo << j;
          bigb |= plo << j;
          if (crashr) {
            const uint32_t inhi = inlo | ((uint32_t)(CNa.w[j] >> P.lane) & 1u);
            const uint32_t hhi = (hhi_u ? 1u : 0u) | sd;
            const uint32_t phi = phi_u + (int)(self & (1u - inhi)) > need ? 1u : 0u;
            // undetermined: hc open, or no decider heard for sure and |M| > need open
            und |= (live_j & ((hlo ^ hhi) | ((1u - hlo) & (plo ^ phi)))) << j;
          }
        }
        if (crashr && pk_any(und)) {
          uint32_t cw = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) cw |= CNa.w[w] ? 1u << w : 0u;
#pragma unroll 1
          for (int j = 0; j < W; ++j) {  // one copy of the draw: the slot index is a loop variable
            if (!pk_any((und >> j) & 1u)) continue;
            const int pid = P.pid(j);
            Mask<W> S = mzero<W>();  // the crashing senders p hears
#pragma unroll
            for (int c2 = 0; 2 * c2 < W; ++c2) {
              if (!((cw >> (2 * c2)) & 3u)) continue;
              const U4 o = philox10((uint32_t)inst, (uint32_t)(inst >> 32), (uint32_t)k,
                                    (uint32_t)pid + ((uint32_t)c2 << 16), (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
              S.w[2 * c2] = CNa.w[2 * c2] & ((uint64_t)o.x | ((uint64_t)o.y << 32));
              if (2 * c2 + 1 < W) S.w[2 * c2 + 1] = CNa.w[2 * c2 + 1] & ((uint64_t)o.z | ((uint64_t)o.w << 32));
            }
            const bool self = selfb && mtest(act, pid);
            const Mask<W> M = mor(Ulo, S);
            const uint32_t hc = (many(mand(M, Dm)) || (self && mtest(Dm, pid))) ? 1u : 0u;
            const uint32_t big = mpopc(M) + ((self && !mtest(M, pid)) ? 1 : 0) > need ? 1u : 0u;
            hcb = (hcb & ~(1u << j)) | (hc << j);
            bigb = (bigb & ~(1u << j)) | (big << j);
          }
        }
      } else {  // the general schedule: each slot's HO set drawn in full (one copy of the draw)
#pragma unroll 1
        for (int j = 0; j < W; ++j) {
          const Mask<W> M = mand(sc.ho(k, P.pid(j), good, goodS, CB, CN), act);
          hcb |= (many(mand(M, Dm)) ? 1u : 0u) << j;
          bigb |= (mpopc(M) > need ? 1u : 0u) << j;
        }
      }
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const bool halted = halt_round[j] >= 0;
        const uint32_t decider = (fw >> j) & 1u;
        const uint32_t live_j = P.val[j] & (halted ? 0u : 1u) & (1u - decider);
        if (!halted && decider) {  // decide(pick(t)) = pu; exitAtEndOfRound (KSetAgreement.scala:48-50)
          decision[j] = pu;
          fw |= punot << (8 + j);
          halt_round[j] = k;
        }
        fw |= (live_j & ((hcb | bigb) >> j) & 1u) << j;  // adopts, or merges with same > n - k: decider
        al[j] = P.val[j] & (halt_round[j] >= 0 ? 0u : 1u);
      }
      act = P.ballot(al);
    }
    check(k + 1);
    pt.mark(live ? 4 : 5);
  }
  // final x = pick(t): a process halted before the hand-off (halt round < k0) decided pick of its
  // own (frozen) t, every other process holds the common t (formed here, not kept live across the
  // rounds: 4 VGPRs)
  int32_t mainx[W];
#pragma unroll
  for (int j = 0; j < W; ++j) mainx[j] = (halt_round[j] >= 0 && halt_round[j] < k0) ? decision[j] : pu;
  pk_finish<W>(P, a, i, ck, 2, decision, halt_round, halt_round, mainx, bc);
  pt.mark(3);
}

#ifndef PSG_KSET_PK_WPE
#define PSG_KSET_PK_WPE 3  // W = 4: four 256-bit t masks per lane; 2 -> 3 after the per-slot state diet: C4 f=1 2.80 -> 2.18 ms
#endif
#ifndef PSG_KSET_SPLIT
#define PSG_KSET_SPLIT 1  // 1: general rounds here, the uniform-t tail in kset_tail_kernel; 0: one kernel
#endif
template <int W, bool HAND>
__global__ void __launch_bounds__(64 * KsStage<W>::kWaves) __attribute__((amdgpu_waves_per_eu(PSG_KSET_PK_WPE)))
kset_packed_kernel(KArgs a) {
  static_assert(64 * KsStage<W>::kWaves == 256, "launched with 256-thread blocks (launch_w)");
  __shared__ BlockCounters bc;
  __shared__ KsPk<W> L[KsStage<W>::kWaves];
  __shared__ KsStage<W> S;
  __shared__ int32_t x0tab[4][X0Set<W>::kSlots];
  counters_init(&bc);
  S.init();
  __syncthreads();
  Pk<W> P;
  P.setup(a.n);
  const int grp = threadIdx.x >> 6;
  PhaseTimers pt;  // profiling builds only: t0 setup, t1 staging + classes, t2 slot updates, t3 finish,
  pt.start();      // t4 check after a live round, t5 frozen round, t6 the slots' HO sets
  InstanceQueue<1> Q;
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    kset_packed<W, HAND>(P, a, i, inst, L[grp], S, grp * KsStage<W>::kBufs / KsStage<W>::kWaves, x0tab[grp], &bc, pt);
  }
  pt.flush(a.counters, P.lane);
  __syncthreads();
  counters_flush(&bc, a.counters, 2, a.R);
}

#ifndef PSG_KSET_TAIL_WPE
#define PSG_KSET_TAIL_WPE 6  // waves/SIMD of the uniform-t tail kernel
#endif
template <int W, bool LAZY>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LAZY ? PSG_KSET_TAIL_WPE : 4))) kset_tail_kernel(KArgs a) {
  __shared__ BlockCounters bc;
  counters_init(&bc);
  __syncthreads();
  Pk<W> P;
  P.setup(a.n);
  PhaseTimers pt;  // profiling builds only: t0 setup, t3 finish, t4 check after a live round, t5 frozen round
  pt.start();
  InstanceQueue<1, 1> Q;  // the second queue region (the general kernel drained the first)
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t h = a.hand_hdr[i];
    if (h & kHandDone) continue;  // finished by the general kernel
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    kset_tail<W, LAZY>(P, a, i, inst, h, &bc, pt);
  }
  pt.flush(a.counters, P.lane);
  __syncthreads();
  counters_flush(&bc, a.counters, 2, a.R);
}

// Kernel body; SH = NoHook for the library's kernels, spec::SpecHook<GenSpec> in a
// fused Spec module (round_amd/formula.py compile_native(fused=True)).
template <int W, bool XHO, class SH = NoHook>
PSG_DEV void kset_body(const KArgs& a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int32_t crl[W > 1 ? 64 * W : 1];
  __shared__ int64_t red[2 * W];
  __shared__ KsLds<W> L;
  __shared__ int32_t x0tab[Geometry<W>::kGroups][X0Set<W>::kSlots];
  counters_init(&bc);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = a.n;
  const int kk = a.param;
  const int need = a.variant == 1 ? 1 : n - kk;  // same.size > n - k (KSetAgreement.scala:56)
  const Mask<W> full = mfull<W>(n);
  uint64_t* ts = L.ts[grp];
  int32_t* x0s = L.x0s[grp];
  int32_t* ds = L.ds[grp];

  PhaseTimers pt;  // profiling builds only: t0 setup, t1 HO sets, t2 update, t3 finish, t4 check, t5 frozen round
  pt.start();
  InstanceQueue<W> Q;  // dynamic instance distribution (psg_device.hpp)
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    Sched<W, XHO> sc;
    sc.setup(a, inst, g.pid, g.valid);
    CrashSets<W> cs;  // per-instance crash rounds (no per-round exchange for W > 1)
    if (sc.crash_on) cs.prep(g, crl, sc.crash_round);
    sc.prep_good(0, g.lane, a.R);
    const bool crashed = sc.crash_round >= 0;
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? init_x(a, i, inst, g.pid) : sc.init_value(g.pid, PSG_ALG_KSET);
    x0s[g.pid] = x0;
    X0Set<W> X0;
    X0.build(g, x0tab[grp], x0);
    const int32_t xmin = g.min32(x0, true);
    const Mask<W> Emin = g.ballot(x0 == xmin);
    // t = Map(id -> io.initialValue); decider = false (KSetAgreement.scala:27-31)
    Mask<W> t = mzero<W>();
    if (g.valid) mset(t, g.pid);
    bool decider = false, decided = false, halted = false;
    int32_t decision = 0, dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    typename SH::template State<W> sh(g, grp, n);  // fused Spec evaluation state (NoHook: empty)
    auto check = [&](int c) {
      ds[g.pid] = decision;
      lds_sync<W>();
      kagree_check<W>(g, ck, c, kk, full, decided, decision, X0, crashed, ds);
    };
    if constexpr (!SH::kFused) check(0);
    auto trace = [&](int c, int32_t hs) {
      emit_state<W, SH>(sh, g, a, i, c, kset_pick<W>(t, x0s, Emin, xmin), decided ? 1 : 0, decision, 0, 0, 0, 0, 0, hs);
    };
    if (tracing<SH>(a)) trace(0, n);
    pt.mark(0);
    for (int k = 0; k < a.R; ++k) {
      const Mask<W> act = g.ballot(!halted);
      int32_t hs = n;  // |mailbox| of this round (Spec field HOSIZE)
      if (many(act)) {
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) cs.sets(g, k, CB, CN);
        const Mask<W> M = mand(sc.ho(k, g.pid, good, goodS, CB, CN), act);
        pt.mark(1);
        if (tracing<SH>(a) && !halted) hs = mpopc(M);
        const Mask<W> Dm = mand(g.ballot(decider), act);  // senders' decider flags (pre-state)
#pragma unroll
        for (int w = 0; w < W; ++w) ts[g.pid * W + w] = t.w[w];
        lds_sync<W>();
        const Mask<W> cand = mand(M, Dm);
        const bool isDec = decider;
        const bool adopt = !halted && !isDec && many(cand);
        const bool mergep = !halted && !isDec && !many(cand);
        Mask<W> tnew = t;
        bool becomeDecider = false;
        if (g.any(mergep)) {
          // same = mailbox.filter(_._2._2 == t).size; uni = t ++ every received t. The alive
          // senders are taken class by class (equal t, one ballot per class: a class's t is
          // read once, and same = |M & class of t|), at most kClasses classes; senders left
          // after that are walked one by one. Round 0 (every alive sender still holds only
          // its own origin) is closed form: same = [p in M], uni = t | M.
          constexpr int kClasses = 8;
          int same = 0;
          Mask<W> uni = t;
          Mask<W> rem = act;
          Mask<W> own = mzero<W>();
          if (g.valid) mset(own, g.pid);
          if (!many(mand(act, g.ballot(!meq(t, own))))) {
            same = mtest(M, g.pid) ? 1 : 0;
            uni = mor(t, M);
            rem = mzero<W>();
          }
          for (int cls = 0; cls < kClasses && many(rem); ++cls) {
            const Mask<W> tq = load_t<W>(ts, mfirst(rem));
            const bool mine = meq(t, tq);
            const Mask<W> E = mand(g.ballot(mine), rem);
            rem = mandn(rem, E);
            const Mask<W> ME = mand(M, E);
            if (mine) same = mpopc(ME);
            if (many(ME)) uni = mor(uni, tq);
          }
#pragma unroll
          for (int w = 0; w < W; ++w) {
            uint64_t m = rem.w[w];
            while (m) {
              const int q = w * 64 + __builtin_ctzll(m);
              m &= m - 1;
              const Mask<W> tq = load_t<W>(ts, q);
              if (mtest(M, q)) {
                same += meq(tq, t) ? 1 : 0;
                uni = mor(uni, tq);
              }
            }
          }
          if (mergep) {
            if (same > need) becomeDecider = true;
            else tnew = uni;
          }
        }
        if (adopt) {
          // t = content.find(_._1).get._2 — last decider message in iteration order
          tnew = load_t<W>(ts, kset_find<W>(a, ts, M, cand));
          becomeDecider = true;
        }
        if (!halted && isDec) {  // decide(pick(t)); exitAtEndOfRound (KSetAgreement.scala:48-50)
          const int32_t v = kset_pick<W>(t, x0s, Emin, xmin);
          dec_val = v;
          dec_round = k;
          decided = true;
          decision = v;
          halt_round = k;
        }
        lds_sync<W>();  // all reads of ts done before the next round restages it
        if (!halted) {
          t = tnew;
          if (becomeDecider) decider = true;
        }
        if (halt_round == k) halted = true;
      }
      pt.mark(2);
      if constexpr (!SH::kFused) check(k + 1);
      if (tracing<SH>(a)) trace(k + 1, hs);
      pt.mark(many(act) ? 4 : 5);
    }
    const int32_t mainx = g.valid ? kset_pick<W>(t, x0s, Emin, xmin) : 0;
    finish_instance<W>(g, a, i, SH::kFused ? sh.ck : ck, SH::kFused ? SH::kSlots : 2, dec_val, dec_round, halt_round, mainx, &bc);
    lds_sync<W>();
    pt.mark(3);
  }
  pt.flush(a.counters, threadIdx.x & 63);
  __syncthreads();
  counters_flush(&bc, a.counters, SH::kFused ? SH::kSlots : 2, a.R);
}

#ifndef PSG_KSET_WPE
#define PSG_KSET_WPE 4  // W = 4 (C4): 4 waves/SIMD measured 1.2x over the register-bound 3; 5 spills
#endif
template <int W, bool XHO, class SH = NoHook>
__global__ void __launch_bounds__(Geometry<W>::kThreads) __attribute__((amdgpu_waves_per_eu(W == 1 ? 1 : PSG_KSET_WPE)))
kset_kernel(KArgs a) {
  kset_body<W, XHO, SH>(a);
}

#ifndef PSG_FUSED_MODULE  // host launchers (not part of a fused Spec module)
template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if constexpr (W > 1) {  // seeded schedule, built-in checker: lane-packed path
    if (!a.ho_in && !a.trace) {
      if (PSG_KSET_SPLIT && a.hand_hdr) {  // general rounds, then the uniform-t tail (same stream)
        const int pg = pk_grid<PSG_ALG_KSET, W>((const void*)kset_packed_kernel<W, true>, a.count);
        hipLaunchKernelGGL((kset_packed_kernel<W, true>), dim3(pg), dim3(256), 0, s, a);
        if (a.drop_log2 == 0 && a.ho_min < 0) {  // loss-free schedules: uniform mailboxes but crash rounds
          const int tg = pk_grid<PSG_ALG_KSET | 0x100, W>((const void*)kset_tail_kernel<W, true>, a.count);
          hipLaunchKernelGGL((kset_tail_kernel<W, true>), dim3(tg), dim3(256), 0, s, a);
        } else {
          const int tg = pk_grid<PSG_ALG_KSET | 0x300, W>((const void*)kset_tail_kernel<W, false>, a.count);
          hipLaunchKernelGGL((kset_tail_kernel<W, false>), dim3(tg), dim3(256), 0, s, a);
        }
        return hipGetLastError();
      }
      const int pg = pk_grid<PSG_ALG_KSET | 0x200, W>((const void*)kset_packed_kernel<W, false>, a.count);
      hipLaunchKernelGGL((kset_packed_kernel<W, false>), dim3(pg), dim3(256), 0, s, a);
      return hipGetLastError();
    }
  }
  if (a.ho_in) hipLaunchKernelGGL((kset_kernel<W, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((kset_kernel<W, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_kset(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1>(a, grid, s);
    case 2: return launch_w<2>(a, grid, s);
    case 3: return launch_w<3>(a, grid, s);
    case 4: return launch_w<4>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

const void* kset_kernel_ptr(int W) {
  switch (W) {
    case 1: return (const void*)kset_kernel<1, false>;
    case 2: return (const void*)kset_kernel<2, false>;
    case 3: return (const void*)kset_kernel<3, false>;
    case 4: return (const void*)kset_kernel<4, false>;
  }
  return nullptr;
}

#endif  // PSG_FUSED_MODULE

}  // namespace psg
