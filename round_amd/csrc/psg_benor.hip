// psg_benor.hip — Ben-Or randomized binary consensus on gfx950.
//
// Reference: example/BenOr.scala:11-84 (BenOrProcess), 91-115 (spec).
// Payloads are one or two bits per process, so every mailbox statistic is a
// popcount of HO(p) & alive & ballot(bit). The unseeded coin
// `util.Random.nextBoolean` (BenOr.scala:77) is java.util.Random's first
// nextBoolean after setSeed(Philox(seed, instance, round, pid)).
// n = 128 runs as W = 2 waves per instance with the ballot words exchanged in LDS.
#ifndef __HIPCC_RTC__
#include <type_traits>
#endif

#include "psg_device.hpp"
#include "psg_kernels.hpp"
#include "psg_packed.hpp"

namespace psg {

// Slots: 0 Safety, 1 Invariant0 (with roundInvariants(0)(0) after R0),
// 2 Agreement, 3 Irrevocability, 4 SafetyPredicate (|HO(p)| > n/2 on the
// effective heard-of sets, BenOr.scala:92).
template <int W>
PSG_DEV void benor_check(Grp<W>& g, Checks& ck, int c, bool has_old, int n, const Mask<W>& full, bool x, bool cd,
                         int vote, bool decided, bool decision, bool old_decided, bool old_decision, bool pred) {
  // every quantified witness in two ballot exchanges (W > 1: two LDS barriers instead
  // of one per P.exists / P.forall); the second depends on the counts of the first
  const bool p1[6] = {decided || cd, x, (decided && decision) || vote == 1, (decided && !decision) || vote == 0,
                      decided && decision, decided && !decision};
  Mask<W> m1[6];
  g.template ballots<6>(p1, m1);
  const bool noDec = !many(m1[0]);
  const int cntT = mpopc(m1[1]);
  const int cntF = n - cntT;
  bool ex = false;
  if (cntF > n / 2) ex = ex || !many(m1[2]);
  if (cntT > n / 2) ex = ex || !many(m1[3]);
  // after R0 (c odd): P.forall(p => p.vote.isDefined ==> |{i : i.x == p.vote.get}| > n/2)
  const bool p2[3] = {decided, (c & 1) != 0 && ((vote == 1 && !(cntT > n / 2)) || (vote == 0 && !(cntF > n / 2))),
                      has_old && old_decided && !(decided && old_decision == decision)};
  Mask<W> m2[3];
  g.template ballots<3>(p2, m2);
  const bool inv0 = (noDec || ex) && !many(m2[1]);
  const Mask<W> D = m2[0];
  const bool same = !(many(m1[4]) && many(m1[5]));
  const bool irrev = !many(m2[2]);
  const uint32_t fb = fbit(inv0, 0) |
                      fbit(inv0, 1) |
                      fbit(same, 2) |
                      fbit(irrev, 3) |
                      fbit(pred, 4);
  ck.record(fb, meq(D, full), c, g.lane);
}

// ---------------------------------------------------------------- one exchange per round
// The built-in checker and the round step share ONE cross-wave exchange per round
// (the general path below pays four: the round's alive ballot, its pre-state
// ballots and two for the Spec check). At check point c each wave publishes
//   - a summary word: its popcounts of x and of decided, and one "some process"
//     flag per quantified witness of the Spec, plus the SafetyPredicate witness
//     (|HO(p)| <= n/2 on the effective sets) of the round just executed;
//   - the masks the next round's mailbox statistics need: alive, and x / canDecide
//     (next round R0) or vote == Some(true) / Some(false) (next round R1).
// The Spec is evaluated as benor_check does; its roundInvariant witness "vote defined
// and |{i : i.x == vote.get}| <= n/2" is "(|x| <= n/2 and some vote is Some(true)) or
// (|!x| <= n/2 and some vote is Some(false))", |x| being the same for every process.
template <int W>
struct BoXch {
  uint64_t sum[W];   // popc(x) | popc(decided) << 16 | witness flags << 32, per wave
  uint64_t m[3][W];  // alive, x or vote == 1, canDecide or vote == 0
};

template <int W, class SC>
PSG_DEV void benor_fast(Grp<W>& g, const KArgs& a, uint64_t i, SC& sc, CrashSets<W>& cs, BoXch<W> (&X)[2],
                        int32_t x0, BlockCounters* bc) {
  const int n = a.n;
  const int thr = a.variant == 1 ? n / 4 : n / 2;  // BenOr.scala:68, 71 (variant 1: mutation)
  bool x = x0 != 0, cd = false, decided = false, decision = false, halted = false;
  int vote = -1;  // Option[Boolean]: -1 None, 0 Some(false), 1 Some(true)
  bool old_decided = false, old_decision = false;
  bool predw = false;  // this process broke the SafetyPredicate in the round just executed
  int32_t dec_val = 0, dec_round = -1, halt_round = -1;
  Checks ck;
  ck.reset();
  Mask<W> act, T1, T2;  // the next round's alive set and payload masks
  auto check = [&](int c, bool has_old) {
    const bool r0next = (c & 1) == 0;  // round c is an R0
    const bool fl[9] = {decided || cd, (decided && decision) || vote == 1, (decided && !decision) || vote == 0,
                        decided && decision, decided && !decision, vote == 1, vote == 0,
                        has_old && old_decided && !(decided && old_decision == decision), predw};
    uint32_t flags = 0;
#pragma unroll
    for (int b = 0; b < 9; ++b) flags |= (__builtin_amdgcn_ballot_w64(g.valid && fl[b]) != 0ull) ? 1u << b : 0u;
    const uint64_t bx = __builtin_amdgcn_ballot_w64(g.valid && x);
    const uint64_t bd = __builtin_amdgcn_ballot_w64(g.valid && decided);
    const uint64_t mw[3] = {__builtin_amdgcn_ballot_w64(g.valid && !halted),
                            __builtin_amdgcn_ballot_w64(g.valid && (r0next ? x : vote == 1)),
                            __builtin_amdgcn_ballot_w64(g.valid && (r0next ? cd : vote == 0))};
    int cntT = __popcll(bx), cntD = __popcll(bd);
    if constexpr (W == 1) {
      act.w[0] = mw[0];
      T1.w[0] = mw[1];
      T2.w[0] = mw[2];
    } else {
      BoXch<W>& e = X[c & 1];
      if (g.lane == 0) {
        e.sum[g.wv] = (uint64_t)cntT | ((uint64_t)cntD << 16) | ((uint64_t)flags << 32);
        e.m[0][g.wv] = mw[0];
        e.m[1][g.wv] = mw[1];
        e.m[2][g.wv] = mw[2];
      }
      __syncthreads();
      cntT = 0;
      cntD = 0;
      flags = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const uint64_t sw = rfl64(e.sum[w]);
        cntT += (int)(sw & 0xFFFFu);
        cntD += (int)((sw >> 16) & 0xFFFFu);
        flags |= (uint32_t)(sw >> 32);
        act.w[w] = rfl64(e.m[0][w]);
        T1.w[w] = rfl64(e.m[1][w]);
        T2.w[w] = rfl64(e.m[2][w]);
      }
    }
    const int cntF = n - cntT;
    const bool noDec = !(flags & 1u);
    const bool ex = (cntF > n / 2 && !(flags & 2u)) || (cntT > n / 2 && !(flags & 4u));
    const bool rfail = (c & 1) != 0 && ((!(cntT > n / 2) && (flags & 32u)) || (!(cntF > n / 2) && (flags & 64u)));
    const bool inv0 = (noDec || ex) && !rfail;
    const bool same = !((flags & 8u) && (flags & 16u));
    const bool irrev = !(flags & 128u);
    const bool pred = !(flags & 256u);
    ck.record(fbit(inv0, 0) | fbit(inv0, 1) | fbit(same, 2) | fbit(irrev, 3) | fbit(pred, 4), cntD == n, c, g.lane);
  };
  check(0, false);
  for (int k = 0; k < a.R; ++k) {
    old_decided = decided;
    old_decision = decision;
    predw = false;
    if (many(act)) {
      Mask<W> goodS;
      const bool good = sc.good_round(k, g.lane, a.R, goodS);
      Mask<W> CB = mzero<W>(), CN = mzero<W>();
      if (sc.crash_on) cs.sets(g, k, CB, CN);
      const Mask<W> M = mand(sc.template ho<false>(k, g.pid, good, goodS, CB, CN), act);
      const int size = mpopc(M);
      predw = !halted && size <= n / 2;
      if ((k & 1) == 0) {  // R0: broadcast (x, canDecide) — BenOr.scala:31-53
        const Mask<W> Tm = mand(T1, act);
        const Mask<W> CDm = mand(T2, act);
        if (!halted) {
          if (cd) {
            dec_val = x ? 1 : 0;
            dec_round = k;
            decided = true;
            decision = x;
            halt_round = k;
          } else {
            const Mask<W> MT = mand(M, Tm);
            const int cT = mpopc(MT);
            const int cF = size - cT;
            const bool exT = many(mand(MT, CDm));
            const bool exF = many(mand(mandn(M, Tm), CDm));
            if (cT > n / 2 || exT) vote = 1;
            else if (cF > n / 2 || exF) vote = 0;
            else vote = -1;
            cd = many(mand(M, CDm));
          }
        }
      } else {  // R1: broadcast vote — BenOr.scala:57-79
        const Mask<W> VT = mand(T1, act);
        const Mask<W> VF = mand(T2, act);
        if (!halted) {
          const int t = mpopc(mand(M, VT));
          const int f = mpopc(mand(M, VF));
          if (t > thr) {
            x = true;
            cd = true;
          } else if (f > thr) {
            x = false;
            cd = true;
          } else if (t > 1) {
            x = true;
          } else if (f > 1) {
            x = false;
          } else {
            x = sc.coin(k, g.pid);
          }
        }
      }
      if (halt_round == k) halted = true;
    }
    check(k + 1, true);
  }
  finish_instance<W>(g, a, i, ck, 5, dec_val, dec_round, halt_round, x ? 1 : 0, bc);
}

// ---------------------------------------------------------------- built-in checker, lane-packed
// benor_fast for n > 64 with one wave per instance, the W processes l + 64 j in lane l
// (psg_packed.hpp): the Spec's existential witnesses are one wave OR of a per-lane flag
// word (the lane's OR over its slots), the counts and the next round's payload masks
// are wave ballots, and no round needs a barrier.
#ifndef PSG_BO_FLAGS_DPP
#define PSG_BO_FLAGS_DPP 1  // one DPP OR of the flag word; 9 ballots measured 2 % slower (C5)
#endif
template <int W>
PSG_DEV void benor_packed(const Pk<W>& P, const KArgs& a, uint64_t i, uint64_t inst, BlockCounters* bc) {
  const int n = a.n;
  const int thr = a.variant == 1 ? n / 4 : n / 2;  // BenOr.scala:68, 71 (variant 1: mutation)
  Sched<W, false> sc;
  sc.setup(a, inst, P.lane, false);  // uniform parts; crash rounds per slot below
  sc.prep_good(0, P.lane, a.R);
  int32_t cr[W];
  pk_crash_rounds<W>(P, a, inst, cr);
  // BenOrProcess state after init(io) (BenOr.scala:13-28), 0/1 words per slot
  uint32_t x[W], cd[W], decided[W], decision[W], halted[W], old_decided[W], old_decision[W], predw[W];
  int32_t vote[W];  // Option[Boolean]: -1 None, 0 Some(false), 1 Some(true)
  int32_t dec_val[W], dec_round[W], halt_round[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    int32_t x0 = 0;
    if (P.val[j])
      x0 = a.init ? a.init[init_row(a, i, inst) * (uint64_t)n + P.pid(j)] : sc.init_value(P.pid(j), PSG_ALG_BENOR);
    x[j] = x0 != 0 ? 1u : 0u;
    cd[j] = decided[j] = decision[j] = halted[j] = old_decided[j] = old_decision[j] = predw[j] = 0;
    vote[j] = -1;
    dec_val[j] = 0;
    dec_round[j] = -1;
    halt_round[j] = -1;
  }
  Checks ck;
  ck.reset();
  Mask<W> act, T1, T2;  // the next round's alive set and payload masks
  // check point c (parity CP = c & 1 at compile time: round c is an R0 iff CP == 0)
  auto check = [&](int c, bool has_old, auto CPc) {
    constexpr int CP = decltype(CPc)::value;
    constexpr bool r0next = CP == 0;
    uint32_t fw = 0;                   // bit b: the Spec witness b holds for some process of the lane
    uint32_t al[W], t1[W], t2[W], xs[W], ds[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const uint32_t v = P.val[j];
      const uint32_t v1 = eq01(vote[j], 1), v0 = eq01(vote[j], 0);
      const uint32_t dT = decided[j] & decision[j], dF = decided[j] & (1u - decision[j]);
      const uint32_t irr = (has_old ? 1u : 0u) & old_decided[j] & (1u - (decided[j] & eq01((int32_t)old_decision[j], (int32_t)decision[j])));
      const uint32_t w = (decided[j] | cd[j]) | ((dT | v1) << 1) | ((dF | v0) << 2) | (dT << 3) | (dF << 4) | (v1 << 5) |
                         (v0 << 6) | (irr << 7) | (predw[j] << 8);
      fw |= v ? w : 0u;
      al[j] = v & (1u - halted[j]);
      t1[j] = v & (r0next ? x[j] : v1);
      t2[j] = v & (r0next ? cd[j] : v0);
      xs[j] = v & x[j];
      ds[j] = v & decided[j];
    }
#if PSG_BO_FLAGS_DPP
    const uint32_t flags = wave_or(fw);
#else
    uint32_t flags = 0;
#pragma unroll
    for (int b = 0; b < 9; ++b) flags |= pk_any((fw >> b) & 1u) ? 1u << b : 0u;
#endif
    act = P.ballot(al);
    T1 = P.ballot(t1);
    T2 = P.ballot(t2);
    const int cntT = mpopc(P.ballot(xs)), cntD = mpopc(P.ballot(ds));
    const int cntF = n - cntT;
    const bool noDec = !(flags & 1u);
    const bool ex = (cntF > n / 2 && !(flags & 2u)) || (cntT > n / 2 && !(flags & 4u));
    const bool rfail = CP != 0 && ((!(cntT > n / 2) && (flags & 32u)) || (!(cntF > n / 2) && (flags & 64u)));
    const bool inv0 = (noDec || ex) && !rfail;
    const bool same = !((flags & 8u) && (flags & 16u));
    const bool irrev = !(flags & 128u);
    const bool pred = !(flags & 256u);
    ck.record(fbit(inv0, 0) | fbit(inv0, 1) | fbit(same, 2) | fbit(irrev, 3) | fbit(pred, 4), cntD == n, c, P.lane);
  };
  check(0, false, Slot<0>{});
  // one round of slot RS = k & 1 (compile time: the R0 / R1 step and the next check specialized)
  auto round = [&](const int k, auto RSc) {
    constexpr int RS = decltype(RSc)::value;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      old_decided[j] = decided[j];
      old_decision[j] = decision[j];
      predw[j] = 0;
    }
    if (many(act)) {
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
      constexpr bool even = RS == 0;
      const Mask<W> A1 = mand(T1, act), A2 = mand(T2, act);  // R0: x / canDecide; R1: vote true / false
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if (halted[j]) continue;  // a halted process neither receives nor updates
        const Mask<W> M = mand(sc.template ho<false>(k, P.pid(j), good, goodS, CB, CN), act);
        const int size = mpopc(M);
        predw[j] = P.val[j] & (size <= n / 2 ? 1u : 0u);
        if constexpr (even) {  // R0: broadcast (x, canDecide) — BenOr.scala:31-53
          if (cd[j]) {
            dec_val[j] = (int32_t)x[j];
            dec_round[j] = k;
            decided[j] = 1;
            decision[j] = x[j];
            halt_round[j] = k;
          } else {
            const Mask<W> MT = mand(M, A1);
            const int cT = mpopc(MT);
            const int cF = size - cT;
            const bool exT = many(mand(MT, A2));
            const bool exF = many(mand(mandn(M, A1), A2));
            vote[j] = (cT > n / 2 || exT) ? 1 : ((cF > n / 2 || exF) ? 0 : -1);
            cd[j] = many(mand(M, A2)) ? 1u : 0u;
          }
        } else {  // R1: broadcast vote — BenOr.scala:57-79
          const int t = mpopc(mand(M, A1));
          const int f = mpopc(mand(M, A2));
          if (t > thr) {
            x[j] = 1;
            cd[j] = 1;
          } else if (f > thr) {
            x[j] = 0;
            cd[j] = 1;
          } else if (t > 1) {
            x[j] = 1;
          } else if (f > 1) {
            x[j] = 0;
          } else {
            x[j] = sc.coin(k, P.pid(j)) ? 1u : 0u;
          }
        }
        if (halt_round[j] == k) halted[j] = 1;
      }
    }
    check(k + 1, true, Slot<(RS + 1) & 1>{});
  };
  for (int k0 = 0; k0 < a.R; k0 += 2) {
    round(k0, Slot<0>{});
    if (k0 + 1 < a.R) round(k0 + 1, Slot<1>{});
  }
  int32_t fx[W];
#pragma unroll
  for (int j = 0; j < W; ++j) fx[j] = (int32_t)x[j];
  pk_finish<W, false>(P, a, i, ck, 5, dec_val, dec_round, halt_round, fx, bc);
}

#ifndef PSG_BO_PK_WPE
#define PSG_BO_PK_WPE 4  // parity-specialized loop: 4 waves/SIMD (no scratch) 37.9 ms vs 5: 38.4 (C5)
#endif
template <int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PSG_BO_PK_WPE))) benor_packed_kernel(KArgs a) {
  __shared__ BlockCounters bc;
  counters_init(&bc);
  __syncthreads();
  Pk<W> P;
  P.setup(a.n);
  InstanceQueue<1> Q;
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    benor_packed<W>(P, a, i, inst, &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, 5, a.R);
}

// Kernel body; SH = NoHook for the library's kernels, spec::SpecHook<GenSpec> in a
// fused Spec module (round_amd/formula.py compile_native(fused=True)).
template <int W, bool XHO, class SH = NoHook>
PSG_DEV void benor_body(const KArgs& a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int32_t crl[W > 1 ? 64 * W : 1];
  __shared__ int64_t red[2 * W];
  __shared__ BoXch<W> BX[2];
  counters_init(&bc);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = a.n;
  const int thr = a.variant == 1 ? n / 4 : n / 2;  // BenOr.scala:68, 71 (variant 1: mutation)
  const Mask<W> full = mfull<W>(n);

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
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? init_x(a, i, inst, g.pid) : sc.init_value(g.pid, PSG_ALG_BENOR);
    if constexpr (!SH::kFused) {
      if (a.trace == nullptr) {  // built-in checker: one exchange per round
        benor_fast<W>(g, a, i, sc, cs, BX, x0, &bc);
        continue;
      }
    }
    // BenOrProcess state after init(io) (BenOr.scala:13-28); vote starts as None
    bool x = x0 != 0, cd = false, decided = false, decision = false, halted = false;
    int vote = -1;  // Option[Boolean]: -1 None, 0 Some(false), 1 Some(true)
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    typename SH::template State<W> sh(g, grp, n);  // fused Spec evaluation state (NoHook: empty)
    if constexpr (!SH::kFused) benor_check<W>(g, ck, 0, false, n, full, x, cd, vote, decided, decision, false, false, true);
    // vote: Option[Boolean] (PSG_NONE32 when empty)
    auto trace = [&](int c, int32_t hs) {
      emit_state<W, SH>(sh, g, a, i, c, x ? 1 : 0, decided ? 1 : 0, decision ? 1 : 0, 0, 0, 0, vote < 0 ? PSG_NONE32 : vote,
                   cd ? 1 : 0, hs);
    };
    if (tracing<SH>(a)) trace(0, n);
    pt.mark(0);
    for (int k = 0; k < a.R; ++k) {
      const bool old_decided = decided, old_decision = decision;
      const Mask<W> act = g.ballot(!halted);
      bool pred = true;
      int32_t hs = n;  // |mailbox| of this round (Spec field HOSIZE)
      if (many(act)) {
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) cs.sets(g, k, CB, CN);
        const Mask<W> M = mand(sc.template ho<false>(k, g.pid, good, goodS, CB, CN), act);
        const int size = mpopc(M);
        pt.mark(1);
        if (!halted) hs = size;
        // the round's pre-state ballots and the SafetyPredicate witness share one exchange
        const bool even = (k & 1) == 0;
        const bool pr[3] = {!halted && size <= n / 2, even ? x : vote == 1, even ? cd : vote == 0};
        Mask<W> pm[3];
        g.template ballots<3>(pr, pm);
        pred = !many(pm[0]);
        if (even) {  // R0: broadcast (x, canDecide) — BenOr.scala:31-53
          const Mask<W> Tm = mand(pm[1], act);
          const Mask<W> CDm = mand(pm[2], act);
          if (!halted) {
            if (cd) {
              dec_val = x ? 1 : 0;
              dec_round = k;
              decided = true;
              decision = x;
              halt_round = k;
            } else {
              const Mask<W> MT = mand(M, Tm);
              const int cT = mpopc(MT);
              const int cF = size - cT;
              const bool exT = many(mand(MT, CDm));
              const bool exF = many(mand(mandn(M, Tm), CDm));
              if (cT > n / 2 || exT) vote = 1;
              else if (cF > n / 2 || exF) vote = 0;
              else vote = -1;
              cd = many(mand(M, CDm));
            }
          }
        } else {  // R1: broadcast vote — BenOr.scala:57-79
          const Mask<W> VT = mand(pm[1], act);
          const Mask<W> VF = mand(pm[2], act);
          if (!halted) {
            const int t = mpopc(mand(M, VT));
            const int f = mpopc(mand(M, VF));
            if (t > thr) {
              x = true;
              cd = true;
            } else if (f > thr) {
              x = false;
              cd = true;
            } else if (t > 1) {
              x = true;
            } else if (f > 1) {
              x = false;
            } else {
              x = sc.coin(k, g.pid);
            }
          }
        }
        if (halt_round == k) halted = true;
        pt.mark(2);
      }
      if constexpr (!SH::kFused) benor_check<W>(g, ck, k + 1, true, n, full, x, cd, vote, decided, decision, old_decided, old_decision, pred);
      if (tracing<SH>(a)) trace(k + 1, hs);
      pt.mark(many(act) ? 4 : 5);
    }
    finish_instance<W>(g, a, i, SH::kFused ? sh.ck : ck, SH::kFused ? SH::kSlots : 5, dec_val, dec_round, halt_round, x ? 1 : 0, &bc);
    pt.mark(3);
  }
  pt.flush(a.counters, threadIdx.x & 63);
  __syncthreads();
  counters_flush(&bc, a.counters, SH::kFused ? SH::kSlots : 5, a.R);
}

#ifndef PSG_BENOR_WPE
#define PSG_BENOR_WPE 5  // W = 2 (C5): 5 waves/SIMD measured 1.14x over the register-bound 4
#endif
template <int W, bool XHO, class SH = NoHook>
__global__ void __launch_bounds__(Geometry<W>::kThreads) __attribute__((amdgpu_waves_per_eu(W == 1 ? 1 : PSG_BENOR_WPE)))
benor_kernel(KArgs a) {
  benor_body<W, XHO, SH>(a);
}

#ifndef PSG_FUSED_MODULE  // host launchers (not part of a fused Spec module)
template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if constexpr (W > 1) {  // seeded schedule, built-in checker: lane-packed path
    if (!a.ho_in && !a.trace) {
      const int pg = pk_grid<PSG_ALG_BENOR, W>((const void*)benor_packed_kernel<W>, a.count);
      hipLaunchKernelGGL((benor_packed_kernel<W>), dim3(pg), dim3(256), 0, s, a);
      return hipGetLastError();
    }
  }
  if (a.ho_in) hipLaunchKernelGGL((benor_kernel<W, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((benor_kernel<W, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_benor(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1>(a, grid, s);
    case 2: return launch_w<2>(a, grid, s);
    case 3: return launch_w<3>(a, grid, s);
    case 4: return launch_w<4>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

const void* benor_kernel_ptr(int W) {
  switch (W) {
    case 1: return (const void*)benor_kernel<1, false>;
    case 2: return (const void*)benor_kernel<2, false>;
    case 3: return (const void*)benor_kernel<3, false>;
    case 4: return (const void*)benor_kernel<4, false>;
  }
  return nullptr;
}

#endif  // PSG_FUSED_MODULE

}  // namespace psg
