// psg_lv.hip — LastVoting (Paxos-style 4-round phase) on gfx950.
//
// Reference: example/LastVoting.scala:80-212 (LVProcess) and 147-198 (spec).
// Coordinator c = (r/4) % n (LastVoting.scala:95) is wave-uniform: its sends are
// a readlane, "mailbox contains coord" is a bit test of HO(p), and the
// coordinator's R0/R2 mailbox is HO(c) & alive & (sender predicate) as a mask.
// maxBy over the R0 mailbox (LastVoting.scala:132) takes the first max in Scala
// Map iteration order: insertion order (ascending pid) up to 4 entries, CHAMP
// order beyond, computed from per-lane CHAMP sort keys and a wave min-reduction.
#ifndef __HIPCC_RTC__
#include <type_traits>
#endif

#include "psg_device.hpp"
#include "psg_kernels.hpp"


namespace psg {

// per-process flag bits (one VGPR word; see nz01 in psg_device.hpp)
enum : uint32_t { F_DECIDED = 1u, F_COMMIT = 2u, F_READY = 4u, F_HALTED = 8u };

template <int W>
struct LvLds {
  int32_t xs[W > 1 ? 64 * W : 1];
  int32_t tss[W > 1 ? 64 * W : 1];
  int32_t votes[W > 1 ? 64 * W : 1];
  int32_t ds[W > 1 ? 64 * W : 1];
  uint64_t hos[W > 1 ? 64 * W * W : 1];
};

template <int W>
PSG_DEV void lv_stage(Grp<W>& g, LvLds<W>& L, int32_t x, int32_t ts, int32_t vote, int32_t decision) {
  if constexpr (W > 1) {
    L.xs[g.pid] = x;
    L.tss[g.pid] = ts;
    L.votes[g.pid] = vote;
    L.ds[g.pid] = decision;
    __syncthreads();
  }
}

// Spec check at check point c (spec r = c). Slots: 0 Safety, 1 Invariant0
// (keepInit && (noDecision || majority)), 2 Invariant1, 3 Agreement, 4 Validity,
// 5 Integrity, 6 Irrevocability. roundInvariants(j-1)(0) is `true` for every j.
// xin01 / din01: 1 iff x / decision is an initial value (tracked by the round step: x and
// decision only ever take the coordinator's uniform vote, whose membership is probed once).
// Scalar-lean form: the kernel is bound by scalar issue, so every "some process" test is one
// ballot of a per-lane VALU predicate, and the binary search's bookkeeping runs in uniform VGPRs.
//
// In two parts: LvState holds every term that reads the process state alone; lv_check_at
// combines it with the terms that read r and coord (the majority clause, (i.ts == r/4) ==>
// coord.commit). lv_check = both, at every check point (the quiescent tail's too).
template <int W>
struct LvState {
  bool same, keep, validity, irrev, noDec, zAny, zOk, anyD, term;
  int32_t z0;
  Mask<W> C;  // processes with commit
};

// FROZEN: a check point of the quiescent tail (lv_body): the pre-round state is the current one, so
// the Irrevocability witness old.decided && !(decided && old.decision == decision) is 0, and no
// process is commit or ready (the tail's condition), so those flags' terms are 0.
template <int W, bool FROZEN = false>
PSG_DEV LvState<W> lv_state(Grp<W>& g, LvLds<W>& L, bool has_old, const Mask<W>& full, int32_t x, int32_t ts,
                            int32_t vote, int32_t decision, uint32_t fl, uint32_t old_fl, int32_t old_decision,
                            uint32_t xin01, uint32_t din01) {
  lv_stage<W>(g, L, x, ts, vote, decision);
  LvState<W> st;
  const uint32_t dec01 = fl & F_DECIDED;  // F_DECIDED == 1
  const Mask<W> D = g.ballot_any(dec01 != 0u);  // never set past n
  st.anyD = many(D);
  st.term = meq(D, full);
  const int32_t d0 = st.anyD ? g.bcast(decision, L.ds, mfirst(D)) : 0;
  // Agreement, keepInit, Validity and Irrevocability from one ballot of a per-process
  // witness word (decision != d0; x or a decision not initial; a changed decision),
  // resolved formula by formula only when some process is a witness
  uint32_t wit = (dec01 & (ne01(decision, d0) | (1u - din01))) | (1u - xin01);
  if (has_old && !FROZEN) wit |= (old_fl & F_DECIDED) & (1u - (dec01 & eq01(old_decision, decision)));
  st.same = st.keep = st.validity = st.irrev = true;
  if (g.any_raw(wit != 0u)) {  // wit, dec01, old_fl & F_DECIDED are 0 past n
    st.same = !g.any_raw(dec01 != 0u && decision != d0);
    st.keep = !g.any(xin01 == 0u);  // P.forall(i => P.exists(j1 => i.x == init(j1.x)))
    st.validity = !g.any_raw(dec01 != 0u && din01 == 0u);
    if constexpr (!FROZEN)
      st.irrev = !has_old || !g.any_raw((old_fl & F_DECIDED) != 0u && !(dec01 != 0u && old_decision == decision));
  }
  if constexpr (FROZEN) {
    // No process is commit or ready in the quiescent tail, so the pinned processes are the
    // deciders: noDec = no decider, the pins' witness z0 is the first decider's decision d0, and
    // "every pinned process agrees with z0" is Agreement (`same`: exact when a witness was found,
    // and true otherwise, as then every decision equals d0). The same terms, from the ballots above.
    st.noDec = !st.anyD;
    st.zAny = st.anyD;
    st.z0 = d0;
    st.zOk = st.same;
    st.C = mzero<W>();
    return st;
  }
  st.noDec = !g.any_raw((fl & (F_DECIDED | F_READY)) != 0u);  // 0 past n but F_HALTED
  // values pinned by (decided ==> decision == v), (commit ==> vote == v), (ready ==> vote == v):
  // z0 = the pinned value of the first pinned process (its decision if it decided, else its
  // vote), and every pinned process must agree with it
  const uint32_t cr01 = (fl & (F_COMMIT | F_READY)) ? 1u : 0u;
  const Mask<W> Pm = g.ballot_any((dec01 | cr01) != 0u);
  st.zAny = many(Pm);
  st.z0 = 0;
  st.zOk = true;
  if (st.zAny) {
    const int32_t zl = dec01 ? decision : vote;
    if constexpr (W > 1) {
      L.votes[g.pid] = zl;  // the staged votes are not read after this point of the check
      __syncthreads();
    }
    st.z0 = g.bcast(zl, L.votes, mfirst(Pm));
    st.zOk = !g.any_raw(((dec01 & ne01(decision, st.z0)) | (cr01 & ne01(vote, st.z0))) != 0u);
  }
  st.C = g.ballot_any((fl & F_COMMIT) != 0u);
  return st;
}

// FROZEN: a check point of the quiescent tail, which starts at a phase boundary 4φ (φ >= 1) where
// every ts <= φ - 1 (ts only takes a phase number in that phase's R1), while every tail check
// point has r/4 >= φ: so no process has ts == r/4 and (i.ts == r/4) ==> coord.commit holds by the
// tail's invariant, as its commit / ready terms are 0.
template <int W, bool FROZEN = false>
PSG_DEV void lv_check_at(Grp<W>& g, LvLds<W>& L, Checks& ck, const LvState<W>& st, int c, int32_t r4, int coord,
                         int n, int32_t x, int32_t ts) {
  // r4 = c / 4, coord = (c / 4) % n: maintained incrementally by the caller (a runtime `% n`
  // is a scalar multiply-high sequence per use on this scalar-issue-bound kernel)
  bool maj = false;
  // (Invariant0 reads maj only when keepInit holds and some process decided or is ready)
  if (c > 0 && st.zOk && st.keep && !st.noDec &&
      // (i.ts == r/4) ==> coord.commit
      (FROZEN || mtest(st.C, coord) || !g.any_raw(ts == r4))) {  // ts = -1 past n
    // exists t <= r/4: A_t = {i : i.ts >= t}, |A_t| > n/2, all x over A_t equal (to the pinned
    // value). The sets A_t shrink as t grows, and "all x over A equal (to z0)" holds on every
    // non-empty subset of a set it holds on, so the exists holds iff it holds at the largest
    // t <= r/4 with |A_t| > n/2. With tv = min(ts, r/4) + 1 in [0, r/4 + 1] that is the
    // largest u with |{tv >= u}| > n/2 (a present value; u = 0 always qualifies): a binary
    // search on the count, ceil(log2(r/4 + 2)) = bit length of r/4 + 1 steps (a step after
    // convergence keeps lo), lo / hi / mid as uniform VGPR values (vector issue)
    const int32_t tsc = ts < r4 ? ts : r4;
    const uint32_t tv = (uint32_t)(tsc + 1);  // ts >= -1 (LastVoting.scala:87)
    const int steps = 32 - __builtin_clz((uint32_t)r4 + 1u);
    uint32_t lo = vgpr_u32(0u), hi = vgpr_u32((uint32_t)r4 + 2u);
    const uint32_t half = (uint32_t)(n / 2);
    for (int s = 0; s < steps; ++s) {
      const uint32_t mid = (lo + hi) >> 1;
      const bool ok = (uint32_t)mpopc_v(g.ballot_any(tv >= mid)) > half;  // tv = 0 past n, mid >= 1
      lo = ok ? mid : lo;
      hi = ok ? hi : mid;
    }
    const Mask<W> A = g.ballot(tv >= lo);
    const int32_t xv = g.bcast(x, L.xs, mfirst(A));
    maj = !g.any(tv >= lo && x != xv) && (!st.zAny || xv == st.z0);
  }
  const bool inv0 = st.keep && (st.noDec || maj);
  const bool d0in = st.same && st.validity;
  const bool inv1 = st.term && d0in;
  const bool integrity = !st.anyD || d0in;
  const uint32_t fb = fbit(inv0 || inv1, 0) | fbit(inv0, 1) | fbit(inv1, 2) | fbit(st.same, 3) |
                      fbit(st.validity, 4) | fbit(integrity, 5) | fbit(st.irrev, 6);
  ck.record(fb, st.term, c, g.lane);
}

template <int W, bool FROZEN = false>
PSG_DEV void lv_check(Grp<W>& g, LvLds<W>& L, Checks& ck, int c, int32_t r4, int coord, bool has_old, int n,
                      const Mask<W>& full, int32_t x, int32_t ts, int32_t vote, int32_t decision, uint32_t fl,
                      uint32_t old_fl, int32_t old_decision, uint32_t xin01, uint32_t din01) {
  const LvState<W> st =
      lv_state<W, FROZEN>(g, L, has_old, full, x, ts, vote, decision, fl, old_fl, old_decision, xin01, din01);
  lv_check_at<W, FROZEN>(g, L, ck, st, c, r4, coord, n, x, ts);
}

// The coordinator's HO mask (uniform).
template <int W>
PSG_DEV Mask<W> ho_of(Grp<W>& g, LvLds<W>& L, const Mask<W>& ho, int c) {
  Mask<W> m;
  if constexpr (W == 1) {
    m.w[0] = readlane64(ho.w[0], c);
  } else {
#pragma unroll
    for (int w = 0; w < W; ++w) L.hos[g.pid * W + w] = ho.w[w];
    __syncthreads();
#pragma unroll
    for (int w = 0; w < W; ++w) m.w[w] = rfl64(L.hos[c * W + w]);
    __syncthreads();
  }
  return m;
}

// R0 and R2 read only the coordinator's HO set (LastVoting.scala:118-135, 166-180).
// Rather than every lane drawing its own HO set in those rounds, lane l draws the
// raw words of the coordinator of the l-th such round (q = l: k = 4*(q/2) + 2*(q%2),
// coord = (k/4) % n), one vector pass of Philox calls per 64 coordinator rounds;
// round k assembles HO(coord) from a readlane of them (Sched::draw / assemble, the
// same words and the same assembly as a per-lane Sched::ho).
template <int W, bool XHO>
struct CoordWords {
  uint64_t dm[W], hf[W];
  int qbase;
  PSG_DEV static int index(int k) { return (k >> 2) * 2 + ((k >> 1) & 1); }  // k even
  PSG_DEV void prep(const Sched<W, XHO>& sc, int q0, int lane, int n) {
    qbase = q0;
    const int q = q0 + lane;
    const int k = 4 * (q >> 1) + 2 * (q & 1);
    sc.draw((uint32_t)k, (uint32_t)((k >> 2) % n), false, sc.crash_on, dm, hf);
  }
  PSG_DEV Mask<W> ho(const Sched<W, XHO>& sc, int k, int c, int lane, int n, bool good, const Mask<W>& goodS,
                     const Mask<W>& CB, const Mask<W>& CN) {
    const int q = index(k);
    if (q - qbase >= 64) prep(sc, q, lane, n);
    const int off = q - qbase;
    uint64_t d[W], h[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      d[w] = readlane64(dm[w], off);
      h[w] = readlane64(hf[w], off);
    }
    return sc.assemble(c, good, goodS, CB, CN, d, h);
  }
};

// Kernel body; SH = NoHook for the library's kernels, spec::SpecHook<GenSpec> in a
// fused Spec module (round_amd/formula.py compile_native(fused=True)).
template <int W, bool XHO, class SH = NoHook, bool TR = true>
PSG_DEV void lv_body(const KArgs& a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int32_t crl[W > 1 ? 64 * W : 1];
  __shared__ int64_t red[2 * W];
  __shared__ LvLds<W> L;
  __shared__ int32_t x0tab[Geometry<W>::kGroups][X0Set<W>::kSlots];
  __shared__ ChampTable<W> CT;  // CHAMP fragment masks per level (maxBy's first max in Map order)
  counters_init(&bc);
  if (a.tiebreak == PSG_TIE_CHAMP) CT.build(a.n);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  // wave-uniform group index (SGPR): measured +3% on this kernel (fewer VGPRs, one more wave/SIMD);
  // the same change cost OTR / ShortLastVoting 1-3%, which keep the VGPR form
  const int grp = W == 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  const int n = a.n;
  const int need2 = a.variant == 1 ? 0 : n / 2;  // R2 quorum (LastVoting.scala:177; variant 1: mutation)
  const Mask<W> full = mfull<W>(n);
  const uint32_t myh = scala_improve((uint32_t)g.pid);

  PhaseTimers pt;  // profiling builds only: t0 setup, t1 HO sets, t2 update, t3 finish, t4 check, t5 frozen round
  pt.start();
  InstanceQueue<W, 0, W == 1 ? PSG_QUEUE_CHUNK_LANE : 0> Q;  // dynamic instance distribution (psg_device.hpp)
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    Sched<W, XHO> sc;
    sc.setup(a, inst, g.pid, g.valid);
    CrashSets<W> cs;  // per-instance crash rounds (no per-round exchange for W > 1)
    if (sc.crash_on) cs.prep(g, crl, sc.crash_round);
    sc.prep_good(0, g.lane, a.R);
    CoordWords<W, XHO> cw;
    if constexpr (!XHO) cw.prep(sc, 0, g.lane, n);
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? init_x(a, i, inst, g.pid) : sc.init_value(g.pid, PSG_ALG_LAST_VOTING);
    X0Set<W> X0;
    X0.build(g, x0tab[grp], x0);
    // LVProcess state after init(io) (LastVoting.scala:82-109)
    int32_t x = x0, ts = -1, vote = 0, decision = -1;
    uint32_t fl = g.valid ? 0u : F_HALTED;
    uint32_t xin = 1u, din = 1u;  // x / decision is an initial value (lv_check)
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    typename SH::template State<W> sh(g, grp, n);  // fused Spec evaluation state (NoHook: empty)
    if constexpr (!SH::kFused) lv_check<W>(g, L, ck, 0, 0, 0, false, n, full, x, ts, vote, decision, fl, 0u, -1, xin, din);
    auto trace = [&](int c, int32_t hs, bool frozen = false) {
      emit_state<W, SH>(sh, g, a, i, c, x, (fl & F_DECIDED) ? 1 : 0, decision, ts, (fl & F_READY) ? 1 : 0,
                        (fl & F_COMMIT) ? 1 : 0, vote, 0, hs, frozen);
    };
    if (tracing<SH, TR>(a)) trace(0, n);
    pt.mark(0);

    // one round of slot RS = k mod 4 (compile time: each slot's step and check specialized)
    // phase = k / 4 and its coordinator (phase % n), and the next phase's, kept incrementally
    int32_t phase = 0;
    int cph = 0, cnx = n > 1 ? 1 : 0;
    auto round = [&](const int k, auto RSc) {
      constexpr int RS = decltype(RSc)::value;
      const uint32_t old_fl = fl;
      const int32_t old_decision = decision;
      const Mask<W> act = g.ballot_any((fl & F_HALTED) == 0u);  // lanes past n are halted
      int32_t hs = n;  // |mailbox| of this round (Spec field HOSIZE)
      if (many(act)) {
        const int c = cph;
        const bool cAlive = mtest(act, c);
        const uint32_t live = (fl & F_HALTED) ? 0u : 1u;
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) cs.sets(g, k, CB, CN);
        // R1 / R3 read bit coord of every HO(p) (a mailbox of at most the coordinator's
        // message); R0 / R2 only HO(coord)
        constexpr bool coordRound = (RS & 1) == 0;
        // R1 / R3: does the coordinator send (commit / ready, LastVoting.scala:141, 187)? When it
        // does not, no mailbox is read and no HO bit of the round is observed
        const bool sent = !coordRound && cAlive && mtest(g.ballot_any((fl & (RS == 1 ? F_COMMIT : F_READY)) != 0u), c);
        Mask<W> HO = mzero<W>(), HOc = mzero<W>();
        if constexpr (XHO) {
          HO = sc.ho(k, g.pid, good, goodS, CB, CN);
        } else if (sent) {
          // only bit coord of HO(p) is read: the crash-round survival words matter only
          // when the coordinator crashes in this round, or when |HO(p)| decides the
          // ho_min rule (other bits are left unspecified otherwise)
          uint64_t dm[W], hf[W];
          const bool crash = sc.crash_on && (mtest(CN, c) || (sc.ho_min >= 0 && many(CN)));
          sc.draw((uint32_t)k, (uint32_t)g.pid, good, crash, dm, hf);
          HO = sc.assemble(g.pid, good, goodS, CB, CN, dm, hf);
        }
        if constexpr (coordRound) {
          if constexpr (XHO) HOc = ho_of<W>(g, L, HO, c);
          else HOc = cw.ho(sc, k, c, g.lane, n, good, goodS, CB, CN);
        }
        pt.mark(1);
        lv_stage<W>(g, L, x, ts, vote, decision);
        if constexpr (RS == 0) {  // R0: send (x, ts) to coord; coord picks vote = x of maxBy ts
          const Mask<W> Mc = mand(HOc, act);
          const int size = mpopc(Mc);
          hs = g.pid == c ? size : 0;
          if (cAlive && (size > n / 2 || (k == 0 && size > 0))) {
            const int32_t v = maxby_ts_x<W>(g, L.xs, Mc, size, x, ts, myh, a.tiebreak, &CT);
            if (g.pid == c) {
              vote = v;
              fl |= F_COMMIT;
            }
          }
        } else if constexpr (RS == 1) {  // R1: coord broadcasts vote if commit; receivers adopt (x, ts = r/4)
          hs = sent && mtest(HO, c) ? 1 : 0;
          if (sent) {
            const int32_t vc = g.bcast(vote, L.votes, c);
            const uint32_t rcv = live & (mtest(HO, c) ? 1u : 0u);
            const uint32_t vin = SH::kFused ? 1u : X0.contains01(vc);  // one probe of a uniform value
            x = rcv ? vc : x;
            xin = rcv ? vin : xin;
            ts = rcv ? phase : ts;
          }
        } else if constexpr (RS == 2) {  // R2: ts == r/4 send x to coord; coord ready on a majority
          const Mask<W> Mc = mand(mand(HOc, act), g.ballot_any(ts == phase));  // ts = -1 past n
          hs = g.pid == c ? mpopc(Mc) : 0;
          if (cAlive && mpopc(Mc) > need2 && g.pid == c) fl |= F_READY;
        } else {  // R3: coord broadcasts vote if ready; receivers decide and exit
          hs = sent && mtest(HO, c) ? 1 : 0;
          if (sent) {
            const int32_t vc = g.bcast(vote, L.votes, c);
            const uint32_t rcv = live & (mtest(HO, c) ? 1u : 0u);
            const uint32_t vin = SH::kFused ? 1u : X0.contains01(vc);
            din = rcv ? vin : din;
            const uint32_t first = rcv & (dec_round < 0 ? 1u : 0u);
            dec_val = first ? vc : dec_val;
            dec_round = first ? k : dec_round;
            decision = rcv ? vc : decision;
            halt_round = rcv ? k : halt_round;
            fl |= rcv ? (F_DECIDED | F_HALTED) : 0u;
          }
          // ready = false; commit = false for every process that took this step
          fl &= live ? ~(F_READY | F_COMMIT) : ~0u;
        }
        pt.mark(2);
      }
      if constexpr (!SH::kFused)
        lv_check<W>(g, L, ck, k + 1, RS == 3 ? phase + 1 : phase, RS == 3 ? cnx : cph, true, n, full, x, ts, vote,
                    decision, fl, old_fl, old_decision, xin, din);
      if (tracing<SH, TR>(a)) trace(k + 1, (old_fl & F_HALTED) ? n : hs);
      pt.mark(many(act) ? 4 : 5);
    };
    // Quiescent tail. At a phase boundary past round 0, once at most n/2 processes are not halted
    // and no process is commit or ready, no process can take an effective step again: R0's
    // commit needs a mailbox of more than n/2 (LastVoting.scala:129), R2's ready more than n/2
    // (177; the unmutated quorum), R1 / R3 send only from a commit / ready coordinator (141,
    // 187), and R3's reset finds the flags already clear — so the state, old included, is final.
    // Rounds kq .. R-1 then draw no HO set and run no step; the Spec is still evaluated at every
    // check point (with old = current: the Irrevocability witness is 0 by algebra, as in OTR's
    // frozen tail). Not taken when a trace or the fused Spec reads |mailbox|.
    const bool hs_read = SH::kFused ? ((SH::kFields >> PSG_FIELD_HOSIZE) & 1u) != 0u
                                    : (TR && a.trace != nullptr && ((a.trace_fields >> PSG_FIELD_HOSIZE) & 1u));
    const bool qok = a.variant == 0 && !hs_read;
    int kq = a.R;
    for (int k0 = 0; k0 < a.R; k0 += 4) {
      if (qok && k0 > 0) {
        const Mask<W> live = g.ballot_any((fl & F_HALTED) == 0u);  // lanes past n are halted
        if (2 * mpopc(live) <= n && !g.any_raw((fl & (F_COMMIT | F_READY)) != 0u)) {
          kq = k0;
          break;
        }
      }
      round(k0, Slot<0>{});
      if (k0 + 1 < a.R) round(k0 + 1, Slot<1>{});
      if (k0 + 2 < a.R) round(k0 + 2, Slot<2>{});
      if (k0 + 3 < a.R) round(k0 + 3, Slot<3>{});
      ++phase;
      cph = cnx;
      cnx = cnx + 1 == n ? 0 : cnx + 1;
    }
    for (int k = kq; k < a.R; ++k) {
      const int RS = k & 3;
      if constexpr (!SH::kFused)
        lv_check<W, true>(g, L, ck, k + 1, RS == 3 ? phase + 1 : phase, RS == 3 ? cnx : cph, true, n, full, x, ts,
                          vote, decision, fl, fl, decision, xin, din);
      if (tracing<SH, TR>(a)) trace(k + 1, n, true);
      if (RS == 3) {
        ++phase;
        cph = cnx;
        cnx = cnx + 1 == n ? 0 : cnx + 1;
      }
      pt.mark(5);
    }
    finish_instance<W>(g, a, i, SH::kFused ? sh.ck : ck, SH::kFused ? SH::kSlots : 7, dec_val, dec_round, halt_round, x, &bc);
    pt.mark(3);
  }
  pt.flush(a.counters, threadIdx.x & 63);
  __syncthreads();
  counters_flush(&bc, a.counters, SH::kFused ? SH::kSlots : 7, a.R);
}

#ifndef PSG_LV_WPE
#define PSG_LV_WPE 7  // W = 1 occupancy target: round 6 (trace-free kernels, 94 SGPR spills) 7 measured 46.9 ms vs 6: 48.4, 8: 50.0 (C3)
#endif
template <int W, bool XHO, class SH = NoHook, bool TR = true>
__global__ void __launch_bounds__(Geometry<W>::kThreads) __attribute__((amdgpu_waves_per_eu(W == 1 ? PSG_LV_WPE : 1)))
lv_kernel(KArgs a) {
  lv_body<W, XHO, SH, TR>(a);
}

#ifndef PSG_FUSED_MODULE  // host launchers (not part of a fused Spec module)
template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if (a.ho_in) hipLaunchKernelGGL((lv_kernel<W, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else if (a.trace) hipLaunchKernelGGL((lv_kernel<W, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((lv_kernel<W, false, NoHook, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_lv(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1>(a, grid, s);
    case 2: return launch_w<2>(a, grid, s);
    case 3: return launch_w<3>(a, grid, s);
    case 4: return launch_w<4>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

const void* lv_kernel_ptr(int W) {
  switch (W) {
    case 1: return (const void*)lv_kernel<1, false, NoHook, false>;
    case 2: return (const void*)lv_kernel<2, false, NoHook, false>;
    case 3: return (const void*)lv_kernel<3, false, NoHook, false>;
    case 4: return (const void*)lv_kernel<4, false, NoHook, false>;
  }
  return nullptr;
}

#endif  // PSG_FUSED_MODULE

}  // namespace psg
