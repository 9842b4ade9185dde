// psg_otr.hip — OTR (one-third rule) and OTR2 on gfx950.
//
// Reference: example/Otr.scala:13-128 (OtrProcess, OTR.spec); example/Otr2.scala:9-104
// (Otr2Process: the same round with decision: Option[Int]; OTR2.spec has no
// keepInit conjunct, Invariant0's first disjunct is "everyone decided" and
// Invariant2 is "all decisions equal").
// One wave64 per instance, lane = process (n <= 64); W waves per instance for
// n > 64. Per round: HO(p) from Philox, mailbox M(p) = HO(p) & alive,
// mmor (Otr.scala:44-49) as a loop over the distinct values v of the alive
// senders: E_v = ballot(x == v), count(p, v) = popc(M(p) & E_v), keep the max
// count, ties to the smaller value. The Spec (Otr.scala:95-120) is evaluated
// after every round with ballots over the same distinct-value structure.
#include "psg_device.hpp"
#include "psg_kernels.hpp"

namespace psg {

template <int W>
struct OtrLds {
  int32_t xs[W > 1 ? 64 * W : 1];
  int32_t ds[W > 1 ? 64 * W : 1];
};

// Spec check at check point c (spec r = c). Slots: 0 Safety (some invariant
// holds), 1..3 invariants, 4 Agreement, 5 Validity, 6 Integrity, 7 Irrevocability.
// Every formula is evaluated from scratch at every check point. The universally
// quantified parts are per-process witnesses:
//   !(i.x == init(j.x) for some j)                  keepInit   (X0-set probe)
//   i.decided && i.decision not initial             Validity
//   i.decided && i.decision != d0                   Agreement  (d0 = a decided value)
//   old(i.decided) && !(i.decided && old(i.decision) == i.decision)  Irrevocability
// Fast path: one VALU word per process holds a bit per witness, where the two X0
// probes only look at the value's two home slots ("maybe not initial"); one ballot
// of "some bit set" settles all four when no process is even a possible witness
// (the common case). Otherwise each is resolved exactly with its own ballot and
// the full probe. (OR-reducing such a word with a DPP chain was measured 28 %
// slower, profiles/s2_ab/ab5.log: the chain's latency; a compare + ballot has none.)
// V.exists(v => |{i : i.x == v}| > 2n/3 && all decisions == v): with decisions only
// v = d0 can qualify; without, v must be a strict majority (Boyer-Moore candidate).
template <int W, bool V2, bool FROZEN = false>
// od / ox: "decision / x maybe not initial" (X0Set::maybe_out01_2 of the current values), probed
// by the caller when the values change (round 0 and executed updates) instead of at every check
// point: the memoized probe of the fused lowering; every formula is still evaluated.
// FROZEN: a check point of the frozen tail, where the pre-round state is the current one, so the
// Irrevocability witness old.decided && !(decided && old.decision == decision) is 0 by algebra.
PSG_DEV void otr_check(Grp<W>& g, OtrLds<W>& L, const X0Set<W>& X0, Checks& ck, int c, bool has_old, int n,
                       const Mask<W>& full, int32_t x, uint32_t dec01, int32_t decision, uint32_t old01,
                       int32_t old_decision, uint32_t valid01, uint32_t od, uint32_t ox) {
  const int sthr = (2 * n) / 3;  // 2*n/3 in the Spec (Otr.scala:101)
  if constexpr (W > 1) {
    L.ds[g.pid] = decision;
    __syncthreads();
  }
  const uint32_t irr01 = (has_old && !FROZEN) ? old01 & (1u - (dec01 & eq01(old_decision, decision))) : 0u;
  {
    // Settled state first (every process decided, every decision equal to process 0's, no
    // witness): one ballot of a per-process word, with process 0's decision as d0 (when all
    // decided, process 0 is the first decider). Then keepInit, Validity, Agreement and
    // Irrevocability hold, so Invariant2 (OTR: term && all decisions equal and initial;
    // OTR2: all decisions equal), Safety and Integrity hold; Invariant0 reduces to e0
    // (OTR2: term), Invariant1 to e1, with the vote count taken at v = d0. The same values
    // as the general path below, in a few instructions (most check points of a run are in
    // this state).
    const int32_t p0 = g.bcast(decision, L.ds, 0);
    uint32_t u = (1u - dec01) | od | ne01(decision, p0) | irr01;
    if constexpr (!V2) u |= ox;  // keepInit (OTR only)
    if (!g.any((u & valid01) != 0u)) {
      const int cnt = mpopc(g.ballot(x == p0));  // (a compare and the valid-lane mask)
      const uint32_t fb = (V2 ? 0u : fbit(cnt > sthr, 1)) | fbit(cnt == n, 2);
      ck.record(fb, true, c, g.lane);
      return;
    }
  }
  // dec01 and the witness word are 0 on lanes past n: ballots without the valid-lane mask
  const Mask<W> D = g.ballot_any(dec01 != 0u);
  const bool anyD = many(D);
  const int32_t d0 = anyD ? g.bcast(decision, L.ds, mfirst(D)) : 0;
  uint32_t wit = od | ne01(decision, d0);
  if constexpr (!V2) wit = (wit & dec01) | ox;  // keepInit (OTR only)
  else wit &= dec01;
  wit |= irr01;
  const Mask<W> Wm = g.ballot_any((wit & valid01) != 0u);
  const bool term = meq(D, full);
  const bool wany = many(Wm);
  bool keep = true, validity = true, same = true, irrev = true;
  if (wany) {  // exact resolution, one ballot per formula
    if constexpr (!V2) keep = X0.all_in(g, full, x);
    validity = X0.all_in(g, D, decision);
    same = !many(mand(D, g.ballot(decision != d0)));
    if (has_old) irrev = !many(mandn(g.ballot(old01 != 0u), mand(D, g.ballot(old_decision == decision))));
  }
  // the vote count's value: d0 once someone decided; before that OTR reads the count only as
  // cnt == n (Invariant1; Invariant0 is keepInit alone with no decision), which holds iff every
  // x equals process 0's — the majority candidate is needed only for OTR2's e0 (and W > 1)
  const int32_t ref = anyD ? d0 : ((!V2 && W == 1) ? readlane32(x, 0) : majority_candidate<W>(g, x));
  const int cnt = mpopc(g.ballot((valid01 & eq01(x, ref)) != 0u));
  const bool condv = !anyD || same;
  const bool e0 = condv && cnt > sthr;
  const bool e1 = condv && cnt == n;
  const bool d0in = same && validity;  // all decisions equal d0 and are initial values
  // OTR: Otr.scala:99-110; OTR2: Otr2.scala:75-87
  const bool inv0 = V2 ? (term || e0) : ((!anyD || e0) && keep);
  const bool inv1 = V2 ? e1 : (e1 && keep);
  const bool inv2 = V2 ? same : (term && d0in);
  const bool integrity = !anyD || d0in;
  const uint32_t fb = fbit(inv0 || inv1 || inv2, 0) | fbit(inv0, 1) | fbit(inv1, 2) | fbit(inv2, 3) |
                      fbit(same, 4) | fbit(validity, 5) | fbit(integrity, 6) | fbit(irrev, 7);
  ck.record(fb, term, c, g.lane);
}

// Kernel body; SH = NoHook for the library's kernels, spec::SpecHook<GenSpec> in a
// fused Spec module (round_amd/formula.py compile_native(fused=True)). TR = false: the
// launch has no Spec-program trace (a.trace == nullptr), known at compile time.
template <int W, bool V2, bool XHO, class SH = NoHook, bool TR = true>
PSG_DEV void otr_body(const KArgs& a) {
  const bool tracing_on = SH::kFused || (TR && a.trace != nullptr);
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int32_t crl[W > 1 ? 64 * W : 1];
  __shared__ int64_t red[2 * W];
  __shared__ OtrLds<W> L;
  __shared__ int32_t x0tab[Geometry<W>::kGroups][X0Set<W>::kSlots];
  counters_init(&bc);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = a.n;
  const int thr = a.variant == 1 ? n / 2 : (2 * n) / 3;  // Otr.scala:64, 67 (variant 1: mutation)
  const Mask<W> full = mfull<W>(n);
  const uint32_t valid01 = g.valid ? 1u : 0u;

  PhaseTimers pt;  // profiling builds only: t0 setup, t1 active round, t2 frozen round, t3 finish
  pt.start();
  InstanceQueue<W, 0, W == 1 ? PSG_QUEUE_CHUNK_LANE : 0> Q;  // dynamic instance distribution (psg_device.hpp)
  StepTally tally;     // per-lane process-round steps, reduced once per wave
  // Host-supplied initial values are loaded one instance ahead: the next row's load is
  // issued when an instance starts and consumed when the next one does, so its latency
  // overlaps the current instance's rounds instead of stalling its setup.
  auto load_x0 = [&](uint64_t ii) -> int32_t {
    if (ii == Q.kDone || !a.init || !g.valid) return 0;
    const uint64_t in_ = a.ids ? a.ids[ii] : a.inst_begin + ii;
    return a.init[init_row(a, ii, in_) * (uint64_t)n + g.pid];
  };
  uint64_t inext = Q.take(a);
  int32_t x0next = load_x0(inext);
  while (inext != Q.kDone) {
    const uint64_t i = inext;
    const int32_t x0host = x0next;
    inext = Q.take(a);
    x0next = load_x0(inext);
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    Sched<W, XHO> sc;
    sc.setup(a, inst, g.pid, g.valid);
    CrashSets<W> cs;  // per-instance crash rounds (no per-round exchange for W > 1)
    if (sc.crash_on) cs.prep(g, crl, sc.crash_round);
    sc.prep_good(0, g.lane, a.R);
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? x0host : sc.init_value(g.pid, PSG_ALG_OTR);
    X0Set<W> X0;
    X0.build(g, x0tab[grp], x0);
    // OtrProcess state after init(io) (Otr.scala:15-26); flags are 0/1 lane words
    int32_t x = x0, decision = -1, after = a.param;
    uint32_t od, ox;  // memoized X0 probes of decision / x (otr_check)
    X0.maybe_out01_2(decision, x, od, ox);
    uint32_t dec01 = 0, halted01 = 1u - valid01;
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    typename SH::template State<W> sh(g, grp, n);  // fused Spec evaluation state (NoHook: empty)
    if constexpr (!SH::kFused) otr_check<W, V2>(g, L, X0, ck, 0, false, n, full, x, dec01, decision, 0u, -1, valid01, od, ox);
    // OTR2's decision is an Option (PSG_NONE32 when empty)
    auto trace = [&](int c, int32_t hs, bool frozen = false) {
      emit_state<W, SH>(sh, g, a, i, c, x, (int32_t)dec01, V2 && !dec01 ? PSG_NONE32 : decision, 0, 0, 0, 0, 0, hs,
                        frozen);
    };
    if (tracing_on) trace(0, n);
    pt.mark(0);

    // does a trace or the fused Spec read |mailbox| (psg.h PSG_FIELD_HOSIZE)?
    const bool hs_needed = SH::kFused ? ((SH::kFields >> PSG_FIELD_HOSIZE) & 1u) != 0u
                                      : (TR && a.trace != nullptr && ((a.trace_fields >> PSG_FIELD_HOSIZE) & 1u));
    int32_t live_rounds = 0;  // rounds in which some process took a step
    int kf = a.R;             // first round in which every process had halted (the state is final)
    for (int k = 0; k < a.R; ++k) {
      const uint32_t old01 = dec01;
      const int32_t old_decision = decision;
      const Mask<W> act = g.ballot_any(halted01 == 0u);  // lanes past n are halted
      int32_t hs = n;  // |mailbox| of this round (Spec field HOSIZE)
      if (!many(act)) {  // every process halted: the frozen tail below (25.3 -> 24.8 ms)
        kf = k;
        break;
      }
      {
        live_rounds = k + 1;
        // Settled round: every live process has decided d and holds x = d. Then every mailbox
        // holds only d, so mmor is d (OtrExample.scala:67-75) and a mailbox above 2n/3 re-decides
        // the d it holds (Otr.scala:63-73): no process's x, decision or decided changes whatever
        // its HO set is, and only `after` counts down (Otr.scala:75-80). The round's HO sets are
        // then not drawn and mmor not run (the schedule is a pure function of (instance, round,
        // pid), so no other draw moves); the check point after it is evaluated as every other.
        // Not taken when a trace or the fused Spec reads |mailbox|.
        bool settled = false;
        if constexpr (W == 1) {
          if (!hs_needed) {
            const int32_t d0 = readlane32(decision, mfirst(act));
            settled = !g.any_raw(halted01 == 0u && !(dec01 != 0u && decision == d0 && x == d0));
          }
        }
        if (!settled) {
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) cs.sets(g, k, CB, CN);
        // mailbox: broadcast(x) from every alive sender in HO(p)
        const Mask<W> M = mand(sc.ho(k, g.pid, good, goodS, CB, CN), act);
        const int32_t msize = mpopc(M);
        if (tracing_on) hs = halted01 ? n : msize;
        const uint32_t upd = (1u - halted01) & gt01(msize, thr);
        if (g.any(upd != 0u)) {
          // mmor: max multiplicity, ties -> smaller value (OtrExample.scala:67-75).
          // The running best is one 64-bit key (count << 32 | v ^ 0x7FFFFFFF): a larger
          // key has a larger count, or the same count and a smaller v, so one 64-bit
          // compare keeps it. The loop walks xv = x ^ 0x7FFFFFFF (the key's low word).
          // E needs neither `& act` nor the valid-lane mask: M lies inside act and rem
          // only loses bits.
          const int32_t xv = x ^ 0x7FFFFFFF;
          if constexpr (W > 1) {
            L.xs[g.pid] = xv;
            __syncthreads();
          }
          uint64_t best = (uint64_t)(uint32_t)(INT32_MAX ^ 0x7FFFFFFF);  // count 0, v = INT32_MAX
          Mask<W> rem = act, passB = mzero<W>(), passS = mzero<W>();
          int stage = 2;  // 2: a single pass over every value
          if constexpr (W == 1) {
            // Round 0 with many distinct values (V = 64: ~40 of 64): a value held by h alive
            // senders counts at most h in any mailbox, so values are folded by decreasing
            // holder classes — h >= 3, then h = 2, then h = 1 — and a class is skipped when
            // every updating lane's best count already exceeds its h (it can neither win
            // nor tie). Holders are counted in LDS (the X0 table is free in bitmap mode:
            // every x is an initial value, x - lo < 64). With few distinct initial values
            // the single pass is already short and the counting is skipped.
            if (k == 0 && X0.bmode && __builtin_popcountll(X0.bm) > 8) {
              int32_t* cnt = x0tab[grp];
              cnt[g.lane] = 0;
              const uint32_t slot = (uint32_t)(x - X0.lo) & 63u;
              if (!halted01) atomicAdd(&cnt[slot], 1);
              const int32_t h = cnt[slot];
              rem = mand(act, g.ballot_any(h >= 3));  // every holder of such a value
              passB = mand(act, g.ballot_any(h == 2));
              passS = mandn(act, mor(rem, passB));
              stage = 0;
            }
          }
          while (true) {
            while (many(rem)) {
              const int32_t kv = g.bcast(xv, L.xs, mfirst(rem));
              const Mask<W> E = g.ballot_any(xv == kv);
              rem = mandn(rem, E);
              const uint64_t key = ((uint64_t)(uint32_t)mpopc(mand(M, E)) << 32) | (uint32_t)kv;
              best = key > best ? key : best;
            }
            if (stage == 2) break;
            const uint32_t beat = stage == 0 ? 3u : 2u;  // the next class's values count < beat
            if (!g.any(upd != 0u && (uint32_t)(best >> 32) < beat)) break;
            rem = stage == 0 ? passB : passS;
            ++stage;
          }
          const int32_t best_c = (int32_t)(best >> 32);
          const int32_t best_v = (int32_t)((uint32_t)best ^ 0x7FFFFFFFu);
          // x = mmor; decide on > 2n/3 copies, callback only the first time (Otr.scala:64-73)
          x = upd ? best_v : x;
          const uint32_t newdec = upd & gt01(best_c, thr);
          const uint32_t first = newdec & (1u - dec01);
          dec_val = first ? best_v : dec_val;
          dec_round = first ? k : dec_round;
          decision = newdec ? best_v : decision;
          dec01 |= newdec;
          if constexpr (!SH::kFused) X0.maybe_out01_2(decision, x, od, ox);
        }
        }  // !settled
        // after -= 1 once decided; exitAtEndOfRound when it reaches 0 (Otr.scala:75-80)
        const uint32_t ad = (1u - halted01) & dec01;
        after -= (int32_t)ad;
        const uint32_t h = ad & gt01(1, after);
        halt_round = h ? k : halt_round;
        halted01 |= h;
      }
      if constexpr (!SH::kFused)
        otr_check<W, V2>(g, L, X0, ck, k + 1, true, n, full, x, dec01, decision, old01, old_decision, valid01, od, ox);
      if (tracing_on) trace(k + 1, hs);
      pt.mark(1);
    }
    // Rounds kf .. R-1: every process has halted, so no process takes a step and the state, the
    // pre-round (old) state included, is the final one; the Spec is still evaluated at each of
    // these check points, kf + 1 .. R (Otr.scala:95-120 over the frozen state).
    for (int k = kf; k < a.R; ++k) {
      if constexpr (!SH::kFused)
        otr_check<W, V2, true>(g, L, X0, ck, k + 1, true, n, full, x, dec01, decision, dec01, decision, valid01, od, ox);
      if (tracing_on) trace(k + 1, n, true);
      pt.mark(2);
    }
    finish_instance<W>(g, a, i, SH::kFused ? sh.ck : ck, SH::kFused ? SH::kSlots : 8, dec_val, dec_round, halt_round, x, &bc,
                       &tally, live_rounds);
    pt.mark(3);
  }
  pt.flush(a.counters, threadIdx.x & 63);
  tally.flush(&bc);
  __syncthreads();
  counters_flush(&bc, a.counters, SH::kFused ? SH::kSlots : 8, a.R);
}

#ifndef PSG_OTR_WPE
#define PSG_OTR_WPE 6
#endif
template <int W, bool V2, bool XHO, class SH = NoHook, bool TR = true>
__global__ void __launch_bounds__(Geometry<W>::kThreads) __attribute__((amdgpu_waves_per_eu(W == 1 ? PSG_OTR_WPE : 1)))
otr_kernel(KArgs a) {
  otr_body<W, V2, XHO, SH, TR>(a);
}

#ifndef PSG_FUSED_MODULE  // host launchers (not part of a fused Spec module)
template <int W, bool V2>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if (a.ho_in) hipLaunchKernelGGL((otr_kernel<W, V2, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else if (a.trace) hipLaunchKernelGGL((otr_kernel<W, V2, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((otr_kernel<W, V2, false, NoHook, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

template <bool V2>
static hipError_t launch_v(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1, V2>(a, grid, s);
    case 2: return launch_w<2, V2>(a, grid, s);
    case 3: return launch_w<3, V2>(a, grid, s);
    case 4: return launch_w<4, V2>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

template <bool V2>
static const void* ptr_v(int W) {
  switch (W) {
    case 1: return (const void*)otr_kernel<1, V2, false, NoHook, false>;
    case 2: return (const void*)otr_kernel<2, V2, false, NoHook, false>;
    case 3: return (const void*)otr_kernel<3, V2, false, NoHook, false>;
    case 4: return (const void*)otr_kernel<4, V2, false, NoHook, false>;
  }
  return nullptr;
}

hipError_t launch_otr(const KArgs& a, int W, int grid, hipStream_t s) { return launch_v<false>(a, W, grid, s); }
hipError_t launch_otr2(const KArgs& a, int W, int grid, hipStream_t s) { return launch_v<true>(a, W, grid, s); }
const void* otr_kernel_ptr(int W) { return ptr_v<false>(W); }
const void* otr2_kernel_ptr(int W) { return ptr_v<true>(W); }

#endif  // PSG_FUSED_MODULE

}  // namespace psg
