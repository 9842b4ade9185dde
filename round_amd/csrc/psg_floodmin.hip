// psg_floodmin.hip — FloodMin on gfx950.
//
// Reference: example/FloodMin.scala:8-36. x = mailbox.foldLeft(x)(min) is
// computed without touching every sender: the distinct sender values are
// visited in ascending order (group min-reduction), and a process resolves at
// the first value v whose sender set E_v intersects its mailbox (or v >= x).
// Values only decrease and converge, so one or two passes are typical.
// Spec: TrivialSpec (FloodMin.scala:40); the build checks k-agreement with
// k = 1 over correct processes and validity (decisions are initial values).
#include "psg_device.hpp"
#include "psg_kernels.hpp"
#include "psg_packed.hpp"

namespace psg {

template <int W>
struct FmLds {
  int32_t ds[W > 1 ? 64 * W : 1];
};

// ---------------------------------------------------------------- crash-stop fast path
// Seeded crash-stop schedules without benign loss, good rounds or ho_min (the C4
// family): HO(p, k) = all \ (CB_k | (CN_k \ S_p)), where CB_k = crashed before k,
// CN_k = crashing in k and S_p = the senders whose crash-round message reaches p
// (p's survival words), plus p itself. So FloodMin's update (FloodMin.scala:25-31)
//   x(p) = min(x(p), min{x_q : q in HO(p) & alive})
// is min(x(p), m_U, min{x_q : q in CN_k & alive & S_p}) with m_U the group minimum
// over U = alive \ (CB_k | CN_k): one group reduction, plus a per-receiver pass over
// the (few) processes crashing in round k. The group minimum over U_{k+1} rides on
// the exchange of the Spec check after round k, with the check's ballots (decided,
// decided-and-correct, decided-a-non-initial-value, alive) and the minimum and
// maximum decision of the correct deciders (k-agreement with k = 1: at most one
// value iff min == max): one block barrier per round, where the general path pays
// one per min-loop step and per exchange.
template <int W>
struct FmXch {  // one wave's part of a round's exchange
  uint64_t b[4];       // ballot words: decided, decided & correct, decided & non-initial, alive
  int32_t mu, dmn, dmx, pad;
};

template <int W>
struct FmFast {
  FmXch<W> ex[2][W];
  int32_t xs[2][64 * W];  // x after the last round, by check parity (the crash-round senders' values)
};

template <int W, class SC>
PSG_DEV void floodmin_fast(Grp<W>& g, const KArgs& a, uint64_t i, SC& sc, CrashSets<W>& cs, FmFast<W>& F,
                           const X0Set<W>& X0, int32_t x0, BlockCounters* bc) {
  const int n = a.n, f = a.param;
  const Mask<W> full = mfull<W>(n);
  const int32_t mycr = g.valid ? sc.crash_round : -1;
  const bool crashed = mycr >= 0;
  int32_t x = x0, decision = 0;
  bool decided = false, halted = false;
  int32_t dec_val = 0, dec_round = -1, halt_round = -1;
  Checks ck;
  ck.reset();
  int32_t mU = INT32_MAX;  // group minimum of x over U of the next round
  Mask<W> act = mzero<W>();
  // check point c (after round c - 1) + the exchange for round c
  auto check = [&](int c) {
    const int par = c & 1;
    const bool alive = g.valid && !halted;
    const bool inU = alive && !(mycr >= 0 && mycr <= c);  // not crashed before or in round c
    const bool dc = g.valid && decided && !crashed;
    const uint64_t b0 = __builtin_amdgcn_ballot_w64(g.valid && decided);
    const uint64_t b1 = __builtin_amdgcn_ballot_w64(g.valid && dc);
    const uint64_t b2 = __builtin_amdgcn_ballot_w64(g.valid && decided && !X0.contains(decision));
    const uint64_t b3 = __builtin_amdgcn_ballot_w64(alive);
    const int32_t wmu = g.wave_min32(inU ? x : INT32_MAX);
    const int32_t wmn = g.wave_min32(dc ? decision : INT32_MAX);
    const int32_t wmx = g.wave_max32(dc ? decision : INT32_MIN);
    Mask<W> D, Y, BAD;
    int32_t dmn, dmx;
    if constexpr (W == 1) {
      D.w[0] = b0;
      Y.w[0] = b1;
      BAD.w[0] = b2;
      act.w[0] = b3;
      mU = wmu;
      dmn = wmn;
      dmx = wmx;
    } else {
      F.xs[par][g.pid] = x;
      FmXch<W>& e = F.ex[par][g.wv];
      if (g.lane == 0) {
        e.b[0] = b0;
        e.b[1] = b1;
        e.b[2] = b2;
        e.b[3] = b3;
        e.mu = wmu;
        e.dmn = wmn;
        e.dmx = wmx;
      }
      __syncthreads();
      mU = INT32_MAX;
      dmn = INT32_MAX;
      dmx = INT32_MIN;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const FmXch<W>& r = F.ex[par][w];
        D.w[w] = rfl64(r.b[0]);
        Y.w[w] = rfl64(r.b[1]);
        BAD.w[w] = rfl64(r.b[2]);
        act.w[w] = rfl64(r.b[3]);
        mU = min(mU, rfl32(r.mu));
        dmn = min(dmn, rfl32(r.dmn));
        dmx = max(dmx, rfl32(r.dmx));
      }
    }
    const bool one = !many(Y) || dmn == dmx;  // KAgreement with k = 1 (kagree_check)
    ck.record(fbit(one, 0) | fbit(!many(BAD), 1), meq(D, full), c, g.lane);
  };
  check(0);
  for (int k = 0; k < a.R; ++k) {
    if (many(act)) {
      Mask<W> CB, CN;
      cs.sets(g, k, CB, CN);
      const Mask<W> CNa = mand(CN, act);
      int32_t nx = min(x, mU);
      if (many(CNa)) {  // crash round of some alive sender: its message reaches p iff p's survival bit
        uint64_t dm[W], hf[W];
        uint32_t cw = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) cw |= CNa.w[w] ? 1u << w : 0u;
        sc.draw((uint32_t)k, (uint32_t)g.pid, false, true, dm, hf, cw);
        Mask<W> rem = CNa;
        while (many(rem)) {
          const int q = mfirst(rem);
          mclear(rem, q);
          int32_t xq;
          if constexpr (W == 1) xq = readlane32(x, q);
          else xq = rfl32(F.xs[k & 1][q]);
          uint64_t word = hf[0];
#pragma unroll
          for (int w = 1; w < W; ++w)
            if ((q >> 6) == w) word = hf[w];
          if ((word >> (q & 63)) & 1ull) nx = min(nx, xq);
        }
      }
      if (!halted) {
        x = nx;
        const bool decideNow = a.variant == 1 ? (k >= f - 1) : (k > f);  // FloodMin.scala:27 (variant 1: mutation)
        if (decideNow) {
          dec_val = x;
          dec_round = k;
          decided = true;
          decision = x;
          halt_round = k;
          halted = true;
        }
      }
    }
    check(k + 1);
  }
  finish_instance<W>(g, a, i, ck, 2, dec_val, dec_round, halt_round, x, bc);
}

// ---------------------------------------------------------------- crash-stop fast path, lane-packed
// The same computation as floodmin_fast for n > 64, one wave per instance with the W
// processes l + 64 j in lane l (psg_packed.hpp): the check's ballots are wave ballots
// (existential ones of the lane's OR over its slots), the minima are wave reductions
// of the lane's minimum over its slots, and a round needs no barrier at all. Only the
// survival words of the crashing senders' 64-pid words are drawn (one Philox call per
// two words), where the group path draws all W.
template <int W>
PSG_DEV void floodmin_packed(const Pk<W>& P, const KArgs& a, uint64_t i, uint64_t inst, int32_t* x0lds,
                             BlockCounters* bc) {
  const int f = a.param;
  Sched<W, false> sc;
  sc.setup(a, inst, P.lane, false);  // uniform parts; crash rounds per slot below
  int32_t cr[W];
  pk_crash_rounds<W>(P, a, inst, cr);
  // Every process decides x and exits in the same round (decideNow is uniform,
  // FloodMin.scala:27-31): the decide / halt round dk is one uniform value (-1 until then), a
  // decision is the process's x, and bit j of nib is "slot j's decision is not an initial
  // value" (its X0 probe, taken when it decides: the decision never changes afterwards).
  int32_t x[W];
  int dk = -1;
  uint32_t nib = 0;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    x[j] = 0;
    if (P.val[j])
      x[j] = a.init ? init_x(a, i, inst, P.pid(j)) : sc.init_value(P.pid(j), PSG_ALG_FLOODMIN);
  }
  X0Set<W> X0;
  pk_x0_build<W>(P, X0, x0lds, x);
  Checks ck;
  ck.reset();
  int32_t mU = INT32_MAX;
  Mask<W> act;
  // check point c (after round c - 1) and the group minimum over U of round c
  auto check = [&](int c) {
    uint32_t anyY = 0, anyBad = 0, undec = 0, alive[W];
    int32_t mu = INT32_MAX, dmn = INT32_MAX, dmx = INT32_MIN;
    const uint32_t dec01 = dk >= 0 ? 1u : 0u;  // every process decided (and halted) in round dk
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const uint32_t crashed = cr[j] >= 0 ? 1u : 0u;
      alive[j] = P.val[j] & (1u - dec01);
      const uint32_t inU = alive[j] & (1u - (crashed & (cr[j] <= c ? 1u : 0u)));  // not crashed before or in round c
      const uint32_t dc = P.val[j] & dec01 & (1u - crashed);
      mu = inU ? min(mu, x[j]) : mu;
      dmn = dc ? min(dmn, x[j]) : dmn;  // decision = x
      dmx = dc ? max(dmx, x[j]) : dmx;
      anyY |= dc;
      anyBad |= P.val[j] & dec01 & ((nib >> j) & 1u);
      undec |= P.val[j] & (1u - dec01);
    }
    act = P.ballot(alive);
    mU = Grp<1>::dpp_reduce32<false>(mu);
    dmn = Grp<1>::dpp_reduce32<false>(dmn);
    dmx = Grp<1>::dpp_reduce32<true>(dmx);
    const bool one = !pk_any(anyY) || dmn == dmx;  // KAgreement with k = 1 (kagree_check)
    ck.record(fbit(one, 0) | fbit(!pk_any(anyBad), 1), !pk_any(undec), c, P.lane);
  };
  check(0);
  for (int k = 0; k < a.R; ++k) {
    if (many(act)) {
      Mask<W> CN;
#pragma unroll
      for (int j = 0; j < W; ++j) CN.w[j] = __builtin_amdgcn_ballot_w64(cr[j] == k);
      const Mask<W> CNa = mand(CN, act);
      int32_t nx[W];
#pragma unroll
      for (int j = 0; j < W; ++j) nx[j] = min(x[j], mU);
      // crash round of some alive sender: its message reaches p iff p's survival bit.
      // Survival word w of p's stream is half w & 1 of Philox call w / 2 (Sched::draw with
      // drop = 0): the senders are taken by call, two 64-pid words at a time.
#pragma unroll
      for (int s = 0; 2 * s < W; ++s) {
        Mask<W> rem = mzero<W>();
        rem.w[2 * s] = CNa.w[2 * s];
        if (2 * s + 1 < W) rem.w[2 * s + 1] = CNa.w[2 * s + 1];
        if (!many(rem)) continue;
        uint64_t h0[W], h1[W];
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const U4 o = philox10((uint32_t)inst, (uint32_t)(inst >> 32), (uint32_t)k,
                                (uint32_t)P.pid(j) + ((uint32_t)s << 16), (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
          h0[j] = (uint64_t)o.x | ((uint64_t)o.y << 32);
          h1[j] = (uint64_t)o.z | ((uint64_t)o.w << 32);
        }
        while (many(rem)) {
          const int q = mtake_first(rem);
          const int32_t xq = P.bcast(x, q);
          const bool hi = (q >> 6) & 1;
          const int qb = q & 63;
#pragma unroll
          for (int j = 0; j < W; ++j)
            if (((hi ? h1[j] : h0[j]) >> qb) & 1ull) nx[j] = min(nx[j], xq);
        }
      }
      const bool decideNow = a.variant == 1 ? (k >= f - 1) : (k > f);  // FloodMin.scala:27 (variant 1: mutation)
      // (the round runs only while every process is alive: they all decide together)
#pragma unroll
      for (int j = 0; j < W; ++j) {
        x[j] = nx[j];
        if (decideNow) nib |= (1u - X0.contains01(x[j])) << j;
      }
      if (decideNow) dk = k;
    }
    check(k + 1);
  }
  int32_t dv[W], dr[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    dv[j] = dk >= 0 ? x[j] : 0;
    dr[j] = dk;
  }
  pk_finish<W>(P, a, i, ck, 2, dv, dr, dr, x, bc);
}

template <int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PSG_PK_WPE))) floodmin_packed_kernel(KArgs a) {
  __shared__ BlockCounters bc;
  __shared__ int32_t x0tab[4][X0Set<W>::kSlots];
  counters_init(&bc);
  __syncthreads();
  Pk<W> P;
  P.setup(a.n);
  int32_t* x0lds = x0tab[threadIdx.x >> 6];
  InstanceQueue<1> Q;
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    floodmin_packed<W>(P, a, i, inst, x0lds, &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, 2, a.R);
}

// Kernel body; SH = NoHook for the library's kernels, spec::SpecHook<GenSpec> in a
// fused Spec module (round_amd/formula.py compile_native(fused=True)).
template <int W, bool XHO, class SH = NoHook>
PSG_DEV void floodmin_body(const KArgs& a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int32_t crl[W > 1 ? 64 * W : 1];
  __shared__ int64_t red[2 * W];
  __shared__ FmLds<W> L;
  __shared__ int32_t x0tab[Geometry<W>::kGroups][X0Set<W>::kSlots];
  __shared__ FmFast<W> FF;  // crash-stop fast path (W == 1 uses registers only)
  counters_init(&bc);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = a.n;
  const int f = a.param;
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
    const bool crashed = sc.crash_round >= 0;
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? init_x(a, i, inst, g.pid) : sc.init_value(g.pid, PSG_ALG_FLOODMIN);
    X0Set<W> X0;
    X0.build(g, x0tab[grp], x0);
    if constexpr (!XHO && !SH::kFused) {
      if (a.trace == nullptr && a.drop_log2 == 0 && a.good_p32 == 0 && a.ho_min < 0) {
        floodmin_fast<W>(g, a, i, sc, cs, FF, X0, x0, &bc);
        continue;
      }
    }
    int32_t x = x0, decision = 0;
    bool decided = false, halted = false;
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    typename SH::template State<W> sh(g, grp, n);  // fused Spec evaluation state (NoHook: empty)
    // The check's first ballot exchange also carries the next round's `act` (alive
    // processes), so a round costs one exchange fewer (fused Spec modules, which
    // skip the built-in check, ballot it at the top of the round instead).
    // W > 1: the staged decisions are published by the barrier of that exchange
    // (read only after it). A write after an executed round is ordered behind the
    // previous check's reads by the round's min exchange; after a frozen round
    // (every process halted) the decisions are unchanged and are not rewritten.
    Mask<W> act_next = mzero<W>();
    auto check = [&](int c, bool restage) {
      if constexpr (W > 1) {
        if (restage) L.ds[g.pid] = decision;
      }
      kagree_check<W>(g, ck, c, 1, full, decided, decision, X0, crashed, L.ds, !halted, &act_next);
    };
    if constexpr (!SH::kFused) check(0, true);
    auto trace = [&](int c, int32_t hs) {
      emit_state<W, SH>(sh, g, a, i, c, x, decided ? 1 : 0, decision, 0, 0, 0, 0, 0, hs);
    };
    if (tracing<SH>(a)) trace(0, n);
    pt.mark(0);
    for (int k = 0; k < a.R; ++k) {
      const Mask<W> act = SH::kFused ? g.ballot(!halted) : act_next;
      int32_t hs = n;  // |mailbox| of this round (Spec field HOSIZE)
      if (many(act)) {
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) cs.sets(g, k, CB, CN);
        const Mask<W> M = mand(sc.ho(k, g.pid, good, goodS, CB, CN), act);
        pt.mark(1);
        if (tracing<SH>(a) && !halted) hs = mpopc(M);
        // x = min(x, min{x_q : q in M}) by ascending distinct sender values
        // (W > 1: the min and "any lane unresolved" share one exchange, E and "any lane
        // still below v" share another; a converged round costs two exchanges)
        bool unres = !halted;
        int32_t nx = x;
        Mask<W> rem = act;
        while (many(rem)) {
          bool anyU;
          const int32_t v = g.min32_any(x, mtest(rem, g.pid), unres, anyU);  // rem non-empty: a sender value
          if (!anyU) break;
          const bool pr[2] = {x == v, unres && v < x};
          Mask<W> m2[2];
          g.template ballots<2>(pr, m2);
          const Mask<W> E = mand(m2[0], rem);
          rem = mandn(rem, E);
          if (unres) {
            if (v >= x) {
              unres = false;
            } else if (many(mand(M, E))) {
              nx = v;
              unres = false;
            }
          }
          if (!many(m2[1])) break;  // every unresolved lane had v >= x: all resolved
        }
        if (!halted) {
          x = nx;
          const bool decideNow = a.variant == 1 ? (k >= f - 1) : (k > f);  // FloodMin.scala:27 (variant 1: mutation)
          if (decideNow) {
            dec_val = x;
            dec_round = k;
            decided = true;
            decision = x;
            halt_round = k;
            halted = true;
          }
        }
      }
      pt.mark(2);
      if constexpr (!SH::kFused) check(k + 1, many(act));
      if (tracing<SH>(a)) trace(k + 1, hs);
      pt.mark(many(act) ? 4 : 5);
    }
    finish_instance<W>(g, a, i, SH::kFused ? sh.ck : ck, SH::kFused ? SH::kSlots : 2, dec_val, dec_round, halt_round, x, &bc);
    pt.mark(3);
  }
  pt.flush(a.counters, threadIdx.x & 63);
  __syncthreads();
  counters_flush(&bc, a.counters, SH::kFused ? SH::kSlots : 2, a.R);
}

#ifndef PSG_FM_WPE
#define PSG_FM_WPE 5  // W = 4: 5 waves/SIMD measured 10 % faster than the register-bound 4 (C4 f = 8)
#endif
template <int W, bool XHO, class SH = NoHook>
__global__ void __launch_bounds__(Geometry<W>::kThreads) __attribute__((amdgpu_waves_per_eu(PSG_FM_WPE)))
floodmin_kernel(KArgs a) {
  floodmin_body<W, XHO, SH>(a);
}

#ifndef PSG_FUSED_MODULE  // host launchers (not part of a fused Spec module)
template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if constexpr (W > 1) {  // seeded crash-stop schedule, built-in checker: lane-packed fast path
    if (!a.ho_in && !a.trace && a.drop_log2 == 0 && a.good_p32 == 0 && a.ho_min < 0) {
      const int pg = pk_grid<PSG_ALG_FLOODMIN, W>((const void*)floodmin_packed_kernel<W>, a.count);
      hipLaunchKernelGGL((floodmin_packed_kernel<W>), dim3(pg), dim3(256), 0, s, a);
      return hipGetLastError();
    }
  }
  if (a.ho_in) hipLaunchKernelGGL((floodmin_kernel<W, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((floodmin_kernel<W, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_floodmin(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1>(a, grid, s);
    case 2: return launch_w<2>(a, grid, s);
    case 3: return launch_w<3>(a, grid, s);
    case 4: return launch_w<4>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

const void* floodmin_kernel_ptr(int W) {
  switch (W) {
    case 1: return (const void*)floodmin_kernel<1, false>;
    case 2: return (const void*)floodmin_kernel<2, false>;
    case 3: return (const void*)floodmin_kernel<3, false>;
    case 4: return (const void*)floodmin_kernel<4, false>;
  }
  return nullptr;
}

#endif  // PSG_FUSED_MODULE

}  // namespace psg
