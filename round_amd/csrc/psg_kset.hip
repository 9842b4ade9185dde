// psg_kset.hip — KSetAgreement on gfx950.
//
// Reference: example/KSetAgreement.scala:21-68. The state t: Map[ProcessID,Int]
// only ever holds entries (q -> initialValue_q) (init `Map(id -> v)` at 30,
// merge `a ++ b` at 36-38), so it is exactly a set of origins over the fixed
// initial vector: a W x 64-bit mask per process; `t == t'` is mask equality,
// `t ++ t'` is OR, pick(t) = min of the initial values of the origins (40).
// Payloads (decider, t) are staged in LDS; each process walks the alive senders
// with broadcast LDS reads. `content.find(_._1)` (53) takes the first decider
// message in Scala Map iteration order (CHAMP for > 4 entries).
#include "psg_device.hpp"
#include "psg_kernels.hpp"

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

template <int W>
PSG_DEV Mask<W> load_t(const uint64_t* ts, int q) {
  Mask<W> m;
#pragma unroll
  for (int w = 0; w < W; ++w) m.w[w] = ts[q * W + w];
  return m;
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
    if (g.valid) x0 = a.init ? a.init[init_row(a, i, inst) * (uint64_t)n + g.pid] : sc.init_value(g.pid, PSG_ALG_KSET);
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
          // t = content.find(_._1).get._2 — first decider message in iteration order
          int qs = mfirst(cand);
          if (a.tiebreak == PSG_TIE_CHAMP && mpopc(M) > 4 && mpopc(cand) > 1) {
            const Mask<W> t0 = load_t<W>(ts, qs);
            bool differ = false;
#pragma unroll
            for (int w = 0; w < W; ++w) {
              uint64_t m = cand.w[w];
              while (m) {
                const int q = w * 64 + __builtin_ctzll(m);
                m &= m - 1;
                if (!meq(load_t<W>(ts, q), t0)) differ = true;
              }
            }
            if (differ) {
              uint64_t best = ~0ull;
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
                  if (key < best) {
                    best = key;
                    qs = q;
                  }
                }
              }
            }
          }
          tnew = load_t<W>(ts, qs);
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
