// psg_kset_es.hip — early-stopping k-set agreement on gfx950.
//
// Reference: example/KSetEarlyStopping.scala:9-44 (KSetESProcess). One round,
// broadcast (est, canDecide); a process decides est and exits once r > t/k or
// canDecide, otherwise est = min of the received estimates and
// canDecide = (some sender could decide) || lastNb - |mailbox| < k.
// est = mailbox.map(_._2._1).min visits the distinct sender estimates in
// ascending order (group min-reduction) and resolves each receiver at the first
// value whose sender set meets its mailbox; with the self bit a receiver also
// stops at its own estimate. Spec: TrivialSpec; the build checks k-agreement over
// never-crashed deciders and validity, like KSetAgreement.
#include "psg_device.hpp"
#include "psg_kernels.hpp"

namespace psg {

template <int W>
struct EsLds {
  int32_t ds[W > 1 ? 64 * W : 1];
};

// Kernel body; SH = NoHook for the library's kernels, spec::SpecHook<GenSpec> in a
// fused Spec module (round_amd/formula.py compile_native(fused=True)).
template <int W, bool XHO, class SH = NoHook>
PSG_DEV void kset_es_body(const KArgs& a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int32_t crl[W > 1 ? 64 * W : 1];
  __shared__ int64_t red[2 * W];
  __shared__ EsLds<W> L;
  __shared__ int32_t x0tab[Geometry<W>::kGroups][X0Set<W>::kSlots];
  counters_init(&bc);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = a.n;
  const int t = a.param, kk = a.param2;
  const Mask<W> full = mfull<W>(n);

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
    if (g.valid) x0 = a.init ? a.init[init_row(a, i, inst) * (uint64_t)n + g.pid] : sc.init_value(g.pid, PSG_ALG_KSET_ES);
    X0Set<W> X0;
    X0.build(g, x0tab[grp], x0);
    // KSetESProcess state after init(io) (KSetEarlyStopping.scala:16-21)
    int32_t est = x0, lastNb = n, decision = 0;
    bool cd = false, decided = false, halted = !g.valid;
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    typename SH::template State<W> sh(g, grp, n);  // fused Spec evaluation state (NoHook: empty)
    auto check = [&](int c) {
      // W > 1: the staged decisions are published by the barrier of kagree_check's
      // first ballot exchange (read only after it); the previous check's reads are
      // ordered before this write by the next round's pre-state exchange
      if constexpr (W > 1) L.ds[g.pid] = decision;
      kagree_check<W>(g, ck, c, kk, full, decided, decision, X0, crashed, L.ds);
    };
    if constexpr (!SH::kFused) check(0);
    auto trace = [&](int c, int32_t hs) {
      emit_state<W, SH>(sh, g, a, i, c, est, decided ? 1 : 0, decision, 0, 0, 0, 0, 0, hs);
    };
    if (tracing<SH>(a)) trace(0, n);
    for (int k = 0; k < a.R; ++k) {
      // pre-state ballots: alive senders, senders' canDecide flags (one exchange)
      const bool pr0[2] = {!halted, cd};
      Mask<W> m0[2];
      g.template ballots<2>(pr0, m0);
      const Mask<W> act = m0[0];
      int32_t hs = n;  // |mailbox| of this round (Spec field HOSIZE)
      if (many(act)) {
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) cs.sets(g, k, CB, CN);
        const Mask<W> M = mand(sc.ho(k, g.pid, good, goodS, CB, CN), act);
        const int currNb = mpopc(M);
        if (!halted) hs = currNb;
        const bool anyCD = many(mand(M, m0[1]));  // mailbox.exists(_._2._2), pre-update flags
        const bool decideNow = !halted && (k > t / kk || cd);
        // est = min over the mailbox's estimates (unchanged if the mailbox is empty)
        bool unres = !halted && !decideNow && currNb > 0;
        const bool selfIn = mtest(M, g.pid);
        int32_t nest = est;
        Mask<W> rem = act;
        while (many(rem)) {
          bool anyU;  // the min and "any lane unresolved" share one exchange
          const int32_t v = g.min32_any(est, mtest(rem, g.pid), unres, anyU);
          if (!anyU) break;
          const Mask<W> E = mand(g.ballot(est == v), rem);
          rem = mandn(rem, E);
          if (unres) {
            if (many(mand(M, E))) {
              nest = v;
              unres = false;
            } else if (selfIn && v >= est) {
              unres = false;  // nothing below the receiver's own estimate reached it
            }
          }
        }
        if (decideNow) {  // callback.decide(est); exitAtEndOfRound (KSetEarlyStopping.scala:32-34)
          dec_val = est;
          dec_round = k;
          decided = true;
          decision = est;
          halt_round = k;
          halted = true;
        } else if (!halted) {  // KSetEarlyStopping.scala:36-38 (variant 1: mutation, always canDecide)
          est = nest;
          cd = a.variant == 1 ? true : (anyCD || lastNb - currNb < kk);
          lastNb = currNb;
        }
      }
      if constexpr (!SH::kFused) check(k + 1);
      if (tracing<SH>(a)) trace(k + 1, hs);
    }
    finish_instance<W>(g, a, i, SH::kFused ? sh.ck : ck, SH::kFused ? SH::kSlots : 2, dec_val, dec_round, halt_round, est, &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, SH::kFused ? SH::kSlots : 2, a.R);
}

#ifndef PSG_KSETES_WPE
#define PSG_KSETES_WPE 5  // W = 4: 5 waves/SIMD measured 1.39x over the register-bound 3
#endif
template <int W, bool XHO, class SH = NoHook>
__global__ void __launch_bounds__(Geometry<W>::kThreads) __attribute__((amdgpu_waves_per_eu(W == 1 ? 1 : PSG_KSETES_WPE)))
kset_es_kernel(KArgs a) {
  kset_es_body<W, XHO, SH>(a);
}

#ifndef PSG_FUSED_MODULE  // host launchers (not part of a fused Spec module)
template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if (a.ho_in) hipLaunchKernelGGL((kset_es_kernel<W, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((kset_es_kernel<W, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_kset_es(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1>(a, grid, s);
    case 2: return launch_w<2>(a, grid, s);
    case 3: return launch_w<3>(a, grid, s);
    case 4: return launch_w<4>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

const void* kset_es_kernel_ptr(int W) {
  switch (W) {
    case 1: return (const void*)kset_es_kernel<1, false>;
    case 2: return (const void*)kset_es_kernel<2, false>;
    case 3: return (const void*)kset_es_kernel<3, false>;
    case 4: return (const void*)kset_es_kernel<4, false>;
  }
  return nullptr;
}

#endif  // PSG_FUSED_MODULE

}  // namespace psg
