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
// Philox round keys formed per call in this translation unit (packed KSetEarlyStopping -3.6 %; the hoisted
// 20-SGPR key schedule spilled here — and won in OTR / LastVoting / FloodMin / BenOr: round-4 A/B)
#ifndef PSG_PHILOX_OPAQUE_KEYS
#define PSG_PHILOX_OPAQUE_KEYS 1
#endif
#include "psg_device.hpp"
#include "psg_kernels.hpp"
#include "psg_packed.hpp"

namespace psg {

template <int W>
struct EsLds {
  int32_t ds[W > 1 ? 64 * W : 1];
};

// ---------------------------------------------------------------- lane-packed path (n > 64)
// kset_es_body's built-in-checker path, one wave per instance with the W processes
// l + 64 j in lane l (psg_packed.hpp): the ascending walk over the distinct sender
// estimates takes the wave minimum of the lane's minimum over its slots still in the
// walk, and every ballot is a wave ballot (no block barrier per step).
template <int W>
PSG_DEV void kset_es_packed(const Pk<W>& P, const KArgs& a, uint64_t i, uint64_t inst, int32_t* x0lds,
                            BlockCounters* bc) {
  const int n = a.n, t = a.param, kk = a.param2;
  Sched<W, false> sc;
  sc.setup(a, inst, P.lane, false);
  sc.prep_good(0, P.lane, a.R);
  int32_t cr[W];
  pk_crash_rounds<W>(P, a, inst, cr);
  // KSetESProcess state after init(io) (KSetEarlyStopping.scala:16-21). Registers are what
  // bounds this kernel (W mailboxes of W words each per lane), so the state is kept compact:
  // a process decides and exits in the same round with decision = est, so the decide value
  // is `decision`, the decide round is the halt round, and decided = halted on a process
  // slot; canDecide and halted are bits j / 8 + j of one flag word.
  int32_t est[W], decision[W];
  uint32_t nbh[W];  // lastNb (bits 0..15) | halt round + 1 (bits 16..31: 0 = not halted)
  uint32_t fl = 0;  // bit j: canDecide of slot j; bit 8 + j: slot j halted (or not a process);
                    // bit 16 + j: slot j's decision is not an initial value (probed when it decides)
#pragma unroll
  for (int j = 0; j < W; ++j) {
    est[j] = 0;
    if (P.val[j])
      est[j] = a.init ? init_x(a, i, inst, P.pid(j)) : sc.init_value(P.pid(j), PSG_ALG_KSET_ES);
    nbh[j] = (uint32_t)n;
    decision[j] = 0;
    fl |= (1u - P.val[j]) << (8 + j);
  }
  X0Set<W> X0;
  pk_x0_build<W>(P, X0, x0lds, est);
  Checks ck;
  ck.reset();
  auto check = [&](int c) {
    uint32_t decided[W], notinit[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      decided[j] = P.val[j] & ((fl >> (8 + j)) & 1u);
      notinit[j] = (fl >> (16 + j)) & 1u;
    }
    pk_kagree_check_m<W>(P, ck, c, kk, decided, decision, cr, notinit);
  };
  check(0);
  for (int k = 0; k < a.R; ++k) {
    uint32_t al[W], cdw[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
      al[j] = 1u - ((fl >> (8 + j)) & 1u);
      cdw[j] = (fl >> j) & 1u;
    }
    const Mask<W> act = P.ballot(al);  // alive senders
    if (many(act)) {
      const Mask<W> CD = P.ballot(cdw);  // senders' canDecide flags (pre-state)
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
      // The distinct sender estimates are visited in ascending order (the first step's value
      // is the minimum over every alive sender, known before any mailbox); each receiver
      // resolves at the first value whose senders meet its mailbox. A receiver's mailbox
      // (W words) is formed, used for the first step and dropped: the rare receivers still
      // unresolved after it re-form theirs at each later step (Sched::ho is a pure function
      // of (k, pid); with crash-stop HO sets it draws only in the crash rounds), so no W x W
      // words of mailboxes stay live in registers (they spilled to scratch).
      int32_t mn = INT32_MAX;
#pragma unroll
      for (int j = 0; j < W; ++j)
        if ((act.w[j] >> P.lane) & 1ull) mn = min(mn, est[j]);
      const int32_t v1 = Grp<1>::dpp_reduce32<false>(mn);  // act non-empty: a sender value
      uint32_t eq1[W];
#pragma unroll
      for (int j = 0; j < W; ++j) eq1[j] = eq01(est[j], v1);
      const Mask<W> E1 = mand(P.ballot(eq1), act);
      int32_t nest[W];
      uint32_t unres = 0, selfIn = 0, dnow = 0;  // bit j per slot
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const Mask<W> M = mand(sc.ho(k, P.pid(j), good, goodS, CB, CN), act);
        const int32_t currNb = mpopc(M);
        const uint32_t live = 1u - ((fl >> (8 + j)) & 1u);
        const uint32_t cd = (fl >> j) & 1u;
        const uint32_t decideNow = live & ((k > t / kk) ? 1u : cd);
        const uint32_t self = (uint32_t)((M.w[j] >> P.lane) & 1ull);
        nest[j] = est[j];
        // est = min over the mailbox's estimates (unchanged if the mailbox is empty)
        uint32_t u = live & (1u - decideNow) & (currNb > 0 ? 1u : 0u);
        if (u) {
          if (many(mand(M, E1))) {
            nest[j] = v1;
            u = 0;
          } else if (self && v1 >= est[j]) {
            u = 0;  // nothing below the receiver's own estimate reached it
          }
        }
        unres |= u << j;
        selfIn |= self << j;
        dnow |= decideNow << j;
        if (live && !decideNow) {  // KSetEarlyStopping.scala:36-38 (variant 1: mutation, always canDecide)
          const bool anyCD = many(mand(M, CD));  // mailbox.exists(_._2._2), pre-update flags
          const int32_t lastNb = (int32_t)(nbh[j] & 0xFFFFu);
          const uint32_t ncd = a.variant == 1 ? 1u : ((anyCD || lastNb - currNb < kk) ? 1u : 0u);
          fl = (fl & ~(1u << j)) | (ncd << j);
          nbh[j] = (nbh[j] & 0xFFFF0000u) | (uint32_t)currNb;
        }
      }
      Mask<W> rem = mandn(act, E1);
      while (many(rem)) {
        if (!pk_any(unres)) break;
        int32_t mv = INT32_MAX;
#pragma unroll
        for (int j = 0; j < W; ++j)
          if ((rem.w[j] >> P.lane) & 1ull) mv = min(mv, est[j]);
        const int32_t v = Grp<1>::dpp_reduce32<false>(mv);  // rem non-empty: a sender value
        uint32_t eq[W];
#pragma unroll
        for (int j = 0; j < W; ++j) eq[j] = eq01(est[j], v);
        const Mask<W> E = mand(P.ballot(eq), rem);
        rem = mandn(rem, E);
#pragma unroll
        for (int j = 0; j < W; ++j) {
          if ((unres >> j) & 1u) {
            const Mask<W> M = mand(sc.ho(k, P.pid(j), good, goodS, CB, CN), act);
            if (many(mand(M, E))) {
              nest[j] = v;
              unres &= ~(1u << j);
            } else if (((selfIn >> j) & 1u) && v >= est[j]) {
              unres &= ~(1u << j);  // nothing below the receiver's own estimate reached it
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if ((dnow >> j) & 1u) {  // callback.decide(est); exitAtEndOfRound (KSetEarlyStopping.scala:32-34)
          decision[j] = est[j];
          nbh[j] = (nbh[j] & 0xFFFFu) | ((uint32_t)(k + 1) << 16);
          fl |= (1u << (8 + j)) | ((1u - X0.contains01(est[j])) << (16 + j));
        } else if (!((fl >> (8 + j)) & 1u)) {
          est[j] = nest[j];
        }
      }
    }
    check(k + 1);
  }
  int32_t halt_round[W];
#pragma unroll
  for (int j = 0; j < W; ++j) halt_round[j] = (int32_t)(nbh[j] >> 16) - 1;
  pk_finish<W>(P, a, i, ck, 2, decision, halt_round, halt_round, est, bc);
}

#ifndef PSG_KSETES_PK_WPE
#define PSG_KSETES_PK_WPE 4  // W = 4, compact state (no scratch): 4 waves/SIMD 15.7 ms vs 5 (156 B scratch) 16.7 ms
#endif
template <int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PSG_KSETES_PK_WPE)))
kset_es_packed_kernel(KArgs a) {
  __shared__ BlockCounters bc;
  __shared__ int32_t x0tab[4][X0Set<W>::kSlots];
  counters_init(&bc);
  __syncthreads();
  Pk<W> P;
  P.setup(a.n);
  InstanceQueue<1> Q;
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    kset_es_packed<W>(P, a, i, inst, x0tab[threadIdx.x >> 6], &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, 2, a.R);
}

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
    if (g.valid) x0 = a.init ? init_x(a, i, inst, g.pid) : sc.init_value(g.pid, PSG_ALG_KSET_ES);
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
  if constexpr (W > 1) {  // seeded schedule, built-in checker: lane-packed path
    if (!a.ho_in && !a.trace) {
      const int pg = pk_grid<PSG_ALG_KSET_ES, W>((const void*)kset_es_packed_kernel<W>, a.count);
      hipLaunchKernelGGL((kset_es_packed_kernel<W>), dim3(pg), dim3(256), 0, s, a);
      return hipGetLastError();
    }
  }
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
