// psg_lv.hip — LastVoting (Paxos-style 4-round phase) on gfx950.
//
// Reference: example/LastVoting.scala:80-212 (LVProcess) and 147-198 (spec).
// Coordinator c = (r/4) % n (LastVoting.scala:95) is wave-uniform: its sends are
// a readlane, "mailbox contains coord" is a bit test of HO(p), and the
// coordinator's R0/R2 mailbox is HO(c) & alive & (sender predicate) as a mask.
// maxBy over the R0 mailbox (LastVoting.scala:132) takes the first max in Scala
// Map iteration order: insertion order (ascending pid) up to 4 entries, CHAMP
// order beyond, computed from per-lane CHAMP sort keys and a wave min-reduction.
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
template <int W>
PSG_DEV void lv_check(Grp<W>& g, LvLds<W>& L, const X0Set<W>& X0, Checks& ck, int c, bool has_old, int n,
                      const Mask<W>& full, int32_t x, int32_t ts, int32_t vote, int32_t decision, uint32_t fl,
                      uint32_t old_fl, int32_t old_decision) {
  lv_stage<W>(g, L, x, ts, vote, decision);
  const int32_t r4 = c / 4;
  const int coord = r4 % n;
  const Mask<W> D = g.ballot((fl & F_DECIDED) != 0u);
  const Mask<W> C = g.ballot((fl & F_COMMIT) != 0u);
  const Mask<W> Rd = g.ballot((fl & F_READY) != 0u);
  const bool anyD = many(D);
  const int32_t d0 = anyD ? g.bcast(decision, L.ds, mfirst(D)) : 0;
  const bool same = !many(mand(D, g.ballot(decision != d0)));
  const bool keep = X0.all_in(g, full, x);  // P.forall(i => P.exists(j1 => i.x == init(j1.x)))
  const bool noDec = !many(mor(D, Rd));
  // values pinned by (decided ==> decision == v), (commit ==> vote == v), (ready ==> vote == v)
  const Mask<W> CR = mor(C, Rd);
  const Mask<W> Pm = mor(D, CR);
  const bool zAny = many(Pm);
  int32_t z0 = 0;
  bool zOk = true;
  if (zAny) {
    const int q = mfirst(Pm);
    z0 = mtest(D, q) ? g.bcast(decision, L.ds, q) : g.bcast(vote, L.votes, q);
    zOk = !many(mor(mand(D, g.ballot(decision != z0)), mand(CR, g.ballot(vote != z0))));
  }
  const bool c5 = mtest(C, coord) || !g.any(ts == r4);  // (i.ts == r/4) ==> coord.commit
  bool maj = false;
  if (c > 0 && zOk && c5) {
    // exists t: A = {i : i.ts >= t}, |A| > n/2, t <= r/4, all x over A equal (to the pinned value)
    auto tryT = [&](int32_t t) {
      const Mask<W> A = g.ballot(ts >= t);
      if (mpopc(A) > n / 2 && t <= r4) {
        const int32_t xv = g.bcast(x, L.xs, mfirst(A));
        const bool allSame = !many(mand(A, g.ballot(x != xv)));
        if (allSame && (!zAny || xv == z0)) maj = true;
      }
    };
    tryT(INT32_MIN);
    Mask<W> rem = full;
    while (!maj && many(rem)) {
      const int32_t u = g.bcast(ts, L.tss, mfirst(rem));
      rem = mandn(rem, g.ballot(ts == u));
      tryT(u + 1);
    }
  }
  const bool inv0 = keep && (noDec || maj);
  const bool validity = X0.all_in(g, D, decision);
  const bool d0in = same && validity;
  const bool term = meq(D, full);
  const bool inv1 = term && d0in;
  const bool integrity = !anyD || d0in;
  const Mask<W> OLD = g.ballot((old_fl & F_DECIDED) != 0u);
  const bool irrev = !has_old || !many(mandn(OLD, mand(D, g.ballot(old_decision == decision))));
  const uint32_t fb = fbit(inv0 || inv1, 0) | fbit(inv0, 1) | fbit(inv1, 2) | fbit(same, 3) | fbit(validity, 4) |
                      fbit(integrity, 5) | fbit(irrev, 6);
  ck.record(fb, term, c, g.lane);
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

// Kernel body; SH = NoHook for the library's kernels, spec::SpecHook<GenSpec> in a
// fused Spec module (round_amd/formula.py compile_native(fused=True)).
template <int W, bool XHO, class SH = NoHook>
PSG_DEV void lv_body(const KArgs& a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[2 * W];
  __shared__ int64_t red[2 * W];
  __shared__ LvLds<W> L;
  __shared__ int32_t x0tab[Geometry<W>::kGroups][X0Set<W>::kSlots];
  counters_init(&bc);
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

  InstanceQueue<W> Q;  // dynamic instance distribution (psg_device.hpp)
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    Sched<W, XHO> sc;
    sc.setup(a, inst, g.pid, g.valid);
    sc.prep_good(0, g.lane, a.R);
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? a.init[init_row(a, i, inst) * (uint64_t)n + g.pid] : sc.init_value(g.pid, PSG_ALG_LAST_VOTING);
    X0Set<W> X0;
    X0.build(g, x0tab[grp], x0);
    // LVProcess state after init(io) (LastVoting.scala:82-109)
    int32_t x = x0, ts = -1, vote = 0, decision = -1;
    uint32_t fl = g.valid ? 0u : F_HALTED;
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    typename SH::template State<W> sh(g, grp, n);  // fused Spec evaluation state (NoHook: empty)
    if constexpr (!SH::kFused) lv_check<W>(g, L, X0, ck, 0, false, n, full, x, ts, vote, decision, fl, 0u, -1);
    auto trace = [&](int c, int32_t hs) {
      emit_state<W, SH>(sh, g, a, i, c, x, (fl & F_DECIDED) ? 1 : 0, decision, ts, (fl & F_READY) ? 1 : 0,
                   (fl & F_COMMIT) ? 1 : 0, vote, 0, hs);
    };
    if (tracing<SH>(a)) trace(0, n);

    for (int k = 0; k < a.R; ++k) {
      const uint32_t old_fl = fl;
      const int32_t old_decision = decision;
      const Mask<W> act = g.ballot((fl & F_HALTED) == 0u);
      int32_t hs = n;  // |mailbox| of this round (Spec field HOSIZE)
      if (many(act)) {
        const int32_t phase = k >> 2;
        const int c = phase % n;
        const bool cAlive = mtest(act, c);
        const uint32_t live = (fl & F_HALTED) ? 0u : 1u;
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) {
          CB = g.ballot(sc.crash_round >= 0 && sc.crash_round < k);
          CN = g.ballot(sc.crash_round == k);
        }
        const Mask<W> HO = sc.ho(k, g.pid, good, goodS, CB, CN);
        lv_stage<W>(g, L, x, ts, vote, decision);
        switch (k & 3) {
          case 0: {  // R0: send (x, ts) to coord; coord picks vote = x of maxBy ts
            const Mask<W> Mc = mand(ho_of<W>(g, L, HO, c), act);
            const int size = mpopc(Mc);
            hs = g.pid == c ? size : 0;
            if (cAlive && (size > n / 2 || (k == 0 && size > 0))) {
              const int32_t v = maxby_ts_x<W>(g, L.xs, Mc, size, x, ts, myh, a.tiebreak);
              if (g.pid == c) {
                vote = v;
                fl |= F_COMMIT;
              }
            }
            break;
          }
          case 1: {  // R1: coord broadcasts vote if commit; receivers adopt (x, ts = r/4)
            const bool sent = cAlive && mtest(g.ballot((fl & F_COMMIT) != 0u), c);
            hs = sent && mtest(HO, c) ? 1 : 0;
            if (sent) {
              const int32_t vc = g.bcast(vote, L.votes, c);
              const uint32_t rcv = live & (mtest(HO, c) ? 1u : 0u);
              x = rcv ? vc : x;
              ts = rcv ? phase : ts;
            }
            break;
          }
          case 2: {  // R2: ts == r/4 send x to coord; coord ready on a majority
            const Mask<W> Mc = mand(mand(ho_of<W>(g, L, HO, c), act), g.ballot(ts == phase));
            hs = g.pid == c ? mpopc(Mc) : 0;
            if (cAlive && mpopc(Mc) > need2 && g.pid == c) fl |= F_READY;
            break;
          }
          default: {  // R3: coord broadcasts vote if ready; receivers decide and exit
            const bool sent = cAlive && mtest(g.ballot((fl & F_READY) != 0u), c);
            hs = sent && mtest(HO, c) ? 1 : 0;
            if (sent) {
              const int32_t vc = g.bcast(vote, L.votes, c);
              const uint32_t rcv = live & (mtest(HO, c) ? 1u : 0u);
              const uint32_t first = rcv & (dec_round < 0 ? 1u : 0u);
              dec_val = first ? vc : dec_val;
              dec_round = first ? k : dec_round;
              decision = rcv ? vc : decision;
              halt_round = rcv ? k : halt_round;
              fl |= rcv ? (F_DECIDED | F_HALTED) : 0u;
            }
            // ready = false; commit = false for every process that took this step
            fl &= live ? ~(F_READY | F_COMMIT) : ~0u;
            break;
          }
        }
      }
      if constexpr (!SH::kFused) lv_check<W>(g, L, X0, ck, k + 1, true, n, full, x, ts, vote, decision, fl, old_fl, old_decision);
      if (tracing<SH>(a)) trace(k + 1, (old_fl & F_HALTED) ? n : hs);
    }
    finish_instance<W>(g, a, i, SH::kFused ? sh.ck : ck, SH::kFused ? SH::kSlots : 7, dec_val, dec_round, halt_round, x, &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, SH::kFused ? SH::kSlots : 7, a.R);
}

template <int W, bool XHO, class SH = NoHook>
__global__ void __launch_bounds__(Geometry<W>::kThreads) lv_kernel(KArgs a) {
  lv_body<W, XHO, SH>(a);
}

#ifndef PSG_FUSED_MODULE  // host launchers (not part of a fused Spec module)
template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if (a.ho_in) hipLaunchKernelGGL((lv_kernel<W, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((lv_kernel<W, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
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
    case 1: return (const void*)lv_kernel<1, false>;
    case 2: return (const void*)lv_kernel<2, false>;
    case 3: return (const void*)lv_kernel<3, false>;
    case 4: return (const void*)lv_kernel<4, false>;
  }
  return nullptr;
}

#endif  // PSG_FUSED_MODULE

}  // namespace psg
