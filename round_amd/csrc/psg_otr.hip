// psg_otr.hip — OTR (one-third rule) on gfx950.
//
// Reference: example/Otr.scala:13-128 (OtrProcess, OTR.spec).
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
  int32_t x0s[W > 1 ? 64 * W : 1];
  int32_t ds[W > 1 ? 64 * W : 1];
};

// Spec check at check point c (spec r = c). Slots: 0 Safety (some invariant
// holds), 1..3 invariants, 4 Agreement, 5 Validity, 6 Integrity, 7 Irrevocability.
template <int W>
PSG_DEV void otr_check(Grp<W>& g, OtrLds<W>& L, Checks& ck, int c, bool has_old, int n, const Mask<W>& full,
                       int32_t x, int32_t x0, bool decided, int32_t decision, bool old_decided, int32_t old_decision) {
  const int sthr = (2 * n) / 3;  // 2*n/3 in the Spec (Otr.scala:101)
  if constexpr (W > 1) {
    L.xs[g.pid] = x;
    L.ds[g.pid] = decision;
    __syncthreads();
  }
  const Mask<W> D = g.ballot(decided);
  const bool anyD = many(D);
  int32_t d0 = 0;
  bool same = true;
  if (anyD) {
    d0 = g.bcast(decision, L.ds, mfirst(D));
    same = !g.any(decided && decision != d0);
  }
  // V.exists(v => |{i : i.x == v}| ... ) finitized over the current x values;
  // keepInit: P.forall(i => P.exists(j => i.x == init(j.x))).
  Mask<W> rem = full;
  bool e0 = false, e1 = false, keep = true;
  while (many(rem)) {
    const int32_t v = g.bcast(x, L.xs, mfirst(rem));
    const Mask<W> E = g.ballot(x == v);
    rem = mandn(rem, E);
    if (keep) keep = g.any(x0 == v);
    const int cnt = mpopc(E);
    const bool condv = !anyD || (same && v == d0);
    e0 = e0 || (cnt > sthr && condv);
    e1 = e1 || (cnt == n && condv);
  }
  const bool inv0 = (!anyD || e0) && keep;
  const bool inv1 = e1 && keep;
  const bool d0in = anyD && g.any(x0 == d0);
  const bool term = meq(D, full);
  const bool inv2 = term && same && d0in;
  bool validity = true;
  if (anyD) {
    if (same) {
      validity = d0in;
    } else {
      Mask<W> remD = D;
      while (many(remD)) {
        const int32_t dv = g.bcast(decision, L.ds, mfirst(remD));
        remD = mandn(remD, g.ballot(decided && decision == dv));
        if (validity) validity = g.any(x0 == dv);
      }
    }
  }
  const bool integrity = !anyD || (same && d0in);
  const bool irrev = !has_old || !g.any(old_decided && !(decided && old_decision == decision));
  const uint32_t fb = fbit(inv0 || inv1 || inv2, 0) |
                      fbit(inv0, 1) |
                      fbit(inv1, 2) |
                      fbit(inv2, 3) |
                      fbit(same, 4) |
                      fbit(validity, 5) |
                      fbit(integrity, 6) |
                      fbit(irrev, 7);
  ck.record(fb, term, c, g.lane);
}

template <int W>
__global__ void __launch_bounds__(Geometry<W>::kThreads) otr_kernel(KArgs a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[2 * W];
  __shared__ int64_t red[2 * W];
  __shared__ OtrLds<W> L;
  counters_init(&bc);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  constexpr int G = Geometry<W>::kGroups;
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = a.n;
  const int thr = a.variant == 1 ? n / 2 : (2 * n) / 3;  // Otr.scala:64, 67 (variant 1: mutation)
  const Mask<W> full = mfull<W>(n);

  for (uint64_t i = (uint64_t)blockIdx.x * G + grp; i < a.count; i += (uint64_t)gridDim.x * G) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    Sched<W> sc;
    sc.setup(a, inst, g.pid, g.valid);
    sc.prep_good(0, g.lane, a.R);
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? a.init[i * (uint64_t)n + g.pid] : sc.init_value(g.pid, PSG_ALG_OTR);
    // OtrProcess state after init(io) (Otr.scala:15-26)
    int32_t x = x0, decision = -1, after = a.param;
    bool decided = false, halted = false;
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    otr_check<W>(g, L, ck, 0, false, n, full, x, x0, decided, decision, false, -1);

    for (int k = 0; k < a.R; ++k) {
      const bool old_decided = decided;
      const int32_t old_decision = decision;
      const Mask<W> act = g.ballot(!halted);
      if (many(act)) {
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) {
          CB = g.ballot(sc.crash_round >= 0 && sc.crash_round < k);
          CN = g.ballot(sc.crash_round == k);
        }
        // mailbox: broadcast(x) from every alive sender in HO(p)
        const Mask<W> M = mand(sc.ho(k, g.pid, good, goodS, CB, CN), act);
        const bool upd = !halted && mpopc(M) > thr;
        if (g.any(upd)) {
          if constexpr (W > 1) {
            L.xs[g.pid] = x;
            __syncthreads();
          }
          // mmor: max multiplicity, ties -> smaller value (OtrExample.scala:67-75)
          Mask<W> rem = act;
          int best_c = 0;
          int32_t best_v = INT32_MAX;
          while (many(rem)) {
            const int32_t v = g.bcast(x, L.xs, mfirst(rem));
            const Mask<W> E = mand(g.ballot(x == v), act);
            rem = mandn(rem, E);
            const int cnt = mpopc(mand(M, E));
            const bool better = cnt > best_c || (cnt == best_c && v < best_v);
            best_c = better ? cnt : best_c;
            best_v = better ? v : best_v;
          }
          if (upd) {
            x = best_v;
            if (best_c > thr) {
              if (!decided) {  // callback.decide(v) only the first time (Otr.scala:68-70)
                dec_val = best_v;
                dec_round = k;
              }
              decided = true;
              decision = best_v;
            }
          }
        }
        if (!halted && decided) {  // Otr.scala:75-80
          after -= 1;
          if (after <= 0) {
            halt_round = k;
            halted = true;  // exitAtEndOfRound
          }
        }
      }
      otr_check<W>(g, L, ck, k + 1, true, n, full, x, x0, decided, decision, old_decided, old_decision);
    }
    finish_instance<W>(g, a, i, ck, 8, dec_val, dec_round, halt_round, x, &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, 8, a.R);
}

template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(otr_kernel<W>, dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_otr(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1>(a, grid, s);
    case 2: return launch_w<2>(a, grid, s);
    case 3: return launch_w<3>(a, grid, s);
    case 4: return launch_w<4>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

const void* otr_kernel_ptr(int W) {
  switch (W) {
    case 1: return (const void*)otr_kernel<1>;
    case 2: return (const void*)otr_kernel<2>;
    case 3: return (const void*)otr_kernel<3>;
    case 4: return (const void*)otr_kernel<4>;
  }
  return nullptr;
}

}  // namespace psg
