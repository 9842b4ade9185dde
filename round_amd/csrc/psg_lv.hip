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

template <int W>
struct LvLds {
  int32_t xs[W > 1 ? 64 * W : 1];
  int32_t tss[W > 1 ? 64 * W : 1];
  int32_t votes[W > 1 ? 64 * W : 1];
  int32_t ds[W > 1 ? 64 * W : 1];
  int32_t flags[W > 1 ? 64 * W : 1];  // bit0 decided, bit1 commit, bit2 ready
  uint64_t hos[W > 1 ? 64 * W * W : 1];
};

template <int W>
PSG_DEV void lv_stage(Grp<W>& g, LvLds<W>& L, int32_t x, int32_t ts, int32_t vote, int32_t decision, bool decided,
                      bool commit, bool ready) {
  if constexpr (W > 1) {
    L.xs[g.pid] = x;
    L.tss[g.pid] = ts;
    L.votes[g.pid] = vote;
    L.ds[g.pid] = decision;
    L.flags[g.pid] = (decided ? 1 : 0) | (commit ? 2 : 0) | (ready ? 4 : 0);
    __syncthreads();
  }
}

// Spec check at check point c (spec r = c). Slots: 0 Safety, 1 Invariant0
// (keepInit && (noDecision || majority)), 2 Invariant1, 3 Agreement, 4 Validity,
// 5 Integrity, 6 Irrevocability. roundInvariants(j-1)(0) is `true` for every j.
template <int W>
PSG_DEV void lv_check(Grp<W>& g, LvLds<W>& L, const X0Set<W>& X0, Checks& ck, int c, bool has_old, int n,
                      const Mask<W>& full, int32_t x, int32_t ts, int32_t vote, int32_t decision, bool decided, bool commit, bool ready,
                      bool old_decided, int32_t old_decision) {
  lv_stage<W>(g, L, x, ts, vote, decision, decided, commit, ready);
  const int32_t r4 = c / 4;
  const int coord = r4 % n;
  const Mask<W> D = g.ballot(decided);
  const bool anyD = many(D);
  int32_t d0 = 0;
  bool same = true;
  if (anyD) {
    d0 = g.bcast(decision, L.ds, mfirst(D));
    same = !g.any(decided && decision != d0);
  }
  // keepInit: P.forall(i => P.exists(j1 => i.x == init(j1.x))) — one X0-set probe per lane
  const bool keep = !g.any(!X0.contains(x));
  const bool noDec = !g.any(decided || ready);
  // values pinned by (decided ==> decision == v), (commit ==> vote == v), (ready ==> vote == v)
  const Mask<W> Pm = g.ballot(decided || commit || ready);
  const bool zAny = many(Pm);
  int32_t z0 = 0;
  bool zOk = true;
  if (zAny) {
    const int q = mfirst(Pm);
    const int32_t fq = g.bcast((decided ? 1 : 0), L.flags, q) & 1;
    z0 = fq ? g.bcast(decision, L.ds, q) : g.bcast(vote, L.votes, q);
    zOk = !g.any((decided && decision != z0) || ((commit || ready) && vote != z0));
  }
  const bool commitCoord = (g.bcast((decided ? 1 : 0) | (commit ? 2 : 0) | (ready ? 4 : 0), L.flags, coord) & 2) != 0;
  const bool c5 = commitCoord || !g.any(ts == r4);  // (i.ts == r/4) ==> coord.commit
  bool maj = false;
  if (c > 0 && zOk && c5) {
    // exists t: A = {i : i.ts >= t}, |A| > n/2, t <= r/4, all x over A equal (to the pinned value)
    auto tryT = [&](int32_t t) {
      const Mask<W> A = g.ballot(ts >= t);
      if (mpopc(A) > n / 2 && t <= r4) {
        const int32_t xv = g.bcast(x, L.xs, mfirst(A));
        const bool allSame = !g.any(ts >= t && x != xv);
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
  const bool d0in = anyD && rfl32(X0.contains(d0) ? 1 : 0) != 0;
  const bool term = meq(D, full);
  const bool inv1 = term && same && d0in;
  const bool validity = !g.any(decided && !X0.contains(decision));
  const bool integrity = !anyD || (same && d0in);
  const bool irrev = !has_old || !g.any(old_decided && !(decided && old_decision == decision));
  const uint32_t fb = fbit(inv0 || inv1, 0) |
                      fbit(inv0, 1) |
                      fbit(inv1, 2) |
                      fbit(same, 3) |
                      fbit(validity, 4) |
                      fbit(integrity, 5) |
                      fbit(irrev, 6);
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

template <int W>
__global__ void __launch_bounds__(Geometry<W>::kThreads) lv_kernel(KArgs a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[2 * W];
  __shared__ int64_t red[2 * W];
  __shared__ LvLds<W> L;
  __shared__ int32_t x0tab[Geometry<W>::kGroups][X0Set<W>::kSlots];
  counters_init(&bc);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  constexpr int G = Geometry<W>::kGroups;
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = a.n;
  const int need2 = a.variant == 1 ? 0 : n / 2;  // R2 quorum (LastVoting.scala:177; variant 1: mutation)
  const Mask<W> full = mfull<W>(n);
  const uint32_t myh = scala_improve((uint32_t)g.pid);

  for (uint64_t i = (uint64_t)blockIdx.x * G + grp; i < a.count; i += (uint64_t)gridDim.x * G) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    Sched<W> sc;
    sc.setup(a, inst, g.pid, g.valid);
    sc.prep_good(0, g.lane, a.R);
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? a.init[i * (uint64_t)n + g.pid] : sc.init_value(g.pid, PSG_ALG_LAST_VOTING);
    // LVProcess state after init(io) (LastVoting.scala:82-109)
    X0Set<W> X0;
    X0.build(g, x0tab[grp], x0);
    int32_t x = x0, ts = -1, vote = 0, decision = -1;
    bool ready = false, commit = false, decided = false, halted = false;
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    lv_check<W>(g, L, X0, ck, 0, false, n, full, x, ts, vote, decision, decided, commit, ready, false, -1);

    for (int k = 0; k < a.R; ++k) {
      const bool old_decided = decided;
      const int32_t old_decision = decision;
      const Mask<W> act = g.ballot(!halted);
      if (many(act)) {
        const int32_t phase = k >> 2;
        const int c = phase % n;
        const bool cAlive = mtest(act, c);
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) {
          CB = g.ballot(sc.crash_round >= 0 && sc.crash_round < k);
          CN = g.ballot(sc.crash_round == k);
        }
        const Mask<W> HO = sc.ho(k, g.pid, good, goodS, CB, CN);
        lv_stage<W>(g, L, x, ts, vote, decision, decided, commit, ready);
        const int32_t cflags = g.bcast((decided ? 1 : 0) | (commit ? 2 : 0) | (ready ? 4 : 0), L.flags, c);
        switch (k & 3) {
          case 0: {  // R0: send (x, ts) to coord; coord picks vote = x of maxBy ts
            const Mask<W> Mc = mand(ho_of<W>(g, L, HO, c), act);
            const int size = mpopc(Mc);
            if (cAlive && (size > n / 2 || (k == 0 && size > 0))) {
              const bool inMc = mtest(Mc, g.pid);
              const int32_t maxts = g.max32(ts, inMc);
              const Mask<W> T = g.ballot(inMc && ts == maxts);
              const int q0 = mfirst(T);
              const int32_t xq0 = g.bcast(x, L.xs, q0);
              int win = q0;
              const bool differ = g.any(mtest(T, g.pid) && x != xq0);
              if (differ && a.tiebreak == PSG_TIE_CHAMP && size > 4) {
                // CHAMP order of the coordinator's mailbox: payload depth of each
                // candidate = longest 5-bit hash prefix shared with another entry.
                int depth = 0;
#pragma unroll
                for (int w = 0; w < W; ++w) {
                  uint64_t m = Mc.w[w];
                  while (m) {
                    const int f = w * 64 + __builtin_ctzll(m);
                    m &= m - 1;
                    if (f != g.pid) depth = max(depth, champ_cpl(myh, scala_improve((uint32_t)f)));
                  }
                }
                const bool inT = mtest(T, g.pid);
                const int64_t key = (int64_t)champ_key(myh, depth);
                const int64_t kmin = g.min64(key, inT);
                win = mfirst(g.ballot(inT && key == kmin));
              }
              const int32_t v = g.bcast(x, L.xs, win);
              if (g.pid == c) {
                vote = v;
                commit = true;
              }
            }
            break;
          }
          case 1: {  // R1: coord broadcasts vote if commit; receivers adopt (x, ts = r/4)
            if (cAlive && (cflags & 2)) {
              const int32_t vc = g.bcast(vote, L.votes, c);
              if (!halted && mtest(HO, c)) {
                x = vc;
                ts = phase;
              }
            }
            break;
          }
          case 2: {  // R2: ts == r/4 send x to coord; coord ready on a majority
            const Mask<W> Mc = mand(mand(ho_of<W>(g, L, HO, c), act), g.ballot(ts == phase));
            if (cAlive && mpopc(Mc) > need2 && g.pid == c) ready = true;
            break;
          }
          default: {  // R3: coord broadcasts vote if ready; receivers decide and exit
            if (cAlive && (cflags & 4)) {
              const int32_t vc = g.bcast(vote, L.votes, c);
              if (!halted && mtest(HO, c)) {
                if (dec_round < 0) {
                  dec_val = vc;
                  dec_round = k;
                }
                decision = vc;
                decided = true;
                halt_round = k;
              }
            }
            if (!halted) {
              ready = false;
              commit = false;
            }
            if (halt_round == k) halted = true;
            break;
          }
        }
      }
      lv_check<W>(g, L, X0, ck, k + 1, true, n, full, x, ts, vote, decision, decided, commit, ready, old_decided,
                  old_decision);
    }
    finish_instance<W>(g, a, i, ck, 7, dec_val, dec_round, halt_round, x, &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, 7, a.R);
}

template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(lv_kernel<W>, dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
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
    case 1: return (const void*)lv_kernel<1>;
    case 2: return (const void*)lv_kernel<2>;
    case 3: return (const void*)lv_kernel<3>;
    case 4: return (const void*)lv_kernel<4>;
  }
  return nullptr;
}

}  // namespace psg
