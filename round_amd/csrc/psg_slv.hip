// psg_slv.hip — ShortLastVoting (3-round LastVoting variant) on gfx950.
//
// Reference: example/ShortLastVoting.scala:13-119 (SlvProcess). Phase of three
// rounds with the coordinator coord(r/4) = (r/4) % n taken literally from the
// source (r/4 although the phase has 3 rounds, ShortLastVoting.scala:37):
//   R0  every process sends (x, ts) to the coordinator; with a majority it takes
//       vote = x of mailbox.maxBy(ts) and commits (shared maxby_ts_x helper);
//   R1  a committed coordinator broadcasts vote; receivers adopt x = vote, ts = r/4;
//   R2  processes with ts == r/4 broadcast x; a receiver with a majority decides
//       mailbox.head._2 (first entry in Scala Map iteration order of ITS mailbox)
//       and exits; commit is cleared.
// The R2 head is resolved per receiver: if every R2 sender holds the same x the
// head's value is that x; otherwise each lane walks the CHAMP trie of its own
// mailbox (champ_first over a per-block fragment table). The fallback is
// defensive: an R2 sender at round k = 3φ+2 has ts == k/4, and only the R1 of the
// same phase (k-1) can have set that ts — (3ψ+1)/4 != (3φ+2)/4 for every ψ < φ
// because 4 consecutive integers hold a multiple of 4 — so every R2 sender holds
// that R1's single broadcast vote. champ_first is checked against the oracle's
// Map order by psg_selftest_map_head.
// Spec: TrivialSpec; the build checks uniform agreement (k = 1 over every
// decider, HO-model consensus) and validity.
#ifndef __HIPCC_RTC__
#include <type_traits>
#endif

#include "psg_device.hpp"
#include "psg_kernels.hpp"

namespace psg {

enum : uint32_t { S_DECIDED = 1u, S_COMMIT = 2u, S_HALTED = 4u };

template <int W>
struct SlvLds {
  int32_t xs[W > 1 ? 64 * W : 1];
  int32_t votes[W > 1 ? 64 * W : 1];
  int32_t ds[W > 1 ? 64 * W : 1];
  uint64_t hos[W > 1 ? 64 * W * W : 1];
};

// The coordinator's HO mask (uniform).
template <int W>
PSG_DEV Mask<W> slv_ho_of(Grp<W>& g, SlvLds<W>& L, const Mask<W>& ho, int c) {
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
template <int W, bool XHO, class SH = NoHook, bool TR = true>
PSG_DEV void slv_body(const KArgs& a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int32_t crl[W > 1 ? 64 * W : 1];
  __shared__ int64_t red[2 * W];
  __shared__ SlvLds<W> L;
  __shared__ ChampTable<W> CT;
  __shared__ int32_t x0tab[Geometry<W>::kGroups][X0Set<W>::kSlots];
  counters_init(&bc);
  CT.build(a.n);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = a.n;
  const int need2 = a.variant == 1 ? 0 : n / 2;  // R2 quorum (ShortLastVoting.scala:85; variant 1: mutation)
  const Mask<W> full = mfull<W>(n);
  const uint32_t myh = scala_improve((uint32_t)g.pid);

  InstanceQueue<W, 0, W == 1 ? PSG_QUEUE_CHUNK_LANE : 0> Q;  // dynamic instance distribution (psg_device.hpp)
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    Sched<W, XHO> sc;
    sc.setup(a, inst, g.pid, g.valid);
    CrashSets<W> cs;  // per-instance crash rounds (no per-round exchange for W > 1)
    if (sc.crash_on) cs.prep(g, crl, sc.crash_round);
    sc.prep_good(0, g.lane, a.R);
    int32_t x0 = 0;
    if (g.valid) x0 = a.init ? init_x(a, i, inst, g.pid) : sc.init_value(g.pid, PSG_ALG_SLV);
    X0Set<W> X0;
    X0.build(g, x0tab[grp], x0);
    // SlvProcess state after init(io) (ShortLastVoting.scala:15-31)
    int32_t x = x0, ts = -1, vote = 0, decision = -1;
    uint32_t fl = g.valid ? 0u : S_HALTED;
    int32_t dec_val = 0, dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    typename SH::template State<W> sh(g, grp, n);  // fused Spec evaluation state (NoHook: empty)
    auto check = [&](int c) {
      if constexpr (W > 1) {
        L.ds[g.pid] = decision;
        __syncthreads();
      }
      kagree_check<W>(g, ck, c, 1, full, (fl & S_DECIDED) != 0u, decision, X0, false, L.ds);
    };
    if constexpr (!SH::kFused) check(0);
    auto trace = [&](int c, int32_t hs, bool frozen = false) {
      emit_state<W, SH>(sh, g, a, i, c, x, (fl & S_DECIDED) ? 1 : 0, decision, ts, 0, (fl & S_COMMIT) ? 1 : 0, vote, 0, hs,
                        frozen);
    };
    if (tracing<SH, TR>(a)) trace(0, n);

    // one round of slot RS = k mod 3 (compile time: each slot's step specialized)
    auto round = [&](const int k, auto RSc) {
      constexpr int RS = decltype(RSc)::value;
      const Mask<W> act = g.ballot((fl & S_HALTED) == 0u);
      const uint32_t fl_start = fl;
      int32_t hs = n;  // |mailbox| of this round (Spec field HOSIZE)
      if (many(act)) {
        const int32_t r4 = k >> 2;
        const int c = r4 % n;
        const bool cAlive = mtest(act, c);
        const uint32_t live = (fl & S_HALTED) ? 0u : 1u;
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) cs.sets(g, k, CB, CN);
        // R1 reads only bit coord of HO(p), and only when the coordinator sends
        // (ShortLastVoting.scala:53): the other rounds' and silent R1s' draws are skipped
        const bool sent = RS == 1 && cAlive && mtest(g.ballot((fl & S_COMMIT) != 0u), c);
        Mask<W> HO = mzero<W>();
        if (RS != 1 || sent) HO = sc.ho(k, g.pid, good, goodS, CB, CN);
        if constexpr (W > 1) {
          L.xs[g.pid] = x;
          L.votes[g.pid] = vote;
          __syncthreads();
        }
        if constexpr (RS == 0) {  // R0 (ShortLastVoting.scala:34-47)
          const Mask<W> Mc = mand(slv_ho_of<W>(g, L, HO, c), act);
          const int size = mpopc(Mc);
          hs = g.pid == c ? size : 0;
          if (cAlive && size > n / 2) {
            const int32_t v = maxby_ts_x<W>(g, L.xs, Mc, size, x, ts, myh, a.tiebreak, &CT);
            if (g.pid == c) {
              vote = v;
              fl |= S_COMMIT;
            }
          }
        } else if constexpr (RS == 1) {  // R1 (ShortLastVoting.scala:51-69)
          hs = sent && mtest(HO, c) ? 1 : 0;
          if (sent) {
            const int32_t vc = g.bcast(vote, L.votes, c);
            const uint32_t rcv = live & (mtest(HO, c) ? 1u : 0u);
            x = rcv ? vc : x;
            ts = rcv ? r4 : ts;
          }
        } else {  // R2 (ShortLastVoting.scala:72-98)
          const Mask<W> S = mand(act, g.ballot(ts == r4));
          const Mask<W> M = mand(HO, S);
          hs = mpopc(M);
          const bool upd = live && mpopc(M) > need2 && (fl & S_DECIDED) == 0u;
          if (g.any(upd)) {
            const int32_t xs0 = g.bcast(x, L.xs, mfirst(S));
            const bool uniform = !many(mand(S, g.ballot(x != xs0)));
            int32_t v = xs0;
            if (!uniform) {
              const int h = upd ? champ_first<W>(CT, M, a.tiebreak) : g.pid;  // mailbox.head
              v = g.gather(x, L.xs, h);
            }
            if (upd) {
              dec_val = v;
              dec_round = k;
              decision = v;
              fl |= S_DECIDED;
            }
          }
          if (live) {
            fl &= ~S_COMMIT;
            if (fl & S_DECIDED) {
              fl |= S_HALTED;
              halt_round = k;
            }
          }
        }
      }
      if constexpr (!SH::kFused) check(k + 1);
      if (tracing<SH, TR>(a)) trace(k + 1, (fl_start & S_HALTED) ? n : hs);
    };
    // Quiescent tail (as lv_body's). At a phase boundary, once at most n/2 processes are not
    // halted and none of them is commit, no process can take an effective step again: R0's
    // commit needs a mailbox of more than n/2 (ShortLastVoting.scala:39), R2's decision more
    // than n/2 (85; the unmutated quorum), R1 sends only from a commit coordinator (53), and R2's
    // reset finds the flag clear — the state is final. Rounds kq .. R-1 then draw no HO set and
    // run no step; the check is still evaluated at every check point. Not taken when a trace or
    // the fused Spec reads |mailbox|.
    const bool hs_read = SH::kFused ? ((SH::kFields >> PSG_FIELD_HOSIZE) & 1u) != 0u
                                    : (TR && a.trace != nullptr && ((a.trace_fields >> PSG_FIELD_HOSIZE) & 1u));
    const bool qok = a.variant == 0 && !hs_read;
    int kq = a.R;
    for (int k0 = 0; k0 < a.R; k0 += 3) {
      if (qok && k0 > 0) {
        const Mask<W> live = g.ballot((fl & S_HALTED) == 0u);
        if (2 * mpopc(live) <= n && !g.any((fl & (S_HALTED | S_COMMIT)) == S_COMMIT)) {
          kq = k0;
          break;
        }
      }
      round(k0, Slot<0>{});
      if (k0 + 1 < a.R) round(k0 + 1, Slot<1>{});
      if (k0 + 2 < a.R) round(k0 + 2, Slot<2>{});
    }
    for (int k = kq; k < a.R; ++k) {
      if constexpr (!SH::kFused) check(k + 1);
      if (tracing<SH, TR>(a)) trace(k + 1, n, true);
    }
    finish_instance<W>(g, a, i, SH::kFused ? sh.ck : ck, SH::kFused ? SH::kSlots : 2, dec_val, dec_round, halt_round, x, &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, SH::kFused ? SH::kSlots : 2, a.R);
}

#ifndef PSG_SLV_WPE
#define PSG_SLV_WPE 7  // W = 1 occupancy target: 7 measured 65.2 ms vs 6: 66.0, compiler (5): 70.5 (W2 row)
#endif
template <int W, bool XHO, class SH = NoHook, bool TR = true>
__global__ void __launch_bounds__(Geometry<W>::kThreads) __attribute__((amdgpu_waves_per_eu(W == 1 ? PSG_SLV_WPE : 1)))
slv_kernel(KArgs a) {
  slv_body<W, XHO, SH, TR>(a);
}

#ifndef PSG_FUSED_MODULE  // host launchers (not part of a fused Spec module)
template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if (a.ho_in) hipLaunchKernelGGL((slv_kernel<W, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else if (a.trace) hipLaunchKernelGGL((slv_kernel<W, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((slv_kernel<W, false, NoHook, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_slv(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1>(a, grid, s);
    case 2: return launch_w<2>(a, grid, s);
    case 3: return launch_w<3>(a, grid, s);
    case 4: return launch_w<4>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

const void* slv_kernel_ptr(int W) {
  switch (W) {
    case 1: return (const void*)slv_kernel<1, false, NoHook, false>;
    case 2: return (const void*)slv_kernel<2, false, NoHook, false>;
    case 3: return (const void*)slv_kernel<3, false, NoHook, false>;
    case 4: return (const void*)slv_kernel<4, false, NoHook, false>;
  }
  return nullptr;
}

// Self-test of champ_first (psg_selftest_map_head): one lane per pid set (n <= 64).
__global__ void __launch_bounds__(256) champ_selftest_kernel(const uint64_t* sets, int count, int tiebreak,
                                                            int32_t* out) {
  __shared__ ChampTable<1> CT;
  CT.build(64);
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) {
    Mask<1> m;
    m.w[0] = sets[i];
    out[i] = champ_first<1>(CT, m, tiebreak);
  }
}

hipError_t launch_champ_selftest(const uint64_t* sets, int count, int tiebreak, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(champ_selftest_kernel, dim3((count + 255) / 256), dim3(256), 0, s, sets, count, tiebreak, out);
  return hipGetLastError();
}

#endif  // PSG_FUSED_MODULE

}  // namespace psg
