// psg_packed.hpp — lane-packed instances: one wave64 runs one instance of
// n <= 64*W processes, lane l holding the W processes l + 64*j ("slot" j).
//
// The group kernels (Grp<W>, W waves per instance) pay a block barrier and an LDS
// round trip for every cross-wave ballot or reduction, and every wave repeats the
// instance's uniform (scalar) work. Packed, a ballot of a per-process predicate is
// W wave ballots (slot j -> mask word j) with no exchange, "some process" is one
// ballot of the lane's OR over its slots, and the scalar work is done once per
// instance. Used by the fast paths whose per-process state is small (FloodMin's
// crash-stop path, BenOr's built-in checker).
#pragma once
#include "psg_device.hpp"

#ifndef PSG_PK_WPE
#define PSG_PK_WPE 5  // waves/SIMD the packed kernels are register-allocated for: 4 -> 5 measured
                      // +6 % (FloodMin C4 f=8 6.60 -> 6.26 ms) and +7 % (BenOr C5 42.6 -> 39.8 ms)
#endif

namespace psg {

template <int W>
struct Pk {
  int lane;
  uint64_t vm[W];    // uniform: lanes whose slot j is a process (pid < n)
  uint32_t val[W];   // per lane: 1 if slot j is a process
  PSG_DEV void setup(int n) {
    lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const int lo = j * 64;
      vm[j] = n >= lo + 64 ? ~0ull : (n <= lo ? 0ull : ((1ull << (n - lo)) - 1ull));
      val[j] = lane + lo < n ? 1u : 0u;
    }
  }
  PSG_DEV int pid(int j) const { return 64 * j + lane; }
  // mask of the processes whose 0/1 word is non-zero (slot j -> word j)
  PSG_DEV Mask<W> ballot(const uint32_t (&p)[W]) const {
    Mask<W> m;
#pragma unroll
    for (int j = 0; j < W; ++j) m.w[j] = __builtin_amdgcn_ballot_w64(p[j] != 0u) & vm[j];
    return m;
  }
  // value of process q (uniform) of a per-slot array
  PSG_DEV int32_t bcast(const int32_t (&v)[W], int q) const {
    int32_t r = readlane32(v[0], q & 63);
#pragma unroll
    for (int j = 1; j < W; ++j)
      if ((q >> 6) == j) r = readlane32(v[j], q & 63);
    return r;
  }
};

// First set pid of a non-empty mask, cleared from it (word-wise selects: a dynamic
// word index would send the mask to scratch memory).
template <int W>
PSG_DEV int mtake_first(Mask<W>& a) {
  int q = 0;
  bool done = false;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const bool here = !done && a.w[i] != 0ull;
    q = here ? i * 64 + (int)__builtin_ctzll(a.w[i]) : q;
    a.w[i] = here ? a.w[i] & (a.w[i] - 1ull) : a.w[i];
    done = done || here;
  }
  return q;
}

// Some lane's 0/1 word is set (uniform).
PSG_DEV bool pk_any(uint32_t p) { return __builtin_amdgcn_ballot_w64(p != 0u) != 0ull; }

// Crash rounds of the lane's W processes (Sched::setup's draw for each slot; -1 = correct).
template <int W>
PSG_DEV void pk_crash_rounds(const Pk<W>& P, const KArgs& a, uint64_t inst, int32_t (&cr)[W]) {
#pragma unroll
  for (int j = 0; j < W; ++j) cr[j] = -1;
  if (a.crash_fmax < 0) return;
  const uint64_t w0 = rword(a.seed, inst, ROUND_CRASH, PID_GLOBAL, 0);
  const uint64_t w1 = rword(a.seed, inst, ROUND_CRASH, PID_GLOBAL, 1);
#pragma unroll
  for (int j = 0; j < W; ++j)
    if (P.val[j]) cr[j] = Sched<W>::crash_of(a, inst, (uint32_t)P.pid(j), w0, w1);
}

// X0Set of the lane-packed instance's initial values (hash mode; the table is this wave's).
template <int W>
PSG_DEV void pk_x0_build(const Pk<W>& P, X0Set<W>& X, int32_t* lds, const int32_t (&x0)[W]) {
  constexpr int kSlots = X0Set<W>::kSlots;
  constexpr int32_t kEmpty = X0Set<W>::kEmpty;
  X.tab = lds;
  X.bmode = false;
  X.lo = 0;
  X.bm = 0;
  for (int t = P.lane; t < kSlots; t += 64) lds[t] = kEmpty;
  lds_sync<1>();
  uint32_t emp = 0;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const int32_t v = x0[j];
    emp |= P.val[j] & eq01(v, kEmpty);
    if (P.val[j] && v != kEmpty) {
      uint32_t h = X0Set<W>::slot(v);
      while (true) {
        const int32_t prev = atomicCAS(&lds[h], kEmpty, v);
        if (prev == kEmpty || prev == v) break;
        h = (h + 1) & (uint32_t)(kSlots - 1);
      }
    }
  }
  X.has_empty = pk_any(emp);
  lds_sync<1>();
}

// k-agreement over a packed instance (kagree_check): slot 0 — the decisions of never-
// crashed deciders number <= k; slot 1 — every decision is an initial value; termination
// when every process decided. notinit: per slot, "decided and its decision is not an initial
// value" — the X0 probe of a decision, taken by the caller when the decision is made (a
// decision never changes afterwards).
template <int W>
PSG_DEV void pk_kagree_check_m(const Pk<W>& P, Checks& ck, int c, int kk, const uint32_t (&decided)[W],
                               const int32_t (&decision)[W], const int32_t (&cr)[W], const uint32_t (&notinit)[W]) {
  uint32_t dc[W], undec = 0, bad = 0;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    dc[j] = P.val[j] & decided[j] & (cr[j] >= 0 ? 0u : 1u);
    undec |= P.val[j] & (1u - decided[j]);
    bad |= P.val[j] & decided[j] & notinit[j];
  }
  // |distinct decisions| from the deciders' min and max (two independent DPP reductions, no
  // scalar walk): none (mn > mx), one (mn == mx), or two plus a ballot for a third value; only
  // k >= 3 with a third value walks the values one by one
  uint32_t anyd = 0;
  int32_t lmn = INT32_MAX, lmx = INT32_MIN;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    anyd |= dc[j];
    lmn = dc[j] ? min(lmn, decision[j]) : lmn;
    lmx = dc[j] ? max(lmx, decision[j]) : lmx;
  }
  int distinct = 0;
  int32_t mn = 0, mx = 0;
  if (pk_any(anyd)) {  // (no correct decider: one ballot)
    mn = Grp<1>::dpp_reduce32<false>(lmn);
    mx = Grp<1>::dpp_reduce32<true>(lmx);
    distinct = mn == mx ? 1 : 2;
  }
  if (distinct == 2 && kk >= 2) {
    uint32_t third = 0;
#pragma unroll
    for (int j = 0; j < W; ++j) third |= dc[j] & ne01(decision[j], mn) & ne01(decision[j], mx);
    if (pk_any(third)) {
      distinct = 3;
      if (kk >= 3) {  // the general walk: one value per step, stopping past k
        Mask<W> Y = P.ballot(dc);
        distinct = 0;
        while (many(Y) && distinct <= kk) {
          const int32_t dv = P.bcast(decision, mfirst(Y));
          uint32_t eq[W];
#pragma unroll
          for (int j = 0; j < W; ++j) eq[j] = dc[j] & eq01(decision[j], dv);
          Y = mandn(Y, P.ballot(eq));
          ++distinct;
        }
      }
    }
  }
  ck.record(fbit(distinct <= kk, 0) | fbit(!pk_any(bad), 1), !pk_any(undec), c, P.lane);
}

// Per-instance epilogue of a packed instance (finish_instance for W slots per lane):
// the same digest (a sum over processes), decide results, summaries and counters.
template <int W, bool OPAQUE = true>
PSG_DEV void pk_finish(const Pk<W>& P, const KArgs& a, uint64_t i, const Checks& ck, int nchecks,
                       const int32_t (&dec_val)[W], const int32_t (&dec_round)[W], const int32_t (&halt_round)[W],
                       const int32_t (&main_x)[W], BlockCounters* bc) {
  const int n = a.n;
  uint64_t d = 0;
  uint32_t nd_l = 0, steps_l = 0;
  int32_t live_l = INT32_MIN;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    if (!P.val[j]) continue;
    const int pid = P.pid(j);
    const bool decided = dec_round[j] >= 0;
    d += proc_digest<OPAQUE>(pid, dec_val[j], dec_round[j], halt_round[j], main_x[j]);
    nd_l += decided ? 1u : 0u;
    const int32_t steps = halt_round[j] >= 0 ? halt_round[j] + 1 : a.R;
    steps_l += (uint32_t)steps;
    live_l = steps > live_l ? steps : live_l;
    const uint64_t off = i * (uint64_t)n + (uint64_t)pid;
    if (a.out_decision) a.out_decision[off] = dec_val[j];
    if (a.out_dround) a.out_dround[off] = decided ? (uint8_t)dec_round[j] : (uint8_t)0xFF;
    if (a.out_rec) {
      psg_process_record r;
      r.decision = dec_val[j];
      r.decision_round = dec_round[j];
      r.halt_round = halt_round[j];
      r.final_x = main_x[j];
      a.out_rec[off] = r;
    }
  }
  Grp<1> g1;
  const uint64_t dig = g1.wave_sum64(d);
  const uint32_t nd = Grp<1>::wave_sum32(nd_l);
  const uint32_t wave_steps = Grp<1>::wave_sum32(steps_l);
  const int32_t live = Grp<1>::dpp_reduce32<true>(live_l);
  const uint32_t term = ck.term_round();
  if (a.out_inst) {
    uint8_t* o = reinterpret_cast<uint8_t*>(a.out_inst + i);
    if (P.lane < PSG_MAX_CHECKS) o[8 + P.lane] = (uint8_t)ck.ffv;  // first_fail[lane]
    if (P.lane == 0) {
      *reinterpret_cast<uint64_t*>(o) = dig;
      o[8 + PSG_MAX_CHECKS] = (uint8_t)term;
      o[9 + PSG_MAX_CHECKS] = (uint8_t)nchecks;
      *reinterpret_cast<uint16_t*>(o + 10 + PSG_MAX_CHECKS) = (uint16_t)nd;
    }
  }
  if (P.lane < nchecks && ck.failed_here()) atomicAdd(&bc->fail[P.lane], 1u);
  if (P.lane == 0) {
    atomicAdd(&bc->hist[term == PSG_NEVER ? a.R + 1 : term], 1u);
    atomicAdd(&bc->decided, nd);
    atomicAdd(&bc->digest, (unsigned long long)dig);
    atomicAdd(&bc->live, (unsigned long long)live);
    atomicAdd(&bc->active, (unsigned long long)wave_steps);
  }
}

#ifndef PSG_FUSED_MODULE  // host code: not part of a fused Spec module (hiprtc has no host API)
// Blocks of packed kernels: 256 threads = 4 instances; grid = resident blocks
// (one cached occupancy per kernel, keyed by algorithm and W).
template <int ALG, int W>
static int pk_grid(const void* kernel, uint64_t count) {
  static const int resident = [kernel] {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0);
    return (per_cu < 1 ? 1 : per_cu) * (cus < 1 ? 1 : cus);
  }();
  const uint64_t want = (count + 3) / 4;
  return (int)(want < (uint64_t)resident ? (want < 1 ? 1 : want) : (uint64_t)resident);
}
#endif  // PSG_FUSED_MODULE

}  // namespace psg
