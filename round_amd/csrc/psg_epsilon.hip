// psg_epsilon.hip — EpsilonConsensus (approximate agreement on Doubles) on gfx950.
//
// Reference: example/Epsilon.scala:16-70 (EpsilonProcess). One round: broadcast
// (x, r > maxR); V = mailbox values ++ halted.values; at r = 0
// maxR = ceil(log(diff(V)/eps) / log(c(n-3f, 2f))) and x = reduce(2f, V).head;
// while r <= maxR, x = mean of every 2f-th element of V sorted with its f lowest
// and f highest dropped; afterwards decide(x) and exit.
//
// Per round the group sorts all n current values once (rank by a 64-bit
// Double.compare total-order key, scatter to LDS), and every lane walks the
// sorted list keeping only the members of its own V: its mailbox plus the
// halted senders it heard announce (a per-lane pid mask; a halted process's x is
// frozen, so the value it announced is its current x). Every arithmetic step is
// the IEEE operation the Scala code performs in the same order (ascending left
// fold from 0.0, one division), so values match the oracle bit for bit; only
// log() can differ by an ulp between libm implementations, which moves maxR
// only when r1 is within an ulp of an integer (parity tolerance in the tests).
#include "psg_device.hpp"
#include "psg_kernels.hpp"

namespace psg {

// java.lang.Double.compare order as a signed 64-bit key (-0.0 < 0.0, canonical NaN last)
PSG_DEV int64_t total_key(double d) {
  int64_t b = __double_as_longlong(d);
  if (d != d) b = 0x7ff8000000000000LL;
  return b ^ ((b >> 63) & 0x7fffffffffffffffLL);
}
PSG_DEV double key_value(int64_t k) { return __longlong_as_double(k ^ ((k >> 63) & 0x7fffffffffffffffLL)); }

// Java narrowing double -> int (math.ceil(r1).toInt)
PSG_DEV int32_t d2i(double d) {
  if (d != d) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}

PSG_DEV int32_t fold32d(double d) {
  const uint64_t b = (uint64_t)__double_as_longlong(d);
  return (int32_t)(uint32_t)(b ^ (b >> 32));
}

template <int W>
struct EpsLds {
  double sx[Geometry<W>::kGroups][64 * W];
  int32_t spid[Geometry<W>::kGroups][64 * W];
  int64_t keys[W > 1 ? 64 * W : 1];
};

// Ascending bitonic sort of (key, pid) pairs over the 64 lanes of a wave (pairs must
// be distinct; pids are). Stage (size, d): partners lane ^ d exchange through the LDS
// crossbar; the lower lane of a pair keeps the smaller pair in an ascending block.
template <int SIZE, int D>
PSG_DEV void sort_stage(int64_t& key, int32_t& pid, int lane) {
  const int64_t pk = (int64_t)xshfl64<D>((uint64_t)key, lane);
  const int32_t pp = (int32_t)xshfl<D>((uint32_t)pid, lane);
  const bool less = pk < key || (pk == key && pp < pid);  // partner's pair precedes mine
  const bool take = less != (((lane & D) != 0) != ((lane & SIZE) != 0));
  key = take ? pk : key;
  pid = take ? pp : pid;
  if constexpr (D > 1) sort_stage<SIZE, D / 2>(key, pid, lane);
}
template <int SIZE = 2>
PSG_DEV void wave_sort_key_pid(int64_t& key, int32_t& pid, int lane) {
  sort_stage<SIZE, SIZE / 2>(key, pid, lane);  // partners exchange in registers (xshfl)
  if constexpr (SIZE < 64) wave_sort_key_pid<SIZE * 2>(key, pid, lane);
}

// 64 x 64 bit-matrix transpose across a wave: lane i holds row i; afterwards lane j holds
// column j (bit i = bit j of row i). The six swap stages of the block transpose: at stage
// s, the lane pair (i, i ^ s) exchanges the off-diagonal s x s blocks of its 2s x 2s block.
template <int S, uint64_t LO>
PSG_DEV uint64_t transpose_stage(uint64_t r, int lane) {
  const uint64_t p = xshfl64<S>(r, lane);
  return (lane & S) ? ((r & ~LO) | ((p & ~LO) >> S)) : ((r & LO) | ((p & LO) << S));
}
PSG_DEV uint64_t wave_transpose64(uint64_t r, int lane) {
  r = transpose_stage<32, 0x00000000FFFFFFFFull>(r, lane);
  r = transpose_stage<16, 0x0000FFFF0000FFFFull>(r, lane);
  r = transpose_stage<8, 0x00FF00FF00FF00FFull>(r, lane);
  r = transpose_stage<4, 0x0F0F0F0F0F0F0F0Full>(r, lane);
  r = transpose_stage<2, 0x3333333333333333ull>(r, lane);
  return transpose_stage<1, 0x5555555555555555ull>(r, lane);
}

// Slots: 0 EpsAgreement (no NaN decision, max - min <= eps), 1 EpsValidity (every
// decision within [min, max] of the non-NaN initial values), 2 SafetyPredicate
// (|V| >= n - f for every process that took a step). Termination: all decided.
template <int W>
PSG_DEV void eps_check(Grp<W>& g, Checks& ck, int c, const Mask<W>& full, bool decided, double decision, double eps,
                       bool anyI, double lo, double hi, bool pred) {
  const bool nanD = g.any(decided && decision != decision);
  const bool ok = decided && decision == decision;
  const bool anyD = g.any(ok);
  const int64_t kd = total_key(decision);
  const double mx = key_value(g.max64(kd, ok));
  const double mn = key_value(g.min64(kd, ok));
  const bool agree = !nanD && (!anyD || mx - mn <= eps);
  const bool valid = !g.any(decided && !(anyI && lo <= decision && decision <= hi));
  ck.record(fbit(agree, 0) | fbit(valid, 1) | fbit(pred, 2), meq(g.ballot(decided), full), c, g.lane);
}

#ifndef PSG_EPS_WPE
#define PSG_EPS_WPE 6  // W = 1 occupancy target: 6 is scratch-free (7 spilled 40 B: log()'s hoisted f64 constants); 14.23 vs 14.13 ms at 7 (W2 row, round-4 A/B)
#endif
template <int W, bool XHO>
__global__ void __launch_bounds__(Geometry<W>::kThreads) __attribute__((amdgpu_waves_per_eu(W == 1 ? PSG_EPS_WPE : 1)))
epsilon_kernel(KArgs a) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int32_t crl[W > 1 ? 64 * W : 1];
  __shared__ int64_t red[2 * W];
  __shared__ EpsLds<W> L;
  counters_init(&bc);
  __syncthreads();
  Grp<W> g;
  grp_setup(g, a, xb, red);
  // wave-uniform group index (SGPR): measured +3% on this kernel (fewer VGPRs, one more wave/SIMD);
  // the same change cost OTR / ShortLastVoting 1-3%, which keep the VGPR form
  const int grp = W == 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  const int n = a.n;
  const int f = a.param;
  const double eps = a.real_param;
  const double logc = log((double)((n - 3 * f - 1) / (2 * f) + 1));  // log(c(n-3f, 2f))
  const Mask<W> full = mfull<W>(n);
  double* sx = L.sx[grp];
  int32_t* spid = L.spid[grp];

  InstanceQueue<W> Q;  // dynamic instance distribution (psg_device.hpp)
  for (uint64_t i = Q.take(a); i != Q.kDone; i = Q.take(a)) {
    const uint64_t inst = a.ids ? a.ids[i] : a.inst_begin + i;
    Sched<W, XHO> sc;
    sc.setup(a, inst, g.pid, g.valid);
    CrashSets<W> cs;  // per-instance crash rounds (no per-round exchange for W > 1)
    if (sc.crash_on) cs.prep(g, crl, sc.crash_round);
    sc.prep_good(0, g.lane, a.R);
    double x0 = 0.0;
    if (g.valid) {
      if (a.init_f64) {
        x0 = a.init_f64[init_row(a, i, inst) * (uint64_t)n + g.pid];
      } else {  // uniform [0,1) with 53 bits (Random.nextDouble shape, Epsilon.scala:94)
        const uint64_t w = rword(a.seed, inst, ROUND_INIT, (uint32_t)g.pid, 0);
        x0 = (double)(w >> 11) * 0x1.0p-53;
      }
    }
    const bool inOk = g.valid && x0 == x0;
    const bool anyI = g.any(inOk);
    const double lo = key_value(g.min64(total_key(x0), inOk));
    const double hi = key_value(g.max64(total_key(x0), inOk));
    // EpsilonProcess state after init(io) (Epsilon.scala:18-26)
    double x = x0, decision = 0.0;
    int32_t maxR = 0;
    Mask<W> H = mzero<W>();  // keys of the `halted` map
    bool halted = !g.valid, decided = false;
    int32_t dec_round = -1, halt_round = -1;
    Checks ck;
    ck.reset();
    eps_check<W>(g, ck, 0, full, decided, decision, eps, anyI, lo, hi, true);

    for (int k = 0; k < a.R; ++k) {
      const Mask<W> act = g.ballot(!halted);
      bool pred = true;
      if (many(act)) {
        Mask<W> goodS;
        const bool good = sc.good_round(k, g.lane, a.R, goodS);
        Mask<W> CB = mzero<W>(), CN = mzero<W>();
        if (sc.crash_on) cs.sets(g, k, CB, CN);
        const Mask<W> M = mand(sc.ho(k, g.pid, good, goodS, CB, CN), act);
        const Mask<W> Fl = mand(g.ballot(!(k <= maxR)), act);  // senders announcing their halt
        const Mask<W> U = mor(M, H);                             // V = mailbox ++ halted.values
        const int m = mpopc(U);
        pred = !g.any(!halted && m < n - f);
        // sort every process's current x in total order (ties by pid): W = 1 a wave bitonic
        // network over (key, pid) pairs, lane t ends with the t-th pair; W > 1 a rank count
        // over the keys staged in LDS. Sorted values go to LDS (position = rank).
        const int64_t key = total_key(x);
        int32_t spid_r = 0;  // W = 1: pid at sorted position = lane
        if constexpr (W == 1) {
          int64_t skey = g.valid ? key : INT64_MAX;  // padding lanes sort last
          spid_r = g.lane;
          wave_sort_key_pid(skey, spid_r, g.lane);
          const double xs = __shfl(x, spid_r);
          if (g.lane < n) sx[g.lane] = xs;
        } else {
          L.keys[g.pid] = key;
          __syncthreads();
          int rank = 0;
          for (int j = 0; j < n; ++j) {
            const int64_t kj = L.keys[j];
            rank += (kj < key || (kj == key && j < g.pid)) ? 1 : 0;
          }
          if (g.valid) {
            sx[rank] = x;
            spid[rank] = g.pid;
          }
        }
        lds_sync<W>();
        // per lane: min, max, V(2f) and the trimmed every-2f-th sum over the members of
        // its own V (Epsilon.scala:31-42)
        double first = 0.0, last = 0.0, e2f = 0.0, sum = 0.0;
        int cnt = 0;
        if constexpr (W == 1) {
          // Us = V as a mask over sorted positions (bit t: the process at position t is in
          // V), from the sorted pid column read at uniform positions. The selected members
          // j = f, 3f, 5f, ... < m - f are then found by dropping the lowest set bits, and
          // only those positions are read from LDS.
          // Us(p) bit t = [sorted position t's process is in U(p)]: transpose U (lane q: the
          // receivers whose V holds q), fetch that column for position t's process, and
          // transpose back (two bit-matrix transposes and one shuffle; padding processes
          // sort last and are in no U)
          const uint64_t Ut = wave_transpose64(U.w[0], g.lane);
          const uint64_t Us = wave_transpose64((uint64_t)__shfl((unsigned long long)Ut, spid_r), g.lane);
          if (!halted && m > 0) {
            if (k == 0) {
              first = sx[__builtin_ctzll(Us)];
              last = sx[63 - __builtin_clzll(Us)];
              if (m > 2 * f) {
                uint64_t S = Us;
                for (int d = 0; d < 2 * f; ++d) S &= S - 1;
                e2f = sx[__builtin_ctzll(S)];
              }
            } else if (k <= maxR) {
              uint64_t S = Us;
              for (int d = 0; d < f; ++d) S &= S - 1;
              for (int j = f; j < m - f; j += 2 * f) {  // ascending left fold from 0.0
                sum += sx[__builtin_ctzll(S)];
                ++cnt;
                for (int d = 0; d < 2 * f; ++d) S &= S - 1;
              }
            }
          }
        } else {
          // W > 1: every lane walks the sorted list once with broadcast LDS reads;
          // the selected members are tracked with a running index (no modulo)
          int j = 0, nsel = f;
          const int jhi = m - f;
          for (int t = 0; t < n; ++t) {
            if (mtest(U, spid[t])) {
              const double v = sx[t];
              if (j == 0) first = v;
              last = v;
              if (j == 2 * f) e2f = v;
              if (j == nsel && j < jhi) {
                sum += v;
                ++cnt;
                nsel += 2 * f;
              }
              ++j;
            }
          }
        }
        if (!halted) {
          H = mor(H, mand(M, Fl));  // halted ++ mailbox.filter(_._2._2)
          if (k == 0) {
            if (m > 0) {  // (empty V: Scala throws; left unchanged)
              const double r1 = log((last - first) / eps) / logc;
              maxR = d2i(ceil(r1));
              if (a.variant == 1) maxR = 0;  // variant 1: mutation, no approximation rounds
              if (m > 4 * f) x = e2f;  // reduce(2f, V).head
            }
          } else if (k <= maxR) {
            x = sum / (double)cnt;  // sel.sum / sel.size (NaN for an empty sel)
          } else {
            decided = true;  // callback.decide(x); exitAtEndOfRound
            decision = x;
            dec_round = k;
            halt_round = k;
            halted = true;
          }
        }
        lds_sync<W>();
      }
      eps_check<W>(g, ck, k + 1, full, decided, decision, eps, anyI, lo, hi, pred);
    }
    if (g.valid) {
      const uint64_t off = i * (uint64_t)n + (uint64_t)g.pid;
      if (a.out_dec_f64) a.out_dec_f64[off] = decided ? decision : 0.0;
      if (a.out_rec_f64) {
        a.out_rec_f64[2 * off] = decided ? decision : 0.0;
        a.out_rec_f64[2 * off + 1] = x;
      }
    }
    finish_instance<W>(g, a, i, ck, 3, decided ? fold32d(decision) : 0, dec_round, halt_round, fold32d(x), &bc);
  }
  __syncthreads();
  counters_flush(&bc, a.counters, 3, a.R);
}

template <int W>
static hipError_t launch_w(const KArgs& a, int grid, hipStream_t s) {
  if (a.ho_in) hipLaunchKernelGGL((epsilon_kernel<W, true>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  else hipLaunchKernelGGL((epsilon_kernel<W, false>), dim3(grid), dim3(Geometry<W>::kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_epsilon(const KArgs& a, int W, int grid, hipStream_t s) {
  switch (W) {
    case 1: return launch_w<1>(a, grid, s);
    case 2: return launch_w<2>(a, grid, s);
    case 3: return launch_w<3>(a, grid, s);
    case 4: return launch_w<4>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

const void* epsilon_kernel_ptr(int W) {
  switch (W) {
    case 1: return (const void*)epsilon_kernel<1, false>;
    case 2: return (const void*)epsilon_kernel<2, false>;
    case 3: return (const void*)epsilon_kernel<3, false>;
    case 4: return (const void*)epsilon_kernel<4, false>;
  }
  return nullptr;
}

}  // namespace psg
