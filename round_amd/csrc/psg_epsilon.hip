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

// log(x): OCML's __ocml_log_f64 (ROCm device libs, ocml.bc), restated operation for operation so
// the result is the same double. Inlined from the library, its nine 64-bit literals are
// loop-invariant: the compiler hoists them out of the instance loop into VGPR pairs that stay live
// across every round and spill (96 B of scratch at 6 waves/SIMD, round 5). Here each literal passes
// an opaque copy at its use, so it is materialized where log runs (once per instance, maxR).
template <uint64_t BITS>
PSG_DEV double lit64() {  // the double with these bits, materialized here (two v_mov_b32 in asm)
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t lo, hi;
  asm volatile("v_mov_b32 %0, %1" : "=v"(lo) : "n"((int32_t)(uint32_t)BITS));
  asm volatile("v_mov_b32 %0, %1" : "=v"(hi) : "n"((int32_t)(uint32_t)(BITS >> 32)));
  return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
#else
  return __builtin_bit_cast(double, BITS);
#endif
}
PSG_DEV double log_ocml(double x) {
#pragma clang fp contract(off)
  int e0;
  const double m0 = __builtin_frexp(x, &e0);
  const bool lo = m0 < lit64<0x3FE5555555555555ULL>();
  const double m = m0 * (lo ? 2.0 : 1.0);
  const int e = e0 + (lo ? -1 : 0);
  const double a = m + -1.0, b = m + 1.0;
  const double bl = m - (b + -1.0);
  const double r0 = __builtin_amdgcn_rcp(b);
  const double r1 = fma(fma(-b, r0, 1.0), r0, r0);
  const double r = fma(fma(-b, r1, 1.0), r1, r1);
  const double q0 = a * r;  // (a / b) in double-double: q0 + q1
  const double p = b * q0;
  const double pl = fma(q0, bl, fma(q0, b, -p));
  const double s = p + pl;
  const double sl = pl - (s - p);
  const double d = a - s;
  const double dl = ((a - d) - s) - sl;
  const double q1c = r * (d + dl);
  const double q = q0 + q1c;
  const double ql = q1c - (q - q0);
  const double z = q * q;
  double t = fma(z, lit64<0x3FC3AB76BF559E2BULL>(), lit64<0x3FC385386B47B09AULL>());
  t = fma(z, t, lit64<0x3FC7474DD7F4DF2EULL>());
  t = fma(z, t, lit64<0x3FCC71C016291751ULL>());
  t = fma(z, t, lit64<0x3FD249249B27ACF1ULL>());
  t = fma(z, t, lit64<0x3FD99999998EF7B6ULL>());
  t = fma(z, t, lit64<0x3FE5555555555780ULL>());
  const double h2 = __builtin_ldexp(q, 1), l2 = __builtin_ldexp(ql, 1);
  const double w = (q * z) * t;
  const double u = h2 + w;
  const double ul = l2 + (w - (u - h2));
  const double v = u + ul;
  const double vl = ul - (v - u);
  const double fe = (double)e, ln2h = lit64<0x3FE62E42FEFA39EFULL>();
  const double k0 = fe * ln2h;
  const double kl = fma(fe, lit64<0x3C7ABC9E3B39803FULL>(), fma(fe, ln2h, -k0));
  const double k = k0 + kl;
  const double kr = kl - (k - k0);
  const double s1 = k + v;
  const double s1b = s1 - k;
  const double s1l = (v - s1b) + (k - (s1 - s1b));
  const double s2 = kr + vl;
  const double s2b = s2 - kr;
  const double s2l = (vl - s2b) + (kr - (s2 - s2b));
  const double s3 = s2 + s1l;
  const double s4 = s1 + s3;
  const double res = s4 + (s2l + (s3 - (s4 - s1)));
  const double ax = __builtin_fabs(x);
  double out = ax == __builtin_inf() ? x : res;
  out = x < 0.0 ? __builtin_nan("") : out;
  return x == 0.0 ? -__builtin_inf() : out;
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
  uint8_t sel8[W == 1 ? 256 * 8 : 1];  // W = 1: sel8[v * 8 + r] = bit index of the r-th set bit of byte v
};

// per-byte popcounts of a 32-bit word (each byte of the result: 0..8)
PSG_DEV uint32_t bytepop(uint32_t v) {
  v = v - ((v >> 1) & 0x55555555u);
  v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
  return (v + (v >> 4)) & 0x0F0F0F0Fu;
}

// Rank select over a 64-bit member mask (W = 1): the position of its j-th set bit (0-based,
// j < popcount), from per-byte prefix counts instead of dropping the j lowest bits one by one.
// cum_* byte b = set bits in bytes 0..b of that half (<= 32, so the SWAR compare below cannot
// borrow across bytes); the byte holding the target is the number of bytes whose prefix count
// is <= j, and the bit inside it comes from the sel8 table.
struct RankSel {
  uint32_t w[2], cum[2], nlo;
  PSG_DEV explicit RankSel(uint64_t m) {
    w[0] = (uint32_t)m;
    w[1] = (uint32_t)(m >> 32);
    cum[0] = bytepop(w[0]) * 0x01010101u;
    cum[1] = bytepop(w[1]) * 0x01010101u;
    nlo = cum[0] >> 24;
  }
  PSG_DEV int at(uint32_t j, const uint8_t* sel8) const {
    const bool hi = j >= nlo;
    const uint32_t r = hi ? j - nlo : j;
    const uint32_t c = hi ? cum[1] : cum[0];
    const uint32_t v = hi ? w[1] : w[0];
    const uint32_t ge = ((c | 0x80808080u) - (r + 1u) * 0x01010101u) & 0x80808080u;  // bytes with prefix > r
    const uint32_t b8 = (4u - (uint32_t)__builtin_popcount(ge)) * 8u;                  // target byte * 8
    const uint32_t before = (c << 8) >> b8 & 0xFFu;                                    // prefix of the bytes below
    const uint32_t byte = (v >> b8) & 0xFFu;
    return (hi ? 32 : 0) + (int)b8 + sel8[byte * 8u + (r - before)];
  }
};

// Ascending bitonic sort of (key, pid) pairs over the 64 lanes of a wave (pairs must
// be distinct; pids are), in the all-ascending form: each merge of two sorted blocks of
// SIZE/2 starts by pairing lane l with its mirror l ^ (SIZE - 1), then half-cleans with
// partners l ^ D, D = SIZE/4 .. 1; in every step the lower lane of a pair keeps the smaller
// pair. The upper-lane test is one lane bit (6 distinct masks over the 21 steps, instead of
// 21 direction masks that do not fit the SGPRs).
// lane l receives lane l ^ X's v. Within a quad (X = 1, 2, 3) and the mirrors of a half row
// / row (X = 7, 15) one DPP move; the rest through the LDS crossbar (ds_bpermute). The sort
// is a chain of 21 dependent exchanges, so exchange latency, not issue, sets its cost: the
// DPP moves took the W2 row 11.65 -> 10.92 ms; X = 4, 8 as a DPP row shift each way and a
// select (11.54), and X = 16, 31, 63 by v_permlane16/32_swap (11.50) measured slower.
template <int CTRL>
PSG_DEV uint32_t dpp_mov(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false); }
template <int X>
PSG_DEV uint32_t xchg(uint32_t v) {
  if constexpr (X == 1) return dpp_mov<0xB1>(v);          // quad_perm [1,0,3,2]
  else if constexpr (X == 2) return dpp_mov<0x4E>(v);     // quad_perm [2,3,0,1]
  else if constexpr (X == 3) return dpp_mov<0x1B>(v);     // quad_perm [3,2,1,0]
  else if constexpr (X == 7) return dpp_mov<0x141>(v);    // row_half_mirror
  else if constexpr (X == 15) return dpp_mov<0x140>(v);   // row_mirror
  else return (uint32_t)__shfl_xor((int)v, X);
}
template <int X>
PSG_DEV uint64_t xchg64(uint64_t v) {
  return (uint64_t)xchg<X>((uint32_t)v) | ((uint64_t)xchg<X>((uint32_t)(v >> 32)) << 32);
}
template <int X, int UP>
PSG_DEV void sort_step(int64_t& key, int32_t& pid, int lane) {
  const int64_t pk = (int64_t)xchg64<X>((uint64_t)key);
  const int32_t pp = (int32_t)xchg<X>((uint32_t)pid);
  const bool less = pk < key || (pk == key && pp < pid);  // partner's pair precedes mine
  const bool take = less != ((lane & UP) != 0);
  key = take ? pk : key;
  pid = take ? pp : pid;
}
template <int D>
PSG_DEV void half_clean(int64_t& key, int32_t& pid, int lane) {
  sort_step<D, D>(key, pid, lane);
  if constexpr (D > 1) half_clean<D / 2>(key, pid, lane);
}
template <int SIZE = 2>
PSG_DEV void wave_sort_key_pid(int64_t& key, int32_t& pid, int lane) {
  sort_step<SIZE - 1, SIZE / 2>(key, pid, lane);  // mirror step
  if constexpr (SIZE >= 4) half_clean<SIZE / 4>(key, pid, lane);
  if constexpr (SIZE < 64) wave_sort_key_pid<SIZE * 2>(key, pid, lane);
}

// The same network over one 64-bit word: the key's top 58 bits with the pid in the low 6
// (distinct words, so the order is total). Sorted by that word, the list is in (key, pid)
// order unless two keys that agree in their top 58 bits differ below them and sit against
// their pid order — the caller checks adjacent full keys and sorts again by (key, pid) then.
// Two 32-bit moves and one compare per step instead of three moves and three compares.
template <int X, int UP>
PSG_DEV void sort_step1(int64_t& c, int lane) {
  const int64_t pc = (int64_t)xchg64<X>((uint64_t)c);
  const bool take = (pc < c) != ((lane & UP) != 0);
  c = take ? pc : c;
}
template <int D>
PSG_DEV void half_clean1(int64_t& c, int lane) {
  sort_step1<D, D>(c, lane);
  if constexpr (D > 1) half_clean1<D / 2>(c, lane);
}
template <int SIZE = 2>
PSG_DEV void wave_sort_packed(int64_t& c, int lane) {
  sort_step1<SIZE - 1, SIZE / 2>(c, lane);
  if constexpr (SIZE >= 4) half_clean1<SIZE / 4>(c, lane);
  if constexpr (SIZE < 64) wave_sort_packed<SIZE * 2>(c, lane);
}

// 64 x 64 bit-matrix transpose across a wave: lane i holds row i; afterwards lane j holds
// column j (bit i = bit j of row i). Stage S (any order: each swaps one bit of the row index
// with the same bit of the column index): the lane pair (i, i ^ S) exchanges the off-diagonal
// S x S blocks of its 2S x 2S block — the lower lane keeps its LO blocks and takes the
// partner's LO blocks into its ~LO ones, the upper lane the mirror image. On the two 32-bit
// halves of the row:
//   S = 32  one v_permlane32_swap (the lower lanes' high words <-> the upper lanes' low words);
//   S = 16  per word one v_permlane16_swap (own and partner's word land in the two outputs)
//           and one v_perm_b32 byte select (bytes 0, 1 / 2, 3 of each);
//   S = 8   per word a ds_bpermute and one v_perm_b32 byte select;
//   S < 8   per word a ds_bpermute, a rotate (v_alignbit: the wrapped bits fall in the blocks
//           the lane keeps) and a bit-field select.
// (round 5: a 64-bit shift / select form of every stage; this one has no 64-bit operations.)
PSG_DEV void transpose_s32(uint32_t& lo, uint32_t& hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
  lo = (uint32_t)r[0];
  hi = (uint32_t)r[1];
}
PSG_DEV uint32_t transpose_s16(uint32_t w, uint32_t sel) {
  const auto r = __builtin_amdgcn_permlane16_swap(w, w, false, false);  // even rows: (own, partner); odd: (partner, own)
  return __builtin_amdgcn_perm((uint32_t)r[1], (uint32_t)r[0], sel);
}
template <int S>
PSG_DEV uint32_t transpose_small(uint32_t w, bool up, int lane) {
  constexpr uint32_t LO = S == 4 ? 0x0F0F0F0Fu : S == 2 ? 0x33333333u : 0x55555555u;
  const uint32_t p = xshfl<S>(w, lane);
  const uint32_t moved = __builtin_amdgcn_alignbit(p, p, up ? S : 32 - S);  // rotate right
  const uint32_t keep = up ? ~LO : LO;
  return (w & keep) | (moved & ~keep);
}
PSG_DEV uint64_t wave_transpose64(uint64_t r, int lane) {
  uint32_t lo = (uint32_t)r, hi = (uint32_t)(r >> 32);
  transpose_s32(lo, hi);
  {
    // v_perm_b32(s0 = r[1], s1 = r[0]): bytes 0-3 of r[0] are selectors 0-3, of r[1] 4-7
    const uint32_t sel = (lane & 16) ? 0x07060302u : 0x05040100u;
    lo = transpose_s16(lo, sel);
    hi = transpose_s16(hi, sel);
  }
  {
    // lower: (w.b0, p.b0, w.b2, p.b2); upper: (p.b1, w.b1, p.b3, w.b3); s0 = p, s1 = w
    const uint32_t sel = (lane & 8) ? 0x03070105u : 0x06020400u;
    lo = __builtin_amdgcn_perm(xshfl<8>(lo, lane), lo, sel);
    hi = __builtin_amdgcn_perm(xshfl<8>(hi, lane), hi, sel);
  }
  {
    const bool up = (lane & 4) != 0;
    lo = transpose_small<4>(lo, up, lane);
    hi = transpose_small<4>(hi, up, lane);
  }
  {
    const bool up = (lane & 2) != 0;
    lo = transpose_small<2>(lo, up, lane);
    hi = transpose_small<2>(hi, up, lane);
  }
  {
    const bool up = (lane & 1) != 0;
    lo = transpose_small<1>(lo, up, lane);
    hi = transpose_small<1>(hi, up, lane);
  }
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Slots: 0 EpsAgreement (no NaN decision, max - min <= eps), 1 EpsValidity (every
// decision within [min, max] of the non-NaN initial values), 2 SafetyPredicate
// (|V| >= n - f for every process that took a step). Termination: all decided.
template <int W>
PSG_DEV void eps_check(Grp<W>& g, Checks& ck, int c, const Mask<W>& full, bool decided, double decision, double eps,
                       bool anyI, double lo, double hi, bool pred) {
  bool agree = true, valid = true;
  if (g.any(decided)) {  // uniform: before the first decision both hold by definition
    const bool nanD = g.any(decided && decision != decision);
    const bool ok = decided && decision == decision;
    const bool anyD = g.any(ok);
    bool close = true;
    if (anyD) {
      const int64_t kd = total_key(decision);
      close = key_value(g.max64(kd, ok)) - key_value(g.min64(kd, ok)) <= eps;
    }
    agree = !nanD && close;
    valid = !g.any(decided && !(anyI && lo <= decision && decision <= hi));
  }
  ck.record(fbit(agree, 0) | fbit(valid, 1) | fbit(pred, 2), meq(g.ballot(decided), full), c, g.lane);
}

#ifndef PSG_EPS_WPE
#define PSG_EPS_WPE 6  // W = 1 occupancy target (round 4: 14.23 vs 14.13 ms at 7); round 5: 96 B scratch at 6 (log()'s hoisted f64 constants, reloaded once per instance), 5 measured slower (12.17 vs 11.63 ms)
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
  const double logc = log_ocml((double)((n - 3 * f - 1) / (2 * f) + 1));  // log(c(n-3f, 2f))
  const Mask<W> full = mfull<W>(n);
  double* sx = L.sx[grp];
  int32_t* spid = L.spid[grp];
  if constexpr (W == 1) {
    for (uint32_t t = threadIdx.x; t < 256u * 8u; t += blockDim.x) {
      uint32_t v = t >> 3, r = t & 7u;
      for (; r > 0 && v != 0; --r) v &= v - 1u;  // drop r lowest set bits
      L.sel8[t] = v ? (uint8_t)__builtin_ctz(v) : 0;
    }
    __syncthreads();
  }

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
        // pid through an opaque copy: the lane's element pointer is formed here, once per
        // instance, instead of hoisted out of the instance loop (a 64-bit VGPR pair spilled to
        // scratch at 6 waves/SIMD)
        int pid = g.pid;
        asm volatile("" : "+v"(pid));
        x0 = a.init_f64[init_row(a, i, inst) * (uint64_t)n + (uint64_t)pid];
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
        // per lane: min, max, V(2f) and the trimmed every-2f-th sum over the members of
        // its own V (Epsilon.scala:31-42); no V is read in a round where every process that
        // still runs decides (r > maxR), so that round skips the sort
        // round 0: span = max - min of V and acc = V(2f); later rounds: acc = the trimmed sum
        // (one pair of doubles for both: they are never live together)
        double span = 0.0, acc = 0.0;
        int cnt = 0;
        if (g.any(!halted && k <= maxR)) {
          // sort every process's current x in total order (ties by pid): W = 1 a wave bitonic
          // network over (key, pid) pairs, lane t ends with the t-th pair; W > 1 a rank count
          // over the keys staged in LDS. Sorted values go to LDS (position = rank).
          const int64_t key = total_key(x);
          int32_t spid_r = 0;  // W = 1: pid at sorted position = lane
          if constexpr (W == 1) {
            // padding lanes sort last: no valid key reaches INT64_MAX's top 58 bits (NaN's is 0x7ff8 << 48)
            int64_t c = ((g.valid ? key : INT64_MAX) & ~(int64_t)63) | g.lane;
            wave_sort_packed(c, g.lane);
            spid_r = (int32_t)(c & 63);
            double xs = __shfl(x, spid_r);
            // position t's full key against position t - 1's (DPP wave_shr:1, no LDS round trip)
            const int64_t ks = total_key(xs);
            const int64_t kp = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)ks, 0x138, 0xF, 0xF, false) |
                                         ((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(ks >> 32), 0x138, 0xF, 0xF, false) << 32));
            if (g.any(g.lane >= 1 && g.lane < n && kp > ks)) {  // rare: keys within 64 ulp out of pid order
              int64_t skey = g.valid ? key : INT64_MAX;
              spid_r = g.lane;
              wave_sort_key_pid(skey, spid_r, g.lane);
              xs = __shfl(x, spid_r);
            }
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
          if constexpr (W == 1) {
            // Us = V as a mask over sorted positions (bit t: the process at position t is in
            // V), from the sorted pid column read at uniform positions. The selected members
            // j = f, 3f, 5f, ... < m - f are then found by rank select (RankSel), and only
            // those positions are read from LDS.
            // Us(p) bit t = [sorted position t's process is in U(p)]: transpose U (lane q: the
            // receivers whose V holds q), fetch that column for position t's process, and
            // transpose back (two bit-matrix transposes and one shuffle; padding processes
            // sort last and are in no U)
            const uint64_t Ut = wave_transpose64(U.w[0], g.lane);
            const uint64_t Us = wave_transpose64((uint64_t)__shfl((unsigned long long)Ut, spid_r), g.lane);
            if (!halted && m > 0) {
              const RankSel rs(Us);
              if (k == 0) {
                span = sx[63 - __builtin_clzll(Us)] - sx[__builtin_ctzll(Us)];
                if (m > 2 * f) acc = sx[rs.at((uint32_t)(2 * f), L.sel8)];
              } else if (k <= maxR) {
                for (int j = f; j < m - f; j += 2 * f) {  // ascending left fold from 0.0
                  acc += sx[rs.at((uint32_t)j, L.sel8)];
                  ++cnt;
                }
              }
            }
          } else {
            // W > 1: every lane walks the sorted list once with broadcast LDS reads;
            // the selected members are tracked with a running index (no modulo)
            double first = 0.0, last = 0.0, e2f = 0.0, sum = 0.0;
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
            span = last - first;
            acc = k == 0 ? e2f : sum;
          }
        }
        if (!halted) {
          H = mor(H, mand(M, Fl));  // halted ++ mailbox.filter(_._2._2)
          if (k == 0) {
            if (m > 0) {  // (empty V: Scala throws; left unchanged)
              const double r1 = log_ocml(span / eps) / logc;
              maxR = d2i(ceil(r1));
              if (a.variant == 1) maxR = 0;  // variant 1: mutation, no approximation rounds
              if (m > 4 * f) x = acc;  // reduce(2f, V).head
            }
          } else if (k <= maxR) {
            x = acc / (double)cnt;  // sel.sum / sel.size (NaN for an empty sel)
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
