// psg_spec_native.hpp — runtime of Spec programs lowered to native wave code.
//
// round_amd/formula.py (compile_native) turns a Spec's Formula tree into a HIP
// source that includes this header: every slot becomes a C++ expression over
// the quantifier templates below, compiled for gfx950 into a code object and
// launched by psg_run_batch_spec instead of the bytecode interpreter (SURVEY §8f
// rank 1: "Formula -> wave-reduction lowering"). The kernel reads the state
// trace written by the round kernels (trace_put) and evaluates every check point.
//
// Lowering rules (mirroring the hand-written checks):
//  * the outermost process quantifier binds the lane's own pid (one lane per
//    process) and reduces with a ballot: forall -> !any(!b), exists -> any(b),
//    filter(...).size -> popcount of the ballot;
//  * nested process quantifiers loop over the pids with a per-lane accumulator
//    and leave as soon as no lane can change (one ballot per step);
//  * a field of a uniform process (loop variable, coord) is a readlane (W = 1)
//    or a broadcast LDS read (W > 1); of a per-lane process, a ds_bpermute /
//    LDS gather;
//  * V.exists over Int visits the distinct values of the compared fields and
//    expressions (+-1) and Int.MinValue / Int.MaxValue, exactly as the
//    interpreter and the oracle finitize it.
#pragma once
#include "psg_device.hpp"

namespace psg {
namespace spec {

template <int W>
struct Ctx {
  Grp<W>& g;
  int n, r;
  int32_t c[PSG_NFIELDS];  // this lane's process: current, old, init values
  int32_t o[PSG_NFIELDS];
  int32_t i[PSG_NFIELDS];
  int32_t* sc;             // W > 1: staged copies [3][PSG_NFIELDS][64W]
  X0Set<W> iset[2];        // membership sets of init(field) values (S::kInitSet0 / kInitSet1)
  // per check point: majority candidates already computed (key field | tag << 8, -1 = empty);
  // scalar slots, not an array, so they stay in registers
  int32_t maj_k0, maj_v0, maj_k1, maj_v1;
  // member_init_own: per memo slot M, the lane's last probed value and its membership
  // (valid once bit M of mok is set; a Ctx lives for one instance)
  uint32_t mok = 0;
  int32_t mv[4] = {0, 0, 0, 0}, mr[4] = {0, 0, 0, 0};
  // symmetric check point (uniform<>): every process holds the same current / old value of each
  // field the uniform lowering reads, process 0's in uc / uo; uni says whether it holds
  bool uni = false;
  int32_t uc[PSG_NFIELDS] = {0}, uo[PSG_NFIELDS] = {0};
  // check points since the state last changed (fused hook, 0..2): at 2 the current and old fields
  // are those of the previous check point, so what depends on the fields alone (the symmetric
  // test, majority candidates, the staged copies) is still valid; the formulas are re-evaluated
  int unch = 0;
  // member_init_u: per memo slot, the last probed (uniform) value and its membership
  uint32_t muok = 0;
  int32_t muv[4] = {0, 0, 0, 0}, mur[4] = {0, 0, 0, 0};
  PSG_DEV const int32_t* stage(int tag, int f) const { return sc + (tag * PSG_NFIELDS + f) * 64 * W; }
  PSG_DEV int32_t own(int tag, int f) const { return tag == PSG_TAG_CUR ? c[f] : (tag == PSG_TAG_OLD ? o[f] : i[f]); }
  PSG_DEV int32_t uf(int tag, int f) const { return tag == PSG_TAG_CUR ? uc[f] : uo[f]; }
};

// ---------------------------------------------------------------- symmetric check points
// A check point is symmetric for a Spec when every process holds the same value of each
// current / old field the Spec reads (settled OTR states: all decided on one value). Then a
// process quantifier whose body reads its variable only through such fields has the same
// body value for every process: forall / exists give that value, count gives n or 0, and a
// field of any process is process 0's. The generator emits a second lowering of the Spec
// under that assumption (scalar code, no ballots for those quantifiers) and this test picks
// it per check point; it is exact for every state (n >= 1: process 0 exists).
// The lowest current field is tested alone first: a Spec whose states are rarely symmetric
// (LastVoting: crashed processes never decide) pays one broadcast and one ballot. Process 0's
// values are kept in (uniform) VGPRs: the symmetric lowering's arithmetic then issues on the
// vector pipe, not on the scalar pipe that bounds the fused kernels (fused OTR -3.7 %).
template <int W, uint32_t CUR, uint32_t OLD>
PSG_DEV bool uniform(Ctx<W>& x) {
  if (x.unch >= 2) return x.uni;  // the same fields as at the previous check point
  constexpr int F0 = CUR ? __builtin_ctz(CUR) : -1;
  constexpr bool kTwo = F0 >= 0 && ((CUR & (CUR - 1)) | OLD) != 0u;  // more than one field
  if constexpr (kTwo) {
    x.uc[F0] = (int32_t)vgpr_u32((uint32_t)x.g.bcast(x.c[F0], x.stage(PSG_TAG_CUR, F0), 0));
    if (x.g.any(x.c[F0] != x.uc[F0])) {
      x.uni = false;
      return false;
    }
  }
  uint32_t diff = 0;
#pragma unroll
  for (int f = 0; f < PSG_NFIELDS; ++f) {
    if (((CUR >> f) & 1u) && !(kTwo && f == F0)) {
      x.uc[f] = (int32_t)vgpr_u32((uint32_t)x.g.bcast(x.c[f], x.stage(PSG_TAG_CUR, f), 0));
      diff |= ne01(x.c[f], x.uc[f]);
    }
    if ((OLD >> f) & 1u) {
      x.uo[f] = (int32_t)vgpr_u32((uint32_t)x.g.bcast(x.o[f], x.stage(PSG_TAG_OLD, f), 0));
      diff |= ne01(x.o[f], x.uo[f]);
    }
  }
  x.uni = !x.g.any(diff != 0u);
  return x.uni;
}

// field (tag) of the process with pid q on a symmetric check point (0 for a pid outside
// [0, n), as fld_u / fld_g)
template <int W>
PSG_DEV int32_t fld_uni(Ctx<W>& x, int tag, int f, int32_t q) {
  return (q >= 0 && q < x.n) ? x.uf(tag, f) : 0;
}

// field f (state tag) of the uniform process q
template <int W>
PSG_DEV int32_t fld_u(Ctx<W>& x, int tag, int f, int32_t q) {
  if (q < 0 || q >= x.n) return 0;
  return x.g.bcast(x.own(tag, f), x.stage(tag, f), q);
}

// field f (state tag) of a per-lane process q (converged code only)
template <int W>
PSG_DEV int32_t fld_g(Ctx<W>& x, int tag, int f, int32_t q) {
  const bool ok = q >= 0 && q < x.n;
  const int32_t v = x.g.gather(x.own(tag, f), x.stage(tag, f), ok ? q : 0);
  return ok ? v : 0;
}

// ---------------------------------------------------------------- process quantifiers, lane form
template <int W, class Fn>
PSG_DEV int32_t forall_lane(Ctx<W>& x, Fn fn) {
  const int32_t b = fn(x.g.pid);
  return x.g.any(b == 0) ? 0 : 1;
}
template <int W, class Fn>
PSG_DEV int32_t exists_lane(Ctx<W>& x, Fn fn) {
  const int32_t b = fn(x.g.pid);
  return x.g.any(b != 0) ? 1 : 0;
}
template <int W, class Fn>
PSG_DEV int32_t count_lane(Ctx<W>& x, Fn fn) {
  const int32_t b = fn(x.g.pid);
  return mpopc(x.g.ballot(b != 0));
}

// ---------------------------------------------------------------- process quantifiers, serial form
// Bodies are evaluated on every lane (converged): a body may hold ballots and
// cross-lane reads, which need all lanes; a per-lane short circuit would not
// save issue slots anyway (the wave runs the body while any lane needs it).
template <int W, class Fn>
PSG_DEV int32_t forall_ser(Ctx<W>& x, Fn fn) {
  int32_t acc = 1;
  for (int j = 0; j < x.n; ++j) {
    const int32_t b = fn(j);
    acc = (acc != 0 && b != 0) ? 1 : 0;
    if (!x.g.any(acc != 0)) break;
  }
  return acc;
}
template <int W, class Fn>
PSG_DEV int32_t exists_ser(Ctx<W>& x, Fn fn) {
  int32_t acc = 0;
  for (int j = 0; j < x.n; ++j) {
    const int32_t b = fn(j);
    acc = (acc != 0 || b != 0) ? 1 : 0;
    if (!x.g.any(acc == 0)) break;
  }
  return acc;
}
template <int W, class Fn>
PSG_DEV int32_t count_ser(Ctx<W>& x, Fn fn) {
  int32_t acc = 0;
  for (int j = 0; j < x.n; ++j) acc += fn(j) != 0 ? 1 : 0;
  return acc;
}

// ---------------------------------------------------------------- serial form over distinct states
// A nested process quantifier whose body reads its variable j only through fields
// visits each distinct tuple of those fields once instead of every pid: forall /
// exists are insensitive to repeats, count weighs a tuple by how many processes
// hold it (a popcount). Typically 1-3 tuples (e.g. undecided / decided v) vs n.
template <int F, int T>
struct Fld {
  static constexpr int f = F, tag = T;
};

template <int W, int MODE, class Fn, class... Fs>  // MODE 0 forall, 1 exists, 2 count
PSG_DEV int32_t quant_tup(Ctx<W>& x, Fn fn, Fs...) {
  int32_t acc = MODE == 0 ? 1 : 0;
  Mask<W> rem = x.g.ballot(true);
  while (many(rem)) {
    const int q = mfirst(rem);
    Mask<W> E = rem;
    auto val = [&](auto fld) -> int32_t {
      using FL = decltype(fld);
      const int32_t mine = x.own(FL::tag, FL::f);
      const int32_t v = x.g.bcast(mine, x.stage(FL::tag, FL::f), q);
      E = mand(E, x.g.ballot(mine == v));
      return v;
    };
    const int32_t b = fn(val(Fs{})...);
    rem = mandn(rem, E);
    if constexpr (MODE == 0) {
      acc = (acc != 0 && b != 0) ? 1 : 0;
      if (!x.g.any(acc != 0)) break;
    } else if constexpr (MODE == 1) {
      acc = (acc != 0 || b != 0) ? 1 : 0;
      if (!x.g.any(acc == 0)) break;
    } else {
      acc += b != 0 ? mpopc(E) : 0;
    }
  }
  return acc;
}

// The distinct-state quantifier's tuple, when every process holds the same one (per
// check point, shared by the quantifiers over that field tuple): then quant_tup has one
// iteration and needs no ballots — forall / exists give the body's value at the tuple,
// count gives n or 0. (Settled states: every process decided the same value; early
// rounds: nobody decided.)
template <int NF>
struct TupU {
  bool uni;
  int32_t v[NF];
};

template <int W, class... Fs>
PSG_DEV TupU<(int)sizeof...(Fs)> tup_uniform(Ctx<W>& x, Fs...) {
  TupU<(int)sizeof...(Fs)> t;
  uint32_t diff = 0;
  int k = 0;
  auto one = [&](auto fld) {
    using FL = decltype(fld);
    const int32_t mine = x.own(FL::tag, FL::f);
    t.v[k] = x.g.bcast(mine, x.stage(FL::tag, FL::f), 0);  // process 0 (n >= 1)
    diff |= ne01(mine, t.v[k]);
    ++k;
  };
  (one(Fs{}), ...);
  t.uni = !x.g.any(diff != 0u);
  return t;
}

template <int W, int MODE, int NF, class Fn, class... Fs>
PSG_DEV int32_t quant_tup_c(Ctx<W>& x, const TupU<NF>& tu, Fn fn, Fs... fs) {
  if (tu.uni) {
    int32_t b;
    if constexpr (NF == 1) b = fn(tu.v[0]);
    else if constexpr (NF == 2) b = fn(tu.v[0], tu.v[1]);
    else if constexpr (NF == 3) b = fn(tu.v[0], tu.v[1], tu.v[2]);
    else b = fn(tu.v[0], tu.v[1], tu.v[2], tu.v[3]);
    if constexpr (MODE == 2) return b != 0 ? x.n : 0;
    else return b != 0 ? 1 : 0;
  }
  return quant_tup<W, MODE>(x, fn, fs...);
}

// Guarded distinct-state quantifiers: P.forall(j => A(j) ==> B), P.exists(j => A(j) && B) and
// the count of A(j) && B visit only the processes where A holds (A reads only j's fields; the
// others contribute nothing), so their tuples are those of the guard set G — one tuple when
// every guarded process agrees (LastVoting's Agreement over the deciders while crashed
// processes never decide). tup_uniform_g: G = ballot(guard), the tuple of G's first process
// and whether every process of G holds it; G empty: the quantifier's identity.
template <int W, int NF>
struct TupG {
  bool uni, empty;
  Mask<W> G;
  int32_t v[NF];
};

template <int W, class... Fs>
PSG_DEV TupG<W, (int)sizeof...(Fs)> tup_uniform_g(Ctx<W>& x, int32_t guard, Fs...) {
  TupG<W, (int)sizeof...(Fs)> t;
  t.G = x.g.ballot(guard != 0);
  t.empty = !many(t.G);
  const int q0 = t.empty ? 0 : mfirst(t.G);
  uint32_t diff = 0;
  int k = 0;
  auto one = [&](auto fld) {
    using FL = decltype(fld);
    const int32_t mine = x.own(FL::tag, FL::f);
    t.v[k] = x.g.bcast(mine, x.stage(FL::tag, FL::f), q0);
    diff |= ne01(mine, t.v[k]);
    ++k;
  };
  (one(Fs{}), ...);
  t.uni = !x.g.any(guard != 0 && diff != 0u);
  return t;
}

template <int W, int MODE, int NF, class Fn, class... Fs>
PSG_DEV int32_t quant_tup_gc(Ctx<W>& x, const TupG<W, NF>& tu, Fn fn, Fs...) {
  if (tu.empty) return MODE == 0 ? 1 : 0;
  if (tu.uni) {
    int32_t b;
    if constexpr (NF == 1) b = fn(tu.v[0]);
    else if constexpr (NF == 2) b = fn(tu.v[0], tu.v[1]);
    else if constexpr (NF == 3) b = fn(tu.v[0], tu.v[1], tu.v[2]);
    else b = fn(tu.v[0], tu.v[1], tu.v[2], tu.v[3]);
    if constexpr (MODE == 2) return b != 0 ? mpopc(tu.G) : 0;
    else return b != 0 ? 1 : 0;
  }
  int32_t acc = MODE == 0 ? 1 : 0;
  Mask<W> rem = tu.G;
  while (many(rem)) {
    const int q = mfirst(rem);
    Mask<W> E = rem;
    auto val = [&](auto fld) -> int32_t {
      using FL = decltype(fld);
      const int32_t mine = x.own(FL::tag, FL::f);
      const int32_t v = x.g.bcast(mine, x.stage(FL::tag, FL::f), q);
      E = mand(E, x.g.ballot(mine == v));
      return v;
    };
    const int32_t b = fn(val(Fs{})...);
    rem = mandn(rem, E);
    if constexpr (MODE == 0) {
      acc = (acc != 0 && b != 0) ? 1 : 0;
      if (!x.g.any(acc != 0)) break;
    } else if constexpr (MODE == 1) {
      acc = (acc != 0 || b != 0) ? 1 : 0;
      if (!x.g.any(acc == 0)) break;
    } else {
      acc += b != 0 ? mpopc(E) : 0;
    }
  }
  return acc;
}

// P.exists(j => init(j.f) == t): membership of t in the instance's set of initial
// values of f — an LDS hash set built once per instance (X0Set), as the
// hand-lowered checks do, instead of a loop over the processes.
template <int W, int K>
PSG_DEV int32_t member_init(Ctx<W>& x, int32_t t) {
  return (int32_t)x.iset[K].contains01(t);
}

// member_init of the lane's own current field F: the membership only changes with the
// value, so each lane keeps its last probed value and answer (memo slot M) and the set
// is probed again only when some lane's value changed (a group-uniform test)
template <int W, int K, int F, int M>
PSG_DEV int32_t member_init_own(Ctx<W>& x) {
  const int32_t v = x.c[F];
  if (!((x.mok >> M) & 1u) || x.g.any(v != x.mv[M])) {
    x.mr[M] = (int32_t)x.iset[K].contains01(v);
    x.mv[M] = v;
    x.mok |= 1u << M;
  }
  return x.mr[M];
}

// member_init of a group-uniform value t (symmetric check points): the same memo per slot M as
// member_init_own, kept in scalar registers; the set is probed only when t changed
template <int W, int K, int M>
PSG_DEV int32_t member_init_u(Ctx<W>& x, int32_t t) {
  if (!((x.muok >> M) & 1u) || t != x.muv[M]) {
    x.mur[M] = rfl32((int32_t)x.iset[K].contains01(t));
    x.muv[M] = t;
    x.muok |= 1u << M;
  }
  return x.mur[M];
}

// ---------------------------------------------------------------- connectives with an expensive right side
// a && b, a || b, a ==> b where b holds a quantifier: b is skipped when no lane of
// the group needs it (a group-uniform decision, so b still runs converged).
template <int W, class Fn>
PSG_DEV int32_t and_sc(Ctx<W>& x, int32_t a, Fn fb) {
  if (!x.g.any(a != 0)) return 0;
  const int32_t b = fb();
  return (a != 0 && b != 0) ? 1 : 0;
}
template <int W, class Fn>
PSG_DEV int32_t or_sc(Ctx<W>& x, int32_t a, Fn fb) {
  if (!x.g.any(a == 0)) return 1;
  const int32_t b = fb();
  return (a != 0 || b != 0) ? 1 : 0;
}
template <int W, class Fn>
PSG_DEV int32_t impl_sc(Ctx<W>& x, int32_t a, Fn fb) {
  if (!x.g.any(a != 0)) return 1;
  const int32_t b = fb();
  return (a == 0 || b != 0) ? 1 : 0;
}

// ---------------------------------------------------------------- value domains
template <int W, class Fn>
PSG_DEV int32_t exists_bool(Ctx<W>& x, Fn fn) {
  int32_t acc = fn(0) != 0 ? 1 : 0;
  if (x.g.any(acc == 0)) {
    const int32_t b = fn(1);
    acc = (acc != 0 || b != 0) ? 1 : 0;
  }
  return acc;
}

// V.exists over Int. Candidate sources: per-lane expression values `ev[0..ne)`
// (their distinct values over the lanes) and field sets `fs[0..nf)` (field | tag
// << 8: the distinct values of that field over all processes); each value v
// contributes v-1, v, v+1 (EQ: v only); then Int.MinValue and Int.MaxValue
// (EQ: one value outside the candidate set).
template <int W, class Fn, bool EQ = false>
struct ExistsInt {
  Ctx<W>& x;
  Fn& fn;
  int32_t acc;
  int32_t lo, hi;  // extreme candidate values visited (EQ)
  bool any_v;
  PSG_DEV bool done() { return !x.g.any(acc == 0); }
  PSG_DEV void test(int32_t cand) {
    const int32_t b = fn(cand);
    acc = (acc != 0 || b != 0) ? 1 : 0;
  }
  uint32_t shifts = 7u;  // breakpoint mode (exists_int_bp): bit d+1 -> test v + d, d in {-1, 0, 1}
  PSG_DEV void visit(int32_t v) {
    if constexpr (EQ) {
      test(v);
      lo = any_v && lo < v ? lo : v;
      hi = any_v && hi > v ? hi : v;
      any_v = true;
    } else {
      for (int d = -1; d <= 1; ++d)
        if ((shifts >> (d + 1)) & 1u) test((int32_t)((uint32_t)v + (uint32_t)d));
    }
  }
  // distinct values of the per-lane `val` over the lanes in `m`
  PSG_DEV bool over(int32_t val, Mask<W> m, const int32_t* staged) {
    while (many(m)) {
      const int32_t v = x.g.bcast(val, staged, mfirst(m));
      m = mandn(m, x.g.ballot(val == v));
      visit(v);
      if (done()) return true;
    }
    return false;
  }
};

template <int W, int NE, int NF, class Fn, bool EQ>
PSG_DEV bool exists_int_scan(ExistsInt<W, Fn, EQ>& e, Ctx<W>& x, const int32_t (&ev)[NE > 0 ? NE : 1],
                             const int32_t (&fs)[NF > 0 ? NF : 1], int32_t* scratch,
                             const uint32_t* shifts = nullptr) {
  const Mask<W> all = x.g.ballot(true);
  for (int k = 0; k < NE; ++k) {
    if (shifts) e.shifts = shifts[k];
    if constexpr (W > 1) {
      scratch[x.g.pid] = ev[k];
      __syncthreads();
    }
    const bool d = e.over(ev[k], all, scratch);
    if constexpr (W > 1) __syncthreads();
    if (d) return true;
  }
  for (int k = 0; k < NF; ++k) {
    if (shifts) e.shifts = shifts[NE + k];
    const int f = fs[k] & 0xff, tag = (fs[k] >> 8) & 0xff;
    if (e.over(x.own(tag, f), all, x.stage(tag, f))) return true;
  }
  return false;
}

template <int W, int NE, int NF, class Fn>
PSG_DEV int32_t exists_int(Ctx<W>& x, const int32_t (&ev)[NE > 0 ? NE : 1], const int32_t (&fs)[NF > 0 ? NF : 1],
                           int32_t* scratch, Fn fn) {
  ExistsInt<W, Fn, false> e{x, fn, 0, 0, 0, false};
  if (exists_int_scan<W, NE, NF>(e, x, ev, fs, scratch)) return e.acc;
  e.test(INT32_MIN);
  e.test(INT32_MAX);
  return e.acc;
}

// V.exists over Int by breakpoints: every atom of the body that reads the variable t is
// `t <= b` or its negation for a breakpoint b of its compared term e (t <= e, t > e: b = e;
// t < e, t >= e: b = e - 1; t == e, t != e: both), so the body is constant on each interval
// (b_j, b_j+1] and on (b_max, Int.MaxValue]: the breakpoints (right ends) plus Int.MaxValue
// decide it. shifts[k] (bit d+1: b = e + d) per candidate source, sources as exists_int.
template <int W, int NE, int NF, class Fn>
PSG_DEV int32_t exists_int_bp(Ctx<W>& x, const int32_t (&ev)[NE > 0 ? NE : 1], const int32_t (&fs)[NF > 0 ? NF : 1],
                              const uint32_t (&shifts)[NE + NF > 0 ? NE + NF : 1], int32_t* scratch, Fn fn) {
  ExistsInt<W, Fn, false> e{x, fn, 0, 0, 0, false};
  if (exists_int_scan<W, NE, NF>(e, x, ev, fs, scratch, shifts)) return e.acc;
  e.test(INT32_MAX);
  return e.acc;
}

// V.exists over Int whose variable is only compared with == / != : the body has
// one truth value on all values outside the candidate set W, so the candidates
// plus ONE value outside W decide it (max+1 or min-1; when W holds both Int
// extremes, the general +-1 finitization).
template <int W, int NE, int NF, class Fn>
PSG_DEV int32_t exists_int_eq(Ctx<W>& x, const int32_t (&ev)[NE > 0 ? NE : 1],
                              const int32_t (&fs)[NF > 0 ? NF : 1], int32_t* scratch, Fn fn) {
  ExistsInt<W, Fn, true> e{x, fn, 0, 0, 0, false};
  if (exists_int_scan<W, NE, NF>(e, x, ev, fs, scratch)) return e.acc;
  if (!e.any_v) e.test(0);
  else if (e.hi != INT32_MAX) e.test(e.hi + 1);
  else if (e.lo != INT32_MIN) e.test(e.lo - 1);
  else return exists_int<W, NE, NF>(x, ev, fs, scratch, fn);
  return e.acc;
}

// V.exists(v => ... && P.filter(i => i.t == v).size >= L && ...): a witness v is
// a value of the per-process term t held by at least L processes. With 2L > n
// that is the strict majority (Boyer-Moore candidate, one body evaluation);
// otherwise the distinct values of t filtered by their count. Requires L >= 1.
template <int W, int KEY, class Fn>
PSG_DEV int32_t exists_int_guard(Ctx<W>& x, int32_t t, const int32_t* staged, int32_t L, Fn fn) {
  if ((int64_t)L >= (int64_t)x.n) {
    // held by every process (a count == n guard): the only candidate is process 0's t, no
    // majority vote (the hand-lowered OTR check does the same before the first decision)
    const int32_t m = x.g.bcast(t, staged, 0);
    if (mpopc(x.g.ballot(t == m)) < L) return 0;
    return fn(m) != 0 ? 1 : 0;
  }
  if (2 * (int64_t)L > (int64_t)x.n) {
    // the candidate depends only on the field's values: computed once per check point
    int32_t m;
    if (x.maj_k0 == KEY) {
      m = x.maj_v0;
    } else if (x.maj_k1 == KEY) {
      m = x.maj_v1;
    } else {
      m = majority_candidate<W>(x.g, t);
      if (x.maj_k0 < 0) {
        x.maj_k0 = KEY;
        x.maj_v0 = m;
      } else if (x.maj_k1 < 0) {
        x.maj_k1 = KEY;
        x.maj_v1 = m;
      }
    }
    if (mpopc(x.g.ballot(t == m)) < L) return 0;
    return fn(m) != 0 ? 1 : 0;
  }
  int32_t acc = 0;
  Mask<W> rem = x.g.ballot(true);
  while (many(rem)) {
    const int32_t v = x.g.bcast(t, staged, mfirst(rem));
    const Mask<W> E = x.g.ballot(t == v);
    rem = mandn(rem, E);
    if (mpopc(E) < L) continue;
    const int32_t b = fn(v);
    acc = (acc != 0 || b != 0) ? 1 : 0;
    if (!x.g.any(acc == 0)) break;
  }
  return acc;
}

// V.exists(v => ... && P.forall(i => ... && (cond(i) ==> term(i) == v) && ...) && ...): once
// some process has an active pin (cond true), a witness must equal that process's term, so
// the body is evaluated at that one value (the first pinned process, its first active pin);
// with no pin active, `general` (the finitization) decides it. `act` / `val`: the lane's
// process's pin flag and pinned value.
template <int W, class FA, class FV, class Fn, class Gen>
PSG_DEV int32_t exists_int_pin(Ctx<W>& x, FA act, FV val, int32_t* scratch, Fn fn, Gen general) {
  const int32_t mine = val(x.g.pid);
  const Mask<W> m = x.g.ballot(act(x.g.pid) != 0);
  if (many(m)) {
    int32_t v;
    if constexpr (W == 1) {
      v = readlane32(mine, mfirst(m));
    } else {
      scratch[x.g.pid] = mine;
      __syncthreads();
      v = rfl32(scratch[mfirst(m)]);
      __syncthreads();
    }
    return fn(v) != 0 ? 1 : 0;
  }
  return general();
}

// exists_int_pin on a symmetric check point whose pinning process variable reads only
// symmetric fields: the pin flag and value are the same for every process
template <class Fn, class Gen>
PSG_DEV int32_t pin_uni(int32_t act, int32_t val, Fn fn, Gen general) {
  if (act != 0) return fn(val) != 0 ? 1 : 0;
  return general();
}

// exists_int_guard on a symmetric check point: every process holds t = u, so u is the only
// value held by L >= 1 processes (n of them)
template <int W, class Fn>
PSG_DEV int32_t guard_uni(Ctx<W>& x, int32_t u, int32_t L, Fn fn) {
  if (x.n < L) return 0;
  return fn(u) != 0 ? 1 : 0;
}

// ---------------------------------------------------------------- arithmetic with Scala Int semantics
PSG_DEV int32_t idiv(int32_t a, int32_t b) { return b == 0 ? 0 : (a == INT32_MIN && b == -1) ? a : a / b; }
PSG_DEV int32_t imod(int32_t a, int32_t b) { return (b == 0 || b == -1) ? 0 : a % b; }
PSG_DEV int32_t iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
PSG_DEV int32_t isub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
PSG_DEV int32_t imul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

// ---------------------------------------------------------------- kernel
// S provides: kSlots, kRelational (slot mask vacuous at c = 0), kHasTerm,
// kFields (bit f: field used), kTags (bit t: state tag used) and
// template <int W> static uint32_t fail(Ctx<W>&, int32_t* scratch) / bool term(...).
template <int W, class S>
__device__ void native_kernel_body(const VmArgs& A) {
  __shared__ BlockCounters bc;
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int64_t red[2 * W];
  __shared__ int32_t stg[W > 1 ? 3 * PSG_NFIELDS * 64 * W : 1];
  __shared__ int32_t scratch[Geometry<W>::kGroups][64 * W];
  __shared__ int32_t isets[S::kInitSet0 >= 0 ? (S::kInitSet1 >= 0 ? 2 : 1) : 1][Geometry<W>::kGroups]
                          [S::kInitSet0 >= 0 ? X0Set<W>::kSlots : 1];
  counters_init(&bc);
  __syncthreads();
  KArgs ka;
  ka.n = A.n;
  Grp<W> g;
  grp_setup(g, ka, xb, red);
  constexpr int G = Geometry<W>::kGroups;
  const int grp = W == 1 ? (int)(threadIdx.x >> 6) : 0;
  const int n = A.n;
  const uint64_t rowsz = (uint64_t)PSG_NFIELDS * (uint64_t)n;
  for (uint64_t ii = (uint64_t)blockIdx.x * G + grp; ii < A.count; ii += (uint64_t)gridDim.x * G) {
    const int32_t* base = A.trace + ii * (uint64_t)(A.R + 1) * rowsz;
    Ctx<W> x{g, n, 0, {0}, {0}, {0}, stg};
    auto load = [&](int32_t* dst, const int32_t* row, int tag) {
#pragma unroll
      for (int f = 0; f < PSG_NFIELDS; ++f) {
        if (!((S::kFields >> f) & 1u)) continue;
        dst[f] = g.valid ? row[(uint64_t)f * n + g.pid] : 0;
        if constexpr (W > 1) stg[(tag * PSG_NFIELDS + f) * 64 * W + g.pid] = dst[f];
      }
    };
    load(x.i, base, PSG_TAG_INIT);
    if constexpr (S::kInitSet0 >= 0) x.iset[0].build(g, isets[0][grp], x.i[S::kInitSet0]);
    if constexpr (S::kInitSet1 >= 0) x.iset[1].build(g, isets[1][grp], x.i[S::kInitSet1]);
    Checks ck;
    ck.reset();
    for (int c = 0; c <= A.R; ++c) {
      x.r = c;
      x.maj_k0 = x.maj_k1 = -1;
      if (S::kTags & 2u) {
        // old = the previous check point's current state, already in registers
        // (c = 0: the initial state, read below); halves the trace read traffic
        if (c == 0) {
          load(x.o, base, PSG_TAG_OLD);
        } else {
#pragma unroll
          for (int f = 0; f < PSG_NFIELDS; ++f) {
            if (!((S::kFields >> f) & 1u)) continue;
            x.o[f] = x.c[f];
            if constexpr (W > 1) stg[(PSG_TAG_OLD * PSG_NFIELDS + f) * 64 * W + g.pid] = x.c[f];
          }
        }
      }
      load(x.c, base + (uint64_t)c * rowsz, PSG_TAG_CUR);
      if constexpr (W > 1) __syncthreads();
      uint32_t fb = S::template fail<W>(x, scratch[grp]);
      if (c == 0) fb &= ~S::kRelational;
      const bool term = S::kHasTerm && S::template term<W>(x, scratch[grp]);
      ck.record(fb, term, c, g.lane);
      if constexpr (W > 1) __syncthreads();
    }
    if (g.wv == 0) {
      const uint32_t term = ck.term_round();
      if (A.out_inst) {
        uint8_t* o = reinterpret_cast<uint8_t*>(A.out_inst + ii);
        if (g.lane < PSG_MAX_CHECKS) o[8 + g.lane] = (uint8_t)ck.ffv;
        if (g.lane == 0) {
          o[8 + PSG_MAX_CHECKS] = (uint8_t)term;
          o[9 + PSG_MAX_CHECKS] = (uint8_t)S::kSlots;
        }
      }
      if (g.lane < S::kSlots && ck.failed_here()) atomicAdd(&bc.fail[g.lane], 1u);
      if (g.lane == 0) atomicAdd(&bc.hist[term == PSG_NEVER ? A.R + 1 : term], 1u);
    }
  }
  __syncthreads();
  counters_flush(&bc, A.counters, S::kSlots, A.R);
}

// ---------------------------------------------------------------- fused round kernel hook
// compile_native(fused=True): the algorithm's round kernel is instantiated with
// SpecHook<S> and evaluates S at every check point from its own registers — the
// same per-process values psg_run_batch_spec would trace (emit_state), so the
// results are those of the trace + native_kernel_body path without the trace's
// HBM round trip and second launch.
template <class S>
struct SpecHook {
  static constexpr bool kFused = true;
  static constexpr int kSlots = S::kSlots;
  static constexpr uint32_t kFields = S::kFields;
  template <int W>
  struct State {
    Ctx<W> x;
    Checks ck;
    int grp;
    PSG_DEV static int32_t* stage_lds() {
      __shared__ int32_t b[W > 1 ? 3 * PSG_NFIELDS * 64 * W : 1];
      return b;
    }
    PSG_DEV static int32_t* scratch_lds(int grp) {
      __shared__ int32_t b[Geometry<W>::kGroups][64 * W];
      return b[grp];
    }
    PSG_DEV static int32_t* iset_lds(int k, int grp) {
      __shared__ int32_t b[S::kInitSet0 >= 0 ? (S::kInitSet1 >= 0 ? 2 : 1) : 1][Geometry<W>::kGroups]
                          [S::kInitSet0 >= 0 ? X0Set<W>::kSlots : 1];
      return b[k][grp];
    }
    PSG_DEV State(Grp<W>& g, int grp_, int n) : x{g, n, 0, {0}, {0}, {0}, stage_lds()}, grp(grp_) { ck.reset(); }

    // frozen: no process took a step in the round before check point c (the kernel's frozen
    // tail), so the state, old included, repeats; from the second such check point in a row the
    // fields, their staged copies and what depends on them alone are kept (Ctx::unch)
    PSG_DEV void put(int c, int32_t f0, int32_t f1, int32_t f2, int32_t f3, int32_t f4, int32_t f5, int32_t f6,
                     int32_t f7, int32_t f8, bool frozen = false) {
      Grp<W>& g = x.g;
      const int32_t v[PSG_NFIELDS] = {f0, f1, f2, f3, f4, f5, f6, f7, f8};
      x.r = c;
      x.unch = (frozen && c > 0) ? (x.unch < 2 ? x.unch + 1 : 2) : 0;
      if (x.unch < 2) {
        x.maj_k0 = x.maj_k1 = -1;
#pragma unroll
        for (int f = 0; f < PSG_NFIELDS; ++f) {
          if (!((S::kFields >> f) & 1u)) continue;
          const int32_t val = g.valid ? v[f] : 0;  // the trace holds valid processes only
          if (c == 0) {
            x.i[f] = val;
            if constexpr (W > 1) x.sc[(PSG_TAG_INIT * PSG_NFIELDS + f) * 64 * W + g.pid] = val;
          }
          x.o[f] = c == 0 ? val : x.c[f];
          x.c[f] = val;
          if constexpr (W > 1) {
            x.sc[(PSG_TAG_OLD * PSG_NFIELDS + f) * 64 * W + g.pid] = x.o[f];
            x.sc[(PSG_TAG_CUR * PSG_NFIELDS + f) * 64 * W + g.pid] = val;
          }
        }
        if (c == 0) {
          if constexpr (S::kInitSet0 >= 0) x.iset[0].build(g, iset_lds(0, grp), x.i[S::kInitSet0]);
          if constexpr (S::kInitSet1 >= 0) x.iset[1].build(g, iset_lds(1, grp), x.i[S::kInitSet1]);
        }
        if constexpr (W > 1) __syncthreads();
      }
      // a frozen check point runs the frozen lowering (every old field is the current one, the
      // kernel's frozen-tail facts are constants: GenSpec::fail_frozen); every formula is evaluated
      const bool fz = frozen && c > 0;
      uint32_t fb = fz ? S::template fail_frozen<W>(x, scratch_lds(grp)) : S::template fail<W>(x, scratch_lds(grp));
      if (c == 0) fb &= ~S::kRelational;
      const bool term = S::kHasTerm && (fz ? S::template term_frozen<W>(x, scratch_lds(grp))
                                           : S::template term<W>(x, scratch_lds(grp)));
      ck.record(fb, term, c, g.lane);
      if constexpr (W > 1) __syncthreads();
    }
  };
};

}  // namespace spec
}  // namespace psg

// One extern "C" kernel per wave count (looked up by psg_run_batch_spec).
#define PSG_SPEC_NATIVE_KERNELS(S)                                                                           \
  extern "C" __global__ void __launch_bounds__(256) psg_spec_native_w1(psg::VmArgs A) {                    \
    psg::spec::native_kernel_body<1, S>(A);                                                                  \
  }                                                                                                          \
  extern "C" __global__ void __launch_bounds__(128) psg_spec_native_w2(psg::VmArgs A) {                    \
    psg::spec::native_kernel_body<2, S>(A);                                                                  \
  }                                                                                                          \
  extern "C" __global__ void __launch_bounds__(192) psg_spec_native_w3(psg::VmArgs A) {                    \
    psg::spec::native_kernel_body<3, S>(A);                                                                  \
  }                                                                                                          \
  extern "C" __global__ void __launch_bounds__(256) psg_spec_native_w4(psg::VmArgs A) {                    \
    psg::spec::native_kernel_body<4, S>(A);                                                                  \
  }
