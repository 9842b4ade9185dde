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
  PSG_DEV const int32_t* stage(int tag, int f) const { return sc + (tag * PSG_NFIELDS + f) * 64 * W; }
  PSG_DEV int32_t own(int tag, int f) const { return tag == PSG_TAG_CUR ? c[f] : (tag == PSG_TAG_OLD ? o[f] : i[f]); }
};

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
template <int W, class Fn>
PSG_DEV int32_t forall_ser(Ctx<W>& x, Fn fn) {
  int32_t acc = 1;
  for (int j = 0; j < x.n; ++j) {
    acc = (acc != 0 && fn(j) != 0) ? 1 : 0;
    if (!x.g.any(acc != 0)) break;
  }
  return acc;
}
template <int W, class Fn>
PSG_DEV int32_t exists_ser(Ctx<W>& x, Fn fn) {
  int32_t acc = 0;
  for (int j = 0; j < x.n; ++j) {
    acc = (acc != 0 || fn(j) != 0) ? 1 : 0;
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

// ---------------------------------------------------------------- value domains
template <int W, class Fn>
PSG_DEV int32_t exists_bool(Ctx<W>& x, Fn fn) {
  int32_t acc = fn(0) != 0 ? 1 : 0;
  if (x.g.any(acc == 0)) acc = (acc != 0 || fn(1) != 0) ? 1 : 0;
  return acc;
}

// V.exists over Int. Candidate sources: per-lane expression values `ev[0..ne)`
// (their distinct values over the lanes) and field sets `fs[0..nf)` (field | tag
// << 8: the distinct values of that field over all processes); each value v
// contributes v-1, v, v+1; then Int.MinValue and Int.MaxValue.
template <int W, class Fn>
struct ExistsInt {
  Ctx<W>& x;
  Fn& fn;
  int32_t acc;
  PSG_DEV bool done() { return !x.g.any(acc == 0); }
  PSG_DEV void visit(int32_t v) {
    for (int d = -1; d <= 1; ++d) {
      const int32_t cand = (int32_t)((uint32_t)v + (uint32_t)d);
      acc = (acc != 0 || fn(cand) != 0) ? 1 : 0;
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

template <int W, int NE, int NF, class Fn>
PSG_DEV int32_t exists_int(Ctx<W>& x, const int32_t (&ev)[NE > 0 ? NE : 1], const int32_t (&fs)[NF > 0 ? NF : 1],
                           int32_t* scratch, Fn fn) {
  ExistsInt<W, Fn> e{x, fn, 0};
  const Mask<W> all = x.g.ballot(true);
  for (int k = 0; k < NE; ++k) {
    if constexpr (W > 1) {
      scratch[x.g.pid] = ev[k];
      __syncthreads();
    }
    const bool d = e.over(ev[k], all, scratch);
    if constexpr (W > 1) __syncthreads();
    if (d) return e.acc;
  }
  for (int k = 0; k < NF; ++k) {
    const int f = fs[k] & 0xff, tag = (fs[k] >> 8) & 0xff;
    if (e.over(x.own(tag, f), all, x.stage(tag, f))) return e.acc;
  }
  e.acc = (e.acc != 0 || fn(INT32_MIN) != 0) ? 1 : 0;
  e.acc = (e.acc != 0 || fn(INT32_MAX) != 0) ? 1 : 0;
  return e.acc;
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
  __shared__ uint64_t xb[2 * W];
  __shared__ int64_t red[2 * W];
  __shared__ int32_t stg[W > 1 ? 3 * PSG_NFIELDS * 64 * W : 1];
  __shared__ int32_t scratch[Geometry<W>::kGroups][64 * W];
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
    Checks ck;
    ck.reset();
    for (int c = 0; c <= A.R; ++c) {
      x.r = c;
      if (S::kTags & 2u) load(x.o, base + (uint64_t)(c > 0 ? c - 1 : 0) * rowsz, PSG_TAG_OLD);
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
      if (g.lane < S::kSlots && ((ck.failed >> g.lane) & 1u)) atomicAdd(&bc.fail[g.lane], 1u);
      if (g.lane == 0) atomicAdd(&bc.hist[term == PSG_NEVER ? A.R + 1 : term], 1u);
    }
  }
  __syncthreads();
  counters_flush(&bc, A.counters, S::kSlots, A.R);
}

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
