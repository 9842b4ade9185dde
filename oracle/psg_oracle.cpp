/*
 * psg_oracle.cpp — CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / timed CPU baseline. The product path
 * (round_amd/, libpsg.so) never calls it.
 *
 * A scalar, literal restatement of the reference's round semantics and Specs:
 *   - lockstep HO rounds: psync/Process.scala:45-82 (r/phase bookkeeping),
 *     psync/Round.scala:57-69 (mailbox += (sender -> payload), finishRound),
 *     psync/Round.scala:102-124 (broadcast includes self; self send bypasses the network),
 *     psync/runtime/InstanceHandler.scala:164-258 (send -> receive* -> update, exit);
 *   - algorithms: example/Otr.scala:13-86, example/LastVoting.scala:80-212,
 *     example/FloodMin.scala:8-36, example/KSetAgreement.scala:21-68, example/BenOr.scala:11-84,
 *     example/Otr2.scala:9-66, example/ShortLastVoting.scala:13-105,
 *     example/KSetEarlyStopping.scala:9-44, example/Epsilon.scala:16-70 (Double state);
 *   - Spec: psync/Specs.scala:8-27 and the per-algorithm specs (Otr.scala:95-120,
 *     LastVoting.scala:19-70, BenOr.scala:91-115, Otr2.scala:71-96), evaluated two independent ways:
 *     (a) a Formula-tree interpreter mirroring psync/formula/Formula.scala
 *         (ForAll/Exists/Comprehension/Cardinality, lowering as in
 *         psync/macros/FormulaExtractor.scala:222-233, 297-316, 500-506);
 *     (b) the hand-lowered evaluator the GPU kernel also implements.
 *     Invariant sequencing follows psync/verification/Verifier.scala:111-141, 159-168.
 *   - third-party semantics the reference relies on but does not vendor:
 *     Scala 2.13.1 immutable.Map iteration order (Map1..Map4 insertion order,
 *     CHAMP HashMap order with scala.collection.Hashing.improve), maxBy/minBy
 *     first-wins, Int division; java.util.Random (BenOr coin); Philox4x32-10
 *     (Random123, schedule generator).
 *
 * PARITY STATUS: the reference is Scala and cannot run in this image (no JVM,
 * no sbt, no dependency cache). The reference ships no golden vectors for this
 * path. This oracle is pinned only by (1) hand-traced known-answer tests derived
 * line by line from the algorithm sources (tests/test_oracle_kat.py), (2) the
 * reference's own mmor spec (src/test/scala/psync/logic/OtrExample.scala:67-75),
 * (3) published known-answer vectors of Philox4x32-10 and java.util.Random.
 * For round execution as a whole, parity with the JVM reference is UNPINNED.
 */
#include "../include/psg.h"

#include <algorithm>
#include <atomic>
#include <bitset>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace orc {

using Bits = std::bitset<PSG_MAX_N>;

/* ------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11; Random123 philox4x32_R(10))    */
/* ------------------------------------------------------------------ */
static void philox4x32_10(const uint32_t in[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static const uint32_t ROUND_INIT = 0xFFFFFFFFu;
static const uint32_t ROUND_CRASH = 0xFFFFFFFEu;
static const uint32_t PID_GLOBAL = 0xFFFFu;
static const uint32_t COIN_TAG = 0x80000000u;

/* 64-bit random word j of stream (inst, round, ctr3base): Philox call s = j/2
 * with counter (inst_lo, inst_hi, round, ctr3base + (s << 16)); even j takes
 * out0 | out1<<32, odd j takes out2 | out3<<32. */
static uint64_t rword(uint64_t seed, uint64_t inst, uint32_t round, uint32_t ctr3base, uint32_t j) {
  uint32_t ctr[4] = {(uint32_t)inst, (uint32_t)(inst >> 32), round, ctr3base + ((j / 2u) << 16)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  philox4x32_10(ctr, key, o);
  return (j & 1u) ? ((uint64_t)o[2] | ((uint64_t)o[3] << 32)) : ((uint64_t)o[0] | ((uint64_t)o[1] << 32));
}

static uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

/* java.util.Random: setSeed(s) then nextBoolean() (JDK: seed scramble with
 * 0x5DEECE66D, 48-bit LCG, next(1) = top bit). Used for BenOr's coin,
 * example/BenOr.scala:77, under the seeding convention of SURVEY §8a A8. */
static bool java_random_first_boolean(uint64_t s) {
  const uint64_t mult = 0x5DEECE66DULL, mask = (1ULL << 48) - 1;
  uint64_t seed = (s ^ mult) & mask;
  seed = (seed * mult + 0xBULL) & mask;
  return (seed >> 47) != 0;
}

/* ------------------------------------------------------------------ */
/* Scala 2.13 immutable.Map iteration order over ProcessID keys        */
/* ------------------------------------------------------------------ */
/* scala.collection.Hashing.improve; key.## of ProcessID(id: Short) = id. */
static uint32_t scala_improve(uint32_t h) {
  uint32_t x = h + ~(h << 9);
  x ^= (x >> 14);
  x += (x << 4);
  x ^= (x >> 10);
  return x;
}

/* CHAMP canonical trie, pre-order: a node's payload entries (ascending 5-bit
 * fragment), then its sub-nodes (ascending fragment), recursively. */
static void champ_iter(const std::vector<int>& keys, int shift, std::vector<int>& out) {
  std::map<uint32_t, std::vector<int>> groups;
  for (int k : keys) groups[(scala_improve((uint32_t)k) >> shift) & 31u].push_back(k);
  for (auto& g : groups)
    if (g.second.size() == 1) out.push_back(g.second[0]);
  for (auto& g : groups)
    if (g.second.size() > 1) champ_iter(g.second, shift + 5, out);
}

/* Iteration order of a Map built by `mailbox += (sender -> payload)` with
 * senders inserted in ascending pid order (the HO harness's insertion order). */
static std::vector<int> scala_map_order(std::vector<int> inserted, int tiebreak) {
  if (tiebreak == PSG_TIE_MIN_PID) {
    std::sort(inserted.begin(), inserted.end());
    return inserted;
  }
  if (inserted.size() <= 4) return inserted; /* Map1..Map4 */
  std::vector<int> out;
  champ_iter(inserted, 0, out);
  return out;
}

/* ------------------------------------------------------------------ */
/* Schedule: HO sets per (instance, round, process)                    */
/* ------------------------------------------------------------------ */
struct Schedule {
  const psg_config& cfg;
  uint64_t inst;
  int n, W;
  std::vector<int> crash_round; /* -1: correct process */
  Bits full;

  Schedule(const psg_config& c, uint64_t i) : cfg(c), inst(i), n(c.n), W((c.n + 63) / 64) {
    for (int p = 0; p < n; ++p) full.set(p);
    crash_round.assign(n, -1);
    if (cfg.sched.crash_fmax >= 0) {
      uint64_t w0 = rword(cfg.seed, inst, ROUND_CRASH, PID_GLOBAL, 0);
      uint64_t w1 = rword(cfg.seed, inst, ROUND_CRASH, PID_GLOBAL, 1);
      uint32_t f = mulhi32((uint32_t)w0, (uint32_t)cfg.sched.crash_fmax + 1u);
      uint32_t a = (uint32_t)(w0 >> 32) | 1u;
      uint32_t off = (uint32_t)w1;
      bool pow2 = (n & (n - 1)) == 0;
      for (int p = 0; p < n; ++p) {
        uint32_t pos = pow2 ? ((a * (uint32_t)p + off) & (uint32_t)(n - 1))
                            : (((uint32_t)p + off % (uint32_t)n) % (uint32_t)n);
        if (pos < f) {
          uint64_t wr = rword(cfg.seed, inst, ROUND_CRASH, (uint32_t)p, 0);
          crash_round[p] = (int)mulhi32((uint32_t)wr, (uint32_t)cfg.rounds);
        }
      }
    }
  }

  bool crashed(int p) const { return crash_round[p] >= 0; }

  int good_min() const { return cfg.sched.good_min >= 0 ? cfg.sched.good_min : (2 * n) / 3; }

  Bits word_to_bits(int w, uint64_t v) const {
    Bits b;
    for (int i = 0; i < 64 && w * 64 + i < n; ++i)
      if ((v >> i) & 1) b.set(w * 64 + i);
    return b;
  }

  /* drop set: AND of drop_log2 random words (per mask word) */
  Bits drop_bits(uint32_t round, uint32_t ctr3, uint32_t j0) const {
    Bits b;
    uint32_t d = cfg.sched.drop_log2;
    if (d == 0) return b;
    for (int w = 0; w < W; ++w) {
      uint64_t m = ~0ULL;
      for (uint32_t i = 0; i < d; ++i) m &= rword(cfg.seed, inst, round, ctr3, j0 + (uint32_t)w * d + i);
      b |= word_to_bits(w, m);
    }
    return b;
  }

  bool good_round(int k) const {
    uint64_t g = rword(cfg.seed, inst, (uint32_t)k, PID_GLOBAL, 0);
    return (uint32_t)g < cfg.sched.good_p32;
  }

  /* HO(p) in round k: the set of q whose round-k message p receives. */
  Bits ho(int k, int p) const {
    Bits base;
    if (good_round(k)) {
      base = full & ~drop_bits((uint32_t)k, PID_GLOBAL, 1);
      if ((int)base.count() <= good_min()) base = full;
    } else {
      base = full & ~drop_bits((uint32_t)k, (uint32_t)p, 0);
    }
    if (cfg.sched.crash_fmax >= 0) {
      Bits half;
      uint32_t d = cfg.sched.drop_log2;
      for (int w = 0; w < W; ++w)
        half |= word_to_bits(w, rword(cfg.seed, inst, (uint32_t)k, (uint32_t)p, (uint32_t)W * d + (uint32_t)w));
      for (int q = 0; q < n; ++q) {
        int cr = crash_round[q];
        if (cr < 0) continue;
        if (cr < k || (cr == k && !half.test(q))) base.reset(q);
      }
    }
    if (cfg.sched.self_bit) base.set(p);
    if (cfg.sched.ho_min >= 0 && (int)base.count() <= cfg.sched.ho_min) base = full;
    return base;
  }

  int32_t init_value(int p) const {
    uint64_t w = rword(cfg.seed, inst, ROUND_INIT, (uint32_t)p, 0);
    if (cfg.alg == PSG_ALG_BENOR) return (int32_t)((uint32_t)w & 1u);
    return 1 + (int32_t)mulhi32((uint32_t)w, (uint32_t)cfg.value_range);
  }

  /* RealConsensusIO.initialValue: uniform in [0, 1) with 53 random bits (the
   * shape of Random.nextDouble, Epsilon.scala:94) */
  double init_real(int p) const {
    uint64_t w = rword(cfg.seed, inst, ROUND_INIT, (uint32_t)p, 0);
    return (double)(w >> 11) * 0x1.0p-53;
  }

  bool coin(int k, int p) const {
    return java_random_first_boolean(rword(cfg.seed, inst, (uint32_t)k, COIN_TAG | (uint32_t)p, 0));
  }
};

/* ------------------------------------------------------------------ */
/* Formula IR (mirrors psync/formula/Formula.scala) + interpreter       */
/* ------------------------------------------------------------------ */
enum Field { F_X = 0, F_DECIDED, F_DECISION, F_TS, F_READY, F_COMMIT, F_VOTE, F_CANDECIDE, F_HOSIZE, F_NFIELDS };
enum Tag { T_CUR = 0, T_OLD = 1, T_INIT = 2 };
static const int64_t NONE = INT64_MIN + 7; /* Option None */

enum Op {
  LIT, NVAR, RVAR, BVAR, FIELD, COORD, NOT, AND, OR, IMPLIES, EQ, NEQ, LT, LE, GT, GE,
  PLUS, MINUS, TIMES, DIV, MOD, FORALL_P, EXISTS_P, EXISTS_V_INT, EXISTS_V_BOOL,
  FILTER_P, CARD, CONTAINS, ISDEF, GET
};
struct Node;
using Fm = std::shared_ptr<Node>;
struct Node {
  Op op;
  int64_t lit = 0;
  int var = -1;   /* bound variable slot */
  int field = -1; /* FIELD */
  int tag = T_CUR;
  std::vector<Fm> c;
};
static Fm mk(Op op, std::vector<Fm> c = {}) {
  auto n = std::make_shared<Node>();
  n->op = op;
  n->c = std::move(c);
  return n;
}
static Fm lit(int64_t v) { auto n = mk(LIT); n->lit = v; return n; }
static Fm tru() { return lit(1); }
static Fm nvar() { return mk(NVAR); }
static Fm rvar() { return mk(RVAR); }
static Fm bv(int slot) { auto n = mk(BVAR); n->var = slot; return n; }
static Fm fld(int f, Fm proc, int tag = T_CUR) { auto n = mk(FIELD, {proc}); n->field = f; n->tag = tag; return n; }
static Fm coord() { return mk(COORD); }
static Fm not_(Fm a) { return mk(NOT, {a}); }
static Fm and_(Fm a, Fm b) { return mk(AND, {a, b}); }
static Fm or_(Fm a, Fm b) { return mk(OR, {a, b}); }
static Fm imp(Fm a, Fm b) { return mk(IMPLIES, {a, b}); }
static Fm eq(Fm a, Fm b) { return mk(EQ, {a, b}); }
static Fm le(Fm a, Fm b) { return mk(LE, {a, b}); }
static Fm gt(Fm a, Fm b) { return mk(GT, {a, b}); }
static Fm ge(Fm a, Fm b) { return mk(GE, {a, b}); }
static Fm times(Fm a, Fm b) { return mk(TIMES, {a, b}); }
static Fm div_(Fm a, Fm b) { return mk(DIV, {a, b}); }
static Fm forallP(int s, Fm body) { auto n = mk(FORALL_P, {body}); n->var = s; return n; }
static Fm existsP(int s, Fm body) { auto n = mk(EXISTS_P, {body}); n->var = s; return n; }
static Fm existsVInt(int s, Fm body) { auto n = mk(EXISTS_V_INT, {body}); n->var = s; return n; }
static Fm existsVBool(int s, Fm body) { auto n = mk(EXISTS_V_BOOL, {body}); n->var = s; return n; }
static Fm filterP(int s, Fm body) { auto n = mk(FILTER_P, {body}); n->var = s; return n; }
static Fm card(Fm set) { return mk(CARD, {set}); }
static Fm contains(Fm set, Fm e) { return mk(CONTAINS, {set, e}); }
static Fm isdef(Fm a) { return mk(ISDEF, {a}); }
static Fm get(Fm a) { return mk(GET, {a}); }

/* State snapshot the Spec quantifies over: per process, per field, cur/old/init. */
struct SpecState {
  int n = 0;
  int64_t r = 0; /* spec r = completed rounds (Verifier.scala:159-168, 237-243) */
  std::vector<int64_t> v[3][F_NFIELDS];
  int64_t get(int f, int tag, int p) const { return v[tag][f][p]; }
};

struct Interp {
  const SpecState& st;
  int64_t bvars[16];
  std::vector<int64_t> int_dom;
  Interp(const SpecState& s, const std::vector<Fm>& roots) : st(s) {
    /* Finitization of V.exists over Int: the truth value of the body can only
     * change at values compared against state terms, so {t-1, t, t+1} for every
     * int term in reach plus the extremes covers every region exactly. */
    std::set<int64_t> base = {0, st.r, st.r / 4, (int64_t)st.n};
    std::function<void(const Fm&)> walk = [&](const Fm& f) {
      if (f->op == FIELD && f->field != F_DECIDED && f->field != F_READY && f->field != F_COMMIT &&
          f->field != F_CANDECIDE && f->field != F_HOSIZE)
        for (int p = 0; p < st.n; ++p) {
          int64_t x = st.get(f->field, f->tag, p);
          if (x != NONE) base.insert(x);
        }
      for (auto& k : f->c) walk(k);
    };
    for (auto& r : roots) walk(r);
    std::set<int64_t> dom = {INT32_MIN, INT32_MAX};
    for (int64_t b : base) { dom.insert(b - 1); dom.insert(b); dom.insert(b + 1); }
    int_dom.assign(dom.begin(), dom.end());
  }
  int64_t ev(const Fm& f) {
    switch (f->op) {
      case LIT: return f->lit;
      case NVAR: return st.n;
      case RVAR: return st.r;
      case BVAR: return bvars[f->var];
      case FIELD: return st.get(f->field, f->tag, (int)ev(f->c[0]));
      case COORD: return (st.r / 4) % st.n;
      case NOT: return !ev(f->c[0]);
      case AND: return ev(f->c[0]) && ev(f->c[1]);
      case OR: return ev(f->c[0]) || ev(f->c[1]);
      case IMPLIES: return !ev(f->c[0]) || ev(f->c[1]);
      case EQ: return ev(f->c[0]) == ev(f->c[1]);
      case NEQ: return ev(f->c[0]) != ev(f->c[1]);
      case LT: return ev(f->c[0]) < ev(f->c[1]);
      case LE: return ev(f->c[0]) <= ev(f->c[1]);
      case GT: return ev(f->c[0]) > ev(f->c[1]);
      case GE: return ev(f->c[0]) >= ev(f->c[1]);
      case PLUS: return ev(f->c[0]) + ev(f->c[1]);
      case MINUS: return ev(f->c[0]) - ev(f->c[1]);
      case TIMES: return ev(f->c[0]) * ev(f->c[1]);
      case DIV: return ev(f->c[0]) / ev(f->c[1]); /* Scala Int division truncates */
      case MOD: return ev(f->c[0]) % ev(f->c[1]);
      case FORALL_P:
        for (int p = 0; p < st.n; ++p) { bvars[f->var] = p; if (!ev(f->c[0])) return 0; }
        return 1;
      case EXISTS_P:
        for (int p = 0; p < st.n; ++p) { bvars[f->var] = p; if (ev(f->c[0])) return 1; }
        return 0;
      case EXISTS_V_INT:
        for (int64_t v : int_dom) { bvars[f->var] = v; if (ev(f->c[0])) return 1; }
        return 0;
      case EXISTS_V_BOOL:
        for (int64_t v = 0; v <= 1; ++v) { bvars[f->var] = v; if (ev(f->c[0])) return 1; }
        return 0;
      case CARD: {
        const Fm& s = f->c[0]; /* FILTER_P */
        int64_t cnt = 0;
        for (int p = 0; p < st.n; ++p) { bvars[s->var] = p; if (ev(s->c[0])) ++cnt; }
        return cnt;
      }
      case CONTAINS: {
        const Fm& s = f->c[0];
        int64_t e = ev(f->c[1]);
        bvars[s->var] = e;
        return ev(s->c[0]);
      }
      case ISDEF: return ev(f->c[0]) != NONE;
      case GET: return ev(f->c[0]);
      case FILTER_P: break;
    }
    return 0;
  }
};

/* A Spec as the reference states it (psync/Specs.scala:8-16). */
struct SpecDef {
  Fm safetyPredicate; /* null = True() (psync/Specs.scala:9) */
  std::vector<Fm> invariants;
  std::vector<std::vector<Fm>> roundInvariants;
  std::vector<std::pair<std::string, Fm>> properties; /* Termination excluded: reported as a round */
  Fm termination;
  std::vector<Fm> all_roots() const {
    std::vector<Fm> r = invariants;
    for (auto& l : roundInvariants) for (auto& f : l) r.push_back(f);
    for (auto& p : properties) r.push_back(p.second);
    if (termination) r.push_back(termination);
    if (safetyPredicate) r.push_back(safetyPredicate);
    return r;
  }
};

/* The five consensus properties shared by OTR and LastVoting
 * (example/Otr.scala:113-119, example/LastVoting.scala:191-197). */
static void consensus_properties(SpecDef& s, bool with_validity_integrity) {
  Fm i = bv(0), j = bv(1);
  s.termination = forallP(0, fld(F_DECIDED, i));
  s.properties.push_back({"Agreement",
      forallP(0, forallP(1, imp(and_(fld(F_DECIDED, i), fld(F_DECIDED, j)),
                                eq(fld(F_DECISION, i), fld(F_DECISION, j)))))});
  if (with_validity_integrity) {
    s.properties.push_back({"Validity",
        forallP(0, imp(fld(F_DECIDED, i), existsP(1, eq(fld(F_X, j, T_INIT), fld(F_DECISION, i)))))});
    s.properties.push_back({"Integrity",
        existsP(1, forallP(0, imp(fld(F_DECIDED, i), eq(fld(F_DECISION, i), fld(F_X, j, T_INIT)))))});
  }
  s.properties.push_back({"Irrevocability",
      forallP(0, imp(fld(F_DECIDED, i, T_OLD),
                     and_(fld(F_DECIDED, i), eq(fld(F_DECISION, i, T_OLD), fld(F_DECISION, i)))))});
}

/* example/Otr.scala:95-120 */
static SpecDef otr_spec() {
  SpecDef s;
  Fm i = bv(0), j1 = bv(1), v = bv(2), ii = bv(3), j = bv(4);
  Fm twoThirds = div_(times(lit(2), nvar()), lit(3));
  /* P.forall(i => P.exists(j1 => i.x == init(j1.x))) */
  Fm keepInit = forallP(0, existsP(1, eq(fld(F_X, i), fld(F_X, j1, T_INIT))));
  /* val A = P.filter(i => i.x == v) */
  Fm A = filterP(3, eq(fld(F_X, ii), v));
  Fm allDecV = forallP(0, imp(fld(F_DECIDED, i), eq(fld(F_DECISION, i), v)));
  Fm inv0 = and_(or_(forallP(0, not_(fld(F_DECIDED, i))),
                     existsVInt(2, and_(gt(card(A), twoThirds), allDecV))),
                 keepInit);
  Fm inv1 = and_(existsVInt(2, and_(eq(card(A), nvar()), allDecV)), keepInit);
  Fm inv2 = existsP(4, forallP(0, and_(fld(F_DECIDED, i), eq(fld(F_DECISION, i), fld(F_X, j, T_INIT)))));
  s.invariants = {inv0, inv1, inv2};
  consensus_properties(s, true);
  return s;
}

/* example/Otr2.scala:71-96. decision is an Option[Int]: field F_DECISION holds
 * the value or NONE, so isDefined / get / Option equality are literal. */
static SpecDef otr2_spec() {
  SpecDef s;
  Fm i = bv(0), j = bv(1), v = bv(2), ii = bv(3);
  Fm twoThirds = div_(times(lit(2), nvar()), lit(3));
  Fm dec = fld(F_DECISION, i);
  Fm A = filterP(3, eq(fld(F_X, ii), v));
  Fm allDecV = forallP(0, imp(isdef(dec), eq(get(dec), v)));
  Fm inv0 = or_(forallP(0, not_(not_(isdef(dec)))), /* P.forall(i => !i.decision.isEmpty) */
                existsVInt(2, and_(gt(card(A), twoThirds), allDecV)));
  Fm inv1 = existsVInt(2, and_(eq(card(A), nvar()), allDecV));
  Fm inv2 = existsVInt(2, allDecV);
  s.invariants = {inv0, inv1, inv2};
  s.termination = forallP(0, isdef(dec));
  Fm decj = fld(F_DECISION, j);
  s.properties.push_back({"Agreement",
      forallP(0, forallP(1, imp(and_(isdef(dec), isdef(decj)), eq(dec, decj))))});
  s.properties.push_back({"Validity",
      forallP(0, imp(isdef(dec), existsP(1, eq(fld(F_X, j, T_INIT), get(dec)))))});
  s.properties.push_back({"Integrity",
      existsP(1, forallP(0, imp(isdef(dec), eq(get(dec), fld(F_X, j, T_INIT)))))});
  Fm odec = fld(F_DECISION, i, T_OLD);
  s.properties.push_back({"Irrevocability", forallP(0, imp(isdef(odec), eq(odec, dec)))});
  return s;
}

/* example/LastVoting.scala:147-198 */
static SpecDef lv_spec() {
  SpecDef s;
  Fm i = bv(0), j1 = bv(1), v = bv(2), t = bv(3), ia = bv(4), j = bv(5);
  Fm half = div_(nvar(), lit(2));
  Fm r4 = div_(rvar(), lit(4));
  Fm noDecision = forallP(0, and_(not_(fld(F_DECIDED, i)), not_(fld(F_READY, i))));
  /* val A = P.filter(i => i.ts >= t) */
  Fm A = filterP(4, ge(fld(F_TS, ia), t));
  Fm body = forallP(0,
      and_(and_(and_(and_(imp(contains(A, i), eq(fld(F_X, i), v)),
                          imp(fld(F_DECIDED, i), eq(fld(F_DECISION, i), v))),
                     imp(fld(F_COMMIT, i), eq(fld(F_VOTE, i), v))),
                imp(fld(F_READY, i), eq(fld(F_VOTE, i), v))),
           imp(eq(fld(F_TS, i), r4), fld(F_COMMIT, coord()))));
  Fm majority = existsVInt(2, existsVInt(3,
      and_(and_(and_(gt(card(A), half), gt(rvar(), lit(0))), le(t, r4)), body)));
  Fm keepInit = forallP(0, existsP(1, eq(fld(F_X, i), fld(F_X, j1, T_INIT))));
  Fm safetyInv = and_(keepInit, or_(noDecision, majority));
  Fm inv1 = existsP(5, forallP(0, and_(fld(F_DECIDED, i), eq(fld(F_DECISION, i), fld(F_X, j, T_INIT)))));
  s.invariants = {safetyInv, inv1};
  /* roundInvariants: index 0 of every list is `true` (LastVoting.scala:176-189) */
  Fm r1 = existsP(0, fld(F_COMMIT, i));
  Fm r2 = existsP(0, and_(fld(F_COMMIT, i), forallP(5, and_(eq(fld(F_TS, j), r4), eq(fld(F_X, j), fld(F_VOTE, i))))));
  Fm r3 = existsP(0, and_(and_(fld(F_COMMIT, i), fld(F_READY, i)),
                          forallP(5, and_(eq(fld(F_TS, j), r4), eq(fld(F_X, j), fld(F_VOTE, i))))));
  s.roundInvariants = {{tru(), r1}, {tru(), r2}, {tru(), r3}};
  consensus_properties(s, true);
  return s;
}

/* example/BenOr.scala:90-115 (V = Domain[Boolean]) */
static SpecDef benor_spec() {
  SpecDef s;
  Fm i = bv(0), j = bv(1), v = bv(2), ia = bv(3), p = bv(4);
  Fm half = div_(nvar(), lit(2));
  Fm A = filterP(3, eq(fld(F_X, ia), v));
  Fm inv0 = or_(forallP(0, and_(not_(fld(F_DECIDED, i)), not_(fld(F_CANDECIDE, i)))),
                existsVBool(2, and_(gt(card(A), half),
                                    forallP(0, and_(imp(fld(F_DECIDED, i), eq(fld(F_DECISION, i), v)),
                                                    imp(isdef(fld(F_VOTE, i)), eq(fld(F_VOTE, i), v)))))));
  s.invariants = {inv0};
  /* P.forall(p => p.vote.isDefined ==> P.filter(i => i.x == p.vote.get).size > n/2) */
  Fm Ap = filterP(3, eq(fld(F_X, ia), get(fld(F_VOTE, p))));
  s.roundInvariants = {{forallP(4, imp(isdef(fld(F_VOTE, p)), gt(card(Ap), half)))}};
  s.properties.push_back({"Agreement",
      forallP(0, forallP(1, imp(and_(fld(F_DECIDED, i), fld(F_DECIDED, j)),
                                eq(fld(F_DECISION, i), fld(F_DECISION, j)))))});
  s.properties.push_back({"Irrevocability",
      forallP(0, imp(fld(F_DECIDED, i, T_OLD),
                     and_(fld(F_DECIDED, i), eq(fld(F_DECISION, i, T_OLD), fld(F_DECISION, i)))))});
  s.termination = forallP(0, fld(F_DECIDED, i));
  /* safetyPredicate: P.forall(p => p.HO.size > n/2), BenOr.scala:92. HO(p) is
   * the effective heard-of set of the round just executed (a halted sender
   * sends nothing); a halted receiver takes no step and is vacuous. */
  s.safetyPredicate = forallP(4, gt(fld(F_HOSIZE, p), half));
  return s;
}

/* Check-slot layout (must match psg_check_name and the device kernels). */
static int n_checks_of(int alg) {
  switch (alg) {
    case PSG_ALG_OTR: return 8;
    case PSG_ALG_LAST_VOTING: return 7;
    case PSG_ALG_BENOR: return 5;
    case PSG_ALG_FLOODMIN: return 2;
    case PSG_ALG_KSET: return 2;
    case PSG_ALG_OTR2: return 8;
    case PSG_ALG_SLV: return 2;
    case PSG_ALG_KSET_ES: return 2;
    case PSG_ALG_EPSILON: return 3;
  }
  return 0;
}

/* Invariant i at check point c with phase position j = c mod L holds iff
 * invariants(i) && (j != 0 ==> roundInvariants(j-1)(0)) — Verifier.getInvariant
 * uses index 0 of the round-invariant list for every invariant
 * (psync/verification/Verifier.scala:111-141). Slot 0 = "Safety": some invariant
 * holds. Properties follow; relational ones (old) are vacuous at c = 0. */
static void eval_spec_interp(const SpecDef& sd, const SpecState& st, int L, bool has_old, std::vector<bool>& checks,
                             bool& term) {
  Interp in(st, sd.all_roots());
  int j = (int)(st.r % L);
  bool rinv = true;
  if (j != 0 && (int)sd.roundInvariants.size() > j - 1 && !sd.roundInvariants[j - 1].empty())
    rinv = in.ev(sd.roundInvariants[j - 1][0]) != 0;
  checks.clear();
  checks.push_back(false);
  bool any = false;
  for (auto& inv : sd.invariants) {
    bool h = rinv && in.ev(inv) != 0;
    checks.push_back(h);
    any = any || h;
  }
  checks[0] = any;
  for (auto& pr : sd.properties) {
    if (!has_old && pr.first == "Irrevocability") checks.push_back(true);
    else checks.push_back(in.ev(pr.second) != 0);
  }
  term = in.ev(sd.termination) != 0;
  if (sd.safetyPredicate) checks.push_back(in.ev(sd.safetyPredicate) != 0);
}

/* ------------------------------------------------------------------ */
/* Algorithms (literal restatements)                                   */
/* ------------------------------------------------------------------ */
/* fold32 of the IEEE-754 bits: how a Double enters the int32 record fields and the digest */
static int32_t fold32(double d) {
  uint64_t b;
  std::memcpy(&b, &d, 8);
  return (int32_t)(uint32_t)(b ^ (b >> 32));
}

struct Callback { /* ConsensusIO.decide / RealConsensusIO.decide */
  int32_t value = 0;
  int32_t round = -1;
  double fvalue = 0.0;
  void decide(int32_t v, int k) {
    if (round < 0) { value = v; round = k; }
  }
  void decide_real(double v, int k) {
    if (round < 0) { fvalue = v; value = fold32(v); round = k; }
  }
};

template <class A>
struct Msg { int src; A payload; };


/* Otr2.scala:32-36, the `ensuring` clause of mmor, literally:
 *   mailbox.forall{ case (k, v2) =>
 *     mailbox.count{ case (k, v3) => v1 == v3 } > mailbox.count{ case (k, v3) => v2 == v3 } || v1 <= v2 }
 * evaluated on every mmor the oracle executes (OTR and OTR2 share the round) while the pin
 * tests have it on (oracle_set_mmor_check; off by default, so the CPU baseline times the round
 * alone, not this O(|mailbox|^2) check); the counters are read by
 * tests/test_reference_pins.py through oracle_mmor_ensuring_stats. */
static std::atomic<int> g_mmor_check{0};
static std::atomic<uint64_t> g_mmor_calls{0}, g_mmor_ensuring_failures{0};
static void mmor_ensuring(const std::vector<Msg<int32_t>>& mb, int32_t v1) {
  if (!g_mmor_check.load(std::memory_order_relaxed)) return;
  auto count = [&](int32_t v) {
    int c = 0;
    for (auto& m : mb) c += m.payload == v;
    return c;
  };
  bool ok = true;
  for (auto& m : mb) ok = ok && (count(v1) > count(m.payload) || v1 <= m.payload);
  g_mmor_calls.fetch_add(1, std::memory_order_relaxed);
  if (!ok) g_mmor_ensuring_failures.fetch_add(1, std::memory_order_relaxed);
}

/* ---------------- OTR: example/Otr.scala:13-86 ---------------- */
struct Otr {
  struct P {
    int32_t x = 0, decision = -1;
    bool decided = false;
    int32_t after = 2;
  };
  using Payload = int32_t;
  int n, afterDecision, variant;
  int thr() const { return variant == 1 ? n / 2 : 2 * n / 3; }
  static const int L = 1;
  void init(P& s, int32_t initValue) { /* Otr.scala:21-26 */
    s.x = initValue; s.decided = false; s.after = afterDecision;
  }
  /* send(): broadcast(x) */
  bool sends_to(const P&, int, int, int) const { return true; }
  Payload payload(const P& s, int, int, int) const { return s.x; }
  /* mmor, Otr.scala:44-49: groupBy value, minBy (-size, v). Every result is checked against
   * the post-condition the reference states for the same function (Otr2.scala:32-36):
   * mailbox.forall{ (k, v2) => count(v1) > count(v2) || v1 <= v2 } (mmor_ensuring below). */
  int32_t mmor(const std::vector<Msg<int32_t>>& mb) const {
    std::map<int32_t, int> byValue;
    for (auto& m : mb) byValue[m.payload]++;
    bool first = true;
    std::pair<int, int32_t> best{0, 0};
    for (auto& kv : byValue) {
      /* variant 2 (oracle-only mutant, tests): ties go to the LARGER value */
      std::pair<int, int32_t> key{-kv.second, variant == 2 ? -kv.first : kv.first};
      if (first || key < best) { best = key; first = false; }
    }
    if (variant == 2) best.second = -best.second;
    mmor_ensuring(mb, best.second);
    return best.second;
  }
  /* update, Otr.scala:63-81; returns true on exitAtEndOfRound */
  bool update(P& s, int, int k, const std::vector<Msg<int32_t>>& mb, Callback& cb, const Schedule&, int) {
    bool exit = false;
    if ((int)mb.size() > thr()) {
      int32_t v = mmor(mb);
      s.x = v;
      int cnt = 0;
      for (auto& m : mb) if (m.payload == v) ++cnt;
      if (cnt > thr()) {
        if (!s.decided) cb.decide(v, k);
        s.decided = true;
        s.decision = v;
      }
    }
    if (s.decided) {
      s.after = s.after - 1;
      if (s.after <= 0) exit = true;
    }
    return exit;
  }
  void fields(const P& s, int64_t* f) const {
    f[F_X] = s.x; f[F_DECIDED] = s.decided; f[F_DECISION] = s.decision;
  }
  int32_t main_x(const P& s) const { return s.x; }
};

/* ---------------- LastVoting: example/LastVoting.scala:80-212 ---------------- */
struct LV {
  struct P {
    int32_t x = 0, ts = -1;
    bool ready = false, commit = false;
    int32_t vote = 0, decision = -1;
    bool decided = false;
  };
  struct Payload { int32_t x; int32_t ts; };
  int n, variant, tiebreak;
  static const int L = 4;
  int coord(int k) const { return (k / 4) % n; } /* LastVoting.scala:95 */
  void init(P& s, int32_t initValue) { /* LastVoting.scala:97-109 */
    s.x = initValue; s.ts = -1; s.decided = false; s.ready = false; s.commit = false;
  }
  bool sends_to(const P& s, int self, int k, int dst) const {
    int c = coord(k);
    switch (k % 4) {
      case 0: return dst == c;                              /* Map(coord -> (x, ts)) */
      case 1: return self == c && s.commit;                 /* broadcast(vote) if coord && commit */
      case 2: return s.ts == k / 4 && dst == c;             /* Map(coord -> x) if ts == r/4 */
      default: return self == c && s.ready;                 /* broadcast(vote) if coord && ready */
    }
  }
  Payload payload(const P& s, int, int k, int) const {
    switch (k % 4) {
      case 0: return {s.x, s.ts};
      case 1: return {s.vote, 0};
      case 2: return {s.x, 0};
      default: return {s.vote, 0};
    }
  }
  bool update(P& s, int self, int k, const std::vector<Msg<Payload>>& mb, Callback& cb, const Schedule&, int) {
    int c = coord(k);
    auto contains_coord = [&](int32_t& v) {
      for (auto& m : mb) if (m.src == c) { v = m.payload.x; return true; }
      return false;
    };
    switch (k % 4) {
      case 0: { /* LastVoting.scala:112-138 */
        if (self == c && ((int)mb.size() > n / 2 || (k == 0 && mb.size() > 0))) {
          /* vote = mailbox.maxBy(_._2._2)._2._1 — first max in Map iteration order */
          std::vector<int> ins;
          for (auto& m : mb) ins.push_back(m.src);
          std::vector<int> order = scala_map_order(ins, tiebreak);
          bool first = true;
          int32_t maxTs = 0, vote = 0;
          for (int q : order) {
            for (auto& m : mb) if (m.src == q) {
              if (first || m.payload.ts > maxTs) { maxTs = m.payload.ts; vote = m.payload.x; first = false; }
            }
          }
          s.vote = vote;
          s.commit = true;
        }
        return false;
      }
      case 1: { /* LastVoting.scala:140-160 */
        int32_t v;
        if (contains_coord(v)) { s.x = v; s.ts = k / 4; }
        return false;
      }
      case 2: { /* LastVoting.scala:163-181 */
        int need = variant == 1 ? 0 : n / 2;
        if (self == c && (int)mb.size() > need) s.ready = true;
        return false;
      }
      default: { /* LastVoting.scala:183-208 */
        bool exit = false;
        int32_t v;
        if (contains_coord(v)) {
          cb.decide(v, k);
          s.decision = v;
          s.decided = true;
          exit = true;
        }
        s.ready = false;
        s.commit = false;
        return exit;
      }
    }
  }
  void fields(const P& s, int64_t* f) const {
    f[F_X] = s.x; f[F_DECIDED] = s.decided; f[F_DECISION] = s.decision; f[F_TS] = s.ts;
    f[F_READY] = s.ready; f[F_COMMIT] = s.commit; f[F_VOTE] = s.vote;
  }
  int32_t main_x(const P& s) const { return s.x; }
};

/* ---------------- FloodMin: example/FloodMin.scala:8-36 ---------------- */
struct FloodMin {
  struct P { int32_t x = 0; bool decided = false; int32_t decision = 0; };
  using Payload = int32_t;
  int n, f, variant;
  static const int L = 1;
  void init(P& s, int32_t v) { s.x = v; }
  bool sends_to(const P&, int, int, int) const { return true; }
  Payload payload(const P& s, int, int, int) const { return s.x; }
  bool update(P& s, int, int k, const std::vector<Msg<int32_t>>& mb, Callback& cb, const Schedule&, int) {
    int32_t acc = s.x; /* mailbox.foldLeft(x)(min) */
    for (auto& m : mb) acc = std::min(acc, m.payload);
    s.x = acc;
    bool decideNow = variant == 1 ? (k >= f - 1) : (k > f);
    if (decideNow) {
      cb.decide(s.x, k);
      s.decided = true; s.decision = s.x;
      return true;
    }
    return false;
  }
  void fields(const P& s, int64_t* fv) const { fv[F_X] = s.x; fv[F_DECIDED] = s.decided; fv[F_DECISION] = s.decision; }
  int32_t main_x(const P& s) const { return s.x; }
};

/* ---------------- KSetAgreement: example/KSetAgreement.scala:21-68 ---------------- */
struct KSet {
  struct P {
    std::map<int, int32_t> t; /* Map[ProcessID, Int] */
    bool decider = false;
    bool decided = false;
    int32_t decision = 0;
  };
  struct Payload { bool decider; std::shared_ptr<const std::map<int, int32_t>> t; };
  int n, k, variant, tiebreak;
  static const int L = 1;
  int self_init_pid = 0;
  void init(P&, int32_t) {}
  bool sends_to(const P&, int, int, int) const { return true; }
  Payload payload(const P& s, int, int, int) const {
    return {s.decider, std::make_shared<const std::map<int, int32_t>>(s.t)};
  }
  static int32_t pick(const std::map<int, int32_t>& t) { /* a.values.min */
    int32_t m = INT32_MAX;
    for (auto& kv : t) m = std::min(m, kv.second);
    return m;
  }
  bool update(P& s, int, int r, const std::vector<Msg<Payload>>& mb, Callback& cb, const Schedule&, int) {
    if (s.decider) { /* KSetAgreement.scala:48-50 */
      cb.decide(pick(s.t), r);
      s.decided = true; s.decision = pick(s.t);
      return true;
    }
    /* val content = mailbox.map{ case (k,v) => v } (KSetAgreement.scala:47): v is a pair
     * (Boolean, Map[ProcessID,Int]), so Scala 2.13 picks MapOps.map[K2,V2] and content is a
     * Map[Boolean, Map[ProcessID,Int]] built by inserting every message in the mailbox's
     * iteration order; a later message with the same flag overwrites the value. Hence
     * content.find(_._1).get._2 (:53) is the t of the LAST decider in iteration order. */
    bool anyDecider = false; /* content.exists(_._1) (:51) */
    for (auto& m : mb) anyDecider = anyDecider || m.payload.decider;
    if (anyDecider) {
      std::vector<int> ins;
      for (auto& m : mb) ins.push_back(m.src);
      std::map<bool, std::shared_ptr<const std::map<int, int32_t>>> content;
      for (int q : scala_map_order(ins, tiebreak))
        for (auto& m : mb)
          if (m.src == q) content[m.payload.decider] = m.payload.t;
      s.decider = true;
      s.t = *content.at(true);
    } else {
      int same = 0;
      for (auto& m : mb) if (*m.payload.t == s.t) ++same;
      int need = variant == 1 ? 1 : n - k;
      if (same > need) {
        s.decider = true;
      } else {
        for (auto& m : mb) /* t = t ++ v */
          for (auto& kv : *m.payload.t) s.t[kv.first] = kv.second;
      }
    }
    return false;
  }
  void fields(const P& s, int64_t* fv) const { fv[F_X] = pick(s.t); fv[F_DECIDED] = s.decided; fv[F_DECISION] = s.decision; }
  int32_t main_x(const P& s) const { return pick(s.t); }
};

/* ---------------- BenOr: example/BenOr.scala:11-84 ---------------- */
struct BenOr {
  struct P {
    bool x = false, canDecide = false;
    int8_t vote = -1; /* Option[Boolean]: -1 None, 0 Some(false), 1 Some(true) */
    bool decision = false, decided = false;
  };
  struct Payload { bool a; bool b; int8_t vote; };
  int n, variant;
  static const int L = 2;
  void init(P& s, int32_t v) { s.x = v != 0; s.canDecide = false; s.decided = false; }
  bool sends_to(const P&, int, int, int) const { return true; }
  Payload payload(const P& s, int, int k, int) const {
    if (k % 2 == 0) return {s.x, s.canDecide, -1};
    return {false, false, s.vote};
  }
  bool update(P& s, int self, int k, const std::vector<Msg<Payload>>& mb, Callback& cb, const Schedule& sch, int) {
    if (k % 2 == 0) { /* BenOr.scala:37-53 */
      if (s.canDecide) {
        cb.decide(s.x ? 1 : 0, k);
        s.decided = true; s.decision = s.x;
        return true;
      }
      int cT = 0, cF = 0;
      bool exT = false, exF = false, exCD = false;
      for (auto& m : mb) {
        if (m.payload.a) ++cT; else ++cF;
        if (m.payload.a && m.payload.b) exT = true;
        if (!m.payload.a && m.payload.b) exF = true;
        if (m.payload.b) exCD = true;
      }
      if (cT > n / 2 || exT) s.vote = 1;
      else if (cF > n / 2 || exF) s.vote = 0;
      else s.vote = -1;
      s.canDecide = exCD;
      return false;
    }
    /* BenOr.scala:63-79 */
    int t = 0, f = 0;
    for (auto& m : mb) { if (m.payload.vote == 1) ++t; if (m.payload.vote == 0) ++f; }
    int thr = variant == 1 ? n / 4 : n / 2;
    if (t > thr) { s.x = true; s.canDecide = true; }
    else if (f > thr) { s.x = false; s.canDecide = true; }
    else if (t > 1) s.x = true;
    else if (f > 1) s.x = false;
    else s.x = sch.coin(k, self); /* util.Random.nextBoolean, seeded per (inst, round, pid) */
    return false;
  }
  void fields(const P& s, int64_t* fv) const {
    fv[F_X] = s.x; fv[F_DECIDED] = s.decided; fv[F_DECISION] = s.decision; fv[F_CANDECIDE] = s.canDecide;
    fv[F_VOTE] = s.vote < 0 ? NONE : s.vote;
  }
  int32_t main_x(const P& s) const { return s.x ? 1 : 0; }
};

/* ---------------- OTR2: example/Otr2.scala:9-66 ----------------
 * Same round as OTR (Otr2.scala:26-61: mmor, > 2n/3 adopt / decide, callback
 * only while decision.isEmpty, decision = Some(v), after countdown); the
 * difference is decision: Option[Int], which the Spec sees as value-or-None. */
struct Otr2 : Otr {
  void fields(const P& s, int64_t* f) const {
    f[F_X] = s.x; f[F_DECIDED] = s.decided; f[F_DECISION] = s.decided ? (int64_t)s.decision : NONE;
  }
};

/* ---------------- ShortLastVoting: example/ShortLastVoting.scala:13-105 ---------------- */
struct SLV {
  struct P {
    int32_t x = 0, ts = -1;
    bool commit = false;
    int32_t vote = 0, decision = -1;
    bool decided = false;
  };
  struct Payload { int32_t x; int32_t ts; };
  int n, variant, tiebreak;
  static const int L = 3;
  int coord(int k) const { return (k / 4) % n; } /* coord(r/4), ShortLastVoting.scala:23, 37 (r/4 literal) */
  void init(P& s, int32_t v) { /* ShortLastVoting.scala:25-31 */
    s.x = v; s.ts = -1; s.decided = false; s.commit = false;
  }
  bool sends_to(const P& s, int self, int k, int dst) const {
    switch (k % 3) {
      case 0: return dst == coord(k);              /* Map(coord(r/4) -> (x, ts)) */
      case 1: return self == coord(k) && s.commit; /* broadcast(vote) if coord && commit */
      default: return s.ts == k / 4;               /* broadcast(x) if ts == r/4 */
    }
  }
  Payload payload(const P& s, int, int k, int) const {
    switch (k % 3) {
      case 0: return {s.x, s.ts};
      case 1: return {s.vote, 0};
      default: return {s.x, 0};
    }
  }
  static int first_in_map_order(const std::vector<Msg<Payload>>& mb, int tiebreak) {
    std::vector<int> ins;
    for (auto& m : mb) ins.push_back(m.src);
    return scala_map_order(ins, tiebreak)[0];
  }
  bool update(P& s, int self, int k, const std::vector<Msg<Payload>>& mb, Callback& cb, const Schedule&, int) {
    const int c = coord(k);
    switch (k % 3) {
      case 0: { /* ShortLastVoting.scala:39-46 */
        if (self == c && (int)mb.size() > n / 2) {
          /* vote = mailbox.maxBy(_._2._2)._2._1: first max in Map iteration order */
          std::vector<int> ins;
          for (auto& m : mb) ins.push_back(m.src);
          bool first = true;
          int32_t maxTs = 0, vote = 0;
          for (int q : scala_map_order(ins, tiebreak))
            for (auto& m : mb)
              if (m.src == q && (first || m.payload.ts > maxTs)) { maxTs = m.payload.ts; vote = m.payload.x; first = false; }
          s.vote = vote;
          s.commit = true;
        }
        return false;
      }
      case 1: /* ShortLastVoting.scala:63-68 */
        for (auto& m : mb) if (m.src == c) { s.x = m.payload.x; s.ts = k / 4; }
        return false;
      default: { /* ShortLastVoting.scala:84-97 */
        const int need = variant == 1 ? 0 : n / 2;
        if ((int)mb.size() > need) {
          const int h = first_in_map_order(mb, tiebreak); /* mailbox.head._2 */
          int32_t v = 0;
          for (auto& m : mb) if (m.src == h) v = m.payload.x;
          if (!s.decided) {
            cb.decide(v, k);
            s.decision = v;
            s.decided = true;
          }
        }
        s.commit = false;
        return s.decided;
      }
    }
  }
  void fields(const P& s, int64_t* f) const {
    f[F_X] = s.x; f[F_DECIDED] = s.decided; f[F_DECISION] = s.decision; f[F_TS] = s.ts;
    f[F_COMMIT] = s.commit; f[F_VOTE] = s.vote;
  }
  int32_t main_x(const P& s) const { return s.x; }
};

/* ---------------- KSetEarlyStopping: example/KSetEarlyStopping.scala:9-44 ---------------- */
struct KSetES {
  struct P { int32_t est = 0; bool canDecide = false; int32_t lastNb = 0; bool decided = false; int32_t decision = 0; };
  struct Payload { int32_t est; bool canDecide; };
  int n, t, k, variant;
  static const int L = 1;
  void init(P& s, int32_t v) { s.canDecide = false; s.lastNb = n; s.est = v; } /* :16-21 */
  bool sends_to(const P&, int, int, int) const { return true; }                   /* broadcast((est, canDecide)) */
  Payload payload(const P& s, int, int, int) const { return {s.est, s.canDecide}; }
  bool update(P& s, int, int r, const std::vector<Msg<Payload>>& mb, Callback& cb, const Schedule&, int) {
    const int currNb = (int)mb.size(); /* :31-41 */
    if (r > t / k || s.canDecide) {
      cb.decide(s.est, r);
      s.decided = true; s.decision = s.est;
      return true;
    }
    /* est = mailbox.map(_._2._1).min. An empty mailbox (pure HO mode only: with
     * the self bit a running process always hears itself) would throw in Scala;
     * here est is left unchanged. */
    bool ex = false;
    for (auto& m : mb) ex = ex || m.payload.canDecide; /* mailbox.exists(_._2._2) */
    if (!mb.empty()) {
      int32_t mn = INT32_MAX;
      for (auto& m : mb) mn = std::min(mn, m.payload.est);
      s.est = mn;
    }
    s.canDecide = variant == 1 ? true : (ex || s.lastNb - currNb < k);
    s.lastNb = currNb;
    return false;
  }
  void fields(const P& s, int64_t* fv) const { fv[F_X] = s.est; fv[F_DECIDED] = s.decided; fv[F_DECISION] = s.decision; }
  int32_t main_x(const P& s) const { return s.est; }
};

/* ---------------- EpsilonConsensus: example/Epsilon.scala:16-70 ---------------- */
/* Java narrowing of double to int (math.ceil(r1).toInt). */
static int32_t d2i(double d) {
  if (std::isnan(d)) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}
/* Ordering.Double.TotalOrdering (java.lang.Double.compare): -0.0 < 0.0, NaN last. */
static int64_t total_key(double d) {
  int64_t b;
  if (std::isnan(d)) b = 0x7ff8000000000000LL; /* doubleToLongBits canonical NaN */
  else std::memcpy(&b, &d, 8);
  return b ^ ((b >> 63) & 0x7fffffffffffffffLL);
}

struct Epsilon {
  struct P {
    double x = 0.0;
    int32_t maxR = 0;                /* var maxR = new Time(0) */
    std::map<int, double> halted;    /* var halted = Map[ProcessID, Double]() */
    bool decided = false;
    double decision = 0.0;
  };
  struct Payload { double x; bool flag; };
  int n, f, variant;
  double eps;
  static const int L = 1;
  void init(P& s, double v) { s.x = v; } /* Epsilon.scala:23-26 */
  bool sends_to(const P&, int, int, int) const { return true; }
  /* if (r <= maxR) broadcast(x -> false) else broadcast(x -> true), Epsilon.scala:44-50 */
  Payload payload(const P& s, int, int k, int) const { return {s.x, !(k <= s.maxR)}; }
  static std::vector<double> sorted(std::vector<double> v) {
    std::stable_sort(v.begin(), v.end(), [](double a, double b) { return total_key(a) < total_key(b); });
    return v;
  }
  /* Epsilon.scala:52-67 */
  bool update(P& s, int, int k, const std::vector<Msg<Payload>>& mb, Callback& cb, const Schedule&, int) {
    std::vector<double> V;
    for (auto& m : mb) V.push_back(m.payload.x);          /* mailbox.toSeq.map(_._2._1) */
    for (auto& kv : s.halted) V.push_back(kv.second);     /* ++ halted.values */
    for (auto& m : mb) if (m.payload.flag) s.halted[m.src] = m.payload.x;
    if (k == 0) {
      /* diff(V) of an empty V and reduce(2f, V).head with |V| <= 4f throw in Scala;
       * here they leave maxR / x unchanged (needs a pure-HO schedule or tiny mailboxes) */
      if (V.empty()) return false;
      std::vector<double> sv = sorted(V);
      const double diff = sv.back() - sv.front();       /* s.max - s.min */
      const int c = (n - 3 * f - 1) / (2 * f) + 1;       /* c(n-3f, 2f) = (m-1)/k + 1 */
      const double r1 = std::log(diff / eps) / std::log((double)c);
      s.maxR = d2i(std::ceil(r1));
      if (variant == 1) s.maxR = 0; /* mutation: no approximation rounds, decide in round 1 */
      if ((int)sv.size() > 4 * f) s.x = sv[2 * f];       /* reduce(2f, V).head */
    } else if (k <= s.maxR) {
      /* _new(2f, f, V): red = sorted.drop(f).dropRight(f); sel = red.grouped(2f).map(_.head);
       * sel.sum / sel.size (left fold from 0.0; 0.0 / 0 = NaN for an empty sel) */
      std::vector<double> sv = sorted(V);
      const int m = (int)sv.size();
      double sum = 0.0;
      int cnt = 0;
      for (int j = f; j < m - f; j += 2 * f) { sum += sv[j]; ++cnt; }
      s.x = sum / (double)cnt;
    } else {
      cb.decide_real(s.x, k);
      s.decided = true;
      s.decision = s.x;
      return true;
    }
    return false;
  }
  void fields(const P& s, int64_t* fv) const {
    fv[F_X] = fold32(s.x); fv[F_DECIDED] = s.decided; fv[F_DECISION] = fold32(s.decision);
  }
  int32_t main_x(const P& s) const { return fold32(s.x); }
  /* Build-defined checks (TrivialSpec, Epsilon.scala:74): 0 EpsAgreement — decisions
   * are not NaN and max - min <= epsilon; 1 EpsValidity — every decision lies within
   * [min, max] of the (non-NaN) initial values; 2 SafetyPredicate — every process
   * that took a step had |V| = |mailbox| + |halted| >= n - f values (the commented
   * assert mailbox.size >= n - f, Epsilon.scala:57, with the remembered values of
   * halted senders standing in for their messages after they exit). */
  void checks(const std::vector<P>& st, const std::vector<double>& x0, const std::vector<int>& hosize,
              std::vector<bool>& ck, bool& term) const {
    bool anyD = false, nanD = false, anyI = false;
    double mx = 0, mn = 0, lo = 0, hi = 0;
    for (double v : x0)
      if (!std::isnan(v)) {
        if (!anyI) { lo = hi = v; anyI = true; }
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
      }
    bool valid = true;
    term = true;
    for (size_t p = 0; p < st.size(); ++p) {
      if (!st[p].decided) { term = false; continue; }
      const double d = st[p].decision;
      if (std::isnan(d)) { nanD = true; valid = false; continue; }
      if (!anyD) { mx = mn = d; anyD = true; }
      mx = d > mx ? d : mx;
      mn = d < mn ? d : mn;
      if (!(anyI && lo <= d && d <= hi)) valid = false;
    }
    const bool agree = !nanD && (!anyD || mx - mn <= eps);
    bool pred = true;
    for (int h : hosize) if (h < n - f) pred = false;
    ck = {agree, valid, pred};
  }
};

/* ------------------------------------------------------------------ */
/* Hand-lowered Spec evaluator (what the GPU kernel implements)         */
/* ------------------------------------------------------------------ */
struct Direct {
  /* inputs */
  int n, alg, kparam, kparam2;
  int64_t r;
  const std::vector<int64_t>* cur;  /* [F][p] */
  const std::vector<int64_t>* old;
  const std::vector<int64_t>* init;
  const std::vector<bool>* crashed;
  bool has_old;

  bool inX0(int64_t v) const {
    for (int p = 0; p < n; ++p) if (init[F_X][p] == v) return true;
    return false;
  }
  bool keepInit() const {
    for (int p = 0; p < n; ++p) if (!inX0(cur[F_X][p])) return false;
    return true;
  }
  /* all decided processes agree: returns (anyDecided, same, d0) */
  void decisions(bool& any, bool& same, int64_t& d0) const {
    any = false; same = true; d0 = 0;
    for (int p = 0; p < n; ++p) if (cur[F_DECIDED][p]) {
      if (!any) { any = true; d0 = cur[F_DECISION][p]; }
      else if (cur[F_DECISION][p] != d0) same = false;
    }
  }
  bool irrevocability() const {
    if (!has_old) return true;
    for (int p = 0; p < n; ++p)
      if (old[F_DECIDED][p] && !(cur[F_DECIDED][p] && old[F_DECISION][p] == cur[F_DECISION][p])) return false;
    return true;
  }
  bool allDecided() const {
    for (int p = 0; p < n; ++p) if (!cur[F_DECIDED][p]) return false;
    return true;
  }
  bool validity() const {
    for (int p = 0; p < n; ++p) if (cur[F_DECIDED][p] && !inX0(cur[F_DECISION][p])) return false;
    return true;
  }

  void eval(std::vector<bool>& ck, bool& term) const {
    ck.clear();
    term = allDecided();
    bool any, same; int64_t d0;
    decisions(any, same, d0);
    if (alg == PSG_ALG_OTR) {
      int thr = 2 * n / 3;
      bool ki = keepInit();
      bool e0 = false, e1 = false;
      std::set<int64_t> xs;
      for (int p = 0; p < n; ++p) xs.insert(cur[F_X][p]);
      for (int64_t v : xs) {
        int cnt = 0;
        for (int p = 0; p < n; ++p) if (cur[F_X][p] == v) ++cnt;
        bool condv = !any || (same && v == d0);
        if (cnt > thr && condv) e0 = true;
        if (cnt == n && condv) e1 = true;
      }
      bool inv0 = (!any || e0) && ki;
      bool inv1 = e1 && ki;
      bool d0in = any && inX0(d0);
      bool inv2 = term && same && d0in;
      ck = {inv0 || inv1 || inv2, inv0, inv1, inv2, same, validity(), !any || (same && d0in), irrevocability()};
    } else if (alg == PSG_ALG_LAST_VOTING) {
      int64_t r4 = r / 4;
      int c = (int)(r4 % n);
      bool ki = keepInit();
      bool noDec = true;
      for (int p = 0; p < n; ++p) if (cur[F_DECIDED][p] || cur[F_READY][p]) noDec = false;
      /* values pinned by decided / commit / ready processes */
      bool zAny = false, zOk = true; int64_t z0 = 0;
      auto pin = [&](int64_t z) { if (!zAny) { zAny = true; z0 = z; } else if (z != z0) zOk = false; };
      for (int p = 0; p < n; ++p) {
        if (cur[F_DECIDED][p]) pin(cur[F_DECISION][p]);
        if (cur[F_COMMIT][p] || cur[F_READY][p]) pin(cur[F_VOTE][p]);
      }
      bool c5 = true;
      for (int p = 0; p < n; ++p) if (cur[F_TS][p] == r4 && !cur[F_COMMIT][c]) c5 = false;
      bool maj = false;
      if (r > 0 && zOk && c5) {
        std::set<int64_t> cands = {(int64_t)INT32_MIN};
        for (int p = 0; p < n; ++p) cands.insert(cur[F_TS][p] + 1);
        for (int64_t t : cands) {
          if (t > r4) continue;
          int cnt = 0; bool allSame = true, first = true; int64_t xv = 0;
          for (int p = 0; p < n; ++p) if (cur[F_TS][p] >= t) {
            ++cnt;
            if (first) { xv = cur[F_X][p]; first = false; } else if (cur[F_X][p] != xv) allSame = false;
          }
          if (cnt > n / 2 && allSame && (!zAny || xv == z0)) { maj = true; break; }
        }
      }
      bool inv0 = ki && (noDec || maj);
      bool inv1 = term && same && any && inX0(d0);
      ck = {inv0 || inv1, inv0, inv1, same, validity(), !any || (same && inX0(d0)), irrevocability()};
    } else if (alg == PSG_ALG_BENOR) {
      bool noDec = true;
      for (int p = 0; p < n; ++p) if (cur[F_DECIDED][p] || cur[F_CANDECIDE][p]) noDec = false;
      int cnt[2] = {0, 0};
      for (int p = 0; p < n; ++p) cnt[cur[F_X][p] ? 1 : 0]++;
      bool ex = false;
      for (int v = 0; v <= 1; ++v) {
        if (!(cnt[v] > n / 2)) continue;
        bool ok = true;
        for (int p = 0; p < n; ++p) {
          if (cur[F_DECIDED][p] && cur[F_DECISION][p] != v) ok = false;
          if (cur[F_VOTE][p] != NONE && cur[F_VOTE][p] != v) ok = false;
        }
        if (ok) ex = true;
      }
      bool inv0 = noDec || ex;
      if (r % 2 == 1) { /* roundInvariants(0)(0) after R0 */
        for (int p = 0; p < n; ++p)
          if (cur[F_VOTE][p] != NONE && !(cnt[cur[F_VOTE][p]] > n / 2)) inv0 = false;
      }
      bool pred = true;
      for (int p = 0; p < n; ++p) if (!(cur[F_HOSIZE][p] > n / 2)) pred = false;
      ck = {inv0, inv0, same, irrevocability(), pred};
    } else if (alg == PSG_ALG_OTR2) {
      /* Otr2.scala:75-87: no keepInit; inv0's first disjunct is "all decided" */
      int thr = 2 * n / 3;
      bool e0 = false, e1 = false;
      std::set<int64_t> xs;
      for (int p = 0; p < n; ++p) xs.insert(cur[F_X][p]);
      for (int64_t v : xs) {
        int cnt = 0;
        for (int p = 0; p < n; ++p) if (cur[F_X][p] == v) ++cnt;
        bool condv = !any || (same && v == d0);
        if (cnt > thr && condv) e0 = true;
        if (cnt == n && condv) e1 = true;
      }
      bool inv0 = term || e0, inv1 = e1, inv2 = same;
      bool d0in = any && inX0(d0);
      ck = {inv0 || inv1 || inv2, inv0, inv1, inv2, same, validity(), !any || (same && d0in), irrevocability()};
    } else {
      /* TrivialSpec algorithms: build-defined k-agreement + validity
       * (KSetAgreement.scala:73). FloodMin / KSet / KSetEarlyStopping (crash-stop
       * algorithms): over never-crashed deciders; ShortLastVoting (HO model,
       * consensus): uniform, over every decider. */
      int k = alg == PSG_ALG_KSET ? kparam : alg == PSG_ALG_KSET_ES ? kparam2 : 1;
      bool uniform = alg == PSG_ALG_SLV;
      std::set<int64_t> Y;
      for (int p = 0; p < n; ++p)
        if (cur[F_DECIDED][p] && (uniform || !(*crashed)[p])) Y.insert(cur[F_DECISION][p]);
      ck = {(int)Y.size() <= k, validity()};
    }
  }
};

/* ------------------------------------------------------------------ */
/* Lockstep HO engine                                                  */
/* ------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
static uint64_t proc_digest(int pid, int32_t dec, int32_t dround, int32_t hround, int32_t mainx) {
  uint64_t y = ((uint64_t)(uint32_t)pid << 32) | ((uint64_t)((uint32_t)dround & 0xFFFFu) << 16) |
               (uint64_t)((uint32_t)hround & 0xFFFFu);
  uint64_t z = ((uint64_t)(uint32_t)dec << 32) | (uint64_t)(uint32_t)mainx;
  return splitmix64(z ^ splitmix64(y));
}

enum SpecMode { SPEC_DIRECT = 0, SPEC_INTERP = 1, SPEC_BOTH = 2 };

struct InstOut {
  psg_instance_summary sum;
  std::vector<psg_process_record> rec;
  std::vector<double> fdec, fx; /* real-valued algorithms: Double decision / final x per process */
  std::vector<int32_t>* vtrace = nullptr; /* Spec-program trace: [R+1][F][n] int32, None = INT32_MIN */
  std::vector<uint16_t>* ckbits = nullptr; /* per check point: bit s = slot s holds, bit 15 = Termination */
  std::vector<int64_t> trace; /* optional: per check point, per process F_X / decided */
  bool mismatch = false;
  std::string msg;
};

/* Explicit HO schedule of one instance (psg_load_schedule semantics, psg.h):
 * ho[(k * n + p) * W + w] = word w of HO(p) in round k, used verbatim (bits >= n
 * ignored). crash (nullable) = crash round per process for the never-crashed
 * classification; `legacy` keeps the single-instance KAT hook's behaviour
 * (crash classification from the seeded draw). */
struct ExplicitHO {
  const uint64_t* ho = nullptr;
  int W = 1;
  const int32_t* crash = nullptr;
  bool legacy = true;
};

template <class Alg>
static void run_engine(Alg& alg, const psg_config& cfg, uint64_t inst, const int32_t* init_in, int spec_mode,
                       const ExplicitHO* eho, InstOut& out, bool want_trace, const double* init_real = nullptr) {
  constexpr bool kReal = std::is_same<Alg, Epsilon>::value;
  const int n = cfg.n, R = cfg.rounds;
  Schedule sch(cfg, inst);
  std::vector<typename Alg::P> st(n);
  std::vector<Callback> cb(n);
  std::vector<bool> halted(n, false);
  std::vector<int32_t> halt_round(n, -1);
  std::vector<int32_t> x0(n);
  std::vector<double> x0r(n);
  for (int p = 0; p < n; ++p) {
    if constexpr (kReal) {
      x0r[p] = init_real ? init_real[p] : sch.init_real(p);
      alg.init(st[p], x0r[p]);
    } else {
      x0[p] = init_in ? init_in[p] : sch.init_value(p);
      alg.init(st[p], x0[p]);
    }
  }
  if constexpr (std::is_same<Alg, KSet>::value) /* t = Map(id -> io.initialValue) */
    for (int p = 0; p < n; ++p) st[p].t = {{p, x0[p]}};

  SpecDef sd;
  bool has_spec = cfg.alg == PSG_ALG_OTR || cfg.alg == PSG_ALG_LAST_VOTING || cfg.alg == PSG_ALG_BENOR ||
                  cfg.alg == PSG_ALG_OTR2;
  if (cfg.alg == PSG_ALG_OTR) sd = otr_spec();
  if (cfg.alg == PSG_ALG_OTR2) sd = otr2_spec();
  if (cfg.alg == PSG_ALG_LAST_VOTING) sd = lv_spec();
  if (cfg.alg == PSG_ALG_BENOR) sd = benor_spec();
  if (spec_mode != SPEC_DIRECT && !has_spec) spec_mode = SPEC_DIRECT;

  std::vector<int64_t> fcur[F_NFIELDS], fold[F_NFIELDS], finit[F_NFIELDS];
  std::vector<int> hosize(n, n); /* effective |HO(p)| of the last round; n if p took no step */
  auto snapshot = [&](std::vector<int64_t>* f) {
    for (int i = 0; i < F_NFIELDS; ++i) f[i].assign(n, 0);
    for (int p = 0; p < n; ++p) {
      int64_t tmp[F_NFIELDS] = {0};
      if (cfg.alg == PSG_ALG_BENOR) tmp[F_VOTE] = NONE;
      alg.fields(st[p], tmp);
      tmp[F_HOSIZE] = hosize[p];
      for (int i = 0; i < F_NFIELDS; ++i) f[i][p] = tmp[i];
    }
  };
  snapshot(finit);
  std::vector<bool> crashed(n);
  for (int p = 0; p < n; ++p)
    crashed[p] = (eho && !eho->legacy) ? (eho->crash != nullptr && eho->crash[p] >= 0) : sch.crashed(p);

  const int nck = n_checks_of(cfg.alg);
  psg_instance_summary& S = out.sum;
  std::memset(&S, 0, sizeof(S));
  for (int i = 0; i < PSG_MAX_CHECKS; ++i) S.first_fail[i] = PSG_NEVER;
  S.term_round = PSG_NEVER;
  S.n_checks = (uint8_t)nck;

  auto check = [&](int c, bool has_old) {
    snapshot(fcur);
    std::vector<bool> ck, ck2;
    bool term = false, term2 = false;
    Direct d{n, cfg.alg, cfg.param, cfg.param2, c, fcur, fold, finit, &crashed, has_old};
    if constexpr (kReal) alg.checks(st, x0r, hosize, ck, term);
    else if (spec_mode != SPEC_INTERP) d.eval(ck, term);
    if (spec_mode != SPEC_DIRECT) {
      SpecState ss;
      ss.n = n; ss.r = c;
      for (int i = 0; i < F_NFIELDS; ++i) { ss.v[T_CUR][i] = fcur[i]; ss.v[T_OLD][i] = fold[i]; ss.v[T_INIT][i] = finit[i]; }
      if (!has_old) for (int i = 0; i < F_NFIELDS; ++i) ss.v[T_OLD][i] = fcur[i];
      eval_spec_interp(sd, ss, Alg::L, has_old, ck2, term2);
      if (spec_mode == SPEC_BOTH && (ck != ck2 || term != term2)) {
        if (!out.mismatch) {
          char buf[256];
          std::snprintf(buf, sizeof buf, "spec mismatch inst %llu check %d", (unsigned long long)inst, c);
          out.msg = buf;
        }
        out.mismatch = true;
      }
      if (spec_mode == SPEC_INTERP) { ck = ck2; term = term2; }
    }
    for (int i = 0; i < nck; ++i)
      if (!ck[i] && S.first_fail[i] == PSG_NEVER) S.first_fail[i] = (uint8_t)c;
    if (term && S.term_round == PSG_NEVER) S.term_round = (uint8_t)c;
    if (out.ckbits) {
      uint16_t b = term ? (uint16_t)0x8000 : (uint16_t)0;
      for (int i = 0; i < nck; ++i) if (ck[i]) b |= (uint16_t)(1u << i);
      out.ckbits->push_back(b);
    }
    if (out.vtrace)
      for (int f = 0; f < F_NFIELDS; ++f)
        for (int p = 0; p < n; ++p)
          out.vtrace->push_back(fcur[f][p] == NONE ? INT32_MIN : (int32_t)fcur[f][p]);
    if (want_trace) {
      for (int p = 0; p < n; ++p) out.trace.push_back(fcur[F_X][p]);
      for (int p = 0; p < n; ++p) out.trace.push_back(fcur[F_DECIDED][p]);
    }
  };

  check(0, false);
  using Payload = typename Alg::Payload;
  for (int k = 0; k < R; ++k) {
    snapshot(fold);
    /* send: every non-halted process computes its messages from the pre-state */
    std::vector<std::vector<std::pair<int, Payload>>> inbox(n);
    std::vector<Payload> sent(n); /* every payload here is destination-independent */
    for (int q = 0; q < n; ++q) if (!halted[q]) sent[q] = alg.payload(st[q], q, k, -1);
    for (int p = 0; p < n; ++p) {
      if (halted[p]) continue;
      Bits ho;
      if (eho && eho->ho) {
        const uint64_t* m = eho->ho + ((size_t)k * n + p) * (size_t)eho->W;
        for (int q = 0; q < n; ++q) if ((m[q >> 6] >> (q & 63)) & 1) ho.set(q);
      } else {
        ho = sch.ho(k, p);
      }
      /* mailbox of p: senders q in HO(p), alive, that address p; inserted in ascending pid */
      for (int q = 0; q < n; ++q) {
        if (!ho.test(q) || halted[q]) continue;
        if (!alg.sends_to(st[q], q, k, p)) continue;
        inbox[p].push_back({q, sent[q]});
      }
    }
    std::vector<bool> exiting(n, false);
    for (int p = 0; p < n; ++p) hosize[p] = halted[p] ? n : (int)inbox[p].size();
    if constexpr (kReal) /* Epsilon: |V| = |mailbox| + |halted| (disjoint: a halted sender is silent) */
      for (int p = 0; p < n; ++p) if (!halted[p]) hosize[p] += (int)st[p].halted.size();
    for (int p = 0; p < n; ++p) {
      if (halted[p]) continue;
      std::vector<Msg<Payload>> mb;
      for (auto& e : inbox[p]) mb.push_back({e.first, e.second});
      exiting[p] = alg.update(st[p], p, k, mb, cb[p], sch, 0);
    }
    for (int p = 0; p < n; ++p)
      if (exiting[p]) { halted[p] = true; halt_round[p] = k; }
    check(k + 1, true);
  }

  out.rec.resize(n);
  uint64_t dig = 0;
  int nd = 0;
  for (int p = 0; p < n; ++p) {
    psg_process_record& pr = out.rec[p];
    pr.decision = cb[p].value;
    pr.decision_round = cb[p].round;
    pr.halt_round = halt_round[p];
    pr.final_x = alg.main_x(st[p]);
    if constexpr (kReal) {
      out.fdec.push_back(cb[p].fvalue);
      out.fx.push_back(st[p].x);
    }
    if (cb[p].round >= 0) ++nd;
    dig += proc_digest(p, pr.decision, pr.decision_round, pr.halt_round, pr.final_x);
  }
  S.digest = dig;
  S.n_decided = (uint16_t)nd;
}

static int validate(const psg_config* c, std::string& err) {
  if (!c) { err = "null config"; return PSG_EINVAL; }
  if (c->n < 1 || c->n > PSG_MAX_N) { err = "n out of range"; return PSG_EINVAL; }
  if (c->rounds < 1 || c->rounds > PSG_MAX_ROUNDS) { err = "rounds out of range"; return PSG_EINVAL; }
  if (c->alg < PSG_ALG_OTR || c->alg > PSG_ALG_EPSILON) { err = "unknown alg"; return PSG_EINVAL; }
  if (c->alg == PSG_ALG_KSET_ES && (c->param < 0 || c->param2 < 1)) { err = "KSetEarlyStopping needs t >= 0, k >= 1"; return PSG_EINVAL; }
  if (c->alg == PSG_ALG_EPSILON && (c->param < 1 || !(c->real_param > 0.0))) { err = "EpsilonConsensus needs f >= 1, epsilon > 0"; return PSG_EINVAL; }
  if (c->alg != PSG_ALG_BENOR && c->alg != PSG_ALG_EPSILON && c->value_range < 1) { err = "value_range < 1"; return PSG_EINVAL; }
  return 0;
}

static void run_one(const psg_config& cfg, uint64_t inst, const int32_t* init, int spec_mode, const ExplicitHO* eho,
                    InstOut& out, bool trace, const double* init_real = nullptr) {
  switch (cfg.alg) {
    case PSG_ALG_EPSILON: {
      Epsilon a{cfg.n, cfg.param, cfg.variant, cfg.real_param};
      run_engine(a, cfg, inst, init, spec_mode, eho, out, trace, init_real);
      break;
    }
    case PSG_ALG_OTR: { Otr a{cfg.n, cfg.param, cfg.variant}; run_engine(a, cfg, inst, init, spec_mode, eho, out, trace); break; }
    case PSG_ALG_LAST_VOTING: { LV a{cfg.n, cfg.variant, cfg.tiebreak}; run_engine(a, cfg, inst, init, spec_mode, eho, out, trace); break; }
    case PSG_ALG_FLOODMIN: { FloodMin a{cfg.n, cfg.param, cfg.variant}; run_engine(a, cfg, inst, init, spec_mode, eho, out, trace); break; }
    case PSG_ALG_KSET: { KSet a{cfg.n, cfg.param, cfg.variant, cfg.tiebreak}; run_engine(a, cfg, inst, init, spec_mode, eho, out, trace); break; }
    case PSG_ALG_BENOR: { BenOr a{cfg.n, cfg.variant}; run_engine(a, cfg, inst, init, spec_mode, eho, out, trace); break; }
    case PSG_ALG_OTR2: { Otr2 a; a.n = cfg.n; a.afterDecision = cfg.param; a.variant = cfg.variant; run_engine(a, cfg, inst, init, spec_mode, eho, out, trace); break; }
    case PSG_ALG_SLV: { SLV a{cfg.n, cfg.variant, cfg.tiebreak}; run_engine(a, cfg, inst, init, spec_mode, eho, out, trace); break; }
    case PSG_ALG_KSET_ES: { KSetES a{cfg.n, cfg.param, cfg.param2, cfg.variant}; run_engine(a, cfg, inst, init, spec_mode, eho, out, trace); break; }
  }
}

/* ------------------------------------------------------------------ */
/* Spec-program interpreter (CPU reference of psg_spec_vm.hip)          */
/* ------------------------------------------------------------------ */
/* Executes the bytecode of include/psg.h scalar-wise: lane-form process
 * quantifiers are plain loops over pids (the lane form is only the device's
 * evaluation strategy), V.exists over Int visits the same finitized candidate
 * set (distinct values of the compared fields / expressions, +-1, MIN, MAX). */
struct CpuVm {
  const psg_spec_program& P;
  const int32_t *cur, *old, *init;
  int n, r;
  int32_t var[16] = {0};
  int err = 0;

  int32_t field(int f, int tag, int32_t p) const {
    if (p < 0 || p >= n || f < 0 || f >= F_NFIELDS) return 0;
    const int32_t* t = tag == T_CUR ? cur : (tag == T_OLD ? old : init);
    return t[f * n + p];
  }
  static int32_t binop(int op, int32_t x, int32_t y) {
    switch (op) {
      case PSG_OP_AND: return x != 0 && y != 0;
      case PSG_OP_OR: return x != 0 || y != 0;
      case PSG_OP_IMPL: return x == 0 || y != 0;
      case PSG_OP_EQ: return x == y;
      case PSG_OP_NE: return x != y;
      case PSG_OP_LT: return x < y;
      case PSG_OP_LE: return x <= y;
      case PSG_OP_GT: return x > y;
      case PSG_OP_GE: return x >= y;
      case PSG_OP_ADD: return (int32_t)((uint32_t)x + (uint32_t)y);
      case PSG_OP_SUB: return (int32_t)((uint32_t)x - (uint32_t)y);
      case PSG_OP_MUL: return (int32_t)((uint32_t)x * (uint32_t)y);
      case PSG_OP_DIV: return y == 0 ? 0 : (x == INT32_MIN && y == -1) ? x : x / y;
      default: return (y == 0 || y == -1) ? 0 : x % y;
    }
  }
  /* Run code from pc with the given stack until HALT (returns top) or until the
   * QEND that closes the current quantifier body (returns the body value and the
   * pc of that QEND through *endpc). */
  int32_t run(int pc, std::vector<int32_t>& st, int* endpc) {
    const int32_t* code = P.code;
    while (pc < P.n_words) {
      const int32_t w = code[pc];
      const int op = w & 0xff, a = (w >> 8) & 0xff, b = w >> 16;
      ++pc;
      switch (op) {
        case PSG_OP_HALT: return st.empty() ? 0 : st.back();
        case PSG_OP_IMM: st.push_back(b); break;
        case PSG_OP_IMM32: st.push_back(code[pc++]); break;
        case PSG_OP_N: st.push_back(n); break;
        case PSG_OP_R: st.push_back(r); break;
        case PSG_OP_COORD: st.push_back((r / 4) % n); break;
        case PSG_OP_VAR: st.push_back(var[a]); break;
        case PSG_OP_FIELD: { int32_t p = st.back(); st.back() = field(a, b, p); break; }
        case PSG_OP_NOT: st.back() = st.back() == 0; break;
        case PSG_OP_NEG: st.back() = (int32_t)(0u - (uint32_t)st.back()); break;
        case PSG_OP_ISDEF: st.back() = st.back() != INT32_MIN; break;
        case PSG_OP_BIND: var[a] = st.back(); st.pop_back(); break;
        case PSG_OP_QEND: if (endpc) *endpc = pc - 1; return st.empty() ? 0 : st.back();
        case PSG_OP_QBEGIN: {
          const int end = code[pc++];
          std::vector<int64_t> cands;
          if (a == PSG_Q_EXISTS_VI) {
            const int32_t desc = code[pc++];
            const int nexpr = desc & 0xffff, nfs = (desc >> 16) & 0xffff;
            std::set<int32_t> bases;
            for (int e = 0; e < nexpr; ++e) { bases.insert(st.back()); st.pop_back(); }
            for (int f = 0; f < nfs; ++f) {
              const int32_t fw = code[pc++];
              for (int p = 0; p < n; ++p) bases.insert(field(fw & 0xff, (fw >> 8) & 0xff, p));
            }
            for (int32_t v : bases)
              for (int d = -1; d <= 1; ++d) cands.push_back((int32_t)((uint32_t)v + (uint32_t)d));
            cands.push_back(INT32_MIN);
            cands.push_back(INT32_MAX);
          } else if (a == PSG_Q_EXISTS_VB) {
            cands = {0, 1};
          } else {
            for (int p = 0; p < n; ++p) cands.push_back(p);
          }
          const bool forall = a == PSG_Q_FORALL_P || a == PSG_Q_FORALL_PL;
          const bool count = a == PSG_Q_COUNT_P || a == PSG_Q_COUNT_PL;
          int32_t acc = forall ? 1 : 0;
          for (int64_t cv : cands) {
            var[b] = (int32_t)cv;
            std::vector<int32_t> sub;
            int e = -1;
            const int32_t res = run(pc, sub, &e);
            if (e != end) { err = 1; return 0; }
            if (count) acc += res != 0;
            else if (forall) { if (res == 0) { acc = 0; break; } }
            else if (res != 0) { acc = 1; break; }
          }
          st.push_back(acc);
          pc = end + 1;
          break;
        }
        default: {
          if (op >= PSG_OP_AND && op <= PSG_OP_MOD) {
            int32_t y = st.back(); st.pop_back();
            st.back() = binop(op, st.back(), y);
          } else {
            err = 1;
            return 0;
          }
        }
      }
    }
    err = 1;
    return 0;
  }
  int32_t eval(int pc) {
    std::vector<int32_t> st;
    return run(pc, st, nullptr);
  }
};

} // namespace orc

/* ------------------------------------------------------------------ */
/* C ABI for tests / bench cpu_baseline (ctypes)                       */
/* ------------------------------------------------------------------ */
extern "C" {

static thread_local std::string g_oracle_err;

const char* oracle_last_error(void) { return g_oracle_err.c_str(); }

void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) { orc::philox4x32_10(ctr, key, out); }

/* Otr2.scala:32-36's ensuring clause on every mmor: on (1) for the pin tests, off (0, the
 * default) otherwise */
void oracle_set_mmor_check(int32_t on) { orc::g_mmor_check = on ? 1 : 0; }

/* mmor calls and violations of Otr2.scala:32-36's ensuring clause since the last reset */
void oracle_mmor_ensuring_stats(uint64_t* calls, uint64_t* failures, int32_t reset) {
  if (calls) *calls = orc::g_mmor_calls.load();
  if (failures) *failures = orc::g_mmor_ensuring_failures.load();
  if (reset) {
    orc::g_mmor_calls = 0;
    orc::g_mmor_ensuring_failures = 0;
  }
}

int oracle_java_first_boolean(int64_t seed) { return orc::java_random_first_boolean((uint64_t)seed) ? 1 : 0; }

uint32_t oracle_scala_improve(uint32_t h) { return orc::scala_improve(h); }

/* Scala Map iteration order of keys inserted in the given order. */
int oracle_scala_map_order(const int32_t* keys, int32_t m, int32_t tiebreak, int32_t* out) {
  std::vector<int> ins(keys, keys + m);
  std::vector<int> o = orc::scala_map_order(ins, tiebreak);
  for (int i = 0; i < m; ++i) out[i] = o[i];
  return 0;
}

/* HO mask of (inst, round k, pid p), n <= 64 only (word 0). */
uint64_t oracle_ho_mask(const psg_config* cfg, uint64_t inst, int32_t k, int32_t p) {
  orc::Schedule s(*cfg, inst);
  orc::Bits b = s.ho(k, p);
  uint64_t m = 0;
  for (int q = 0; q < cfg->n && q < 64; ++q) if (b.test(q)) m |= 1ULL << q;
  return m;
}

int32_t oracle_init_value(const psg_config* cfg, uint64_t inst, int32_t p) {
  orc::Schedule s(*cfg, inst);
  return s.init_value(p);
}

int32_t oracle_crash_round(const psg_config* cfg, uint64_t inst, int32_t p) {
  orc::Schedule s(*cfg, inst);
  return s.crash_round[p];
}

/* Run instances [inst_begin, inst_begin+count) (or the explicit ids list) on
 * `threads` host threads. init: optional [count][n]; per_inst/recs optional.
 * spec_mode: 0 hand-lowered, 1 Formula interpreter, 2 both (returns -EIO on
 * any disagreement). */
static int run_impl(const psg_config* cfg, uint64_t inst_begin, uint64_t count, const uint64_t* ids,
                    const int32_t* init, const double* init_real, psg_summary* out, psg_instance_summary* per_inst,
                    psg_process_record* recs, double* fdec, double* fx, int32_t threads, int32_t spec_mode,
                    const uint64_t* sched_ho = nullptr, const int32_t* sched_crash = nullptr);

int oracle_run(const psg_config* cfg, uint64_t inst_begin, uint64_t count, const uint64_t* ids,
               const int32_t* init, psg_summary* out, psg_instance_summary* per_inst,
               psg_process_record* recs, int32_t threads, int32_t spec_mode) {
  return run_impl(cfg, inst_begin, count, ids, init, nullptr, out, per_inst, recs, nullptr, nullptr, threads,
                  spec_mode);
}

/* Real-valued algorithms: Double initial values (nullable = seeded) and the Double
 * decision / final x of every process ([count][n] each, nullable). */
int oracle_run_real(const psg_config* cfg, uint64_t inst_begin, uint64_t count, const uint64_t* ids,
                    const double* init, psg_summary* out, psg_instance_summary* per_inst,
                    psg_process_record* recs, double* fdec, double* fx, int32_t threads) {
  return run_impl(cfg, inst_begin, count, ids, nullptr, init, out, per_inst, recs, fdec, fx, threads, 0);
}

static int run_impl(const psg_config* cfg, uint64_t inst_begin, uint64_t count, const uint64_t* ids,
                    const int32_t* init, const double* init_real, psg_summary* out, psg_instance_summary* per_inst,
                    psg_process_record* recs, double* fdec, double* fx, int32_t threads, int32_t spec_mode,
                    const uint64_t* sched_ho, const int32_t* sched_crash) {
  std::string err;
  int rc = orc::validate(cfg, err);
  if (rc) { g_oracle_err = err; return rc; }
  if (threads < 1) threads = 1;
  const int n = cfg->n, R = cfg->rounds, nck = orc::n_checks_of(cfg->alg);
  std::vector<psg_summary> part(threads);
  std::vector<std::string> errs(threads);
  std::atomic<int> bad{0};
  auto worker = [&](int t) {
    psg_summary& s = part[t];
    std::memset(&s, 0, sizeof(s));
    uint64_t lo = count * (uint64_t)t / threads, hi = count * (uint64_t)(t + 1) / threads;
    for (uint64_t i = lo; i < hi; ++i) {
      uint64_t inst = ids ? ids[i] : inst_begin + i;
      orc::InstOut o;
      orc::ExplicitHO e;
      if (sched_ho) {
        const int W = (n + 63) / 64;
        e.ho = sched_ho + i * (uint64_t)R * (uint64_t)n * (uint64_t)W;
        e.W = W;
        e.crash = sched_crash ? sched_crash + i * (uint64_t)n : nullptr;
        e.legacy = false;
      }
      orc::run_one(*cfg, inst, init ? init + i * (uint64_t)n : nullptr, spec_mode, sched_ho ? &e : nullptr, o, false,
                   init_real ? init_real + i * (uint64_t)n : nullptr);
      if (o.mismatch) { bad = 1; errs[t] = o.msg; }
      s.instances += 1;
      s.process_rounds += (int64_t)n * R;
      {  // rounds each process took a step in (Round.scala:42-55: halted after its exit round)
        int32_t live = 0;
        for (int p = 0; p < n; ++p) {
          const int32_t st = o.rec[p].halt_round >= 0 ? o.rec[p].halt_round + 1 : R;
          s.active_process_rounds += st;
          live = std::max(live, st);
        }
        s.live_instance_rounds += live;
      }
      for (int c = 0; c < nck; ++c) if (o.sum.first_fail[c] != PSG_NEVER) s.fail_count[c] += 1;
      s.decided_processes += o.sum.n_decided;
      s.digest = (int64_t)((uint64_t)s.digest + o.sum.digest);
      s.term_hist[o.sum.term_round == PSG_NEVER ? R + 1 : o.sum.term_round] += 1;
      if (per_inst) per_inst[i] = o.sum;
      if (recs) std::memcpy(recs + i * (uint64_t)n, o.rec.data(), sizeof(psg_process_record) * n);
      if (fdec && !o.fdec.empty()) std::memcpy(fdec + i * (uint64_t)n, o.fdec.data(), sizeof(double) * n);
      if (fx && !o.fx.empty()) std::memcpy(fx + i * (uint64_t)n, o.fx.data(), sizeof(double) * n);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  psg_summary total;
  std::memset(&total, 0, sizeof(total));
  for (auto& s : part) {
    total.instances += s.instances;
    total.process_rounds += s.process_rounds;
    total.active_process_rounds += s.active_process_rounds;
    total.live_instance_rounds += s.live_instance_rounds;
    for (int c = 0; c < PSG_MAX_CHECKS; ++c) total.fail_count[c] += s.fail_count[c];
    total.decided_processes += s.decided_processes;
    total.digest = (int64_t)((uint64_t)total.digest + (uint64_t)s.digest);
    for (int c = 0; c < PSG_MAX_ROUNDS + 2; ++c) total.term_hist[c] += s.term_hist[c];
  }
  if (out) *out = total;
  if (bad) {
    for (auto& e : errs) if (!e.empty()) { g_oracle_err = e; break; }
    return PSG_EIO;
  }
  return 0;
}

/* Spec-program trace of instances [inst_begin, inst_begin+count) (init: optional
 * [count][n] initial values, else seeded): out receives
 * count x (R+1) x F x n int32 (the device trace layout; Option None = INT32_MIN). */
int oracle_trace(const psg_config* cfg, uint64_t inst_begin, uint64_t count, const int32_t* init, int32_t* out,
                 int32_t threads) {
  std::string err;
  int rc = orc::validate(cfg, err);
  if (rc) { g_oracle_err = err; return rc; }
  if (threads < 1) threads = 1;
  const uint64_t per = (uint64_t)(cfg->rounds + 1) * orc::F_NFIELDS * (uint64_t)cfg->n;
  auto worker = [&](int t) {
    uint64_t lo = count * (uint64_t)t / threads, hi = count * (uint64_t)(t + 1) / threads;
    for (uint64_t i = lo; i < hi; ++i) {
      orc::InstOut o;
      std::vector<int32_t> tr;
      o.vtrace = &tr;
      orc::run_one(*cfg, inst_begin + i, init ? init + i * (uint64_t)cfg->n : nullptr, 0, nullptr, o, false);
      std::memcpy(out + i * per, tr.data(), sizeof(int32_t) * per);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  return 0;
}

/* oracle_trace plus the checker's verdict at every check point: bits [count][R+1]
 * (bit s = slot s holds at that check point, bit 15 = Termination holds), from the
 * hand-lowered evaluator (spec_mode 0), the Formula interpreter (1) or both, required
 * equal (2). trace (nullable) as oracle_trace. Test infrastructure: the per-check-point
 * view the reference-model pins (tests/test_reference_otr_spec.py) compare against. */
int oracle_trace_checks(const psg_config* cfg, uint64_t inst_begin, uint64_t count, const int32_t* init,
                        int32_t* trace, uint16_t* bits, int32_t threads, int32_t spec_mode) {
  std::string err;
  int rc = orc::validate(cfg, err);
  if (rc) { g_oracle_err = err; return rc; }
  if (threads < 1) threads = 1;
  const uint64_t per = (uint64_t)(cfg->rounds + 1) * orc::F_NFIELDS * (uint64_t)cfg->n;
  std::vector<std::string> errs(threads);
  auto worker = [&](int t) {
    uint64_t lo = count * (uint64_t)t / threads, hi = count * (uint64_t)(t + 1) / threads;
    for (uint64_t i = lo; i < hi; ++i) {
      orc::InstOut o;
      std::vector<int32_t> tr;
      std::vector<uint16_t> ck;
      o.vtrace = &tr;
      o.ckbits = &ck;
      orc::run_one(*cfg, inst_begin + i, init ? init + i * (uint64_t)cfg->n : nullptr, spec_mode, nullptr, o, false);
      if (o.mismatch && errs[t].empty()) errs[t] = o.msg;
      if (trace) std::memcpy(trace + i * per, tr.data(), sizeof(int32_t) * per);
      std::memcpy(bits + i * (uint64_t)(cfg->rounds + 1), ck.data(), sizeof(uint16_t) * ck.size());
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  for (auto& e : errs)
    if (!e.empty()) { g_oracle_err = e; return PSG_EIO; }
  return 0;
}

/* Evaluate a Spec program over traces (count x (R+1) x F x n): first_fail
 * [count][PSG_MAX_CHECKS] and term_round [count] in psg_instance_summary terms. */
int oracle_vm_run(const psg_spec_program* prog, const int32_t* trace, uint64_t count, int32_t n, int32_t R,
                  uint8_t* first_fail, uint8_t* term_round) {
  const uint64_t row = (uint64_t)orc::F_NFIELDS * (uint64_t)n;
  for (uint64_t i = 0; i < count; ++i) {
    const int32_t* base = trace + i * (uint64_t)(R + 1) * row;
    uint8_t* ff = first_fail + i * PSG_MAX_CHECKS;
    for (int s = 0; s < PSG_MAX_CHECKS; ++s) ff[s] = PSG_NEVER;
    term_round[i] = PSG_NEVER;
    for (int c = 0; c <= R; ++c) {
      orc::CpuVm vm{*prog, base + (uint64_t)c * row, base + (uint64_t)(c > 0 ? c - 1 : 0) * row, base, n, c};
      for (int s = 0; s < prog->n_slots; ++s) {
        const bool vac = c == 0 && (prog->slot_flags[s] & PSG_SPEC_RELATIONAL);
        if (!vac && vm.eval(prog->slot_entry[s]) == 0 && ff[s] == PSG_NEVER) ff[s] = (uint8_t)c;
      }
      if (prog->term_entry >= 0 && term_round[i] == PSG_NEVER && vm.eval(prog->term_entry) != 0)
        term_round[i] = (uint8_t)c;
      if (vm.err) { g_oracle_err = "bad spec program"; return PSG_EINVAL; }
    }
  }
  return 0;
}

/* Single instance with an explicit HO schedule ho[R][n] (n <= 64) and init
 * values; trace receives (R+1) * 2n int64 (x then decided per check point). */
/* Explicit HO schedule for a real-valued algorithm: Double init [n]; fdec / fx [n]. */
int oracle_run_explicit_real(const psg_config* cfg, const double* init, const uint64_t* ho, psg_instance_summary* sum,
                             psg_process_record* recs, double* fdec, double* fx) {
  std::string err;
  int rc = orc::validate(cfg, err);
  if (rc) { g_oracle_err = err; return rc; }
  if (cfg->n > 64) { g_oracle_err = "explicit HO needs n <= 64"; return PSG_EINVAL; }
  orc::ExplicitHO e{ho};
  orc::InstOut o;
  orc::run_one(*cfg, 0, nullptr, 0, &e, o, false, init);
  if (sum) *sum = o.sum;
  if (recs) std::memcpy(recs, o.rec.data(), sizeof(psg_process_record) * cfg->n);
  if (fdec && !o.fdec.empty()) std::memcpy(fdec, o.fdec.data(), sizeof(double) * cfg->n);
  if (fx && !o.fx.empty()) std::memcpy(fx, o.fx.data(), sizeof(double) * cfg->n);
  return 0;
}

int oracle_run_explicit(const psg_config* cfg, const int32_t* init, const uint64_t* ho, psg_instance_summary* sum,
                        psg_process_record* recs, int64_t* trace, int32_t spec_mode) {
  std::string err;
  int rc = orc::validate(cfg, err);
  if (rc) { g_oracle_err = err; return rc; }
  if (cfg->n > 64) { g_oracle_err = "explicit HO needs n <= 64"; return PSG_EINVAL; }
  orc::ExplicitHO e{ho};
  orc::InstOut o;
  orc::run_one(*cfg, 0, init, spec_mode, &e, o, trace != nullptr);
  if (sum) *sum = o.sum;
  if (recs) std::memcpy(recs, o.rec.data(), sizeof(psg_process_record) * cfg->n);
  if (trace) std::memcpy(trace, o.trace.data(), sizeof(int64_t) * o.trace.size());
  if (o.mismatch) { g_oracle_err = o.msg; return PSG_EIO; }
  return 0;
}

/* Instances [inst_begin, inst_begin+count) under an explicit schedule
 * ho [count][R][n][W] (crash [count][n] nullable), psg_load_schedule semantics.
 * init: [count][n] int32 (nullable = seeded); init_real likewise for Doubles. */
int oracle_run_schedule(const psg_config* cfg, uint64_t inst_begin, uint64_t count, const int32_t* init,
                        const double* init_real, const uint64_t* ho, const int32_t* crash, psg_summary* out,
                        psg_instance_summary* per_inst, psg_process_record* recs, double* fdec, double* fx,
                        int32_t threads) {
  if (!ho && count) { g_oracle_err = "null schedule"; return PSG_EINVAL; }
  return run_impl(cfg, inst_begin, count, nullptr, init, init_real, out, per_inst, recs, fdec, fx, threads, 0, ho,
                  crash);
}

/* The seeded schedule of instances [inst_begin, inst_begin+count) in the explicit
 * layout (psg_materialize_schedule): ho [count][R][n][W], crash [count][n] (nullable). */
int oracle_materialize_schedule(const psg_config* cfg, uint64_t inst_begin, uint64_t count, uint64_t* ho,
                                int32_t* crash) {
  std::string err;
  int rc = orc::validate(cfg, err);
  if (rc) { g_oracle_err = err; return rc; }
  const int n = cfg->n, R = cfg->rounds, W = (n + 63) / 64;
  for (uint64_t i = 0; i < count; ++i) {
    orc::Schedule s(*cfg, inst_begin + i);
    if (crash) for (int p = 0; p < n; ++p) crash[i * (uint64_t)n + p] = s.crash_round[p];
    for (int k = 0; k < R; ++k)
      for (int p = 0; p < n; ++p) {
        orc::Bits b = s.ho(k, p);
        uint64_t* q = ho + ((i * (uint64_t)R + (uint64_t)k) * (uint64_t)n + (uint64_t)p) * (uint64_t)W;
        for (int w = 0; w < W; ++w) q[w] = 0;
        for (int x = 0; x < n; ++x) if (b.test(x)) q[x >> 6] |= 1ULL << (x & 63);
      }
  }
  return 0;
}

} // extern "C"
