// psg_spec_gen.cpp — psg_spec_compile_native: a Spec given as Formula text lowered to native
// gfx950 code in-process. It is the only Spec generator: the C ABI (and so the JVM,
// integration/scala/GpuSpec.scala) calls it directly, round_amd/formula.py compile_native
// writes a DSL Spec as Formula text and calls it. The code object is compiled with hiprtc (no
// process is started) and cached by a hash of the toolchain, the source and the kernel
// headers. Host C++ only.
//
// Reference: the Spec being lowered is a psync.Spec (psync/Specs.scala:8-16) whose Formula
// trees (psync/formula/Formula.scala:5-585) arrive as text; the rewrites below are exact
// for every input (equality pins, count guards, breakpoint finitization, tuple quantifiers,
// memoized init membership, common closed subformulas, split foralls; DESIGN.md §5;
// psg_spec_rewrite_text exposes the tree rewrites to the tests).
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <fstream>
#include <functional>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

#include "psg_spec_ir.hpp"

namespace psgspec {
namespace {

// ------------------------------------------------------------------ tree helpers
bool is_var(const Tree& T, int e, int uid) { return T.nodes[e].k == VAR && T.nodes[e].uid == uid; }

// Generator options (experiments and profiling builds), comma-separated: "nosym" (no
// symmetric-check-point lowering), "sym" (that lowering also where it is off by default: fused
// LastVoting modules), "nosplit" (no split foralls / hoisted conjuncts),
// "D<NAME>=<VALUE>" (a #define at the top of the module, e.g. DPSG_PHASE_TIMERS=1). They change
// the source, hence the cache key. Per thread: psg_spec_set_options sets the calling thread's
// string, otherwise the environment variable PSG_SPEC_OPTIONS is read; every entry point parses
// them into its own thread's GenOptions, so concurrent callers (JVM threads) never share state.
struct GenOptions {
  bool symmetric = true, split = true, frozen = true;
  bool sym_explicit = false;  // "sym" / "nosym" given: no per-algorithm default
  std::vector<std::string> defines;
};
thread_local GenOptions g_opts;        // this thread's options for the generation in progress
thread_local std::string t_options;     // psg_spec_set_options (this thread)
thread_local bool t_options_set = false;

GenOptions parse_options(const std::string& t) {
  GenOptions o;
  size_t i = 0;
  while (i <= t.size()) {
    const size_t j = t.find(',', i);
    const std::string tok = t.substr(i, j == std::string::npos ? std::string::npos : j - i);
    if (tok == "nosym" || tok == "sym") {
      o.symmetric = tok == "sym";
      o.sym_explicit = true;
    }
    else if (tok == "nosplit") o.split = false;
    else if (tok == "nofrozen") o.frozen = false;
    else if (tok.size() > 1 && tok[0] == 'D') {
      const size_t eq = tok.find('=');
      const std::string name = tok.substr(1, eq == std::string::npos ? std::string::npos : eq - 1);
      const std::string value = eq == std::string::npos ? std::string() : tok.substr(eq + 1);
      if (name.empty() || name.find_first_not_of("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789_") !=
                              std::string::npos)
        throw SpecError("PSG_SPEC_OPTIONS: bad define " + tok);
      // every knob is an integer: the value never carries source text (a newline would paste
      // arbitrary code into the generated module)
      if (value.find_first_not_of("0123456789") != std::string::npos && !(value.size() > 1 && value[0] == '-' &&
                                                                          value.find_first_not_of("0123456789", 1) == std::string::npos))
        throw SpecError("PSG_SPEC_OPTIONS: define " + name + " takes an integer value");
#ifndef PSG_PROBE_BUILD
      // allow-list: the profiling switch and the knobs whose settings are exact alternatives
      // (occupancy targets, instance-queue chunking, instruction-selection forms); anything
      // else (PSG_MAX_CHECKS, PSG_FUSED_MODULE, probe switches) would change what a product
      // module computes
      static const char* const kKnobs[] = {"PSG_PHASE_TIMERS", "PSG_PHILOX_OPAQUE_KEYS", "PSG_PHILOX_MAD64",
                                           "PSG_XSHFL_MASK",   "PSG_QUEUE_CHUNK",        "PSG_QUEUE_CHUNK_WIDE",   "PSG_QUEUE_CHUNK_LANE",
                                           "PSG_MAJ_BITVOTE",  "PSG_BO_FLAGS_DPP"};
      bool ok = name.size() > 8 && name.compare(0, 4, "PSG_") == 0 && name.compare(name.size() - 4, 4, "_WPE") == 0;
      for (const char* k : kKnobs) ok = ok || name == k;
      if (!ok) throw SpecError("PSG_SPEC_OPTIONS: " + name + " is not a generator knob (or needs a probe build)");
#endif
      o.defines.push_back(tok.substr(1));
    } else if (!tok.empty()) throw SpecError("PSG_SPEC_OPTIONS: unknown option " + tok);
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return o;
}
void load_options() {
  if (t_options_set) {
    g_opts = parse_options(t_options);
  } else {
    const char* e = std::getenv("PSG_SPEC_OPTIONS");
    g_opts = parse_options(e ? e : "");
  }
}

// Python's `is` on the trees formula.py from_text builds: a variable is one object per binder
bool same_obj(const Tree& T, int a, int b) {
  return a == b || (T.nodes[a].k == VAR && T.nodes[b].k == VAR && T.nodes[a].uid == T.nodes[b].uid);
}

std::set<int> free_of(const Tree& T, int e) {
  std::set<int> bound, out;
  T.free_vars(e, bound, out);
  return out;
}

void conjuncts(const Tree& T, int e, std::vector<int>& out) {
  const Node& n = T.nodes[e];
  if (n.k == BIN && n.op == PSG_OP_AND) {
    conjuncts(T, n.a, out);
    conjuncts(T, n.b, out);
  } else {
    out.push_back(e);
  }
}

bool expensive(const Tree& T, int e) {  // a quantifier or a set membership inside
  std::vector<int> w;
  T.walk(e, w);
  for (int x : w)
    if (T.nodes[x].k == QUANT || T.nodes[x].k == CONTAINS) return true;
  return false;
}

int and_all(Tree& T, const std::vector<int>& xs) {
  int out = xs[0];
  for (size_t k = 1; k < xs.size(); ++k) out = T.bin(PSG_OP_AND, out, xs[k]);
  return out;
}

// P.exists(j => init(j.f) == t) with t free of j: (f, t), else (-1, -1)
std::pair<int, int> init_member(const Tree& T, int q) {
  const Node& Q = T.nodes[q];
  const Node& b = T.nodes[Q.a];
  if (Q.qk != QEXISTS || b.k != BIN || b.op != PSG_OP_EQ) return {-1, -1};
  const int pairs[2][2] = {{b.a, b.b}, {b.b, b.a}};
  for (auto& pr : pairs) {
    const Node& a = T.nodes[pr[0]];
    if (a.k == FIELD && a.tag == PSG_TAG_INIT && is_var(T, a.a, Q.uid)) {
      std::vector<int> w;
      T.walk(pr[1], w);
      bool uses = false;
      for (int x : w) uses = uses || is_var(T, x, Q.uid);
      if (!uses) return {a.f, pr[1]};
    }
  }
  return {-1, -1};
}

// Fields (field, tag) through which the body reads the quantified process, or false if the
// variable is used otherwise
bool tuple_fields(const Tree& T, int q, std::vector<std::pair<int, int>>& out) {
  const Node& Q = T.nodes[q];
  std::vector<int> w;
  T.walk(Q.a, w);
  bool as_field = false;
  for (int x : w) {
    const Node& f = T.nodes[x];
    if (f.k == FIELD && is_var(T, f.a, Q.uid)) {
      as_field = true;
      const std::pair<int, int> key{f.f, f.tag};
      if (std::find(out.begin(), out.end(), key) == out.end()) out.push_back(key);
    }
  }
  for (int x : w)
    if (is_var(T, x, Q.uid) && !as_field) return false;
  return out.size() <= 4;
}

// Structural key of node e, bound variables numbered by binding depth from e:
// two closed subformulas with equal keys are the same formula.
std::string skey_rec(const Tree& T, int e, std::map<int, int>& env) {
  const Node& n = T.nodes[e];
  switch (n.k) {
    case VAR: {
      auto it = env.find(n.uid);
      return it != env.end() ? "V" + std::to_string(it->second) : "free" + std::to_string(n.uid);
    }
    case LIT: return "L" + std::to_string(n.v);
    case NV: return "N";
    case RV: return "R";
    case COORDV: return "K";
    case FIELD: return "F(" + std::to_string(n.f) + "," + std::to_string(n.tag) + "," + skey_rec(T, n.a, env) + ")";
    case UN: return "U(" + std::to_string(n.op) + "," + skey_rec(T, n.a, env) + ")";
    case BIN:
      return "B(" + std::to_string(n.op) + "," + skey_rec(T, n.a, env) + "," + skey_rec(T, n.b, env) + ")";
    case QUANT:
    case CONTAINS: {
      const std::string pre = n.k == QUANT ? "Q(" + std::to_string(n.qk) + "," : "C(" + skey_rec(T, n.a, env) + ",";
      const bool had = env.count(n.uid) > 0;
      const int old = had ? env[n.uid] : 0;
      const int level = (int)env.size();  // binding depth
      env[n.uid] = level;
      const std::string body = skey_rec(T, n.k == QUANT ? n.a : n.b, env);
      if (had) env[n.uid] = old;
      else env.erase(n.uid);
      return pre + body + ")";
    }
  }
  throw SpecError("unsupported node");
}

// Does the body of process quantifier q read its variable only through current / old fields
// (no init field, no use as a pid)?
bool symmetric(const Tree& T, int q) {
  const int uid = T.nodes[q].uid;
  std::vector<int> w;
  T.walk(T.nodes[q].a, w);
  int nvar = 0, nfield = 0;
  for (int x : w) {
    const Node& n = T.nodes[x];
    if (n.k == VAR && n.uid == uid) {
      ++nvar;
    } else if (n.k == FIELD && is_var(T, n.a, uid)) {
      if (n.tag == PSG_TAG_INIT) return false;
      ++nfield;
    }
  }
  return nvar == nfield;
}

// Conjuncts A of forall(j => A && .. ==> B) / exists, count(j => A && .. && B) that read only j
//: the processes where one fails contribute nothing
std::vector<int> tuple_guard(const Tree& T, int q) {
  const Node& Q = T.nodes[q];
  std::vector<int> cs, out;
  if (Q.qk == QFORALL) {
    const Node& b = T.nodes[Q.a];
    if (!(b.k == BIN && b.op == PSG_OP_IMPL)) return out;
    conjuncts(T, b.a, cs);
  } else {
    conjuncts(T, Q.a, cs);
  }
  for (int c : cs) {
    const std::set<int> fv = free_of(T, c);
    if (fv.size() == 1 && fv.count(Q.uid) && !expensive(T, c)) out.push_back(c);
  }
  return out;
}

// breakpoint offsets (bit d+1: b = e + d) of an atom `t OP e`, t the V.exists variable
int bp_shift(int op) {
  switch (op) {
    case PSG_OP_LE: case PSG_OP_GT: return 2;
    case PSG_OP_LT: case PSG_OP_GE: return 1;
    case PSG_OP_EQ: case PSG_OP_NE: return 3;
  }
  return 0;
}
int flip_op(int op) {
  switch (op) {
    case PSG_OP_LE: return PSG_OP_GE;
    case PSG_OP_GE: return PSG_OP_LE;
    case PSG_OP_LT: return PSG_OP_GT;
    case PSG_OP_GT: return PSG_OP_LT;
  }
  return op;
}

std::vector<int> breakpoint_shifts(const Tree& T, int q, const std::vector<int>& exprs,
                                   const std::vector<std::pair<int, int>>& fsets) {
  const int uid = T.nodes[q].uid;
  std::vector<int> es(exprs.size(), 0), fm(fsets.size(), 0);
  std::vector<int> w;
  T.walk(T.nodes[q].a, w);
  for (int x : w) {
    const Node& b = T.nodes[x];
    if (b.k != BIN || !bp_shift(b.op)) continue;
    const int sides[2][3] = {{b.a, b.b, b.op}, {b.b, b.a, flip_op(b.op)}};
    for (auto& sd : sides) {
      if (!is_var(T, sd[0], uid)) continue;
      const Node& t = T.nodes[sd[1]];
      if (t.k == FIELD) {
        for (size_t k = 0; k < fsets.size(); ++k)
          if (fsets[k] == std::make_pair(t.f, t.tag)) fm[k] |= bp_shift(sd[2]);
      } else {
        bool hit = false;
        for (size_t k = 0; k < exprs.size(); ++k)
          if (same_obj(T, exprs[k], sd[1])) {
            es[k] |= bp_shift(sd[2]);
            hit = true;
          }
        if (!hit) return std::vector<int>(exprs.size() + fsets.size(), 7);  // unmatched: every offset
      }
    }
  }
  std::vector<int> out = es;
  out.insert(out.end(), fm.begin(), fm.end());
  for (int& m : out) m = m ? m : 7;
  return out;
}

bool eq_only(const Tree& T, int q) {
  const int uid = T.nodes[q].uid;
  std::vector<int> w;
  T.walk(T.nodes[q].a, w);
  for (int x : w) {
    const Node& b = T.nodes[x];
    if (b.k == BIN && b.op >= PSG_OP_LT && b.op <= PSG_OP_GE && (is_var(T, b.a, uid) || is_var(T, b.b, uid)))
      return false;
  }
  return true;
}

struct Pins {
  int forall = -1;
  std::vector<std::pair<int, int>> list;  // (cond or -1, term)
};

bool intersects(const std::set<int>& a, const std::set<int>& b) {
  for (int x : a)
    if (b.count(x)) return true;
  return false;
}

// Equality pins of the V.exists variable uid in body
bool pins(const Tree& T, int body, int uid, const std::set<int>& banned, Pins& out) {
  std::vector<int> cs;
  conjuncts(T, body, cs);
  for (int c : cs) {
    const Node& C = T.nodes[c];
    if (C.k == QUANT && C.qk == QVINT) {
      std::set<int> b2 = banned;
      b2.insert(C.uid);
      if (pins(T, C.a, uid, b2, out)) return true;
      continue;
    }
    if (!(C.k == QUANT && C.qk == QFORALL)) continue;
    std::vector<int> ds;
    conjuncts(T, C.a, ds);
    std::vector<std::pair<int, int>> found;
    for (int d : ds) {
      const Node& D = T.nodes[d];
      int cond = -1, eq = d;
      if (D.k == BIN && D.op == PSG_OP_IMPL) {
        cond = D.a;
        eq = D.b;
      }
      if (cond >= 0) {
        const std::set<int> fc = free_of(T, cond);
        if (fc.count(uid) || intersects(fc, banned)) continue;
      }
      const Node& E = T.nodes[eq];
      if (!(E.k == BIN && E.op == PSG_OP_EQ)) continue;
      const int pairs[2][2] = {{E.a, E.b}, {E.b, E.a}};
      for (auto& pr : pairs) {
        const std::set<int> ft = free_of(T, pr[0]);
        if (is_var(T, pr[1], uid) && !ft.count(uid) && !intersects(ft, banned)) {
          found.emplace_back(cond, pr[0]);
          break;
        }
      }
    }
    if (!found.empty()) {
      out.forall = c;
      out.list = found;
      return true;
    }
  }
  return false;
}

struct CountGuard {
  int f = -1, tag = 0, thr = -1, op = 0;
};

// A conjunct `P.filter(i => i.f == v).size OP thr` (OP in >, >=, ==; thr uniform) of V.exists(v => body)
bool count_guard(const Tree& T, int q, CountGuard& g) {
  const int uid = T.nodes[q].uid;
  std::vector<int> cs;
  conjuncts(T, T.nodes[q].a, cs);
  for (int c : cs) {
    const Node& C = T.nodes[c];
    if (C.k != BIN || !(C.op == PSG_OP_GT || C.op == PSG_OP_GE || C.op == PSG_OP_EQ || C.op == PSG_OP_LT ||
                         C.op == PSG_OP_LE))
      continue;
    int cnt = C.a, thr = C.b, op = C.op;
    if (!(T.nodes[cnt].k == QUANT && T.nodes[cnt].qk == QCOUNT)) {
      cnt = C.b;
      thr = C.a;
      op = C.op == PSG_OP_LT ? PSG_OP_GT : C.op == PSG_OP_LE ? PSG_OP_GE : C.op == PSG_OP_GT ? PSG_OP_LT
         : C.op == PSG_OP_GE ? PSG_OP_LE : PSG_OP_EQ;
    }
    if (!(op == PSG_OP_GT || op == PSG_OP_GE || op == PSG_OP_EQ) ||
        !(T.nodes[cnt].k == QUANT && T.nodes[cnt].qk == QCOUNT))
      continue;
    std::vector<int> w;
    T.walk(thr, w);
    bool uniform = true;
    for (int x : w) {
      const Kind k = T.nodes[x].k;
      uniform = uniform && !(k == VAR || k == QUANT || k == FIELD || k == CONTAINS);
    }
    if (!uniform) continue;  // the threshold must be uniform (n, r, literals)
    const Node& B = T.nodes[T.nodes[cnt].a];
    if (!(B.k == BIN && B.op == PSG_OP_EQ)) continue;
    const int pairs[2][2] = {{B.a, B.b}, {B.b, B.a}};
    for (auto& pr : pairs) {
      const Node& fld = T.nodes[pr[0]];
      if (fld.k == FIELD && is_var(T, fld.a, T.nodes[cnt].uid) && is_var(T, pr[1], uid)) {
        g.f = fld.f;
        g.tag = fld.tag;
        g.thr = thr;
        g.op = op;
        return true;
      }
    }
  }
  return false;
}

// e reads a field of a process other than uid, or holds a quantifier / set membership
//
bool cross(const Tree& T, int e, int uid) {
  std::vector<int> w;
  T.walk(e, w);
  for (int x : w) {
    const Node& n = T.nodes[x];
    if (n.k == QUANT || n.k == CONTAINS) return true;
    if (n.k == FIELD && !is_var(T, n.a, uid)) return true;
  }
  return false;
}

// V.exists(v => A && B(v)) -> A && V.exists(v => B(v)) for the conjuncts A free of v, a conjunct
// P.forall(i => A && B) split into P.forall(A) && P.forall(B) first, A the conjuncts free of v
// doing cross-lane work (shared subformulas stay shared)
// the conjuncts of quantifier q's body, each P.forall(i => A && B) among them split into
// P.forall(A), P.forall(B): A the conjuncts free of q's variable (and doing cross-lane work,
// cross_only)
void split_conjuncts(Tree& T, int q, bool cross_only, std::vector<int>& cs) {
  const int uid = T.nodes[q].uid;
  std::vector<int> cs0;
  conjuncts(T, T.nodes[q].a, cs0);
  for (int c : cs0) {
    const Node C = T.nodes[c];
    if (g_opts.split && C.k == QUANT && C.qk == QFORALL) {
      std::vector<int> ds, dfr, dbd;
      conjuncts(T, C.a, ds);
      for (int d : ds) (!free_of(T, d).count(uid) && (!cross_only || cross(T, d, C.uid)) ? dfr : dbd).push_back(d);
      if (!dfr.empty() && !dbd.empty()) {
        const int a = and_all(T, dfr);
        cs.push_back(T.quant(QFORALL, C.uid, a));
        const int b = and_all(T, dbd);
        cs.push_back(T.quant(QFORALL, C.uid, b));
        continue;
      }
    }
    cs.push_back(c);
  }
}

// P.exists(j => A && B(j)) -> A && P.exists(j => B(j)), the same for P.forall (n >= 1), for the
// conjuncts A free of j
int proc_step(Tree& T, int q) {
  if (!g_opts.split) return q;
  const int uid = T.nodes[q].uid, qk = T.nodes[q].qk;
  std::vector<int> cs, fr, bd;
  split_conjuncts(T, q, false, cs);
  for (int c : cs) (free_of(T, c).count(uid) ? bd : fr).push_back(c);
  if (!fr.empty() && !bd.empty()) {
    std::vector<int> all = fr;
    all.push_back(T.quant(qk, uid, and_all(T, bd)));
    return and_all(T, all);
  }
  return q;
}

int vint_step(Tree& T, int q) {
  const int uid = T.nodes[q].uid;
  std::vector<int> cs, fr, bd;
  split_conjuncts(T, q, true, cs);
  for (int c : cs) (free_of(T, c).count(uid) ? bd : fr).push_back(c);
  if (!fr.empty() && !bd.empty()) {
    std::vector<int> all = fr;
    all.push_back(T.quant(QVINT, uid, and_all(T, bd)));
    return and_all(T, all);
  }
  return q;
}

int rewrite_vint(Tree& T, int e, std::map<int, int>& memo) {
  auto it = memo.find(e);
  if (it != memo.end()) return it->second;
  int out = e;
  const Node n = T.nodes[e];  // a copy: rewriting appends nodes
  if (n.k == QUANT) {
    const int b = rewrite_vint(T, n.a, memo);
    out = b == n.a ? e : T.quant(n.qk, n.uid, b);
    if (T.nodes[out].qk == QVINT) out = vint_step(T, out);
    else if (T.nodes[out].qk == QEXISTS || T.nodes[out].qk == QFORALL) out = proc_step(T, out);
  } else if (n.k == BIN) {
    const int x = rewrite_vint(T, n.a, memo);
    const int y = rewrite_vint(T, n.b, memo);
    out = (x == n.a && y == n.b) ? e : T.bin(n.op, x, y);
  } else if (n.k == UN) {
    const int x = rewrite_vint(T, n.a, memo);
    out = x == n.a ? e : T.un(n.op, x);
  } else if (n.k == CONTAINS) {
    const int b = rewrite_vint(T, n.b, memo);
    const int x = rewrite_vint(T, n.a, memo);
    if (!(b == n.b && x == n.a)) {
      Node c{CONTAINS};
      c.uid = n.uid;
      c.a = x;
      c.b = b;
      out = T.add(c);
    }
  }
  memo[e] = out;
  return out;
}

std::string c_int(int32_t v) { return v == INT32_MIN ? "(-2147483647 - 1)" : "((int32_t)" + std::to_string(v) + ")"; }
std::string S(int v) { return std::to_string(v); }

using Code = std::pair<std::string, bool>;  // (C++ expression, depends on the lane)

// ------------------------------------------------------------------ the generator
struct Gen {
  Tree& T;
  bool restrict_fields;
  std::set<int> fields_available;
  struct Name {
    std::string name;
    bool lane = false, own = false;
  };
  std::map<int, Name> names;
  int k = 0;
  std::set<int> fields, tags;
  int max_vi = 0;
  std::map<int, std::map<std::pair<int, int>, std::string>> tuples;
  std::vector<int> init_sets;
  std::map<std::string, std::string> cse;  // structural key of a closed subformula -> its hoisted value
  std::map<int, std::string> skeys;         // skey memo per node
  const std::string& skey(int e) {
    auto it = skeys.find(e);
    if (it != skeys.end()) return it->second;
    std::map<int, int> env;
    return skeys[e] = skey_rec(T, e, env);
  }
  // (field tuple, guard code or "") -> TupU / TupG name
  using TupKey = std::pair<std::vector<std::pair<int, int>>, std::string>;
  std::vector<std::pair<TupKey, std::string>> tup_sets;
  std::set<TupKey> tup_used;
  std::map<std::pair<int, int>, int> memo_slots;
  bool uni = false;                          // lowering for symmetric check points (spec::uniform)
  std::set<int> pvars;                       // variables bound to a process (a pid in [0, n))
  std::vector<std::pair<int, int>> uft;      // (field, tag) current / old fields the symmetric lowering reads
  std::map<std::pair<int, std::string>, int> umemo;  // (init set, C++ expression) -> member_init_u slot
  // lowering for the kernel's frozen check points (fail_frozen): no process took a step since the
  // previous check point, so every old field is the current one, and `facts` (field -> value) hold
  // for every process (the algorithm's frozen-tail invariants, frozen_facts)
  bool frozen = false;
  std::map<int, int> facts;

  bool own(int uid) const {
    auto it = names.find(uid);
    return it != names.end() && it->second.own;
  }
  void check_field(int f) const {
    if (restrict_fields && !fields_available.count(f))
      throw SpecError("field " + S(f) + " is not part of this algorithm's state");
  }
  std::string next(const char* p) { return p + S(k++); }
  void add_uft(int f, int tag) {
    if (std::find(uft.begin(), uft.end(), std::make_pair(f, tag)) == uft.end()) uft.emplace_back(f, tag);
  }

  Code gen(int e, bool in_lane, int vi) {
    auto c = cse.find(skey(e));
    if (c != cse.end()) return {c->second, false};  // a closed subformula computed once per check point
    const Node n = T.nodes[e];
    switch (n.k) {
      case LIT: return {c_int(n.v), false};
      case NV: return {"x.n", false};
      case RV: return {"x.r", false};
      case COORDV: return {"((x.r / 4) % x.n)", false};
      case VAR: {
        auto it = names.find(n.uid);
        if (it == names.end()) throw SpecError("variable used outside its quantifier");
        return {it->second.name, it->second.lane};
      }
      case FIELD: {
        check_field(n.f);
        fields.insert(n.f);
        tags.insert(n.tag);
        const Node& p = T.nodes[n.a];
        // frozen check point: old(f) is the current f; a fact field of a process (a quantified
        // pid or coord, both in [0, n)) is its constant
        const int tag = (frozen && n.tag == PSG_TAG_OLD) ? PSG_TAG_CUR : n.tag;
        if (frozen && tag == PSG_TAG_CUR && facts.count(n.f) &&
            (p.k == COORDV || (p.k == VAR && pvars.count(p.uid))))
          return {c_int(facts.at(n.f)), false};
        if (uni && tag != PSG_TAG_INIT) {
          // symmetric check point: every process holds process 0's value
          add_uft(n.f, tag);
          if (p.k == COORDV || (p.k == VAR && pvars.count(p.uid))) return {"x.uf(" + S(tag) + ", " + S(n.f) + ")", false};
          const Code pc = gen(n.a, in_lane, vi);
          return {"spec::fld_uni<W>(x, " + S(tag) + ", " + S(n.f) + ", " + pc.first + ")", pc.second};
        }
        if (p.k == VAR && own(p.uid)) return {"x.own(" + S(tag) + ", " + S(n.f) + ")", true};  // the lane's own process
        if (p.k == VAR && tuples.count(p.uid)) return {tuples[p.uid][{n.f, n.tag}], false};  // a distinct-state tuple value
        const Code pc = gen(n.a, in_lane, vi);
        return {std::string("spec::") + (pc.second ? "fld_g" : "fld_u") + "<W>(x, " + S(tag) + ", " + S(n.f) + ", " +
                    pc.first + ")",
                pc.second};
      }
      case UN: {
        const Code a = gen(n.a, in_lane, vi);
        if (n.op == PSG_OP_NOT) return {"(int32_t)((" + a.first + ") == 0)", a.second};
        if (n.op == PSG_OP_NEG) return {"spec::isub(0, " + a.first + ")", a.second};
        return {"(int32_t)((" + a.first + ") != (-2147483647 - 1))", a.second};
      }
      case BIN: {
        const Code a = gen(n.a, in_lane, vi);
        const Code b = gen(n.b, in_lane, vi);
        if ((n.op == PSG_OP_AND || n.op == PSG_OP_OR || n.op == PSG_OP_IMPL) && expensive(T, n.b)) {
          // skip a quantified right side when no lane needs it (group-uniform test)
          if (!a.second) {
            std::string t;
            if (n.op == PSG_OP_AND) t = "(" + a.first + ") != 0 ? (int32_t)((" + b.first + ") != 0) : 0";
            else if (n.op == PSG_OP_OR) t = "(" + a.first + ") != 0 ? 1 : (int32_t)((" + b.first + ") != 0)";
            else t = "(" + a.first + ") == 0 ? 1 : (int32_t)((" + b.first + ") != 0)";
            return {"(" + t + ")", b.second};
          }
          const char* fn = n.op == PSG_OP_AND ? "and_sc" : n.op == PSG_OP_OR ? "or_sc" : "impl_sc";
          return {std::string("spec::") + fn + "<W>(x, " + a.first + ", [&]() -> int32_t { return " + b.first + "; })",
                  true};
        }
        return {bin(n.op, a.first, b.first), a.second || b.second};
      }
      case CONTAINS: {
        const Code val = gen(n.a, in_lane, vi);
        const std::string v = next("b");
        const bool own_e = T.nodes[n.a].k == VAR && own(T.nodes[n.a].uid);
        if (T.nodes[n.a].k == COORDV || (T.nodes[n.a].k == VAR && pvars.count(T.nodes[n.a].uid)))
          pvars.insert(n.uid);  // a process's pid
        // A.contains(i) for the lane's own process i: the comprehension's variable is that
        // process too (its fields are the lane's registers, not a gather)
        names[n.uid] = own_e ? Name{val.first, true, true} : Name{v, val.second, false};
        const Code body = gen(n.b, in_lane, vi);
        return {"([&](int32_t " + v + ") -> int32_t { return " + body.first + "; })(" + val.first + ")",
                val.second || body.second};
      }
      case QUANT: return quant(e, in_lane, vi);
    }
    throw SpecError("unsupported node");
  }

  static std::string bin(int op, const std::string& x, const std::string& y) {
    switch (op) {
      case PSG_OP_AND: return "(int32_t)(((" + x + ") != 0) & ((" + y + ") != 0))";
      case PSG_OP_OR: return "(int32_t)(((" + x + ") != 0) | ((" + y + ") != 0))";
      case PSG_OP_IMPL: return "(int32_t)(((" + x + ") == 0) | ((" + y + ") != 0))";
      case PSG_OP_EQ: return "(int32_t)((" + x + ") == (" + y + "))";
      case PSG_OP_NE: return "(int32_t)((" + x + ") != (" + y + "))";
      case PSG_OP_LT: return "(int32_t)((" + x + ") < (" + y + "))";
      case PSG_OP_LE: return "(int32_t)((" + x + ") <= (" + y + "))";
      case PSG_OP_GT: return "(int32_t)((" + x + ") > (" + y + "))";
      case PSG_OP_GE: return "(int32_t)((" + x + ") >= (" + y + "))";
      case PSG_OP_ADD: return "spec::iadd(" + x + ", " + y + ")";
      case PSG_OP_SUB: return "spec::isub(" + x + ", " + y + ")";
      case PSG_OP_MUL: return "spec::imul(" + x + ", " + y + ")";
      case PSG_OP_DIV: return "spec::idiv(" + x + ", " + y + ")";
      case PSG_OP_MOD: return "spec::imod(" + x + ", " + y + ")";
    }
    throw SpecError("unsupported operator");
  }

  static std::string lam(const std::string& params, const std::string& body) {
    return "[&](" + params + ") -> int32_t { return " + body + "; }";
  }

  Code quant(int q, bool in_lane, int vi) {
    const Node Q = T.nodes[q];
    const std::string v = next("v");
    if (Q.qk == QFORALL || Q.qk == QEXISTS || Q.qk == QCOUNT) {
      const int mode = Q.qk == QFORALL ? 0 : Q.qk == QEXISTS ? 1 : 2;
      pvars.insert(Q.uid);
      // a variable may be bound by several quantifiers (split_conjuncts): drop its last binding
      tuples.erase(Q.uid);
      names.erase(Q.uid);
      if (uni) {
        Code got;
        if (quant_uni(q, v, in_lane, vi, got)) return got;
      }
      if (!in_lane) {
        names[Q.uid] = Name{v, true, true};
        const Code body = gen(Q.a, true, vi);
        const char* fn = mode == 0 ? "forall_lane" : mode == 1 ? "exists_lane" : "count_lane";
        return {std::string("spec::") + fn + "<W>(x, " + lam("int32_t " + v, body.first) + ")", false};
      }
      const std::pair<int, int> mem = init_member(T, q);
      if (mem.first >= 0 && (std::find(init_sets.begin(), init_sets.end(), mem.first) != init_sets.end() ||
                             init_sets.size() < 2)) {
        const int f = mem.first, t = mem.second;
        if (std::find(init_sets.begin(), init_sets.end(), f) == init_sets.end()) init_sets.push_back(f);
        fields.insert(f);
        tags.insert(PSG_TAG_INIT);
        const int K = (int)(std::find(init_sets.begin(), init_sets.end(), f) - init_sets.begin());
        const Node tn = T.nodes[t];
        if (tn.k == FIELD && tn.tag == PSG_TAG_CUR && T.nodes[tn.a].k == VAR && own(T.nodes[tn.a].uid)) {
          // the lane's own current field: memoized probe (member_init_own)
          const std::pair<int, int> key{K, tn.f};
          if (!memo_slots.count(key) && memo_slots.size() < 4) {
            const int slot = (int)memo_slots.size();
            memo_slots[key] = slot;
          }
          if (memo_slots.count(key)) {
            fields.insert(tn.f);
            tags.insert(PSG_TAG_CUR);
            return {"spec::member_init_own<W, " + S(K) + ", " + S(tn.f) + ", " + S(memo_slots[key]) + ">(x)", true};
          }
        }
        const Code tc = gen(t, in_lane, vi);
        return {"spec::member_init<W, " + S(K) + ">(x, " + tc.first + ")", tc.second};
      }
      std::vector<std::pair<int, int>> flds;
      if (tuple_fields(T, q, flds)) {
        // the body reads j only through fields: visit each distinct field tuple once
        // (count: weighted by how many processes hold it)
        const std::vector<int> guard = flds.empty() ? std::vector<int>{} : tuple_guard(T, q);
        std::string gcode;
        if (!guard.empty()) {
          // A(j) of forall(j => A(j) ==> B) / exists, count(j => A(j) && B): only the processes
          // where it holds are visited; evaluated per lane (j = the lane's own process)
          names[Q.uid] = Name{v, true, true};
          for (size_t i = 0; i < guard.size(); ++i)
            gcode += (i ? " & " : "") + std::string("(int32_t)((") + gen(guard[i], true, vi).first + ") != 0)";
          names.erase(Q.uid);
        }
        std::map<std::pair<int, int>, std::string> nm;
        for (size_t i = 0; i < flds.size(); ++i) nm[flds[i]] = v + "_" + S((int)i);
        tuples[Q.uid] = nm;
        for (auto& ft : flds) {
          check_field(ft.first);
          fields.insert(ft.first);
          tags.insert(ft.second);
        }
        const Code body = gen(Q.a, in_lane, vi);
        std::string params, fl;
        for (size_t i = 0; i < flds.size(); ++i) {
          params += (i ? ", " : "") + std::string("int32_t ") + nm[flds[i]];
          fl += (i ? ", " : "") + std::string("spec::Fld<") + S(flds[i].first) + ", " + S(flds[i].second) + ">{}";
        }
        if (flds.empty())
          return {"spec::quant_tup<W, " + S(mode) + ">(x, " + lam(params, body.first) + ")", body.second};
        // per check point: are those fields the same for every (guarded) process (one tuple)?
        const TupKey key{flds, gcode};
        auto ts = std::find_if(tup_sets.begin(), tup_sets.end(), [&](const auto& p) { return p.first == key; });
        if (ts == tup_sets.end()) {
          tup_sets.emplace_back(key, "tu" + S((int)tup_sets.size()));
          ts = tup_sets.end() - 1;
        }
        tup_used.insert(key);
        return {std::string("spec::") + (gcode.empty() ? "quant_tup_c" : "quant_tup_gc") + "<W, " + S(mode) + ">(x, " +
                    ts->second + ", " + lam(params, body.first) + ", " + fl + ")",
                body.second};
      }
      names[Q.uid] = Name{v, false, false};
      const Code body = gen(Q.a, in_lane, vi);
      const char* fn = mode == 0 ? "forall_ser" : mode == 1 ? "exists_ser" : "count_ser";
      return {std::string("spec::") + fn + "<W>(x, " + lam("int32_t " + v, body.first) + ")", body.second};
    }
    names[Q.uid] = Name{v, false, false};
    if (Q.qk == QVBOOL) {
      const Code body = gen(Q.a, in_lane, vi);
      return {"spec::exists_bool<W>(x, " + lam("int32_t " + v, body.first) + ")", body.second};
    }
    Pins P;
    if (!in_lane && pins(T, Q.a, Q.uid, {}, P)) {
      // equality pins: a conjunct P.forall(i => ... && (cond(i) ==> term(i) == v) && ...)
      // leaves v = term(i) as the only candidate once some process has cond(i); with
      // none active, the finitization below decides it
      const std::string pl = next("p");
      names[T.nodes[P.forall].uid] = Name{pl, true, true};
      pvars.insert(T.nodes[P.forall].uid);
      std::vector<std::string> conds, vals;
      bool plane = false;
      for (auto& ct : P.list) {
        if (ct.first < 0) {
          conds.push_back("1");
        } else {
          const Code cc = gen(ct.first, true, vi);
          conds.push_back("(int32_t)((" + cc.first + ") != 0)");
          plane = plane || cc.second;
        }
        const Code tc = gen(ct.second, true, vi);
        vals.push_back(tc.first);
        plane = plane || tc.second;
      }
      std::string act;
      for (size_t i = 0; i < conds.size(); ++i) act += (i ? " | " : "") + conds[i];
      std::string val = vals.back();
      for (int i = (int)conds.size() - 2; i >= 0; --i)
        val = "((" + conds[i] + ") != 0 ? (" + vals[i] + ") : (" + val + "))";
      const Code general = vint_unpinned(q, v, in_lane, vi);
      names[Q.uid] = Name{v, false, false};
      const Code body = gen(Q.a, in_lane, vi + 1);
      max_vi = std::max(max_vi, vi + 1);
      if (uni && !plane)  // symmetric check point: every process has the same pin flag and value
        return {"spec::pin_uni(" + act + ", " + val + ", " + lam("int32_t " + v, body.first) +
                    ", [&]() -> int32_t { return " + general.first + "; })",
                body.second || general.second};
      return {"spec::exists_int_pin<W>(x, " + lam("int32_t " + pl, act) + ", " + lam("int32_t " + pl, val) +
                  ", scratch + " + S(vi) + " * 64 * W, " + lam("int32_t " + v, body.first) +
                  ", [&]() -> int32_t { return " + general.first + "; })",
              true};
    }
    return vint_unpinned(q, v, in_lane, vi);
  }

  // A process quantifier on a symmetric check point, false for the
  // general rules: a body reading its variable only through current / old fields has one value
  // for every process; P.exists(j => init(j.f) == t) with a group-uniform t is a scalar-memoized probe
  bool quant_uni(int q, const std::string& v, bool in_lane, int vi, Code& out) {
    const Node Q = T.nodes[q];
    const int mode = Q.qk == QFORALL ? 0 : Q.qk == QEXISTS ? 1 : 2;
    if (symmetric(T, q)) {
      names[Q.uid] = Name{"0", false, false};  // never read but through its fields
      const Code body = gen(Q.a, in_lane, vi);
      if (body.second && !in_lane) {
        // a group-uniform value in a lane register: reduced over the valid lanes
        const char* fn = mode == 0 ? "forall_lane" : mode == 1 ? "exists_lane" : "count_lane";
        out = {std::string("spec::") + fn + "<W>(x, " + lam("int32_t " + v, body.first) + ")", false};
        return true;
      }
      if (mode == 2) out = {"((" + body.first + ") != 0 ? x.n : 0)", body.second};
      else out = {"(int32_t)((" + body.first + ") != 0)", body.second};
      return true;
    }
    const std::pair<int, int> mem = init_member(T, q);
    if (mem.first >= 0 && (std::find(init_sets.begin(), init_sets.end(), mem.first) != init_sets.end() ||
                           init_sets.size() < 2)) {
      const int f = mem.first;
      const Code tc = gen(mem.second, in_lane, vi);
      if (tc.second) return false;
      if (std::find(init_sets.begin(), init_sets.end(), f) == init_sets.end()) init_sets.push_back(f);
      fields.insert(f);
      tags.insert(PSG_TAG_INIT);
      const int K = (int)(std::find(init_sets.begin(), init_sets.end(), f) - init_sets.begin());
      const std::pair<int, std::string> key{K, tc.first};
      if (!umemo.count(key) && umemo.size() < 4) {
        const int slot = (int)umemo.size();
        umemo[key] = slot;
      }
      if (umemo.count(key))
        out = {"spec::member_init_u<W, " + S(K) + ", " + S(umemo[key]) + ">(x, " + tc.first + ")", false};
      else
        out = {"spec::member_init<W, " + S(K) + ">(x, " + tc.first + ")", false};
      return true;
    }
    return false;
  }

  // V.exists over Int: count-guarded candidates, else the general finitization
  Code vint_unpinned(int q, const std::string& v, bool in_lane, int vi) {
    const int uid = T.nodes[q].uid;
    names[uid] = Name{v, false, false};
    CountGuard g;
    bool guard = count_guard(T, q, g);
    std::string tc;
    if (guard) {
      // a conjunct P.filter(i => i.f == v).size >= L restricts the witnesses to values
      // of f held by >= L processes (runtime L >= 1; else the general finitization)
      fields.insert(g.f);
      tags.insert(g.tag);
      const Code t = gen(g.thr, in_lane, vi);
      tc = t.first;
      if (t.second) guard = false;
    }
    if (guard) {
      const std::string L = g.op == PSG_OP_GT ? "((" + tc + ") + 1)" : "(" + tc + ")";
      const Code general = vint_general(q, v, in_lane, vi);
      names[uid] = Name{v, false, false};
      const Code body = gen(T.nodes[q].a, in_lane, vi + 1);
      max_vi = std::max(max_vi, vi + 1);
      if (uni && g.tag != PSG_TAG_INIT) {
        // symmetric check point: process 0's value is the only one, held by n processes
        add_uft(g.f, g.tag);
        return {"([&]() -> int32_t { const int32_t L_ = " + L + "; if (L_ >= 1) return spec::guard_uni<W>(x, x.uf(" +
                    S(g.tag) + ", " + S(g.f) + "), L_, " + lam("int32_t " + v, body.first) + "); return " +
                    general.first + "; })()",
                body.second || general.second};
      }
      return {"([&]() -> int32_t { const int32_t L_ = " + L + "; if (L_ >= 1) return spec::exists_int_guard<W, " +
                  S(g.f | (g.tag << 8)) + ">(x, x.own(" + S(g.tag) + ", " + S(g.f) + "), x.stage(" + S(g.tag) + ", " +
                  S(g.f) + "), L_, " + lam("int32_t " + v, body.first) + "); return " + general.first + "; })()",
              true};
    }
    return vint_general(q, v, in_lane, vi);
  }

  // V.exists over Int by finitization over the compared terms (equality-only: no +-1)
  Code vint_general(int q, const std::string& v, bool in_lane, int vi) {
    names[T.nodes[q].uid] = Name{v, false, false};
    std::vector<int> exprs;
    std::vector<std::pair<int, int>> fsets;
    witnesses(T, q, exprs, fsets);
    const bool eqo = eq_only(T, q);
    std::vector<std::string> evs;
    for (int t : exprs) evs.push_back(gen(t, in_lane, vi).first);
    for (auto& ft : fsets) {
      fields.insert(ft.first);
      tags.insert(ft.second);
    }
    max_vi = std::max(max_vi, vi + 1);
    const Code body = gen(T.nodes[q].a, in_lane, vi + 1);
    // its value is group-uniform outside a lane quantifier (the candidates are); the general
    // lowering keeps the conservative lane flag
    const bool vlane = uni ? (in_lane || body.second) : true;
    const int ne = (int)evs.size(), nf = (int)fsets.size();
    std::string ev, fs;
    for (int i = 0; i < ne; ++i) ev += (i ? ", " : "") + evs[i];
    for (int i = 0; i < nf; ++i) fs += (i ? ", " : "") + S(fsets[i].first | (fsets[i].second << 8));
    if (ev.empty()) ev = "0";
    if (fs.empty()) fs = "0";
    const std::string head = "([&]() -> int32_t { const int32_t ev_[" + S(std::max(ne, 1)) + "] = {" + ev +
                             "}; const int32_t fs_[" + S(std::max(nf, 1)) + "] = {" + fs + "}; ";
    const std::string tail = lam("int32_t " + v, body.first) + "); })()";
    if (eqo)
      return {head + "return spec::exists_int_eq<W, " + S(ne) + ", " + S(nf) + ">(x, ev_, fs_, scratch + " + S(vi) +
                  " * 64 * W, " + tail,
              vlane};
    // order comparisons: one candidate per breakpoint (exists_int_bp) instead of v-1, v, v+1
    const std::vector<int> sh = breakpoint_shifts(T, q, exprs, fsets);
    std::string shs;
    for (size_t i = 0; i < sh.size(); ++i) shs += (i ? ", " : "") + S(sh[i]) + "u";
    if (shs.empty()) shs = "0u";
    return {head + "const uint32_t sh_[" + S(std::max(ne + nf, 1)) + "] = {" + shs + "}; return spec::exists_int_bp<W, " +
                S(ne) + ", " + S(nf) + ">(x, ev_, fs_, sh_, scratch + " + S(vi) + " * 64 * W, " + tail,
            vlane};
  }
};

// The native checker's source for a parsed + compiled Spec.
// The algorithm kernels' frozen-tail invariants (fields by psg.h PSG_FIELD_*: x 0, decided 1,
// decision 2, ts 3, ready 4, commit 5, vote 6): facts that hold for every process at a frozen
// check point of that kernel. OTR / OTR2: the frozen tail starts when every process halted, and a
// process halts only after deciding (Otr.scala:75-80). LastVoting: the quiescent tail starts when
// no process is commit or ready (psg_lv.hip), and no step runs after it.
std::map<int, int> frozen_facts(int alg) {
  switch (alg) {
    case PSG_ALG_OTR:
    case PSG_ALG_OTR2: return {{PSG_FIELD_DECIDED, 1}};
    case PSG_ALG_LAST_VOTING: return {{PSG_FIELD_READY, 0}, {PSG_FIELD_COMMIT, 0}};
    default: return {};
  }
}

std::string codegen_hip(ParsedSpec& P, const Compiled& prog, int alg) {
  Tree& T = P.T;
  Gen gen{T, alg != 0, alg != 0 ? alg_fields(alg) : std::set<int>{}};
  std::map<int, int> memo;
  std::vector<int> invs;
  for (int inv : P.invs) invs.push_back(rewrite_vint(T, inv, memo));
  std::vector<std::pair<std::string, int>> props;
  for (auto& p : P.props) props.emplace_back(p.first, rewrite_vint(T, p.second, memo));
  const int safety = P.sp < 0 ? -1 : rewrite_vint(T, P.sp, memo);
  // common closed subformulas (structurally equal, skey): hoisted, evaluated once per check point
  std::vector<int> roots = invs;
  for (auto& p : props)
    if (p.first != "Termination") roots.push_back(p.second);
  if (safety >= 0) roots.push_back(safety);
  std::map<std::string, int> seen;
  std::vector<int> order;
  for (int rt : roots) {
    struct V {
      static void visit(Gen& G, int e, std::map<std::string, int>& seen, std::vector<int>& order) {
        if (++seen[G.skey(e)] > 1) return;
        std::vector<int> ch;
        G.T.children(e, ch);
        for (int c : ch) visit(G, c, seen, order);
        order.push_back(e);  // post-order: inner subformulas first
      }
    };
    V::visit(gen, rt, seen, order);
  }
  auto tup_decls = [&](const std::set<Gen::TupKey>& used, const std::string& ind) {
    std::vector<std::string> out;
    for (auto& ts : gen.tup_sets) {
      if (!used.count(ts.first)) continue;
      const auto& flds = ts.first.first;
      std::string fl;
      for (size_t i = 0; i < flds.size(); ++i)
        fl += (i ? ", " : "") + std::string("spec::Fld<") + S(flds[i].first) + ", " + S(flds[i].second) + ">{}";
      if (ts.first.second.empty())
        out.push_back(ind + "const auto " + ts.second + " = spec::tup_uniform<W>(x, " + fl + ");");
      else
        out.push_back(ind + "const auto " + ts.second + " = spec::tup_uniform_g<W>(x, " + ts.first.second + ", " + fl +
                      ");");
    }
    return out;
  };
  struct Block {
    std::vector<std::string> lines, term_decls;
    std::string term;
    bool has_term = false;
    int slot = 0;
  };
  // the slot lines of fail() and the Termination expression, under the general or the
  // symmetric-check-point lowering
  auto block = [&](bool uni) {
    gen.uni = uni;
    gen.cse.clear();
    gen.tup_used.clear();
    const std::string ind = uni ? "      " : "    ", pre = uni ? "ucse" : "cse", iv = uni ? "uinv" : "inv";
    Block B;
    std::vector<std::string> lines;
    // a distinct-state tuple test is declared just before the first line that uses it
    auto add = [&](int e, const std::function<std::string(const std::string&)>& fmt) {
      const std::set<Gen::TupKey> before = gen.tup_used;
      const Code c = gen.gen(e, false, 0);
      std::set<Gen::TupKey> fresh;
      for (auto& k : gen.tup_used)
        if (!before.count(k)) fresh.insert(k);
      for (auto& d : tup_decls(fresh, ind)) lines.push_back(d);
      lines.push_back(fmt(c.first));
    };
    int slot = 0;
    for (int e : order) {
      const Kind kd = T.nodes[e].k;
      if (seen[gen.skey(e)] > 1 && (kd == QUANT || kd == CONTAINS) && free_of(T, e).empty()) {
        const std::string name = pre + S((int)gen.cse.size());
        add(e, [&](const std::string& c) { return ind + "const int32_t " + name + " = " + c + ";"; });
        gen.cse[gen.skey(e)] = name;
      }
    }
    if (!invs.empty()) {
      for (size_t k = 0; k < invs.size(); ++k)
        add(invs[k], [&](const std::string& c) { return ind + "const int32_t " + iv + S((int)k) + " = " + c + ";"; });
      std::string any;
      for (size_t k = 0; k < invs.size(); ++k) any += (k ? " | " : "") + std::string("(") + iv + S((int)k) + " != 0)";
      lines.push_back(ind + "if (!(" + any + ")) fb |= 1u << " + S(slot) + ";");
      ++slot;
      for (size_t k = 0; k < invs.size(); ++k) {
        lines.push_back(ind + "if (" + iv + S((int)k) + " == 0) fb |= 1u << " + S(slot) + ";");
        ++slot;
      }
    }
    std::set<Gen::TupKey> term_tups;
    for (auto& p : props) {
      if (p.first == "Termination") {
        // term() is its own function: fail()'s hoisted subformulas (cse*) and tuple tests are
        // not in scope there, so it is lowered with neither
        auto saved = gen.tup_used;
        gen.tup_used.clear();
        auto saved_cse = gen.cse;
        gen.cse.clear();
        B.term = gen.gen(p.second, false, 0).first;
        B.has_term = true;
        term_tups = gen.tup_used;
        gen.tup_used = saved;
        gen.cse = saved_cse;
        continue;
      }
      add(p.second, [&](const std::string& c) {
        return ind + "if ((" + c + ") == 0) fb |= 1u << " + S(slot) + ";  // " + p.first;
      });
      ++slot;
    }
    if (safety >= 0) {
      add(safety, [&](const std::string& c) {
        return ind + "if ((" + c + ") == 0) fb |= 1u << " + S(slot) + ";  // SafetyPredicate";
      });
      ++slot;
    }
    if (slot != (int)prog.entry.size()) throw SpecError("native lowering: slot count mismatch");
    B.lines = lines;
    B.term_decls = tup_decls(term_tups, ind);
    B.slot = slot;
    return B;
  };
  // fail() / term() bodies from the general and the symmetric-check-point blocks; the symmetric
  // one is worth its test only with few fields to compare (uft: the fields it compares)
  auto assemble = [&](const Block& G, const Block& U, const std::vector<std::pair<int, int>>& uft,
                      std::vector<std::string>& body, std::vector<std::string>& term_decls) {
    const bool has_term = G.has_term && !G.term.empty();
    if (g_opts.symmetric && !uft.empty() && uft.size() <= 6) {
      uint32_t cur = 0, old = 0;
      for (auto& ft : uft) {
        if (ft.second == PSG_TAG_CUR) cur |= 1u << ft.first;
        else if (ft.second == PSG_TAG_OLD) old |= 1u << ft.first;
      }
      body.push_back("    if (spec::uniform<W, " + std::to_string(cur) + "u, " + std::to_string(old) + "u>(x)) {");
      body.insert(body.end(), U.lines.begin(), U.lines.end());
      body.push_back("      return fb;");
      body.push_back("    }");
      if (has_term) {
        term_decls.push_back("    if (x.uni) {");
        term_decls.insert(term_decls.end(), U.term_decls.begin(), U.term_decls.end());
        term_decls.push_back("      return (" + U.term + ") != 0;");
        term_decls.push_back("    }");
      }
    }
    body.insert(body.end(), G.lines.begin(), G.lines.end());
    term_decls.insert(term_decls.end(), G.term_decls.begin(), G.term_decls.end());
  };
  Block G = block(false);
  // symmetric check points (every process holds the same value of each current / old field the
  // Spec reads): a second, scalar lowering, chosen per check point by spec::uniform
  Block U = block(true);
  gen.uni = false;
  const int slot = G.slot;
  const bool has_term = G.has_term && !G.term.empty();
  const std::string term = G.term;
  std::vector<std::string> body, term_decls;
  assemble(G, U, gen.uft, body, term_decls);
  // The kernel's frozen check points (SpecHook::put with frozen: no process took a step since the
  // previous check point): the same formulas with every old field read as the current one and the
  // algorithm's frozen-tail facts as constants (frozen_facts), so the compiler folds what they
  // decide (Irrevocability's old.decision == decision, LastVoting's commit / ready terms). Every
  // formula is still evaluated at every check point; only its inputs are known.
  std::vector<std::string> fbody, fterm_decls;
  std::string fterm;
  bool frozen_ok = false;
  if (g_opts.frozen && alg != 0) {
    const auto saved_uft = gen.uft;
    gen.uft.clear();
    gen.frozen = true;
    gen.facts = frozen_facts(alg);
    try {
      Block FG = block(false);
      Block FU = block(true);
      assemble(FG, FU, gen.uft, fbody, fterm_decls);
      fterm = FG.term;
      frozen_ok = true;
    } catch (const SpecError&) {
      frozen_ok = false;  // (not expected: the same tree) fail_frozen falls back to fail
    }
    gen.frozen = false;
    gen.uni = false;
    gen.uft = saved_uft;
  }
  if (gen.max_vi > 4) throw SpecError("more than 4 nested V.exists over Int");
  uint32_t rel = 0, fmask = 0, tmask = 0;
  for (size_t s = 0; s < prog.flags.size(); ++s)
    if (prog.flags[s] & PSG_SPEC_RELATIONAL) rel |= 1u << s;
  for (int f : gen.fields) fmask |= 1u << f;
  for (int t : gen.tags) tmask |= 1u << t;
  std::ostringstream o;
  o << "// generated by psg_spec_gen.cpp: native checker of one Spec\n"
    << "#include \"psg_spec_native.hpp\"\n"
    << "namespace psg {\n"
    << "struct GenSpec {\n"
    << "  static constexpr int kSlots = " << slot << ";\n"
    << "  static constexpr uint32_t kRelational = " << rel << "u;\n"
    << "  static constexpr bool kHasTerm = " << (has_term && !term.empty() ? "true" : "false") << ";\n"
    << "  static constexpr uint32_t kFields = " << fmask << "u;\n"
    << "  static constexpr uint32_t kTags = " << tmask << "u;\n"
    << "  static constexpr int kInitSet0 = " << (gen.init_sets.size() > 0 ? gen.init_sets[0] : -1) << ";\n"
    << "  static constexpr int kInitSet1 = " << (gen.init_sets.size() > 1 ? gen.init_sets[1] : -1) << ";\n"
    << "  template <int W>\n"
    << "  __device__ static uint32_t fail(spec::Ctx<W>& x, int32_t* scratch) {\n"
    << "    (void)scratch;\n"
    << "    uint32_t fb = 0;\n";
  for (auto& l : body) o << l << "\n";
  o << "    return fb;\n"
    << "  }\n"
    << "  template <int W>\n"
    << "  __device__ static bool term(spec::Ctx<W>& x, int32_t* scratch) {\n"
    << "    (void)scratch;\n";
  for (auto& l : term_decls) o << l << "\n";
  o << "    return (" << (has_term && !term.empty() ? term : "0") << ") != 0;\n"
    << "  }\n";
  // frozen check points (SpecHook::put): old fields = current ones, frozen-tail facts constant
  o << "  template <int W>\n"
    << "  __device__ static uint32_t fail_frozen(spec::Ctx<W>& x, int32_t* scratch) {\n";
  if (frozen_ok) {
    o << "    (void)scratch;\n"
      << "    uint32_t fb = 0;\n";
    for (auto& l : fbody) o << l << "\n";
    o << "    return fb;\n";
  } else {
    o << "    return fail<W>(x, scratch);\n";
  }
  o << "  }\n"
    << "  template <int W>\n"
    << "  __device__ static bool term_frozen(spec::Ctx<W>& x, int32_t* scratch) {\n";
  if (frozen_ok) {
    o << "    (void)scratch;\n";
    for (auto& l : fterm_decls) o << l << "\n";
    o << "    return (" << (has_term && !fterm.empty() ? fterm : "0") << ") != 0;\n";
  } else {
    o << "    return term<W>(x, scratch);\n";
  }
  o << "  }\n"
    << "};\n"
    << "}  // namespace psg\n"
    << "PSG_SPEC_NATIVE_KERNELS(psg::GenSpec)\n"
    << "extern \"C\" __device__ int32_t psg_spec_alg = " << alg << ";  // checked by psg_run_batch_spec\n";
  return o.str();
}

// algorithm -> (round-kernel source, body template, leading template arguments)
bool fused_kernel(int alg, std::string& src, std::string& body, std::string& targs_w_prefix, std::string& targs_tail) {
  targs_tail.clear();
  switch (alg) {
    case PSG_ALG_OTR: src = "psg_otr.hip"; body = "otr_body"; targs_tail = ", false"; break;
    case PSG_ALG_OTR2: src = "psg_otr.hip"; body = "otr_body"; targs_tail = ", true"; break;
    case PSG_ALG_LAST_VOTING: src = "psg_lv.hip"; body = "lv_body"; break;
    case PSG_ALG_FLOODMIN: src = "psg_floodmin.hip"; body = "floodmin_body"; break;
    case PSG_ALG_KSET: src = "psg_kset.hip"; body = "kset_body"; break;
    case PSG_ALG_BENOR: src = "psg_benor.hip"; body = "benor_body"; break;
    case PSG_ALG_SLV: src = "psg_slv.hip"; body = "slv_body"; break;
    case PSG_ALG_KSET_ES: src = "psg_kset_es.hip"; body = "kset_es_body"; break;
    default: return false;
  }
  targs_w_prefix.clear();
  return true;
}

// The algorithm's round kernel instantiated with the generated Spec as its hook
std::string fused_source(int alg, const std::vector<int>& waves) {
  std::string src, body, pre, tail;
  if (!fused_kernel(alg, src, body, pre, tail)) throw SpecError("fused lowering needs one of the integer-state algorithms");
  std::ostringstream o;
  o << "#include \"" << src << "\"  // its kernel bodies; host launchers are compiled out (PSG_FUSED_MODULE)";
  // occupancy target of the W = 1 kernels (0: the compiler's); an empty PSG_FUSED_WPE means unset.
  // Measured on MI355X (round 6, scripts/probe_fused.py): LastVoting 5/6/7/8 waves 90.0 / 84.8 /
  // 82.8 / 81.3 ms, OTR compiler's (5) / 6 / 7 waves 38.8 / 36.4 / 37.3 ms; the extra waves cost a
  // few spilled words outside the round loop and hide more of the checker's latency than they add
  int wpe = alg == PSG_ALG_LAST_VOTING ? 8 : (alg == PSG_ALG_OTR || alg == PSG_ALG_OTR2) ? 6 : 0;
  if (const char* e = std::getenv("PSG_FUSED_WPE"))
    if (*e) wpe = std::atoi(e);
  for (int W : waves) {
    const int threads = W == 1 ? 256 : 64 * W;
    const std::string attr =
        W == 1 && wpe > 0 ? "__attribute__((amdgpu_waves_per_eu(" + S(wpe) + "))) " : std::string();
    const char* sfx[2] = {"", "x_"};
    const char* xho[2] = {"false", "true"};
    for (int k = 0; k < 2; ++k) {
      o << "\nextern \"C\" __global__ void __launch_bounds__(" << threads << ") " << attr << "psg_fused_" << sfx[k] << "a"
        << alg << "_w" << W << "(psg::KArgs a) {";
      o << "\n  psg::" << body << "<" << W << tail << ", " << xho[k] << ", psg::spec::SpecHook<psg::GenSpec>>(a);";
      o << "\n}";
    }
  }
  return o.str() + "\n";
}

// ------------------------------------------------------------------ SHA-256 (the cache key, = hashlib.sha256)
struct Sha256 {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  std::string buf;
  uint64_t len = 0;
  static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  void block(const unsigned char* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
        0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
        0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
        0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
        0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
        0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
        0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const std::string& s) {
    len += s.size();
    buf += s;
    size_t off = 0;
    for (; off + 64 <= buf.size(); off += 64) block((const unsigned char*)buf.data() + off);
    buf.erase(0, off);
  }
  std::string hex() {
    std::string pad = buf;
    pad.push_back((char)0x80);
    while (pad.size() % 64 != 56) pad.push_back(0);
    const uint64_t bits = len * 8;
    for (int i = 7; i >= 0; --i) pad.push_back((char)(bits >> (8 * i)));
    for (size_t off = 0; off < pad.size(); off += 64) block((const unsigned char*)pad.data() + off);
    char out[65];
    for (int i = 0; i < 8; ++i) std::snprintf(out + 8 * i, 9, "%08x", h[i]);
    return std::string(out, 64);
  }
};

bool read_file(const std::string& path, std::string& out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return false;
  std::ostringstream ss;
  ss << in.rdbuf();
  out = ss.str();
  return true;
}

// <library dir>: round_amd/ (libpsg.so) -> csrc/ next to it, include/ and build/spec/ one up
std::string lib_dir() {
  Dl_info info;
  if (dladdr((const void*)&lib_dir, &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    const size_t s = p.find_last_of('/');
    return s == std::string::npos ? std::string(".") : p.substr(0, s);
  }
  return ".";
}

std::string env_or(const char* name, const std::string& dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::string(e) : dflt;
}

// The full module source of compile_native(text, alg, fused, n) and its cache key.
std::string module_source(ParsedSpec& P, const Compiled& prog, int alg, bool fused, int n) {
  // fused LastVoting: no symmetric-check-point lowering unless asked for ("sym") — its check points
  // are rarely symmetric, and without the second lowering the module measured 2 % faster (round 6,
  // 81.55 -> 79.90 ms at 8 waves/SIMD, scripts/probe_fused.py)
  const bool sym_saved = g_opts.symmetric;
  if (fused && alg == PSG_ALG_LAST_VOTING && !g_opts.sym_explicit) g_opts.symmetric = false;
  std::string src = codegen_hip(P, prog, alg);
  g_opts.symmetric = sym_saved;
  std::string defs;
  for (const std::string& d : g_opts.defines) {
    const size_t eq = d.find('=');
    defs += "#define " + (eq == std::string::npos ? d : d.substr(0, eq) + " " + d.substr(eq + 1)) + "\n";
  }
  src = defs + src;
  if (fused) {
    std::vector<int> waves;
    if (n > 0) waves.push_back((n + 63) / 64);
    else waves = {1, 2, 3, 4};
    // Philox products: the inline v_mad_u64_u32 form (carry in VCC, the library's round kernels'
    // choice) for OTR / OTR2 — round 6, at 6 waves/SIMD: fused OTR 36.50 -> 35.21 ms; LastVoting
    // neutral (81.46 / 81.55) — and the compiler's mul_lo / mul_hi pair for the others (round 4:
    // the inline form 4-6 % slower there)
    const int mad64 = alg == PSG_ALG_OTR || alg == PSG_ALG_OTR2 ? 2 : 0;
    src = "#define PSG_FUSED_MODULE 1\n#ifndef PSG_PHILOX_MAD64\n#define PSG_PHILOX_MAD64 " + S(mad64) + "\n#endif\n" + src +
          fused_source(alg, waves);
  }
  return src;
}

// A tree as Formula text (the format psg_spec_from_text reads; formula.py to_text)
std::string text_of(const Tree& T, int e) {
  static const char* fields[] = {"x", "decided", "decision", "ts", "ready", "commit", "vote", "canDecide"};
  static const std::map<int, const char*> bins = {
      {PSG_OP_AND, "And"}, {PSG_OP_OR, "Or"},     {PSG_OP_IMPL, "Implies"}, {PSG_OP_EQ, "Eq"},
      {PSG_OP_NE, "Neq"},  {PSG_OP_LT, "Lt"},     {PSG_OP_LE, "Leq"},       {PSG_OP_GT, "Gt"},
      {PSG_OP_GE, "Geq"},  {PSG_OP_ADD, "Plus"},  {PSG_OP_SUB, "Minus"},    {PSG_OP_MUL, "Times"},
      {PSG_OP_DIV, "Divides"}, {PSG_OP_MOD, "Remainder"}};
  const Node& n = T.nodes[e];
  auto var = [](int uid) { return "v" + S(uid); };
  switch (n.k) {
    case LIT: return "(Lit " + S(n.v) + ")";
    case NV: return "(Var n)";
    case RV: return "(Var r)";
    case COORDV: return "(Var coord)";
    case VAR: return "(Var " + var(n.uid) + ")";
    case FIELD: {
      if (n.f == PSG_FIELD_HOSIZE) return "(App Cardinality (App HO " + text_of(T, n.a) + "))";
      const std::string pre = n.tag == PSG_TAG_OLD ? "__old__" : n.tag == PSG_TAG_INIT ? "__init__" : "";
      return "(App " + pre + fields[n.f] + " " + text_of(T, n.a) + ")";
    }
    case UN:
      return std::string("(App ") + (n.op == PSG_OP_NOT ? "Not" : n.op == PSG_OP_NEG ? "Minus" : "IsDefined") + " " +
             text_of(T, n.a) + ")";
    case BIN: return std::string("(App ") + bins.at(n.op) + " " + text_of(T, n.a) + " " + text_of(T, n.b) + ")";
    case CONTAINS:
      return "(App In " + text_of(T, n.a) + " (Comprehension ((" + var(n.uid) + " pid)) " + text_of(T, n.b) + "))";
    case QUANT:
      switch (n.qk) {
        case QFORALL: return "(ForAll ((" + var(n.uid) + " pid)) " + text_of(T, n.a) + ")";
        case QEXISTS: return "(Exists ((" + var(n.uid) + " pid)) " + text_of(T, n.a) + ")";
        case QCOUNT: return "(App Cardinality (Comprehension ((" + var(n.uid) + " pid)) " + text_of(T, n.a) + "))";
        case QVINT: return "(Exists ((" + var(n.uid) + " Int)) " + text_of(T, n.a) + ")";
        default: return "(Exists ((" + var(n.uid) + " Bool)) " + text_of(T, n.a) + ")";
      }
  }
  throw SpecError("text_of: unknown node");
}

std::mutex g_paths_mu;
std::set<std::string>& interned() {  // module paths handed out (valid until the process exits)
  static std::set<std::string> s;
  return s;
}

// The compiler the modules are built with. A process may already hold another HIP toolchain under
// the same sonames: PyTorch's wheel bundles its own libamdhip64 / libhiprtc / libamd_comgr (ROCm
// 7.0 here), and once `import torch` has loaded them, libpsg's libhiprtc.so.7 and the comgr that
// hiprtc loads by name resolve to torch's copies. Both toolchains report the same hiprtcVersion,
// so modules compiled by either shared one cache key, and they differ: ROCm 7.0's comgr gives the
// fused LastVoting kernel 416 B of scratch (187 SGPR spills) where the image's ROCm 7.2 gives none
// — round 5's one-process configuration run loaded such a module and ran fused LastVoting 3.4x
// slower (profiles/r5_configs: Scratch_Size 416 in the dispatch record). So the
// image's comgr and hiprtc (PSG_ROCM_LIB, default /opt/rocm/lib) are loaded into a link-map
// namespace of their own (dlmopen), comgr first, whatever the process has loaded, and the cache
// key carries the files they came from. If that fails, the process's own hiprtc is used and its
// file is in the key.
struct RtcApi {
  decltype(&hiprtcCreateProgram) create = nullptr;
  decltype(&hiprtcCompileProgram) compile = nullptr;
  decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
  decltype(&hiprtcGetProgramLog) log = nullptr;
  decltype(&hiprtcGetCodeSize) code_size = nullptr;
  decltype(&hiprtcGetCode) code = nullptr;
  decltype(&hiprtcDestroyProgram) destroy = nullptr;
  std::string ident;  // the compiler's files (cache key)
};

std::string file_ident(const std::string& path) {
  char real[4096];
  const std::string rp = realpath(path.c_str(), real) ? std::string(real) : path;
  struct stat st;
  return rp + ":" + (stat(rp.c_str(), &st) == 0 ? std::to_string((long long)st.st_size) : std::string("?"));
}

const RtcApi& rtc_api() {
  static const RtcApi api = [] {
    RtcApi a;
    const std::string dir = env_or("PSG_ROCM_LIB", "/opt/rocm/lib");
    const std::string comgr = dir + "/libamd_comgr.so.3", rtc = dir + "/libhiprtc.so.7";
    void* hc = dlmopen(LM_ID_NEWLM, comgr.c_str(), RTLD_NOW | RTLD_LOCAL);
    Lmid_t lm = 0;
    void* hr = nullptr;
    if (hc && dlinfo(hc, RTLD_DI_LMID, &lm) == 0) hr = dlmopen(lm, rtc.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (hr) {
      a.create = (decltype(a.create))dlsym(hr, "hiprtcCreateProgram");
      a.compile = (decltype(a.compile))dlsym(hr, "hiprtcCompileProgram");
      a.log_size = (decltype(a.log_size))dlsym(hr, "hiprtcGetProgramLogSize");
      a.log = (decltype(a.log))dlsym(hr, "hiprtcGetProgramLog");
      a.code_size = (decltype(a.code_size))dlsym(hr, "hiprtcGetCodeSize");
      a.code = (decltype(a.code))dlsym(hr, "hiprtcGetCode");
      a.destroy = (decltype(a.destroy))dlsym(hr, "hiprtcDestroyProgram");
    }
    if (a.create && a.compile && a.log_size && a.log && a.code_size && a.code && a.destroy) {
      a.ident = "isolated " + file_ident(rtc) + " " + file_ident(comgr);
      return a;
    }
    a = RtcApi();  // the process's own hiprtc (whichever copy the dynamic linker bound)
    a.create = &hiprtcCreateProgram;
    a.compile = &hiprtcCompileProgram;
    a.log_size = &hiprtcGetProgramLogSize;
    a.log = &hiprtcGetProgramLog;
    a.code_size = &hiprtcGetCodeSize;
    a.code = &hiprtcGetCode;
    a.destroy = &hiprtcDestroyProgram;
    Dl_info info;
    a.ident = std::string("process ") +
              (dladdr((const void*)&hiprtcCompileProgram, &info) && info.dli_fname ? file_ident(info.dli_fname) : "?");
    return a;
  }();
  return api;
}

int compile_module(const std::string& src, int alg, bool fused, const char* cache_dir, std::string& path,
                   std::string& err) {
  const std::string lib = lib_dir();
  const std::string csrc = env_or("PSG_CSRC", lib + "/csrc");
  const std::string inc = env_or("PSG_INCLUDE", lib + "/../include");
  std::vector<std::string> hdr_names = {"psg_spec_native.hpp", "psg_device.hpp"};
  if (fused) {
    std::string ksrc, body, pre, tail;
    fused_kernel(alg, ksrc, body, pre, tail);
    hdr_names.push_back(ksrc);  // everything it includes
    hdr_names.push_back("psg_kernels.hpp");
    hdr_names.push_back("psg_packed.hpp");
  }
  // the cache key: the source, the kernel headers and psg.h, and the compiler's identity (the
  // files of the hiprtc and comgr that compile it, and the options), so a module built by another
  // toolchain is never reused
  const RtcApi& R = rtc_api();
  int rtc_major = 0, rtc_minor = 0;
  (void)hiprtcVersion(&rtc_major, &rtc_minor);
  const std::string toolchain = "hiprtc " + S(rtc_major) + "." + S(rtc_minor) + " " + R.ident +
                                " --offload-arch=gfx950 -O3 -std=c++17";
  Sha256 h;
  h.update(toolchain);
  h.update(src);
  for (auto& nm : hdr_names) {
    std::string t;
    if (!read_file(csrc + "/" + nm, t)) {
      err = "native spec: cannot read " + csrc + "/" + nm;
      return PSG_EIO;
    }
    h.update(t);
  }
  std::string psgh;
  if (!read_file(inc + "/psg.h", psgh)) {
    err = "native spec: cannot read " + inc + "/psg.h";
    return PSG_EIO;
  }
  h.update(psgh);
  const std::string dir = cache_dir && *cache_dir ? std::string(cache_dir) : lib + "/../build/spec";
  path = dir + "/spec_" + h.hex().substr(0, 24) + ".co";
  if (access(path.c_str(), R_OK) == 0) return PSG_OK;  // compiled before
  for (size_t i = 1; i <= dir.size(); ++i)  // mkdir -p
    if (i == dir.size() || dir[i] == '/') {
      const std::string d = dir.substr(0, i);
      if (!d.empty()) (void)::mkdir(d.c_str(), 0755);
    }
  hiprtcProgram prog;
  if (R.create(&prog, src.c_str(), "spec.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    err = "native spec: hiprtcCreateProgram failed";
    return PSG_EIO;
  }
  const std::string oi = "-I" + csrc, oj = "-I" + inc;
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", oi.c_str(), oj.c_str()};
  const hiprtcResult rc = R.compile(prog, 5, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t ls = 0;
    R.log_size(prog, &ls);
    std::string log(ls, '\0');
    if (ls) R.log(prog, &log[0]);
    R.destroy(&prog);
    err = "native spec compile failed:\n" + log.substr(log.size() > 4000 ? log.size() - 4000 : 0);
    return PSG_EINVAL;
  }
  size_t cs = 0;
  R.code_size(prog, &cs);
  std::string code(cs, '\0');
  if (cs) R.code(prog, &code[0]);
  R.destroy(&prog);
  const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
  {
    std::ofstream out(tmp, std::ios::binary);
    out.write(code.data(), (std::streamsize)code.size());
    if (!out) {
      err = "native spec: cannot write " + tmp;
      return PSG_EIO;
    }
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) {
    err = "native spec: cannot rename " + tmp;
    return PSG_EIO;
  }
  return PSG_OK;
}

}  // namespace
}  // namespace psgspec

extern "C" {

int psg_spec_set_options(const char* options) {
  using namespace psgspec;
  if (!options) {
    t_options_set = false;
    t_options.clear();
    return PSG_OK;
  }
  try {
    (void)parse_options(options);
  } catch (const std::exception&) {
    return PSG_EINVAL;
  }
  t_options = options;
  t_options_set = true;
  return PSG_OK;
}

int psg_spec_native_source(const char* text, int32_t alg, int32_t fused, int32_t n, char* src, size_t* src_len,
                           char* err, size_t err_len) {
  using namespace psgspec;
  if (!text || !src_len) {
    put(err, err_len, "null argument");
    return PSG_EINVAL;
  }
  try {
    load_options();
    ParsedSpec P = parse_spec(text);
    const Compiled prog = compile_program(P, alg);
    const std::string s = module_source(P, prog, alg, fused != 0, n);
    const size_t cap = *src_len;
    *src_len = s.size() + 1;
    if (!src || cap < s.size() + 1) {
      put(err, err_len, "source buffer too small: " + std::to_string(s.size() + 1) + " bytes needed");
      return PSG_ERANGE;
    }
    std::memcpy(src, s.c_str(), s.size() + 1);
    put(err, err_len, "");
    return PSG_OK;
  } catch (const std::exception& e) {
    put(err, err_len, e.what());
    return PSG_EINVAL;
  }
}

int psg_spec_rewrite_text(const char* text, int32_t alg, char* out, size_t* out_len, char* err, size_t err_len) {
  using namespace psgspec;
  if (!text || !out_len) {
    put(err, err_len, "null argument");
    return PSG_EINVAL;
  }
  try {
    load_options();
    ParsedSpec P = parse_spec(text);
    (void)compile_program(P, alg);  // the same checks as the other entry points
    Tree& T = P.T;
    std::map<int, int> memo;  // one memo for every root, as codegen_hip shares it
    std::string s = "(Spec (phase 1)\n  (invariants";
    for (int inv : P.invs) s += " " + text_of(T, rewrite_vint(T, inv, memo));
    s += ")\n  (properties";
    for (auto& p : P.props) s += " (prop \"" + p.first + "\" " + text_of(T, rewrite_vint(T, p.second, memo)) + ")";
    s += ")";
    if (P.sp >= 0) s += "\n  (safetyPredicate " + text_of(T, rewrite_vint(T, P.sp, memo)) + ")";
    s += ")";
    const size_t cap = *out_len;
    *out_len = s.size() + 1;
    if (!out || cap < s.size() + 1) {
      put(err, err_len, "output buffer too small: " + std::to_string(s.size() + 1) + " bytes needed");
      return PSG_ERANGE;
    }
    std::memcpy(out, s.c_str(), s.size() + 1);
    put(err, err_len, "");
    return PSG_OK;
  } catch (const std::exception& e) {
    put(err, err_len, e.what());
    return PSG_EINVAL;
  }
}

int psg_spec_compile_native(const char* text, int32_t alg, int32_t fused, int32_t n, const char* cache_dir,
                            psg_spec_program* out, char* names, size_t names_len, char* err, size_t err_len) {
  using namespace psgspec;
  if (!text || !out) {
    put(err, err_len, "null argument");
    return PSG_EINVAL;
  }
  std::memset(out, 0, sizeof(*out));
  std::string path, msg;
  try {
    load_options();
    ParsedSpec P = parse_spec(text);
    const Compiled prog = compile_program(P, alg);
    const std::string s = module_source(P, prog, alg, fused != 0, n);
    const int rc = compile_module(s, alg, fused != 0, cache_dir, path, msg);
    if (rc) {
      put(err, err_len, msg);
      return rc;
    }
    const int frc = fill_program(prog, alg, out, names, names_len, err, err_len);
    if (frc) return frc;
  } catch (const std::exception& e) {
    put(err, err_len, e.what());
    return PSG_EINVAL;
  } catch (...) {
    put(err, err_len, "native spec: internal error");
    return PSG_EIO;
  }
  std::lock_guard<std::mutex> lk(g_paths_mu);
  out->module_path = interned().insert(path).first->c_str();
  return PSG_OK;
}

}  // extern "C"
