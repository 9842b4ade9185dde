// psg_spec_text.cpp — psg_spec_from_text: a Spec given as Formula text (the
// S-expression form of the reference's own Formula trees, psync/formula/Formula.scala:
// Binding ForAll / Exists / Comprehension, Application, Variable, Literal; format in
// round_amd/formula.py "Formula text") compiled to the psg_spec_program bytecode that
// psg_run_batch_spec evaluates. This is the JVM plugin's path to generic Specs
// (integration/scala/GpuSpec.scala writes the text from a psync.Spec): host C++,
// no GPU needed. The lowering and the code it emits are the same as
// round_amd/formula.py compile_spec (tests/test_spec_text.py checks them word for
// word); slot assembly follows psync/verification/Verifier.scala:111-141 (Safety = some
// invariant, invariant i guarded by roundInvariants(j-1)(0), properties, Termination
// as a round, SafetyPredicate).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/psg.h"
#include "psg_spec_ir.hpp"

namespace psgspec {
namespace {

// ------------------------------------------------------------------ S-expressions
struct Sx {
  bool atom = false;
  bool str = false;
  std::string tok;
  std::vector<Sx> items;
  bool is(const char* h) const { return !atom && !items.empty() && items[0].atom && items[0].tok == h; }
  const Sx& at(size_t k) const {
    if (atom || k >= items.size()) throw SpecError("Formula text: malformed form");
    return items[k];
  }
  const std::string& name() const {
    if (!atom) throw SpecError("Formula text: expected a name");
    return tok;
  }
};

struct Reader {
  const char* p;
  int depth = 0;  // nesting of the form being read: deep text must not overflow the native stack
  static constexpr int kMaxDepth = 512;
  void skip() {
    while (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r') ++p;
  }
  Sx read() {
    skip();
    Sx s;
    if (!*p) throw SpecError("Formula text: unexpected end");
    if (*p == '(') {
      if (++depth > kMaxDepth) throw SpecError("Formula text: nesting deeper than 512 forms");
      ++p;
      for (;;) {
        skip();
        if (!*p) throw SpecError("Formula text: missing )");
        if (*p == ')') {
          ++p;
          --depth;
          return s;
        }
        s.items.push_back(read());
      }
    }
    if (*p == ')') throw SpecError("Formula text: unexpected )");
    s.atom = true;
    if (*p == '"') {
      const char* q = std::strchr(p + 1, '"');
      if (!q) throw SpecError("Formula text: unterminated string");
      s.str = true;
      s.tok.assign(p + 1, q);
      p = q + 1;
      return s;
    }
    const char* q = p;
    while (*q && *q != ' ' && *q != '\n' && *q != '\t' && *q != '\r' && *q != '(' && *q != ')' && *q != '"') ++q;
    s.tok.assign(p, q);
    p = q;
    return s;
  }
};

const std::map<std::string, int>& field_names() {
  static const std::map<std::string, int> m = {
      {"x", PSG_FIELD_X}, {"decided", PSG_FIELD_DECIDED}, {"decision", PSG_FIELD_DECISION}, {"ts", PSG_FIELD_TS},
      {"ready", PSG_FIELD_READY}, {"commit", PSG_FIELD_COMMIT}, {"vote", PSG_FIELD_VOTE},
      {"canDecide", PSG_FIELD_CANDECIDE}, {"est", PSG_FIELD_X}};
  return m;
}
const std::map<std::string, int>& bin_names() {
  static const std::map<std::string, int> m = {
      {"And", PSG_OP_AND}, {"Or", PSG_OP_OR}, {"Implies", PSG_OP_IMPL}, {"Eq", PSG_OP_EQ}, {"Neq", PSG_OP_NE},
      {"Lt", PSG_OP_LT}, {"Leq", PSG_OP_LE}, {"Gt", PSG_OP_GT}, {"Geq", PSG_OP_GE}, {"Plus", PSG_OP_ADD},
      {"Minus", PSG_OP_SUB}, {"Times", PSG_OP_MUL}, {"Divides", PSG_OP_DIV}, {"Remainder", PSG_OP_MOD}};
  return m;
}

// ------------------------------------------------------------------ text -> IR (= formula.py _from_sexp)
struct Lower {
  Tree& T;
  struct Binding {
    bool is_set;
    int uid;  // VAR uid
    Comp comp;
  };
  using Env = std::map<std::string, Binding>;

  int expr(const Sx& s, const Env& env) {
    if (s.atom || s.items.empty() || !s.items[0].atom) throw SpecError("Formula text: expected a form");
    const std::string& h = s.items[0].tok;
    if (h == "Lit") {
      const std::string& v = s.at(1).name();
      if (v == "true") return T.lit(1);
      if (v == "false") return T.lit(0);
      char* end = nullptr;
      const long long x = std::strtoll(v.c_str(), &end, 10);
      if (!end || *end || x < INT32_MIN || x > INT32_MAX) throw SpecError("Formula text: literal " + v + " is not an Int");
      return T.lit((int32_t)x);
    }
    if (h == "Var") {
      const std::string& nm = s.at(1).name();
      auto it = env.find(nm);
      if (it != env.end()) {
        if (it->second.is_set) throw SpecError("Formula text: set " + nm + " used as a value");
        return T.var(it->second.uid);
      }
      if (nm == "n") return T.add(Node{NV});
      if (nm == "r") return T.add(Node{RV});
      if (nm == "coord") return T.add(Node{COORDV});
      throw SpecError("Formula text: unbound variable " + nm);
    }
    if (h == "ForAll" || h == "Exists") {
      const Sx& decls = s.at(1);
      if (decls.atom || decls.items.empty()) throw SpecError("Formula text: binder without variables");
      return binder(h == "ForAll", decls, 0, s.at(2), env);
    }
    if (h == "Comprehension") throw SpecError("Formula text: a set is only used under Cardinality / In / Contains");
    if (h != "App") throw SpecError("Formula text: unknown form " + h);
    const std::string& sym = s.at(1).name();
    const size_t na = s.items.size() - 2;
    auto arg = [&](size_t k) { return expr(s.at(2 + k), env); };
    if (sym == "And" || sym == "Or") {
      if (na < 1) throw SpecError("Formula text: empty " + sym);
      std::vector<int> xs;
      for (size_t k = 0; k < na; ++k) xs.push_back(arg(k));
      return fold(sym == "And" ? PSG_OP_AND : PSG_OP_OR, xs, 0, xs.size());
    }
    auto bn = bin_names().find(sym);
    if (bn != bin_names().end()) {
      if (sym == "Minus" && na == 1) return T.un(PSG_OP_NEG, arg(0));
      if (na != 2) throw SpecError("Formula text: " + sym + " takes two arguments");
      const int x = arg(0);
      return T.bin(bn->second, x, arg(1));
    }
    if (sym == "Not" && na == 1) return T.un(PSG_OP_NOT, arg(0));
    if (sym == "IsDefined" && na == 1) return T.un(PSG_OP_ISDEF, arg(0));
    if (sym == "IsEmpty" && na == 1) return T.un(PSG_OP_NOT, T.un(PSG_OP_ISDEF, arg(0)));
    // Option get / Some; Time <-> Int conversions of psync.logic.ReduceTime (identities here)
    if ((sym == "Get" || sym == "Some" || sym == "toInt" || sym == "fromInt") && na == 1) return arg(0);
    if (sym == "Cardinality" && na == 1) {
      const Sx& x = s.at(2);
      if (x.is("App") && x.items.size() == 3 && x.at(1).atom && x.at(1).tok == "HO") {
        Node n{FIELD};
        n.f = PSG_FIELD_HOSIZE;
        n.a = expr(x.at(2), env);
        return T.add(n);
      }
      const Comp c = set(x, env);
      return T.quant(QCOUNT, c.var, c.body);
    }
    if ((sym == "In" || sym == "Contains") && na == 2) {
      const Sx& elem = sym == "In" ? s.at(2) : s.at(3);
      const Sx& st = sym == "In" ? s.at(3) : s.at(2);
      const Comp c = set(st, env);
      Node n{CONTAINS};
      n.a = expr(elem, env);
      n.uid = c.var;
      n.b = c.body;
      return T.add(n);
    }
    if (sym == "coord" && na == 0) return T.add(Node{COORDV});
    int tag = PSG_TAG_CUR;
    std::string base = sym;
    if (sym.rfind("__init__", 0) == 0) {
      tag = PSG_TAG_INIT;
      base = sym.substr(8);
    } else if (sym.rfind("__old__", 0) == 0) {
      tag = PSG_TAG_OLD;
      base = sym.substr(7);
    }
    auto fn = field_names().find(base);
    if (fn != field_names().end() && na == 1) {
      Node n{FIELD};
      n.f = fn->second;
      n.tag = tag;
      n.a = arg(0);
      return T.add(n);
    }
    throw SpecError("Formula text: unknown symbol " + sym + "/" + std::to_string(na));
  }

  // An n-ary And / Or: left-deep (the DSL's `a & b & c` shape) up to kLeftFold arguments,
  // halves folded recursively above that, so a wide conjunction stays shallow (depth
  // kLeftFold + log2(arity)) for the recursive lowering and generator passes
  static constexpr size_t kLeftFold = 32;
  int fold(int op, const std::vector<int>& xs, size_t lo, size_t hi) {
    if (hi - lo > kLeftFold) {
      const size_t mid = lo + (hi - lo) / 2;
      const int x = fold(op, xs, lo, mid);
      return T.bin(op, x, fold(op, xs, mid, hi));
    }
    int out = xs[lo];
    for (size_t k = lo + 1; k < hi; ++k) out = T.bin(op, out, xs[k]);
    return out;
  }

  int binder(bool forall, const Sx& decls, size_t k, const Sx& body, const Env& env) {
    const Sx& d = decls.at(k);
    const std::string& nm = d.at(0).name();
    const std::string& typ = d.at(1).name();
    const bool last = k + 1 == decls.items.size();
    auto inner = [&](const Env& e2) { return last ? expr(body, e2) : binder(forall, decls, k + 1, body, e2); };
    if (typ == "Set") {
      if (forall) throw SpecError("Formula text: a Set variable is only bound by a let (Exists)");
      if (!last) throw SpecError("Formula text: a let binds one Set variable");
      return let(nm, body, env);
    }
    const int uid = T.next_uid++;
    Env e2 = env;
    e2[nm] = Binding{false, uid, {}};
    if (typ == "pid") return T.quant(forall ? QFORALL : QEXISTS, uid, inner(e2));
    if (forall) throw SpecError("Formula text: ForAll over " + typ + " cannot be checked (only V.exists)");
    if (typ != "Int" && typ != "Time" && typ != "Bool") throw SpecError("Formula text: unknown type " + typ);
    return T.quant(typ == "Bool" ? QVBOOL : QVINT, uid, inner(e2));
  }

  Comp comp(const Sx& s, const Env& env) {
    const Sx& decls = s.at(1);
    if (decls.atom || decls.items.size() != 1 || decls.at(0).at(1).name() != "pid")
      throw SpecError("Formula text: comprehensions range over one process variable");
    const int uid = T.next_uid++;
    Env e2 = env;
    e2[decls.at(0).at(0).name()] = Binding{false, uid, {}};
    return Comp{uid, expr(s.at(2), e2)};
  }

  Comp set(const Sx& s, const Env& env) {
    if (s.is("Comprehension")) return comp(s, env);
    if (s.is("Var")) {
      auto it = env.find(s.at(1).name());
      if (it != env.end() && it->second.is_set) return it->second.comp;
    }
    throw SpecError("Formula text: expected a set of processes");
  }

  // Exists A: Set. A == {..} && rest  ->  rest with A := {..} (FormulaExtractor's `val A = ...`)
  int let(const std::string& nm, const Sx& body, const Env& env) {
    std::vector<const Sx*> conj;
    std::vector<const Sx*> stack{&body};
    // flatten nested Ands left to right
    struct F {
      static void flat(const Sx& x, std::vector<const Sx*>& out) {
        if (x.is("App") && x.items.size() >= 3 && x.at(1).atom && x.at(1).tok == "And") {
          for (size_t k = 2; k < x.items.size(); ++k) flat(x.items[k], out);
        } else {
          out.push_back(&x);
        }
      }
    };
    F::flat(body, conj);
    for (size_t k = 0; k < conj.size(); ++k) {
      const Sx& c = *conj[k];
      if (!(c.is("App") && c.items.size() == 4 && c.at(1).atom && c.at(1).tok == "Eq")) continue;
      for (int side = 0; side < 2; ++side) {
        const Sx& lhs = c.at(side ? 3 : 2);
        const Sx& rhs = c.at(side ? 2 : 3);
        if (lhs.is("Var") && lhs.at(1).atom && lhs.at(1).tok == nm && rhs.is("Comprehension")) {
          Env e2 = env;
          e2[nm] = Binding{true, -1, comp(rhs, env)};
          std::vector<const Sx*> rest;
          for (size_t j = 0; j < conj.size(); ++j)
            if (j != k) rest.push_back(conj[j]);
          if (rest.empty()) return T.lit(1);
          std::vector<int> xs;
          for (const Sx* x : rest) xs.push_back(expr(*x, e2));
          return fold(PSG_OP_AND, xs, 0, xs.size());
        }
      }
    }
    throw SpecError("Formula text: Set variable " + nm + " is not defined by a conjunct " + nm + " == {...}");
  }
};

// ------------------------------------------------------------------ IR -> bytecode (= formula.py _Compiler)
int32_t word(int op, int a = 0, int b = 0) {
  if (b < -(1 << 15) || b >= (1 << 15)) throw SpecError("immediate out of range");
  return (int32_t)((uint32_t)(op & 0xFF) | ((uint32_t)(a & 0xFF) << 8) | ((uint32_t)(b & 0xFFFF) << 16));
}

}  // namespace

std::set<int> alg_fields(int alg) {
  using S = std::set<int>;
  switch (alg) {
    case PSG_ALG_OTR: case PSG_ALG_OTR2: case PSG_ALG_FLOODMIN: case PSG_ALG_KSET: case PSG_ALG_KSET_ES:
      return S{PSG_FIELD_X, PSG_FIELD_DECIDED, PSG_FIELD_DECISION, PSG_FIELD_HOSIZE};
    case PSG_ALG_LAST_VOTING:
      return S{PSG_FIELD_X, PSG_FIELD_DECIDED, PSG_FIELD_DECISION, PSG_FIELD_TS, PSG_FIELD_READY, PSG_FIELD_COMMIT,
               PSG_FIELD_VOTE, PSG_FIELD_HOSIZE};
    case PSG_ALG_BENOR:
      return S{PSG_FIELD_X, PSG_FIELD_DECIDED, PSG_FIELD_DECISION, PSG_FIELD_CANDECIDE, PSG_FIELD_VOTE,
               PSG_FIELD_HOSIZE};
    case PSG_ALG_SLV:
      return S{PSG_FIELD_X, PSG_FIELD_DECIDED, PSG_FIELD_DECISION, PSG_FIELD_TS, PSG_FIELD_COMMIT, PSG_FIELD_VOTE,
               PSG_FIELD_HOSIZE};
  }
  throw SpecError("algorithm " + std::to_string(alg) + " has no integer state to check");
}

// (= formula.py _Compiler.witnesses)
void witnesses(const Tree& T, int e, std::vector<int>& exprs, std::vector<std::pair<int, int>>& fsets) {
  const Node& q = T.nodes[e];
  const int v = q.uid;
  std::vector<int> w;
  T.walk(q.a, w);
  std::set<int> inner;
  for (int x : w)
    if (T.nodes[x].k == QUANT || T.nodes[x].k == CONTAINS) inner.insert(T.nodes[x].uid);
  bool seen = false;
  for (int x : w) {
    const Node& b = T.nodes[x];
    if (b.k != BIN || b.op < PSG_OP_EQ || b.op > PSG_OP_GE) continue;
    const int pairs[2][2] = {{b.a, b.b}, {b.b, b.a}};
    for (auto& pr : pairs) {
      const Node& a = T.nodes[pr[0]];
      if (a.k != VAR || a.uid != v) continue;
      std::set<int> bound, fv;
      T.free_vars(pr[1], bound, fv);
      if (fv.count(v)) throw SpecError("V.exists variable compared with a term containing itself");
      const Node& t = T.nodes[pr[1]];
      if (t.k == FIELD) {
        const std::pair<int, int> key{t.f, t.tag};
        bool have = false;
        for (auto& k : fsets) have = have || k == key;
        if (!have) fsets.push_back(key);
      } else {
        bool dep = false;
        for (int u : fv) dep = dep || inner.count(u);
        if (dep) throw SpecError("V.exists witness term depends on an inner bound variable and is not a process field");
        exprs.push_back(pr[1]);
      }
      seen = true;
    }
  }
  for (int x : w)
    if (T.nodes[x].k == VAR && T.nodes[x].uid == v && !seen)
      throw SpecError("a V.exists variable may only appear directly in comparisons");
}

bool uses_old(const Tree& T, int e) {
  std::vector<int> w;
  T.walk(e, w);
  for (int x : w)
    if (T.nodes[x].k == FIELD && T.nodes[x].tag == PSG_TAG_OLD) return true;
  return false;
}

namespace {

struct Compiler {
  const Tree& T;
  bool restrict_fields;
  std::set<int> fields_available;
  std::vector<int32_t> code;
  std::map<int, int> slot_of;
  int max_slot = -1;

  int emit(int32_t w) {
    code.push_back(w);
    return (int)code.size() - 1;
  }
  int bind(int uid, int depth) {
    if (depth >= 16) throw SpecError("more than 16 nested bound variables");
    slot_of[uid] = depth;
    max_slot = std::max(max_slot, depth);
    return depth;
  }
  void expr(int e, int depth, bool in_lane) {
    const Node& n = T.nodes[e];
    switch (n.k) {
      case LIT:
        if (n.v >= -(1 << 15) && n.v < (1 << 15)) {
          emit(word(PSG_OP_IMM, 0, n.v));
        } else {
          emit(word(PSG_OP_IMM32));
          emit(n.v);
        }
        break;
      case NV: emit(word(PSG_OP_N)); break;
      case RV: emit(word(PSG_OP_R)); break;
      case COORDV: emit(word(PSG_OP_COORD)); break;
      case VAR: {
        auto it = slot_of.find(n.uid);
        if (it == slot_of.end()) throw SpecError("variable used outside its quantifier");
        emit(word(PSG_OP_VAR, it->second));
        break;
      }
      case FIELD:
        if (restrict_fields && !fields_available.count(n.f))
          throw SpecError("field " + std::to_string(n.f) + " is not part of this algorithm's state");
        expr(n.a, depth, in_lane);
        emit(word(PSG_OP_FIELD, n.f, n.tag));
        break;
      case UN:
        expr(n.a, depth, in_lane);
        emit(word(n.op));
        break;
      case BIN:
        expr(n.a, depth, in_lane);
        expr(n.b, depth, in_lane);
        emit(word(n.op));
        break;
      case CONTAINS: {
        expr(n.a, depth, in_lane);
        const int slot = bind(n.uid, depth);
        emit(word(PSG_OP_BIND, slot));
        expr(n.b, depth + 1, in_lane);
        break;
      }
      case QUANT: quant(e, depth, in_lane); break;
    }
  }
  void quant(int e, int depth, bool in_lane) {
    const Node& q = T.nodes[e];
    const int slot = bind(q.uid, depth);
    bool lane_form = false;
    int32_t head;
    std::vector<int> exprs;
    std::vector<std::pair<int, int>> fsets;
    if (q.qk == QFORALL || q.qk == QEXISTS || q.qk == QCOUNT) {
      lane_form = !in_lane;
      const int base = q.qk == QFORALL ? PSG_Q_FORALL_P : (q.qk == QEXISTS ? PSG_Q_EXISTS_P : PSG_Q_COUNT_P);
      head = word(PSG_OP_QBEGIN, lane_form ? base + 3 : base, slot);
    } else if (q.qk == QVBOOL) {
      head = word(PSG_OP_QBEGIN, PSG_Q_EXISTS_VB, slot);
    } else {
      witnesses(T, e, exprs, fsets);
      for (int t : exprs) expr(t, depth, in_lane);
      head = word(PSG_OP_QBEGIN, PSG_Q_EXISTS_VI, slot);
    }
    emit(head);
    const int end_at = emit(0);
    if (q.qk == QVINT) {
      emit((int32_t)(exprs.size() | (fsets.size() << 16)));
      for (auto& ft : fsets) emit(ft.first | (ft.second << 8));
    }
    expr(q.a, depth + 1, in_lane || lane_form);
    const int end = emit(word(PSG_OP_QEND));
    code[end_at] = end;
  }
  int root(int e) {
    const int at = (int)code.size();
    expr(e, 0, false);
    emit(word(PSG_OP_HALT));
    return at;
  }
};

}  // namespace

static constexpr int kMaxTreeDepth = 1024;

ParsedSpec parse_spec(const char* text) {
  Reader rd{text};
  const Sx s = rd.read();
  rd.skip();
  if (*rd.p) throw SpecError("Formula text: trailing input");
  if (!s.is("Spec")) throw SpecError("Formula text: expected (Spec ...)");
  ParsedSpec P;
  Tree& T = P.T;
  Lower L{T};
  int& phase = P.phase;
  std::vector<int>& invs = P.invs;
  std::vector<std::vector<int>> rinv;
  std::vector<std::pair<std::string, int>>& props = P.props;
  int& sp = P.sp;
  const Lower::Env env;
  for (size_t k = 1; k < s.items.size(); ++k) {
    const Sx& part = s.items[k];
    const std::string& key = part.at(0).name();
    if (key == "phase") {
      phase = std::atoi(part.at(1).name().c_str());
      if (phase < 1) throw SpecError("Formula text: phase length must be >= 1");
    } else if (key == "invariants") {
      for (size_t j = 1; j < part.items.size(); ++j) invs.push_back(L.expr(part.items[j], env));
    } else if (key == "roundInvariants") {
      for (size_t j = 1; j < part.items.size(); ++j) {
        std::vector<int> l;
        for (size_t m = 1; m < part.items[j].items.size(); ++m) l.push_back(L.expr(part.items[j].items[m], env));
        rinv.push_back(l);
      }
    } else if (key == "properties") {
      for (size_t j = 1; j < part.items.size(); ++j) {
        const Sx& p = part.items[j];
        if (!p.is("prop") || !p.at(1).str) throw SpecError("Formula text: expected (prop \"Name\" f)");
        props.emplace_back(p.at(1).tok, L.expr(p.at(2), env));
      }
    } else if (key == "safetyPredicate") {
      sp = L.expr(part.at(1), env);
    } else {
      throw SpecError("Formula text: unknown Spec part " + key);
    }
  }
  // (r % L == j) ==> roundInvariants(j-1)(0) for j = 1..L-1 (Verifier.scala:133-141)
  int guard = -1;
  for (int j = 1; j < phase; ++j) {
    if (j - 1 < (int)rinv.size() && !rinv[j - 1].empty()) {
      const int cond = T.bin(PSG_OP_EQ, T.bin(PSG_OP_MOD, T.add(Node{RV}), T.lit(phase)), T.lit(j));
      const int part = T.bin(PSG_OP_IMPL, cond, rinv[j - 1][0]);
      guard = guard < 0 ? part : T.bin(PSG_OP_AND, guard, part);
    }
  }
  if (guard >= 0)
    for (int& inv : invs) inv = T.bin(PSG_OP_AND, inv, guard);
  // The lowering and the native generator recurse over the tree: bound its depth (children
  // precede their parents in T.nodes, so one pass in index order computes every depth)
  std::vector<int> depth(T.nodes.size(), 1);
  for (size_t e = 0; e < T.nodes.size(); ++e) {
    std::vector<int> ch;
    T.children((int)e, ch);
    for (int c : ch) depth[e] = std::max(depth[e], depth[c] + 1);
    if (depth[e] > kMaxTreeDepth)
      throw SpecError("Formula text: expression tree deeper than " + std::to_string(kMaxTreeDepth));
  }
  return P;
}

Compiled compile_program(ParsedSpec& P, int alg) {
  Tree& T = P.T;
  const std::vector<int>& invs = P.invs;
  const int sp = P.sp;
  Compiler C{T, alg != 0, alg != 0 ? alg_fields(alg) : std::set<int>{}};
  Compiled out;
  if (!invs.empty()) {
    int any = invs[0];
    for (size_t k = 1; k < invs.size(); ++k) any = T.bin(PSG_OP_OR, any, invs[k]);
    out.names.push_back("Safety");
    out.entry.push_back(C.root(any));
    out.flags.push_back(0);
    for (size_t k = 0; k < invs.size(); ++k) {
      out.names.push_back("Invariant" + std::to_string(k));
      out.entry.push_back(C.root(invs[k]));
      out.flags.push_back(0);
    }
  }
  for (auto& p : P.props) {
    if (p.first == "Termination") {
      out.term = C.root(p.second);
      continue;
    }
    out.names.push_back(p.first);
    out.entry.push_back(C.root(p.second));
    out.flags.push_back(uses_old(T, p.second) ? PSG_SPEC_RELATIONAL : 0);
  }
  if (sp >= 0) {
    out.names.push_back("SafetyPredicate");
    out.entry.push_back(C.root(sp));
    out.flags.push_back(uses_old(T, sp) ? PSG_SPEC_RELATIONAL : 0);
  }
  if (out.entry.empty()) throw SpecError("a Spec needs at least one invariant, property or safety predicate");
  if (out.entry.size() > PSG_MAX_CHECKS) throw SpecError("more than 12 check slots");
  out.code = std::move(C.code);
  out.nvars = C.max_slot + 1;
  return out;
}

void put(char* buf, size_t len, const std::string& s) {
  if (!buf || !len) return;
  const size_t k = std::min(len - 1, s.size());
  std::memcpy(buf, s.data(), k);
  buf[k] = 0;
}

int fill_program(const Compiled& c, int alg, psg_spec_program* out, char* names, size_t names_len, char* err,
                 size_t err_len) {
  std::string joined;
  for (size_t k = 0; k < c.names.size(); ++k) joined += (k ? "\n" : "") + c.names[k];
  if (names && names_len <= joined.size()) {  // never a silently truncated slot-name list
    put(err, err_len, "names buffer too small: " + std::to_string(joined.size() + 1) + " bytes needed");
    return PSG_ERANGE;
  }
  int32_t* code = (int32_t*)std::malloc(sizeof(int32_t) * c.code.size());
  int32_t* ent = (int32_t*)std::malloc(sizeof(int32_t) * c.entry.size());
  int32_t* flg = (int32_t*)std::malloc(sizeof(int32_t) * c.flags.size());
  if (!code || !ent || !flg) {
    std::free(code);
    std::free(ent);
    std::free(flg);
    put(err, err_len, "out of host memory");
    return PSG_ENOMEM;
  }
  std::memcpy(code, c.code.data(), sizeof(int32_t) * c.code.size());
  std::memcpy(ent, c.entry.data(), sizeof(int32_t) * c.entry.size());
  std::memcpy(flg, c.flags.data(), sizeof(int32_t) * c.flags.size());
  out->n_slots = (int32_t)c.entry.size();
  out->n_words = (int32_t)c.code.size();
  out->code = code;
  out->slot_entry = ent;
  out->slot_flags = flg;
  out->term_entry = c.term;
  out->n_vars = c.nvars;
  out->module_path = nullptr;
  out->alg = alg;
  put(names, names_len, joined);
  put(err, err_len, "");
  return PSG_OK;
}

}  // namespace psgspec

extern "C" {

int psg_spec_from_text(const char* text, int32_t alg, psg_spec_program* out, char* names, size_t names_len,
                       char* err, size_t err_len) {
  using namespace psgspec;
  if (!text || !out) {
    put(err, err_len, "null argument");
    return PSG_EINVAL;
  }
  std::memset(out, 0, sizeof(*out));
  try {
    ParsedSpec P = parse_spec(text);
    return fill_program(compile_program(P, alg), alg, out, names, names_len, err, err_len);
  } catch (const std::exception& e) {
    put(err, err_len, e.what());
    return PSG_EINVAL;
  } catch (...) {
    put(err, err_len, "Formula text: internal error");
    return PSG_EIO;
  }
}

void psg_spec_release(psg_spec_program* prog) {
  if (!prog) return;
  std::free(const_cast<int32_t*>(prog->code));
  std::free(const_cast<int32_t*>(prog->slot_entry));
  std::free(const_cast<int32_t*>(prog->slot_flags));
  std::memset(prog, 0, sizeof(*prog));
}

}  // extern "C"
