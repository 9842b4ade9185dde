// psg_spec_ir.hpp — the expression IR of a Spec given as Formula text (= round_amd/formula.py
// Expr), shared by the bytecode compiler (psg_spec_text.cpp, psg_spec_from_text) and the
// native generator (psg_spec_gen.cpp, psg_spec_compile_native). Host C++ only.
#pragma once
#include <cstdint>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/psg.h"

namespace psgspec {

struct SpecError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ expression IR (= formula.py Expr)
enum Kind { LIT, NV, RV, COORDV, VAR, FIELD, UN, BIN, QUANT, CONTAINS };
enum QK { QFORALL, QEXISTS, QCOUNT, QVINT, QVBOOL };
struct Node {
  Kind k;
  int32_t v = 0;       // LIT value
  int op = 0;          // UN / BIN opcode (enum psg_op)
  int f = 0, tag = 0;  // FIELD
  int uid = -1;        // VAR uid; QUANT / CONTAINS bound variable uid
  int qk = 0;          // QUANT kind
  int a = -1, b = -1;  // children: FIELD proc=a; UN x=a; BIN x=a y=b; QUANT body=a; CONTAINS elem=a, set body=b
};
struct Comp {  // a set of processes {var. body}
  int var, body;
};

struct Tree {
  std::vector<Node> nodes;
  int next_uid = 0;
  int add(Node n) {
    nodes.push_back(n);
    return (int)nodes.size() - 1;
  }
  int lit(int32_t v) { Node n{LIT}; n.v = v; return add(n); }
  int bin(int op, int x, int y) { Node n{BIN}; n.op = op; n.a = x; n.b = y; return add(n); }
  int un(int op, int x) { Node n{UN}; n.op = op; n.a = x; return add(n); }
  int quant(int kind, int var, int body) { Node n{QUANT}; n.qk = kind; n.uid = var; n.a = body; return add(n); }
  int var(int uid) { Node n{VAR}; n.uid = uid; return add(n); }
  // children in formula.py's Expr.children() order
  void children(int e, std::vector<int>& out) const {
    const Node& n = nodes[e];
    switch (n.k) {
      case FIELD: case UN: case QUANT: out.push_back(n.a); break;
      case BIN: case CONTAINS: out.push_back(n.a); out.push_back(n.b); break;
      default: break;
    }
  }
  void walk(int e, std::vector<int>& out) const {  // pre-order (formula.py _walk)
    out.push_back(e);
    std::vector<int> ch;
    children(e, ch);
    for (int c : ch) walk(c, out);
  }
  void free_vars(int e, std::set<int>& bound, std::set<int>& out) const {
    const Node& n = nodes[e];
    if (n.k == VAR) {
      if (!bound.count(n.uid)) out.insert(n.uid);
      return;
    }
    if (n.k == QUANT || n.k == CONTAINS) {
      if (n.k == CONTAINS) free_vars(n.a, bound, out);
      const int body = n.k == QUANT ? n.a : n.b;
      const bool added = bound.insert(n.uid).second;
      free_vars(body, bound, out);
      if (added) bound.erase(n.uid);
      return;
    }
    std::vector<int> ch;
    children(e, ch);
    for (int c : ch) free_vars(c, bound, out);
  }
};

// A parsed Spec: invariants already guarded by the round invariants (Verifier.scala:133-141),
// properties in text order (Termination included), the safety predicate (-1: none).
struct ParsedSpec {
  Tree T;
  int phase = 1;
  std::vector<int> invs;
  std::vector<std::pair<std::string, int>> props;
  int sp = -1;
};

// The bytecode program of a parsed Spec (= formula.py compile_spec).
struct Compiled {
  std::vector<int32_t> code, entry, flags;
  int32_t term = -1, nvars = 0;
  std::vector<std::string> names;
};

ParsedSpec parse_spec(const char* text);
Compiled compile_program(ParsedSpec& P, int alg);
std::set<int> alg_fields(int alg);
// Candidate sources of V.exists(v => body) (node e): every term v is compared with
void witnesses(const Tree& T, int e, std::vector<int>& exprs, std::vector<std::pair<int, int>>& fsets);
bool uses_old(const Tree& T, int e);
void put(char* buf, size_t len, const std::string& s);
// The program's arrays (malloc, released by psg_spec_release), names '\n'-separated
int fill_program(const Compiled& c, int alg, psg_spec_program* out, char* names, size_t names_len, char* err,
                 size_t err_len);

}  // namespace psgspec
