"""Spec formulas for the GPU checker: a Python mirror of the reference's Spec DSL
and its compiler to the device bytecode (include/psg.h, psg_run_batch_spec).

The reference writes a Spec as Scala expressions over the process state that the
`Formula` macros (psync/macros/FormulaExtractor.scala:219-520) turn into a
`Formula` tree (psync/formula/Formula.scala: ForAll / Exists / Comprehension /
Cardinality, `init(...)` / `old(...)`, Option `isDefined` / `get`). The same
specs read almost verbatim here, e.g. OTR's first invariant
(example/Otr.scala:99-105):

    ( P.forall(lambda i: ~i.decided)
      | V.exists(lambda v: (P.filter(lambda i: i.x == v).size > 2 * n // 3)
                           & P.forall(lambda i: i.decided.implies(i.decision == v))) )
    & P.forall(lambda i: P.exists(lambda j1: i.x == init(j1.x)))

Python operators: `&` `|` `~` for && || !, `.implies(b)` for ==>, `//` and `%`
for Int division / remainder, comparisons as usual. `compile_spec` assembles the
check slots exactly as the built-in checker does (psync/verification/
Verifier.scala:111-141): slot "Safety" = some invariant holds, invariant i at
check point r is `invariants(i) && (r % L != 0 ==> roundInvariants(r%L - 1)(0))`,
then the properties ("Termination" becomes the termination round), then
"SafetyPredicate" if the spec has one.
"""
from __future__ import annotations

import ctypes as C
import itertools
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from . import abi

# --------------------------------------------------------------------------- ABI constants (include/psg.h)
FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_TS, FIELD_READY, FIELD_COMMIT, FIELD_VOTE, FIELD_CANDECIDE, \
    FIELD_HOSIZE = range(9)
TAG_CUR, TAG_OLD, TAG_INIT = range(3)
NONE32 = -(1 << 31)

OP = dict(HALT=0, IMM=1, IMM32=2, N=3, R=4, VAR=5, FIELD=6, NOT=7, NEG=8, ISDEF=9, AND=10, OR=11, IMPL=12,
          EQ=13, NE=14, LT=15, LE=16, GT=17, GE=18, ADD=19, SUB=20, MUL=21, DIV=22, MOD=23, BIND=24,
          QBEGIN=25, QEND=26, COORD=27)
Q_FORALL_P, Q_EXISTS_P, Q_COUNT_P, Q_FORALL_PL, Q_EXISTS_PL, Q_COUNT_PL, Q_EXISTS_VB, Q_EXISTS_VI = range(8)
SPEC_RELATIONAL = 1
MAX_VARS = 16

# fields each algorithm's kernels trace (the rest read as 0)
ALG_FIELDS = {
    abi.PSG_ALG_OTR: {FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_HOSIZE},
    abi.PSG_ALG_OTR2: {FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_HOSIZE},
    abi.PSG_ALG_LAST_VOTING: {FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_TS, FIELD_READY, FIELD_COMMIT,
                              FIELD_VOTE, FIELD_HOSIZE},
    abi.PSG_ALG_FLOODMIN: {FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_HOSIZE},
    abi.PSG_ALG_KSET: {FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_HOSIZE},
    abi.PSG_ALG_BENOR: {FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_CANDECIDE, FIELD_VOTE, FIELD_HOSIZE},
    abi.PSG_ALG_SLV: {FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_TS, FIELD_COMMIT, FIELD_VOTE, FIELD_HOSIZE},
    abi.PSG_ALG_KSET_ES: {FIELD_X, FIELD_DECIDED, FIELD_DECISION, FIELD_HOSIZE},
}


class FormulaError(ValueError):
    pass


# --------------------------------------------------------------------------- expression tree
class Expr:
    """A Formula node. Operators build new nodes (they never evaluate)."""

    def _bin(self, op, other, swap=False):
        other = lift(other)
        return Bin(op, other, self) if swap else Bin(op, self, other)

    def __and__(self, o): return self._bin("AND", o)
    def __rand__(self, o): return self._bin("AND", o, True)
    def __or__(self, o): return self._bin("OR", o)
    def __ror__(self, o): return self._bin("OR", o, True)
    def __invert__(self): return Un("NOT", self)
    def __neg__(self): return Un("NEG", self)
    def __eq__(self, o): return self._bin("EQ", o)  # noqa: PLE0307 (builds a node)
    def __ne__(self, o): return self._bin("NE", o)
    def __lt__(self, o): return self._bin("LT", o)
    def __le__(self, o): return self._bin("LE", o)
    def __gt__(self, o): return self._bin("GT", o)
    def __ge__(self, o): return self._bin("GE", o)
    def __add__(self, o): return self._bin("ADD", o)
    def __radd__(self, o): return self._bin("ADD", o, True)
    def __sub__(self, o): return self._bin("SUB", o)
    def __rsub__(self, o): return self._bin("SUB", o, True)
    def __mul__(self, o): return self._bin("MUL", o)
    def __rmul__(self, o): return self._bin("MUL", o, True)
    def __floordiv__(self, o): return self._bin("DIV", o)  # Scala Int `/` (truncates)
    def __rfloordiv__(self, o): return self._bin("DIV", o, True)
    def __mod__(self, o): return self._bin("MOD", o)
    def __rmod__(self, o): return self._bin("MOD", o, True)
    __hash__ = object.__hash__

    def implies(self, o):
        """`a ==> b`."""
        return self._bin("IMPL", o)

    def __bool__(self):
        raise FormulaError("a Formula has no truth value in Python: use & | ~ and .implies(), not and/or/not")

    # Option[_] accessors (FormulaExtractor: isDefined / isEmpty / get)
    @property
    def isDefined(self): return Un("ISDEF", self)
    @property
    def isEmpty(self): return Un("NOT", Un("ISDEF", self))
    @property
    def get(self): return self

    def children(self):
        return ()


class Lit(Expr):
    def __init__(self, v):
        if isinstance(v, bool):
            v = int(v)
        if not (-(1 << 31) <= int(v) < (1 << 31)):
            raise FormulaError(f"literal {v} is not an Int")
        self.v = int(v)


class NVal(Expr):
    pass


class RVal(Expr):
    pass


class Var(Expr):
    """A bound variable (process id, or a V.exists value)."""
    _ids = itertools.count()

    def __init__(self, kind):
        self.kind = kind  # "proc" | "int" | "bool"
        self.uid = next(Var._ids)

    # process fields (the variables of the reference's Process classes)
    @property
    def x(self): return Field(FIELD_X, self)
    @property
    def decided(self): return Field(FIELD_DECIDED, self)
    @property
    def decision(self): return Field(FIELD_DECISION, self)
    @property
    def ts(self): return Field(FIELD_TS, self)
    @property
    def ready(self): return Field(FIELD_READY, self)
    @property
    def commit(self): return Field(FIELD_COMMIT, self)
    @property
    def vote(self): return Field(FIELD_VOTE, self)
    @property
    def canDecide(self): return Field(FIELD_CANDECIDE, self)
    @property
    def est(self): return Field(FIELD_X, self)
    @property
    def HO(self): return _HO(self)


class _HO:
    def __init__(self, p): self.p = p
    @property
    def size(self): return Field(FIELD_HOSIZE, self.p)


class CoordVal(Expr):
    """coord = (r/4) % n as a process (LastVoting.scala:95)."""
    @property
    def commit(self): return Field(FIELD_COMMIT, self)
    @property
    def ready(self): return Field(FIELD_READY, self)
    @property
    def vote(self): return Field(FIELD_VOTE, self)
    @property
    def x(self): return Field(FIELD_X, self)
    @property
    def ts(self): return Field(FIELD_TS, self)


class Field(Expr):
    def __init__(self, f, proc, tag=TAG_CUR):
        self.f, self.proc, self.tag = f, lift(proc), tag

    def children(self):
        return (self.proc,)


class Un(Expr):
    def __init__(self, op, x):
        self.op, self.x = op, lift(x)

    def children(self):
        return (self.x,)


class Bin(Expr):
    def __init__(self, op, x, y):
        self.op, self.x, self.y = op, lift(x), lift(y)

    def children(self):
        return (self.x, self.y)


class Quant(Expr):
    """ForAll / Exists / Cardinality(Comprehension) over processes; Exists over a value domain."""

    def __init__(self, kind, var, body):
        self.kind, self.var, self.body = kind, var, lift(body)  # kind: forall | exists | count | vint | vbool

    def children(self):
        return (self.body,)


class Contains(Expr):
    def __init__(self, comp, e):
        self.comp, self.e = comp, lift(e)

    def children(self):
        return (self.e, self.comp.body)


class Comprehension:
    """P.filter(i => body): a set of processes (Comprehension in Formula.scala)."""

    def __init__(self, var, body):
        self.var, self.body = var, lift(body)

    @property
    def size(self):
        return Quant("count", self.var, self.body)

    def contains(self, e):
        return Contains(self, e)

    # Scala Set operations on the comprehension, lowered to exactly the shapes
    # FormulaExtractor gives them (tests/macros/FormulaExtractorSuite.scala:42-56):
    #   s.forall(p) -> ForAll(v, Implies(In(v, s), p(v)))
    #   s.exists(p) -> Exists(v, And(In(v, s), p(v)))
    #   s.filter(p) -> Comprehension(v, And(In(v, s), p(v)))
    #   s.count(p)  -> Cardinality(Comprehension(v, And(In(v, s), p(v))))
    def forall(self, fn: Callable):
        v = Var("proc")
        return Quant("forall", v, Implies(Contains(self, v), fn(v)))

    def exists(self, fn: Callable):
        v = Var("proc")
        return Quant("exists", v, And(Contains(self, v), fn(v)))

    def filter(self, fn: Callable):
        v = Var("proc")
        return Comprehension(v, And(Contains(self, v), fn(v)))

    def count(self, fn: Callable):
        return self.filter(fn).size


def lift(v):
    if isinstance(v, Expr):
        return v
    if isinstance(v, (bool, int)):
        return Lit(v)
    raise FormulaError(f"cannot use {v!r} in a Formula")


def Some(e):
    """Some(v) compared with an Option field (None is PSG_NONE32, so Some(v) == v)."""
    return lift(e)


def init(e):
    """init(i.x): the value at check point 0 (FormulaExtractor `init`)."""
    return _retag(e, TAG_INIT)


def old(e):
    """old(i.x): the value before the last round."""
    return _retag(e, TAG_OLD)


def _retag(e, tag):
    if isinstance(e, Field):
        return Field(e.f, e.proc, tag)
    if isinstance(e, Un) and e.op in ("ISDEF", "NOT"):
        return Un(e.op, _retag(e.x, tag))
    raise FormulaError("init/old apply to a process field")


def And(*xs):
    out = lift(xs[0])
    for x in xs[1:]:
        out = out & x
    return out


def Or(*xs):
    out = lift(xs[0])
    for x in xs[1:]:
        out = out | x
    return out


def Implies(a, b):
    return lift(a).implies(b)


class _P:
    """The process domain (psync/Algorithm.scala `P`)."""

    @staticmethod
    def forall(fn: Callable):
        v = Var("proc")
        return Quant("forall", v, fn(v))

    @staticmethod
    def exists(fn: Callable):
        v = Var("proc")
        return Quant("exists", v, fn(v))

    @staticmethod
    def filter(fn: Callable):
        v = Var("proc")
        return Comprehension(v, fn(v))


class _Domain:
    """`new Domain[Int]` / `new Domain[Boolean]` (only `exists` is meaningful to check)."""

    def __init__(self, kind):
        self.kind = kind

    def exists(self, fn: Callable):
        v = Var(self.kind)
        return Quant("vint" if self.kind == "int" else "vbool", v, fn(v))


P = _P()
V = _Domain("int")
VB = _Domain("bool")
n = NVal()
r = RVal()
coord = CoordVal()
true = Lit(1)
false = Lit(0)


# --------------------------------------------------------------------------- Spec
class Spec:
    """psync/Specs.scala:8-16: safetyPredicate, invariants, roundInvariants, properties."""

    def __init__(self, invariants: Sequence[Expr] = (), round_invariants: Sequence[Sequence[Expr]] = (),
                 properties: Sequence[Tuple[str, Expr]] = (), safety_predicate: Optional[Expr] = None,
                 phase_length: int = 1):
        self.invariants = [lift(f) for f in invariants]
        self.round_invariants = [[lift(f) for f in l] for l in round_invariants]
        self.properties = [(name, lift(f)) for name, f in properties]
        self.safety_predicate = None if safety_predicate is None else lift(safety_predicate)
        self.phase_length = int(phase_length)


class Program:
    """A compiled Spec: psg_spec_program plus slot names."""

    def __init__(self, code, slot_entry, slot_flags, term_entry, n_vars, slot_names, fields):
        self.code, self.slot_entry, self.slot_flags = list(code), list(slot_entry), list(slot_flags)
        self.term_entry, self.n_vars, self.slot_names, self.fields = term_entry, n_vars, list(slot_names), fields
        self.module_path = None  # native code object (compile_native) or None: bytecode interpreter
        self.alg = 0             # enum psg_alg the program was compiled for (0: unbound)
        self._keep = None

    def to_c(self) -> abi.SpecProgram:
        code = (C.c_int32 * len(self.code))(*self.code)
        ent = (C.c_int32 * len(self.slot_entry))(*self.slot_entry)
        flg = (C.c_int32 * len(self.slot_flags))(*self.slot_flags)
        self._keep = (code, ent, flg)
        p = abi.SpecProgram()
        p.n_slots = len(self.slot_entry)
        p.n_words = len(self.code)
        p.code = C.cast(code, C.POINTER(C.c_int32))
        p.slot_entry = C.cast(ent, C.POINTER(C.c_int32))
        p.slot_flags = C.cast(flg, C.POINTER(C.c_int32))
        p.term_entry = self.term_entry
        p.n_vars = self.n_vars
        p.module_path = self.module_path.encode() if self.module_path else None
        p.alg = int(self.alg or 0)
        return p


# --------------------------------------------------------------------------- compiler
def _word(op, a=0, b=0):
    if not (-(1 << 15) <= b < (1 << 15)):
        raise FormulaError("immediate out of range")
    w = (OP[op] & 0xFF) | ((a & 0xFF) << 8) | ((b & 0xFFFF) << 16)
    return w - (1 << 32) if w >= (1 << 31) else w


def _walk(e):
    yield e
    for c in e.children():
        yield from _walk(c)


def _free_vars(e, bound=frozenset()):
    """uids of variables used in e but bound outside it."""
    out = set()
    if isinstance(e, Var):
        if e.uid not in bound:
            out.add(e.uid)
        return out
    if isinstance(e, Quant):
        return _free_vars(e.body, bound | {e.var.uid})
    if isinstance(e, Contains):
        return _free_vars(e.e, bound) | _free_vars(e.comp.body, bound | {e.comp.var.uid})
    for c in e.children():
        out |= _free_vars(c, bound)
    return out


def _strip(e):
    return e  # `.get` is the identity on the int encoding


def _uses_old(e):
    return any(isinstance(x, Field) and x.tag == TAG_OLD for x in _walk(e))


class _Compiler:
    def __init__(self, fields_available=None):
        self.code: List[int] = []
        self.slot_of: Dict[int, int] = {}
        self.max_slot = -1
        self.fields_used = set()
        self.fields_available = fields_available

    def emit(self, w):
        self.code.append(w)
        return len(self.code) - 1

    def bind(self, var, depth):
        if depth >= MAX_VARS:
            raise FormulaError(f"more than {MAX_VARS} nested bound variables")
        self.slot_of[var.uid] = depth
        self.max_slot = max(self.max_slot, depth)
        return depth

    def expr(self, e, depth, in_lane):
        if isinstance(e, Lit):
            if -(1 << 15) <= e.v < (1 << 15):
                self.emit(_word("IMM", 0, e.v))
            else:
                self.emit(_word("IMM32"))
                self.emit(e.v)
        elif isinstance(e, NVal):
            self.emit(_word("N"))
        elif isinstance(e, RVal):
            self.emit(_word("R"))
        elif isinstance(e, CoordVal):
            self.emit(_word("COORD"))
        elif isinstance(e, Var):
            if e.uid not in self.slot_of:
                raise FormulaError("variable used outside its quantifier")
            self.emit(_word("VAR", self.slot_of[e.uid]))
        elif isinstance(e, Field):
            if self.fields_available is not None and e.f not in self.fields_available:
                raise FormulaError(f"field {e.f} is not part of this algorithm's state")
            self.fields_used.add(e.f)
            self.expr(e.proc, depth, in_lane)
            self.emit(_word("FIELD", e.f, e.tag))
        elif isinstance(e, Un):
            self.expr(e.x, depth, in_lane)
            self.emit(_word(e.op))
        elif isinstance(e, Bin):
            self.expr(e.x, depth, in_lane)
            self.expr(e.y, depth, in_lane)
            self.emit(_word(e.op))
        elif isinstance(e, Contains):
            # A.contains(e) == body of A with its variable bound to e
            self.expr(e.e, depth, in_lane)
            slot = self.bind(e.comp.var, depth)
            self.emit(_word("BIND", slot))
            self.expr(e.comp.body, depth + 1, in_lane)
        elif isinstance(e, Quant):
            self.quant(e, depth, in_lane)
        else:
            raise FormulaError(f"unsupported node {type(e).__name__}")

    def quant(self, q, depth, in_lane):
        slot = self.bind(q.var, depth)
        lane_form = False
        if q.kind in ("forall", "exists", "count"):
            lane_form = not in_lane
            base = {"forall": Q_FORALL_P, "exists": Q_EXISTS_P, "count": Q_COUNT_P}[q.kind]
            kind = base + 3 if lane_form else base
            head = [_word("QBEGIN", kind, slot)]
        elif q.kind == "vbool":
            head = [_word("QBEGIN", Q_EXISTS_VB, slot)]
        else:  # vint: finitize over what v is compared with
            exprs, fsets = self.witnesses(q)
            for t in exprs:
                self.expr(t, depth, in_lane)
            head = [_word("QBEGIN", Q_EXISTS_VI, slot)]
        at = self.emit(head[0])
        end_at = self.emit(0)
        if q.kind == "vint":
            self.emit(len(exprs) | (len(fsets) << 16))
            for f, tag in fsets:
                self.fields_used.add(f)
                self.emit(f | (tag << 8))
        self.expr(q.body, depth + 1, in_lane or lane_form)
        end = self.emit(_word("QEND"))
        self.code[end_at] = end
        return at

    def witnesses(self, q):
        """Candidate sources of V.exists(v => body): every term v is compared with."""
        v = q.var.uid
        inner = {x.var.uid for x in _walk(q.body) if isinstance(x, Quant)} | \
                {x.comp.var.uid for x in _walk(q.body) if isinstance(x, Contains)}
        exprs, fsets = [], []
        seen_cmp = set()
        for x in _walk(q.body):
            if isinstance(x, Bin) and x.op in ("EQ", "NE", "LT", "LE", "GT", "GE"):
                for a, b in ((x.x, x.y), (x.y, x.x)):
                    if isinstance(a, Var) and a.uid == v:
                        if v in _free_vars(b):
                            raise FormulaError("V.exists variable compared with a term containing itself")
                        t = _strip(b)
                        if isinstance(t, Field):
                            key = (t.f, t.tag)
                            if key not in fsets:
                                fsets.append(key)
                        elif not (_free_vars(t) & inner):
                            exprs.append(t)
                        else:
                            raise FormulaError("V.exists witness term depends on an inner bound variable "
                                               "and is not a process field")
                        seen_cmp.add(id(a))
        for x in _walk(q.body):
            if isinstance(x, Var) and x.uid == v and id(x) not in seen_cmp:
                raise FormulaError("a V.exists variable may only appear directly in comparisons")
        return exprs, fsets

    def root(self, e):
        at = len(self.code)
        self.expr(e, 0, False)
        self.emit(_word("HALT"))
        return at


def _rinv_guard(spec: Spec) -> Optional[Expr]:
    """(r % L == j) ==> roundInvariants(j-1)(0) for j = 1..L-1 (Verifier.scala:133-141)."""
    L = spec.phase_length
    parts = []
    for j in range(1, L):
        if j - 1 < len(spec.round_invariants) and spec.round_invariants[j - 1]:
            parts.append(((r % L) == j).implies(spec.round_invariants[j - 1][0]))
    return And(*parts) if parts else None


def compile_spec(spec: Spec, alg: Optional[int] = None) -> Program:
    comp = _Compiler(ALG_FIELDS.get(alg) if alg is not None else None)
    names, entries, flags = [], [], []
    guard = _rinv_guard(spec)
    invs = [inv if guard is None else (inv & guard) for inv in spec.invariants]
    if invs:
        names.append("Safety")
        entries.append(comp.root(Or(*invs)))
        flags.append(0)
        for k, inv in enumerate(invs):
            names.append(f"Invariant{k}")
            entries.append(comp.root(inv))
            flags.append(0)
    term = -1
    for name, f in spec.properties:
        if name == "Termination":
            term = comp.root(f)
            continue
        names.append(name)
        entries.append(comp.root(f))
        flags.append(SPEC_RELATIONAL if _uses_old(f) else 0)
    if spec.safety_predicate is not None:
        names.append("SafetyPredicate")
        entries.append(comp.root(spec.safety_predicate))
        flags.append(SPEC_RELATIONAL if _uses_old(spec.safety_predicate) else 0)
    if not entries:
        raise FormulaError("a Spec needs at least one invariant, property or safety predicate")
    if len(entries) > abi.PSG_MAX_CHECKS:
        raise FormulaError(f"more than {abi.PSG_MAX_CHECKS} check slots")
    prog = Program(comp.code, entries, flags, term, comp.max_slot + 1, names, comp.fields_used)
    prog.alg = int(alg or 0)
    return prog


# --------------------------------------------------------------------------- the reference specs, restated
def otr_spec() -> Spec:
    """example/Otr.scala:95-120."""
    def A(v): return P.filter(lambda i: i.x == v)
    keep_init = P.forall(lambda i: P.exists(lambda j1: i.x == init(j1.x)))
    inv0 = (P.forall(lambda i: ~i.decided)
            | V.exists(lambda v: (A(v).size > 2 * n // 3)
                       & P.forall(lambda i: i.decided.implies(i.decision == v)))) & keep_init
    inv1 = V.exists(lambda v: (A(v).size == n)
                    & P.forall(lambda i: i.decided.implies(i.decision == v))) & keep_init
    inv2 = P.exists(lambda j: P.forall(lambda i: i.decided & (i.decision == init(j.x))))
    return Spec([inv0, inv1, inv2], properties=_consensus_properties())


def _consensus_properties():
    return [
        ("Termination", P.forall(lambda i: i.decided)),
        ("Agreement", P.forall(lambda i: P.forall(lambda j: (i.decided & j.decided).implies(
            i.decision == j.decision)))),
        ("Validity", P.forall(lambda i: i.decided.implies(P.exists(lambda j: init(j.x) == i.decision)))),
        ("Integrity", P.exists(lambda j: P.forall(lambda i: i.decided.implies(i.decision == init(j.x))))),
        ("Irrevocability", P.forall(lambda i: old(i.decided).implies(
            i.decided & (old(i.decision) == i.decision)))),
    ]


def otr2_spec() -> Spec:
    """example/Otr2.scala:71-96 (decision: Option[Int])."""
    def A(v): return P.filter(lambda i: i.x == v)
    def all_dec(v): return P.forall(lambda i: i.decision.isDefined.implies(i.decision.get == v))
    inv0 = P.forall(lambda i: ~i.decision.isEmpty) | V.exists(lambda v: (A(v).size > 2 * n // 3) & all_dec(v))
    inv1 = V.exists(lambda v: (A(v).size == n) & all_dec(v))
    inv2 = V.exists(lambda v: all_dec(v))
    props = [
        ("Termination", P.forall(lambda i: i.decision.isDefined)),
        ("Agreement", P.forall(lambda i: P.forall(lambda j: (i.decision.isDefined & j.decision.isDefined).implies(
            i.decision == j.decision)))),
        ("Validity", P.forall(lambda i: i.decision.isDefined.implies(
            P.exists(lambda j: init(j.x) == i.decision.get)))),
        ("Integrity", P.exists(lambda j: P.forall(lambda i: i.decision.isDefined.implies(
            i.decision.get == init(j.x))))),
        ("Irrevocability", P.forall(lambda i: old(i.decision).isDefined.implies(old(i.decision) == i.decision))),
    ]
    return Spec([inv0, inv1, inv2], properties=props)


def lv_spec() -> Spec:
    """example/LastVoting.scala:19-70."""
    no_decision = P.forall(lambda i: ~i.decided & ~i.ready)

    def majority_body(v, t):
        A = P.filter(lambda i: i.ts >= t)
        return ((A.size > n // 2) & (r > 0) & (t <= r // 4)
                & P.forall(lambda i: A.contains(i).implies(i.x == v)
                           & i.decided.implies(i.decision == v)
                           & i.commit.implies(i.vote == v)
                           & i.ready.implies(i.vote == v)
                           & (i.ts == r // 4).implies(coord.commit)))

    majority = V.exists(lambda v: V.exists(lambda t: majority_body(v, t)))
    keep_init = P.forall(lambda i: P.exists(lambda j1: i.x == init(j1.x)))
    safety_inv = And(keep_init, Or(no_decision, majority))
    inv1 = P.exists(lambda j: P.forall(lambda i: i.decided & (i.decision == init(j.x))))
    rinv = [
        [true, P.exists(lambda i: i.commit)],
        [true, P.exists(lambda i: i.commit & P.forall(lambda j: (j.ts == r // 4) & (j.x == i.vote)))],
        [true, P.exists(lambda i: i.commit & i.ready & P.forall(lambda j: (j.ts == r // 4) & (j.x == i.vote)))],
    ]
    return Spec([safety_inv, inv1], rinv, _consensus_properties(), phase_length=4)


def benor_spec() -> Spec:
    """example/BenOr.scala:91-115 (V = Domain[Boolean])."""
    inv0 = (P.forall(lambda i: ~i.decided & ~i.canDecide)
            | VB.exists(lambda v: (P.filter(lambda i: i.x == v).size > n // 2)
                        & P.forall(lambda i: i.decided.implies(i.decision == v)
                                   & i.vote.isDefined.implies(i.vote == Some(v)))))
    rinv = [[P.forall(lambda p: p.vote.isDefined.implies(P.filter(lambda i: i.x == p.vote.get).size > n // 2))]]
    props = [
        ("Agreement", P.forall(lambda i: P.forall(lambda j: (i.decided & j.decided).implies(
            i.decision == j.decision)))),
        ("Irrevocability", P.forall(lambda i: old(i.decided).implies(i.decided & (old(i.decision) == i.decision)))),
        ("Termination", P.forall(lambda i: i.decided)),
    ]
    return Spec([inv0], rinv, props, safety_predicate=P.forall(lambda p: p.HO.size > n // 2), phase_length=2)


REFERENCE_SPECS = {
    abi.PSG_ALG_OTR: otr_spec,
    abi.PSG_ALG_OTR2: otr2_spec,
    abi.PSG_ALG_LAST_VOTING: lv_spec,
    abi.PSG_ALG_BENOR: benor_spec,
}


# --------------------------------------------------------------------------- native lowering (HIP)
_CSRC = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "csrc")
_INCLUDE = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(_CSRC)), "include")
CACHE_DIR = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(_CSRC)),
                                        "build", "spec")


def _c_int(v):
    return "(-2147483647 - 1)" if v == -(1 << 31) else f"((int32_t){v})"


class _Gen:
    """Formula tree -> C++ expression over psg_spec_native.hpp (template parameter W)."""

    BIN = {"AND": "(int32_t)((({x}) != 0) & (({y}) != 0))", "OR": "(int32_t)((({x}) != 0) | (({y}) != 0))",
           "IMPL": "(int32_t)((({x}) == 0) | (({y}) != 0))", "EQ": "(int32_t)(({x}) == ({y}))",
           "NE": "(int32_t)(({x}) != ({y}))", "LT": "(int32_t)(({x}) < ({y}))", "LE": "(int32_t)(({x}) <= ({y}))",
           "GT": "(int32_t)(({x}) > ({y}))", "GE": "(int32_t)(({x}) >= ({y}))", "ADD": "spec::iadd({x}, {y})",
           "SUB": "spec::isub({x}, {y})", "MUL": "spec::imul({x}, {y})", "DIV": "spec::idiv({x}, {y})",
           "MOD": "spec::imod({x}, {y})"}

    def __init__(self, fields_available=None):
        self.names = {}       # var uid -> (c name, per-lane?, lane-bound pid?)
        self.k = itertools.count()
        self.fields = set()
        self.tags = set()
        self.fields_available = fields_available
        self.max_vi = 0
        self.tuples = {}      # var uid -> {(field, tag): C++ name} (serial quantifier over distinct states)
        self.init_sets = []   # fields f with an LDS membership set of init(f) (at most 2)
        self.cse = {}         # structural key of a closed subformula -> C++ name of its hoisted value
        self.skeys = {}       # _skey memo
        self.tup_sets = {}    # field tuple of a distinct-state quantifier -> C++ name of its per-check-point TupU
        self.tup_used = set()  # field tuples used by the function being generated
        self.memo_slots = {}   # (init set, field) -> memo slot of member_init_own
        self.uni = False       # lowering for symmetric check points (spec::uniform, psg_spec_native.hpp)
        self.pvars = set()     # uids of variables bound to a process (a pid in [0, n))
        self.uft = []          # (field, tag) current / old fields read by the symmetric lowering
        self.umemo = {}        # (init set, C++ expression) -> memo slot of member_init_u

    def gen(self, e, in_lane, vi_depth):
        """(C++ expression, depends on the lane)."""
        k = _skey(e, self.skeys)
        if k in self.cse:
            return self.cse[k], False  # a closed subformula computed once per check point
        if isinstance(e, Lit):
            return _c_int(e.v), False
        if isinstance(e, NVal):
            return "x.n", False
        if isinstance(e, RVal):
            return "x.r", False
        if isinstance(e, CoordVal):
            return "((x.r / 4) % x.n)", False
        if isinstance(e, Var):
            if e.uid not in self.names:
                raise FormulaError("variable used outside its quantifier")
            name, lane, _ = self.names[e.uid]
            return name, lane
        if isinstance(e, Field):
            if self.fields_available is not None and e.f not in self.fields_available:
                raise FormulaError(f"field {e.f} is not part of this algorithm's state")
            self.fields.add(e.f)
            self.tags.add(e.tag)
            if self.uni and e.tag != TAG_INIT:
                # symmetric check point: every process holds process 0's value
                if (e.f, e.tag) not in self.uft:
                    self.uft.append((e.f, e.tag))
                if isinstance(e.proc, CoordVal) or (isinstance(e.proc, Var) and e.proc.uid in self.pvars):
                    return f"x.uf({e.tag}, {e.f})", False
                p, lane = self.gen(e.proc, in_lane, vi_depth)
                return f"spec::fld_uni<W>(x, {e.tag}, {e.f}, {p})", lane
            if isinstance(e.proc, Var) and self.names.get(e.proc.uid, (None, False, False))[2]:
                return f"x.own({e.tag}, {e.f})", True  # the lane's own process
            if isinstance(e.proc, Var) and e.proc.uid in self.tuples:
                return self.tuples[e.proc.uid][(e.f, e.tag)], False  # a distinct-state tuple value
            p, lane = self.gen(e.proc, in_lane, vi_depth)
            fn = "fld_g" if lane else "fld_u"
            return f"spec::{fn}<W>(x, {e.tag}, {e.f}, {p})", lane
        if isinstance(e, Un):
            a, lane = self.gen(e.x, in_lane, vi_depth)
            if e.op == "NOT":
                return f"(int32_t)(({a}) == 0)", lane
            if e.op == "NEG":
                return f"spec::isub(0, {a})", lane
            return f"(int32_t)(({a}) != (-2147483647 - 1))", lane
        if isinstance(e, Bin):
            a, la = self.gen(e.x, in_lane, vi_depth)
            b, lb = self.gen(e.y, in_lane, vi_depth)
            if e.op in ("AND", "OR", "IMPL") and _expensive(e.y):
                # skip a quantified right side when no lane needs it (group-uniform test)
                if not la:
                    t = {"AND": "({a}) != 0 ? (int32_t)(({b}) != 0) : 0",
                         "OR": "({a}) != 0 ? 1 : (int32_t)(({b}) != 0)",
                         "IMPL": "({a}) == 0 ? 1 : (int32_t)(({b}) != 0)"}[e.op]
                    return "(" + t.format(a=a, b=b) + ")", lb
                fn = {"AND": "and_sc", "OR": "or_sc", "IMPL": "impl_sc"}[e.op]
                return f"spec::{fn}<W>(x, {a}, [&]() -> int32_t {{ return {b}; }})", True
            return self.BIN[e.op].format(x=a, y=b), la or lb
        if isinstance(e, Contains):
            val, lane = self.gen(e.e, in_lane, vi_depth)
            v = f"b{next(self.k)}"
            own = isinstance(e.e, Var) and self.names.get(e.e.uid, (None, False, False))[2]
            if isinstance(e.e, CoordVal) or (isinstance(e.e, Var) and e.e.uid in self.pvars):
                self.pvars.add(e.comp.var.uid)  # a process's pid
            # A.contains(i) for the lane's own process i: the comprehension's variable is that
            # process too (its fields are the lane's registers, not a gather)
            self.names[e.comp.var.uid] = (val, True, True) if own else (v, lane, False)
            body, lb = self.gen(e.comp.body, in_lane, vi_depth)
            return f"([&](int32_t {v}) -> int32_t {{ return {body}; }})({val})", lane or lb
        if isinstance(e, Quant):
            return self.quant(e, in_lane, vi_depth)
        raise FormulaError(f"unsupported node {type(e).__name__}")

    def quant(self, q, in_lane, vi_depth):
        v = f"v{next(self.k)}"
        if q.kind in ("forall", "exists", "count"):
            self.pvars.add(q.var.uid)
            # a variable may be bound by several quantifiers (_split_forall): drop its last binding
            self.tuples.pop(q.var.uid, None)
            self.names.pop(q.var.uid, None)
            if self.uni:
                got = self._quant_uni(q, v, in_lane, vi_depth)
                if got is not None:
                    return got
            if not in_lane:
                self.names[q.var.uid] = (v, True, True)
                body, _ = self.gen(q.body, True, vi_depth)
                fn = {"forall": "forall_lane", "exists": "exists_lane", "count": "count_lane"}[q.kind]
                return f"spec::{fn}<W>(x, [&](int32_t {v}) -> int32_t {{ return {body}; }})", False
            mem = _init_member(q)
            if mem is not None and (mem[0] in self.init_sets or len(self.init_sets) < 2):
                f, t = mem
                if f not in self.init_sets:
                    self.init_sets.append(f)
                self.fields.add(f)
                self.tags.add(TAG_INIT)
                K = self.init_sets.index(f)
                if (isinstance(t, Field) and t.tag == TAG_CUR and isinstance(t.proc, Var)
                        and self.names.get(t.proc.uid, (None, False, False))[2]):
                    # the lane's own current field: memoized probe (member_init_own)
                    key = (K, t.f)
                    if key not in self.memo_slots and len(self.memo_slots) < 4:
                        self.memo_slots[key] = len(self.memo_slots)
                    if key in self.memo_slots:
                        self.fields.add(t.f)
                        self.tags.add(TAG_CUR)
                        return f"spec::member_init_own<W, {K}, {t.f}, {self.memo_slots[key]}>(x)", True
                tc, tl = self.gen(t, in_lane, vi_depth)
                return f"spec::member_init<W, {K}>(x, {tc})", tl
            flds = _tuple_fields(q)
            if flds is not None:
                # the body reads j only through fields: visit each distinct field tuple once
                # (count: weighted by how many processes hold it)
                guard = _tuple_guard(q) if flds else []
                gcode = None
                if guard:
                    # A(j) of forall(j => A(j) ==> B) / exists, count(j => A(j) && B): only the
                    # processes where it holds are visited; evaluated per lane (j = the lane's own)
                    self.names[q.var.uid] = (v, True, True)
                    gcode = " & ".join(f"(int32_t)(({self.gen(c, True, vi_depth)[0]}) != 0)" for c in guard)
                    del self.names[q.var.uid]
                names = {ft: f"{v}_{k}" for k, ft in enumerate(flds)}
                self.tuples[q.var.uid] = names
                for f, tag in flds:
                    if self.fields_available is not None and f not in self.fields_available:
                        raise FormulaError(f"field {f} is not part of this algorithm's state")
                    self.fields.add(f)
                    self.tags.add(tag)
                body, lane = self.gen(q.body, in_lane, vi_depth)
                mode = {"forall": 0, "exists": 1, "count": 2}[q.kind]
                params = ", ".join(f"int32_t {names[ft]}" for ft in flds)
                fl = ", ".join(f"spec::Fld<{f}, {tag}>{{}}" for f, tag in flds)
                if not flds:
                    return (f"spec::quant_tup<W, {mode}>(x, [&]({params}) -> int32_t {{ return {body}; }})"), lane
                # per check point: are those fields the same for every (guarded) process (one tuple)?
                key = tuple(flds) if gcode is None else (tuple(flds), gcode)
                if key not in self.tup_sets:
                    self.tup_sets[key] = f"tu{len(self.tup_sets)}"
                self.tup_used.add(key)
                fn = "quant_tup_c" if gcode is None else "quant_tup_gc"
                return (f"spec::{fn}<W, {mode}>(x, {self.tup_sets[key]}, [&]({params}) -> int32_t "
                        f"{{ return {body}; }}, {fl})"), lane
            self.names[q.var.uid] = (v, False, False)
            body, lane = self.gen(q.body, in_lane, vi_depth)
            fn = {"forall": "forall_ser", "exists": "exists_ser", "count": "count_ser"}[q.kind]
            return f"spec::{fn}<W>(x, [&](int32_t {v}) -> int32_t {{ return {body}; }})", lane
        self.names[q.var.uid] = (v, False, False)
        if q.kind == "vbool":
            body, lane = self.gen(q.body, in_lane, vi_depth)
            return f"spec::exists_bool<W>(x, [&](int32_t {v}) -> int32_t {{ return {body}; }})", lane
        pins = None if in_lane else _pins(q.body, q.var.uid)
        if pins is not None:
            # equality pins: a conjunct P.forall(i => ... && (cond(i) ==> term(i) == v) && ...)
            # leaves v = term(i) as the only candidate once some process has cond(i); with
            # none active, the finitization below decides it
            fq, plist = pins
            pl = f"p{next(self.k)}"
            self.names[fq.var.uid] = (pl, True, True)
            self.pvars.add(fq.var.uid)
            conds, vals, plane = [], [], False
            for cond, term in plist:
                if cond is None:
                    conds.append("1")
                else:
                    cc, cl = self.gen(cond, True, vi_depth)
                    conds.append(f"(int32_t)(({cc}) != 0)")
                    plane = plane or cl
                tc, tl = self.gen(term, True, vi_depth)
                vals.append(tc)
                plane = plane or tl
            act = " | ".join(conds)
            val = vals[-1]
            for cc, tc in reversed(list(zip(conds[:-1], vals[:-1]))):
                val = f"(({cc}) != 0 ? ({tc}) : ({val}))"
            general, lane_g = self._vint_unpinned(q, v, in_lane, vi_depth)
            self.names[q.var.uid] = (v, False, False)
            body, lane_b = self.gen(q.body, in_lane, vi_depth + 1)
            self.max_vi = max(self.max_vi, vi_depth + 1)
            if self.uni and not plane:
                # symmetric check point: every process has the same pin flag and value
                return (f"spec::pin_uni({act}, {val}, [&](int32_t {v}) -> int32_t {{ return {body}; }}, "
                        f"[&]() -> int32_t {{ return {general}; }})"), lane_b or lane_g
            return (f"spec::exists_int_pin<W>(x, [&](int32_t {pl}) -> int32_t {{ return {act}; }}, "
                    f"[&](int32_t {pl}) -> int32_t {{ return {val}; }}, scratch + {vi_depth} * 64 * W, "
                    f"[&](int32_t {v}) -> int32_t {{ return {body}; }}, [&]() -> int32_t {{ return {general}; }})"), True
        return self._vint_unpinned(q, v, in_lane, vi_depth)

    def _quant_uni(self, q, v, in_lane, vi_depth):
        """A process quantifier on a symmetric check point, or None for the general rules:
        a body reading its variable only through current / old fields has one value for every
        process (forall / exists: that value, count: n or 0); P.exists(j => init(j.f) == t)
        with a group-uniform t is a scalar-memoized set probe."""
        if _symmetric(q):
            self.names[q.var.uid] = ("0", False, False)  # never read but through its fields
            body, lane = self.gen(q.body, in_lane, vi_depth)
            if lane and not in_lane:
                # a group-uniform value in a lane register: reduced over the valid lanes
                fn = {"forall": "forall_lane", "exists": "exists_lane", "count": "count_lane"}[q.kind]
                return f"spec::{fn}<W>(x, [&](int32_t {v}) -> int32_t {{ return {body}; }})", False
            if q.kind == "count":
                return f"(({body}) != 0 ? x.n : 0)", lane
            return f"(int32_t)(({body}) != 0)", lane
        mem = _init_member(q)
        if mem is not None and (mem[0] in self.init_sets or len(self.init_sets) < 2):
            f, t = mem
            tc, tl = self.gen(t, in_lane, vi_depth)
            if tl:
                return None
            if f not in self.init_sets:
                self.init_sets.append(f)
            self.fields.add(f)
            self.tags.add(TAG_INIT)
            K = self.init_sets.index(f)
            key = (K, tc)
            if key not in self.umemo and len(self.umemo) < 4:
                self.umemo[key] = len(self.umemo)
            if key in self.umemo:
                return f"spec::member_init_u<W, {K}, {self.umemo[key]}>(x, {tc})", False
            return f"spec::member_init<W, {K}>(x, {tc})", False
        return None

    def _vint_unpinned(self, q, v, in_lane, vi_depth):
        """V.exists over Int: count-guarded candidates, else the general finitization."""
        self.names[q.var.uid] = (v, False, False)
        guard = _count_guard(q)
        if guard is not None:
            # a conjunct P.filter(i => i.f == v).size >= L restricts the witnesses to values
            # of f held by >= L processes (runtime L >= 1; else the general finitization)
            (f, tag), thr, op = guard
            self.fields.add(f)
            self.tags.add(tag)
            tc, tl = self.gen(thr, in_lane, vi_depth)
            if tl:
                guard = None
        if guard is not None:
            L = f"(({tc}) + 1)" if op == "GT" else f"({tc})"
            general, lane_g = self._vint_general(q, v, in_lane, vi_depth)
            self.names[q.var.uid] = (v, False, False)
            body, lane = self.gen(q.body, in_lane, vi_depth + 1)
            self.max_vi = max(self.max_vi, vi_depth + 1)
            if self.uni and tag != TAG_INIT:
                # symmetric check point: process 0's value is the only one, held by n processes
                if (f, tag) not in self.uft:
                    self.uft.append((f, tag))
                return (f"([&]() -> int32_t {{ const int32_t L_ = {L}; if (L_ >= 1) return "
                        f"spec::guard_uni<W>(x, x.uf({tag}, {f}), L_, "
                        f"[&](int32_t {v}) -> int32_t {{ return {body}; }}); return {general}; }})()"), lane or lane_g
            return (f"([&]() -> int32_t {{ const int32_t L_ = {L}; if (L_ >= 1) return "
                    f"spec::exists_int_guard<W, {f | (tag << 8)}>(x, x.own({tag}, {f}), x.stage({tag}, {f}), L_, "
                    f"[&](int32_t {v}) -> int32_t {{ return {body}; }}); return {general}; }})()"), True
        return self._vint_general(q, v, in_lane, vi_depth)

    def _vint_general(self, q, v, in_lane, vi_depth):
        """V.exists over Int by finitization over the compared terms (equality-only: no +-1)."""
        self.names[q.var.uid] = (v, False, False)
        exprs, fsets = _Compiler.witnesses(_Compiler(), q)
        eq_only = _eq_only(q)
        evs = []
        for t in exprs:
            c, _ = self.gen(t, in_lane, vi_depth)
            evs.append(c)
        for f, tag in fsets:
            self.fields.add(f)
            self.tags.add(tag)
        self.max_vi = max(self.max_vi, vi_depth + 1)
        body, lane = self.gen(q.body, in_lane, vi_depth + 1)
        # its value is group-uniform outside a lane quantifier (the candidates are); the general
        # lowering keeps the conservative lane flag
        vlane = (in_lane or lane) if self.uni else True
        ne, nf = len(evs), len(fsets)
        ev = ", ".join(evs) if evs else "0"
        fs = ", ".join(str(f | (t << 8)) for f, t in fsets) if fsets else "0"
        head = (f"([&]() -> int32_t {{ const int32_t ev_[{max(ne, 1)}] = {{{ev}}}; "
                f"const int32_t fs_[{max(nf, 1)}] = {{{fs}}}; ")
        lam = f"[&](int32_t {v}) -> int32_t {{ return {body}; }}); }})()"
        if eq_only:
            return (head + f"return spec::exists_int_eq<W, {ne}, {nf}>(x, ev_, fs_, scratch + {vi_depth} * 64 * W, "
                    + lam), vlane
        # order comparisons: one candidate per breakpoint (exists_int_bp) instead of v-1, v, v+1
        sh = _breakpoint_shifts(q, exprs, fsets)
        return (head + f"const uint32_t sh_[{max(ne + nf, 1)}] = {{{', '.join(f'{m}u' for m in sh) or '0u'}}}; "
                f"return spec::exists_int_bp<W, {ne}, {nf}>(x, ev_, fs_, sh_, scratch + {vi_depth} * 64 * W, "
                + lam), vlane


def _expensive(e) -> bool:
    """Does e hold a quantifier or a set membership (worth a short circuit)?"""
    return any(isinstance(x, (Quant, Contains)) for x in _walk(e))


def _init_member(q):
    """P.exists(j => init(j.f) == t) with t free of j: (f, t), else None."""
    if q.kind != "exists" or not (isinstance(q.body, Bin) and q.body.op == "EQ"):
        return None
    uid = q.var.uid
    for a, b in ((q.body.x, q.body.y), (q.body.y, q.body.x)):
        if (isinstance(a, Field) and a.tag == TAG_INIT and isinstance(a.proc, Var) and a.proc.uid == uid
                and uid not in {x.uid for x in _walk(b) if isinstance(x, Var)}):
            return a.f, b
    return None


def _skey(e, memo):
    """Structural key of e, bound variables numbered by binding depth from e: two closed
    subformulas with equal keys are the same formula (common-subformula hoisting finds the
    repeats of Formula text, where every occurrence is its own tree, as well as those of one
    Python object)."""
    got = memo.get(id(e))
    if got is not None and got[0] is e:  # the key object is kept alive with its entry
        return got[1]

    def rec(x, env):
        if isinstance(x, Var):
            return ("V", env[x.uid]) if x.uid in env else ("free", x.uid)
        if isinstance(x, Lit):
            return ("L", x.v)
        if isinstance(x, NVal):
            return ("N",)
        if isinstance(x, RVal):
            return ("R",)
        if isinstance(x, CoordVal):
            return ("K",)
        if isinstance(x, Field):
            return ("F", x.f, x.tag, rec(x.proc, env))
        if isinstance(x, Un):
            return ("U", x.op, rec(x.x, env))
        if isinstance(x, Bin):
            return ("B", x.op, rec(x.x, env), rec(x.y, env))
        if isinstance(x, Quant):
            return ("Q", x.kind, rec(x.body, {**env, x.var.uid: len(env)}))
        if isinstance(x, Contains):
            return ("C", rec(x.e, env), rec(x.comp.body, {**env, x.comp.var.uid: len(env)}))
        raise FormulaError(f"unsupported node {type(x).__name__}")

    k = rec(e, {})
    memo[id(e)] = (e, k)
    return k


def _symmetric(q):
    """Does the body of process quantifier q read its variable only through current / old
    fields (no init field, no use as a pid)?"""
    uid = q.var.uid
    nvar = nfield = 0
    for x in _walk(q.body):
        if isinstance(x, Var) and x.uid == uid:
            nvar += 1
        elif isinstance(x, Field) and isinstance(x.proc, Var) and x.proc.uid == uid:
            if x.tag == TAG_INIT:
                return False
            nfield += 1
    return nvar == nfield


def _tuple_fields(q):
    """Fields (field, tag) through which the body of a process quantifier reads its
    variable, or None if the variable is used otherwise (compared as a pid, bound by
    a set membership, ...)."""
    uid = q.var.uid
    out = []
    field_procs = set()
    for x in _walk(q.body):
        if isinstance(x, Field) and isinstance(x.proc, Var) and x.proc.uid == uid:
            field_procs.add(id(x.proc))
            if (x.f, x.tag) not in out:
                out.append((x.f, x.tag))
    for x in _walk(q.body):
        if isinstance(x, Var) and x.uid == uid and id(x) not in field_procs:
            return None
    return out if len(out) <= 4 else None


def _tuple_guard(q):
    """Conjuncts A of forall(j => A && .. ==> B) / exists, count(j => A && .. && B) that read
    only j's fields (no quantifier, set or other variable): the processes where one fails
    contribute nothing, so the distinct-state walk visits only those where all hold."""
    uid = q.var.uid
    if q.kind == "forall":
        if not (isinstance(q.body, Bin) and q.body.op == "IMPL"):
            return []
        cs = _conjuncts(q.body.x)
    else:
        cs = _conjuncts(q.body)
    return [c for c in cs if _free_vars(c) == {uid} and not _expensive(c)]


def _conjuncts(e):
    if isinstance(e, Bin) and e.op == "AND":
        return _conjuncts(e.x) + _conjuncts(e.y)
    return [e]


# breakpoint offsets (bit d+1: b = e + d) of an atom `t OP e` with t the V.exists variable
_BP_SHIFT = {"LE": 2, "GT": 2, "LT": 1, "GE": 1, "EQ": 3, "NE": 3}
_FLIP = {"LE": "GE", "GE": "LE", "LT": "GT", "GT": "LT", "EQ": "EQ", "NE": "NE"}


def _breakpoint_shifts(q, exprs, fsets):
    """Per candidate source of _Compiler.witnesses (exprs, then field sets): the union of
    the breakpoint offsets of the atoms comparing the variable with it (exists_int_bp)."""
    uid = q.var.uid
    es = [0] * len(exprs)
    fm = {k: 0 for k in fsets}
    for x in _walk(q.body):
        if not (isinstance(x, Bin) and x.op in _BP_SHIFT):
            continue
        for a, b, op in ((x.x, x.y, x.op), (x.y, x.x, _FLIP[x.op])):
            if not (isinstance(a, Var) and a.uid == uid):
                continue
            t = _strip(b)
            if isinstance(t, Field):
                fm[(t.f, t.tag)] |= _BP_SHIFT[op]
            else:
                hit = [i for i, e in enumerate(exprs) if e is t]
                if not hit:
                    return [7] * (len(exprs) + len(fsets))  # unmatched source: every offset (exact)
                for i in hit:
                    es[i] |= _BP_SHIFT[op]
    out = es + [fm[k] for k in fsets]
    return [m if m else 7 for m in out]


def _eq_only(q) -> bool:
    """Is the V.exists variable of q compared with == / != only?"""
    uid = q.var.uid
    for x in _walk(q.body):
        if isinstance(x, Bin) and x.op in ("LT", "LE", "GT", "GE"):
            for a in (x.x, x.y):
                if isinstance(a, Var) and a.uid == uid:
                    return False
    return True


def _pins(body, uid, banned=frozenset()):
    """Equality pins of the V.exists variable `uid` in `body`: the first top-level conjunct
    P.forall(i => c1 && c2 && ...) having conjuncts `cond ==> term == v` or `term == v`
    (cond, term free of v): (that forall, [(cond or None, term)]), else None. A conjunct
    V.exists(t => B) is searched too, for pins free of t: they constrain v for every t, so
    they pin v across the inner quantifier (LastVoting: decided ==> decision == v)."""
    for c in _conjuncts(body):
        if isinstance(c, Quant) and c.kind == "vint":
            got = _pins(c.body, uid, banned | {c.var.uid})
            if got is not None:
                return got
            continue
        if not (isinstance(c, Quant) and c.kind == "forall"):
            continue
        out = []
        for d in _conjuncts(c.body):
            cond, eq = (d.x, d.y) if isinstance(d, Bin) and d.op == "IMPL" else (None, d)
            if cond is not None and (uid in _free_vars(cond) or _free_vars(cond) & banned):
                continue
            if not (isinstance(eq, Bin) and eq.op == "EQ"):
                continue
            for term, other in ((eq.x, eq.y), (eq.y, eq.x)):
                if (isinstance(other, Var) and other.uid == uid and uid not in _free_vars(term)
                        and not (_free_vars(term) & banned)):
                    out.append((cond, term))
                    break
        if out:
            return c, out
    return None


# The swap below is exact but measured slower on LastVoting's majority clause (fused LV
# n=64: 205 -> 346 ms per 1.25e7 instances, scripts/fused_breakdown.py): the original order
# finds its witness early (the first value candidate with the first passing round), the
# swapped one tries every round candidate. Off by default; the tests exercise both.
SWAP_VINT = False


# The symmetric-check-point lowering (spec::uniform); off only for A/B measurements (the C ABI's
# generator, psg_spec_gen.cpp, always emits it).
SYMMETRIC_LOWERING = True
SYMMETRIC_MAX_FIELDS = 6  # (field, tag) pairs compared by spec::uniform; more: no symmetric lowering


def _rewrite_vint(e, memo=None):
    """Rewrites of V.exists over Int for the native lowering, exact for every input (the
    domain is non-empty and both sides are decided exactly):
      V.exists(v => V.exists(t => B)) -> V.exists(t => V.exists(v => B)) when v has equality
        pins in B and t has none (the pinned variable innermost, where one candidate decides it);
      V.exists(v => A && B(v)) -> A && V.exists(v => B(v)) for the conjuncts A free of v,
        P.forall conjuncts split first (_split_forall: LastVoting's majority clause evaluates
        its v- and t-free implications once, not per candidate).
    Shared subformulas stay shared (memo by object)."""
    memo = {} if memo is None else memo
    k = id(e)
    if k in memo and memo[k][0] is e:  # the key object is kept alive with its entry (ids are reused)
        return memo[k][1]
    out = e
    if (SWAP_VINT and isinstance(e, Quant) and e.kind == "vint" and isinstance(e.body, Quant)
            and e.body.kind == "vint"
            and _pins(e.body.body, e.var.uid) is not None and _pins(e.body.body, e.body.var.uid) is None):
        out = _rewrite_vint(Quant("vint", e.body.var, Quant("vint", e.var, e.body.body)), memo)
    elif isinstance(e, Quant):
        b = _rewrite_vint(e.body, memo)
        out = e if b is e.body else Quant(e.kind, e.var, b)
        if out.kind == "vint":
            out = _vint_step(out, memo)
        elif out.kind in ("exists", "forall") and SPLIT_FORALL:
            out = _proc_step(out)
    elif isinstance(e, Bin):
        x, y = _rewrite_vint(e.x, memo), _rewrite_vint(e.y, memo)
        out = e if (x is e.x and y is e.y) else Bin(e.op, x, y)
    elif isinstance(e, Un):
        x = _rewrite_vint(e.x, memo)
        out = e if x is e.x else Un(e.op, x)
    elif isinstance(e, Contains):
        b, x = _rewrite_vint(e.comp.body, memo), _rewrite_vint(e.e, memo)
        out = e if (b is e.comp.body and x is e.e) else Contains(Comprehension(e.comp.var, b), x)
    memo[k] = (e, out)
    return out


# V.exists(v => ... && P.forall(i => A(i) && B(i, v)) && ...): the forall splits into
# P.forall(A) && P.forall(B) so that A, free of v, leaves the quantifier (_vint_step) when A
# does cross-lane work (reads another process's field: LastVoting's coord.commit); A of the
# lane's own fields stays in the forall (a separate forall would cost one more ballot than it
# saves). Off only for A/B measurements (psg_spec_gen.cpp always splits).
SPLIT_FORALL = True


def _cross(d, uid):
    """d reads a field of a process other than `uid`, or holds a quantifier / set membership."""
    for x in _walk(d):
        if isinstance(x, (Quant, Contains)):
            return True
        if isinstance(x, Field) and not (isinstance(x.proc, Var) and x.proc.uid == uid):
            return True
    return False


def _split_forall(c, v, cross_only=True):
    """P.forall(i => A && B) with conjuncts A free of v (and doing cross-lane work, cross_only)
    and the rest B -> [P.forall(A), P.forall(B)] (forall distributes over &&: exact)."""
    if SPLIT_FORALL and isinstance(c, Quant) and c.kind == "forall":
        ds = _conjuncts(c.body)
        out = [v not in _free_vars(d) and (not cross_only or _cross(d, c.var.uid)) for d in ds]
        fr = [d for d, o in zip(ds, out) if o]
        bd = [d for d, o in zip(ds, out) if not o]
        if fr and bd:
            return [Quant("forall", c.var, And(*fr)), Quant("forall", c.var, And(*bd))]
    return [c]


def _proc_step(q):
    """P.exists(j => A && B(j)) -> A && P.exists(j => B(j)), the same for P.forall (n >= 1: exact),
    for the conjuncts A free of j, a conjunct P.forall(i => A(i) && B(i, j)) split first
    (LastVoting's / OTR's P.exists(j => P.forall(i => i.decided && i.decision == init(j.x))):
    the serial walk over i runs only once every process decided)."""
    v = q.var.uid
    cs = [d for c in _conjuncts(q.body) for d in _split_forall(c, v, cross_only=False)]
    free = [c for c in cs if v not in _free_vars(c)]
    bound = [c for c in cs if v in _free_vars(c)]
    if free and bound:
        return And(*free, Quant(q.kind, q.var, And(*bound)))
    return q


def _vint_step(q, memo):
    v, body = q.var.uid, q.body
    cs = [d for c in _conjuncts(body) for d in _split_forall(c, v)]
    free = [c for c in cs if v not in _free_vars(c)]
    bound = [c for c in cs if v in _free_vars(c)]
    if free and bound:
        return And(*free, Quant("vint", q.var, And(*bound)))
    return q


def _count_guard(q):
    """A top-level conjunct `P.filter(i => i.f == v).size OP thr` (OP in >, >=, ==; thr
    free of bound variables) of V.exists(v => body): ((f, tag), thr, OP) or None."""
    uid = q.var.uid
    for c in _conjuncts(q.body):
        if not isinstance(c, Bin) or c.op not in ("GT", "GE", "EQ", "LT", "LE"):
            continue
        cnt, thr, op = c.x, c.y, c.op
        if not (isinstance(cnt, Quant) and cnt.kind == "count"):
            cnt, thr = c.y, c.x
            op = {"LT": "GT", "LE": "GE", "EQ": "EQ", "GT": "LT", "GE": "LE"}[c.op]
        if op not in ("GT", "GE", "EQ") or not (isinstance(cnt, Quant) and cnt.kind == "count"):
            continue
        if any(isinstance(x, (Var, Quant, Field, Contains)) for x in _walk(thr)):
            continue  # the threshold must be uniform (n, r, literals)
        b = cnt.body
        if not (isinstance(b, Bin) and b.op == "EQ"):
            continue
        for fld, other in ((b.x, b.y), (b.y, b.x)):
            if (isinstance(fld, Field) and isinstance(fld.proc, Var) and fld.proc.uid == cnt.var.uid
                    and isinstance(other, Var) and other.uid == uid):
                return (fld.f, fld.tag), thr, op
    return None


def codegen_hip(spec: Spec, alg: Optional[int] = None) -> Tuple[str, Program]:
    """HIP source of the native checker of `spec` (+ the bytecode Program it replaces)."""
    prog = compile_spec(spec, alg)
    gen = _Gen(ALG_FIELDS.get(alg) if alg is not None else None)
    guard = _rinv_guard(spec)
    memo = {}
    invs = [_rewrite_vint(inv if guard is None else (inv & guard), memo) for inv in spec.invariants]
    props = [(name, _rewrite_vint(f, memo)) for name, f in spec.properties]
    safety = None if spec.safety_predicate is None else _rewrite_vint(spec.safety_predicate, memo)
    # common closed subformulas (the same formula in several places, e.g. OTR's keepInit in
    # Invariant0 and Invariant1; structurally equal, _skey): hoisted, evaluated once per check point
    roots = list(invs) + [f for name, f in props if name != "Termination"]
    if safety is not None:
        roots.append(safety)
    seen, order = {}, []

    def visit(e):
        k = _skey(e, gen.skeys)
        seen[k] = seen.get(k, 0) + 1
        if seen[k] > 1:
            return
        for c in e.children():
            visit(c)
        order.append(e)  # post-order: inner subformulas first

    for rt in roots:
        visit(rt)

    def tup_decls(used, ind):
        out = []
        for k in gen.tup_sets:
            if k not in used:
                continue
            flds, gcode = (k, None) if not (len(k) == 2 and isinstance(k[1], str)) else k
            fl = ", ".join(f"spec::Fld<{f}, {tag}>{{}}" for f, tag in flds)
            if gcode is None:
                out.append(f"{ind}const auto {gen.tup_sets[k]} = spec::tup_uniform<W>(x, {fl});")
            else:
                out.append(f"{ind}const auto {gen.tup_sets[k]} = spec::tup_uniform_g<W>(x, {gcode}, {fl});")
        return out

    def block(uni):
        """The slot lines of fail() and the Termination expression, under the general or the
        symmetric-check-point lowering. A distinct-state tuple test is declared just before the
        first line that uses it (short live ranges: the fused kernels are register-bound)."""
        gen.uni, gen.cse, gen.tup_used = uni, {}, set()
        ind, pre = ("      ", "ucse") if uni else ("    ", "cse")
        lines = []

        def add(e, fmt):
            before = set(gen.tup_used)
            c, _ = gen.gen(e, False, 0)
            lines.extend(tup_decls(gen.tup_used - before, ind))
            lines.append(fmt(c))

        slot = 0
        for e in order:
            if seen[_skey(e, gen.skeys)] > 1 and isinstance(e, (Quant, Contains)) and not _free_vars(e):
                name = f"{pre}{len(gen.cse)}"
                add(e, lambda c, name=name: f"{ind}const int32_t {name} = {c};")
                gen.cse[_skey(e, gen.skeys)] = name
        iv = "uinv" if uni else "inv"
        if invs:
            for k, inv in enumerate(invs):
                add(inv, lambda c, k=k: f"{ind}const int32_t {iv}{k} = {c};")
            lines.append(f"{ind}if (!(" + " | ".join(f"({iv}{k} != 0)" for k in range(len(invs)))
                         + f")) fb |= 1u << {slot};")
            slot += 1
            for k in range(len(invs)):
                lines.append(f"{ind}if ({iv}{k} == 0) fb |= 1u << {slot};")
                slot += 1
        term = None
        term_tups = set()
        for name, f in props:
            if name == "Termination":
                # term() is its own function: fail()'s hoisted subformulas (cse*) and tuple
                # tests are not in scope there, so it is lowered with neither
                saved, gen.tup_used = gen.tup_used, set()
                saved_cse, gen.cse = gen.cse, {}
                term, _ = gen.gen(f, False, 0)
                term_tups, gen.tup_used = gen.tup_used, saved
                gen.cse = saved_cse
                continue
            add(f, lambda c, slot=slot, name=name: f"{ind}if (({c}) == 0) fb |= 1u << {slot};  // {name}")
            slot += 1
        if safety is not None:
            add(safety, lambda c, slot=slot: f"{ind}if (({c}) == 0) fb |= 1u << {slot};  // SafetyPredicate")
            slot += 1
        assert slot == len(prog.slot_entry)
        return lines, term, tup_decls(term_tups, ind), slot

    lines, term, term_decls, slot = block(False)
    # symmetric check points (every process holds the same value of each current / old field
    # the Spec reads): a second, scalar lowering, chosen per check point by spec::uniform
    ulines, uterm, uterm_decls, _ = block(True)
    gen.uni = False
    # worth its test only with few fields to compare: OTR's 5 (x, decided, decision; old decided,
    # decision) are symmetric at 86 % of check points (fused OTR 13.4 -> 11.6 ms per 2.5e6
    # instances), LastVoting's 9 almost never (22.9 -> 24.4 ms: the test is pure overhead)
    if gen.uft and len(gen.uft) <= SYMMETRIC_MAX_FIELDS and SYMMETRIC_LOWERING:
        cur = sum(1 << f for f, t in gen.uft if t == TAG_CUR)
        old = sum(1 << f for f, t in gen.uft if t == TAG_OLD)
        lines = ([f"    if (spec::uniform<W, {cur}u, {old}u>(x)) {{"] + ulines + ["      return fb;", "    }"]
                 + lines)
        if term:
            term_decls = (["    if (x.uni) {"] + uterm_decls + [f"      return ({uterm}) != 0;", "    }"]
                          + term_decls)
    if gen.max_vi > 4:
        raise FormulaError("more than 4 nested V.exists over Int")
    rel = sum(1 << s for s, fl in enumerate(prog.slot_flags) if fl & SPEC_RELATIONAL)
    fmask = sum(1 << f for f in gen.fields)
    tmask = sum(1 << t for t in gen.tags)
    src = [
        "// generated by round_amd/formula.py (codegen_hip): native checker of one Spec",
        '#include "psg_spec_native.hpp"',
        "namespace psg {",
        "struct GenSpec {",
        f"  static constexpr int kSlots = {slot};",
        f"  static constexpr uint32_t kRelational = {rel}u;",
        f"  static constexpr bool kHasTerm = {'true' if term else 'false'};",
        f"  static constexpr uint32_t kFields = {fmask}u;",
        f"  static constexpr uint32_t kTags = {tmask}u;",
        f"  static constexpr int kInitSet0 = {gen.init_sets[0] if len(gen.init_sets) > 0 else -1};",
        f"  static constexpr int kInitSet1 = {gen.init_sets[1] if len(gen.init_sets) > 1 else -1};",
        "  template <int W>",
        "  __device__ static uint32_t fail(spec::Ctx<W>& x, int32_t* scratch) {",
        "    (void)scratch;",
        "    uint32_t fb = 0;",
        *lines,
        "    return fb;",
        "  }",
        "  template <int W>",
        "  __device__ static bool term(spec::Ctx<W>& x, int32_t* scratch) {",
        "    (void)scratch;",
        *term_decls,
        f"    return ({term or '0'}) != 0;",
        "  }",
        "};",
        "}  // namespace psg",
        "PSG_SPEC_NATIVE_KERNELS(psg::GenSpec)",
        f'extern "C" __device__ int32_t psg_spec_alg = {int(alg or 0)};  // checked by psg_run_batch_spec',
        "",
    ]
    return "\n".join(src), prog


# algorithm -> (round-kernel source, body template, leading template arguments) for fused modules
FUSED_KERNELS = {
    abi.PSG_ALG_OTR: ("psg_otr.hip", "otr_body", "{W}, false"),
    abi.PSG_ALG_OTR2: ("psg_otr.hip", "otr_body", "{W}, true"),
    abi.PSG_ALG_LAST_VOTING: ("psg_lv.hip", "lv_body", "{W}"),
    abi.PSG_ALG_FLOODMIN: ("psg_floodmin.hip", "floodmin_body", "{W}"),
    abi.PSG_ALG_KSET: ("psg_kset.hip", "kset_body", "{W}"),
    abi.PSG_ALG_BENOR: ("psg_benor.hip", "benor_body", "{W}"),
    abi.PSG_ALG_SLV: ("psg_slv.hip", "slv_body", "{W}"),
    abi.PSG_ALG_KSET_ES: ("psg_kset_es.hip", "kset_es_body", "{W}"),
}


FUSED_WPE = {abi.PSG_ALG_LAST_VOTING: 6}


def _fused_source(alg: int, waves: Sequence[int]) -> str:
    """The algorithm's round kernel instantiated with the generated Spec as its hook:
    extern "C" psg_fused_a<alg>_w<W> (seeded HO sets) / psg_fused_x_a<alg>_w<W> (explicit)."""
    import os
    src, body, targs = FUSED_KERNELS[alg]
    out = [f'#include "{src}"  // its kernel bodies; host launchers are compiled out (PSG_FUSED_MODULE)']
    # occupancy target of the W = 1 kernels (0: the compiler's); LastVoting's generated check
    # otherwise takes 92 VGPRs (5 waves/SIMD): 6 measured 155.6 -> 147.5 ms on C3 (7: no gain)
    wpe = int(os.environ.get("PSG_FUSED_WPE") or FUSED_WPE.get(alg, 0))
    for W in waves:
        threads = 256 if W == 1 else 64 * W
        attr = f"__attribute__((amdgpu_waves_per_eu({wpe}))) " if W == 1 and wpe > 0 else ""
        for suffix, xho in (("", "false"), ("x_", "true")):
            out.append(f'extern "C" __global__ void __launch_bounds__({threads}) {attr}'
                       f'psg_fused_{suffix}a{alg}_w{W}(psg::KArgs a) {{')
            out.append(f"  psg::{body}<{targs.format(W=W)}, {xho}, psg::spec::SpecHook<psg::GenSpec>>(a);")
            out.append("}")
    return "\n".join(out) + "\n"


def compile_native(spec: Spec, alg: Optional[int] = None, cache_dir: str = None, hipcc: str = None,
                   fused: bool = False, n: Optional[int] = None, defines: Sequence[str] = ()) -> Program:
    """Lower `spec` to native gfx950 code (hipcc --genco, cached by source hash) and
    return a Program whose module_path psg_run_batch_spec launches instead of the
    bytecode interpreter.

    fused=True also instantiates the algorithm's round kernel with the Spec as its
    check hook (spec::SpecHook): psg_run_batch_spec then runs ONE launch that
    executes the rounds and evaluates the Spec from registers, with no state trace.
    `n` (optional) limits the instantiations to that group size's wave count. `defines`: extra
    preprocessor definitions (e.g. "PSG_PHASE_TIMERS=1" for a profiling module; part of the
    cache key)."""
    import hashlib
    import os
    import subprocess
    src, prog = codegen_hip(spec, alg)
    hdr_names = ["psg_spec_native.hpp", "psg_device.hpp"]
    if fused:
        if alg not in FUSED_KERNELS:
            raise FormulaError("fused lowering needs one of the integer-state algorithms")
        waves = [(n + 63) // 64] if n is not None else [1, 2, 3, 4]
        src = "#define PSG_FUSED_MODULE 1\n" + src + _fused_source(alg, waves)
        hdr_names += [FUSED_KERNELS[alg][0], "psg_kernels.hpp", "psg_packed.hpp"]  # everything it includes
    cache_dir = cache_dir or CACHE_DIR
    os.makedirs(cache_dir, exist_ok=True)
    hdrs = "".join(open(os.path.join(_CSRC, h)).read() for h in hdr_names)
    dflags = [f"-D{d}" for d in defines]
    key_src = src + hdrs + open(os.path.join(_INCLUDE, "psg.h")).read() + ("".join(dflags) if dflags else "")
    key = hashlib.sha256(key_src.encode()).hexdigest()[:24]
    out = os.path.join(cache_dir, f"spec_{key}.co")
    if not os.path.exists(out):
        path = os.path.join(cache_dir, f"spec_{key}.hip")
        with open(path, "w") as f:
            f.write(src)
        cmd = [hipcc or os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "--genco", "--offload-arch=gfx950", "-O3",
               "-std=c++17", "-I", _CSRC, "-I", _INCLUDE, *dflags, path, "-o", out + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise FormulaError("native spec compile failed:\n" + r.stderr[-4000:])
        os.replace(out + ".tmp", out)
    prog.module_path = out
    return prog


# --------------------------------------------------------------------------- Formula text (JVM interchange)
# A Spec as the S-expression text of the reference's own Formula trees
# (psync/formula/Formula.scala:20-583: Binding(ForAll | Exists | Comprehension),
# Application(symbol, args), Variable, Literal), as integration/scala/GpuSpec.scala
# writes it from a psync.Spec and as psg_spec_from_text (psg_spec_text.cpp, the C ABI)
# compiles it; `from_text` here gives the same Spec in this DSL (for compile_native).
#
#   spec  := (Spec (phase L) (invariants f*) (roundInvariants (list f*)*)
#                  (properties (prop "Name" f)*) [(safetyPredicate f)])
#   f     := (ForAll (decl+) f) | (Exists (decl+) f) | (Comprehension (decl) f)
#          | (App SYMBOL f*) | (Var NAME) | (Lit INT | true | false)
#   decl  := (NAME pid | Int | Time | Bool | Set)       (Time: the round type, read as Int)
#
# Symbols: the InterpretedFct names And Or Not Implies Eq Neq Lt Leq Gt Geq Plus Minus
# Times Divides In Contains Cardinality IsDefined IsEmpty Get Some (Formula.scala:175-348;
# Remainder is this format's `%`), toInt / fromInt (psync.logic.ReduceTime, Time <-> Int,
# identities here), process fields x decided decision ts ready commit vote
# canDecide est with the `__init__` / `__old__` prefixes of init(...) / old(...)
# (psync/verification/Utils.scala:24-25), HO (Cardinality(HO(p)) = |HO(p)|) and coord.
# Variables n and r and coord are the free ones. FormulaExtractor's
# `val A = P.filter(...); body` arrives as (Exists ((A Set)) (App And (App Eq (Var A)
# (Comprehension ...)) body...)) and is substituted back.
FIELD_NAMES = {"x": FIELD_X, "decided": FIELD_DECIDED, "decision": FIELD_DECISION, "ts": FIELD_TS,
               "ready": FIELD_READY, "commit": FIELD_COMMIT, "vote": FIELD_VOTE, "canDecide": FIELD_CANDECIDE,
               "est": FIELD_X}
_FIELD_TEXT = {FIELD_X: "x", FIELD_DECIDED: "decided", FIELD_DECISION: "decision", FIELD_TS: "ts",
               FIELD_READY: "ready", FIELD_COMMIT: "commit", FIELD_VOTE: "vote", FIELD_CANDECIDE: "canDecide"}
_BIN_TEXT = {"AND": "And", "OR": "Or", "IMPL": "Implies", "EQ": "Eq", "NE": "Neq", "LT": "Lt", "LE": "Leq",
             "GT": "Gt", "GE": "Geq", "ADD": "Plus", "SUB": "Minus", "MUL": "Times", "DIV": "Divides",
             "MOD": "Remainder"}
_TEXT_BIN = {v: k for k, v in _BIN_TEXT.items()}


def _expr_text(e, names) -> str:
    def nm(v):
        if v.uid not in names:
            names[v.uid] = f"{v.kind[0]}{len(names)}"
        return names[v.uid]

    def t(e):
        if isinstance(e, Lit):
            return f"(Lit {e.v})"
        if isinstance(e, NVal):
            return "(Var n)"
        if isinstance(e, RVal):
            return "(Var r)"
        if isinstance(e, CoordVal):
            return "(Var coord)"
        if isinstance(e, Var):
            return f"(Var {nm(e)})"
        if isinstance(e, Field):
            if e.f == FIELD_HOSIZE:
                return f"(App Cardinality (App HO {t(e.proc)}))"
            pre = {TAG_CUR: "", TAG_OLD: "__old__", TAG_INIT: "__init__"}[e.tag]
            return f"(App {pre}{_FIELD_TEXT[e.f]} {t(e.proc)})"
        if isinstance(e, Un):
            op = {"NOT": "Not", "NEG": "Minus", "ISDEF": "IsDefined"}[e.op]
            return f"(App {op} {t(e.x)})"
        if isinstance(e, Bin):
            return f"(App {_BIN_TEXT[e.op]} {t(e.x)} {t(e.y)})"
        if isinstance(e, Contains):
            return f"(App In {t(e.e)} {comp(e.comp)})"
        if isinstance(e, Quant):
            if e.kind == "count":
                return f"(App Cardinality (Comprehension (({nm(e.var)} pid)) {t(e.body)}))"
            typ = {"forall": "pid", "exists": "pid", "vint": "Int", "vbool": "Bool"}[e.kind]
            b = "ForAll" if e.kind == "forall" else "Exists"
            return f"({b} (({nm(e.var)} {typ})) {t(e.body)})"
        raise FormulaError(f"cannot write {type(e).__name__} as Formula text")

    def comp(c):
        return f"(Comprehension (({nm(c.var)} pid)) {t(c.body)})"

    return t(e)


def to_text(spec: Spec) -> str:
    """The Spec as Formula text (the interchange format above)."""
    names: Dict[int, str] = {}
    out = [f"(Spec (phase {spec.phase_length})"]
    out.append("  (invariants " + " ".join(_expr_text(f, names) for f in spec.invariants) + ")")
    out.append("  (roundInvariants " + " ".join(
        "(list " + " ".join(_expr_text(f, names) for f in l) + ")" for l in spec.round_invariants) + ")")
    out.append("  (properties " + " ".join(f'(prop "{nm}" {_expr_text(f, names)})' for nm, f in spec.properties)
               + ")")
    if spec.safety_predicate is not None:
        out.append("  (safetyPredicate " + _expr_text(spec.safety_predicate, names) + ")")
    return "\n".join(out) + ")"


def _sexp(text: str):
    toks, i = [], 0
    while i < len(text):
        ch = text[i]
        if ch.isspace():
            i += 1
        elif ch in "()":
            toks.append(ch)
            i += 1
        elif ch == '"':
            j = text.index('"', i + 1)
            toks.append(("str", text[i + 1:j]))
            i = j + 1
        else:
            j = i
            while j < len(text) and not text[j].isspace() and text[j] not in '()"':
                j += 1
            toks.append(text[i:j])
            i = j
    pos = 0

    def parse():
        nonlocal pos
        if pos >= len(toks):
            raise FormulaError("Formula text: unexpected end")
        tk = toks[pos]
        pos += 1
        if tk == "(":
            lst = []
            while pos < len(toks) and toks[pos] != ")":
                lst.append(parse())
            if pos >= len(toks):
                raise FormulaError("Formula text: missing )")
            pos += 1
            return lst
        if tk == ")":
            raise FormulaError("Formula text: unexpected )")
        return tk

    v = parse()
    if pos != len(toks):
        raise FormulaError("Formula text: trailing input")
    return v


def _from_sexp(s, env):
    if not isinstance(s, list) or not s:
        raise FormulaError(f"Formula text: expected a form, got {s!r}")
    head = s[0]
    if head == "Lit":
        v = s[1]
        return Lit(1 if v == "true" else 0 if v == "false" else int(v))
    if head == "Var":
        name = s[1]
        if name in env:
            return env[name]
        if name == "n":
            return NVal()
        if name == "r":
            return RVal()
        if name == "coord":
            return CoordVal()
        raise FormulaError(f"Formula text: unbound variable {name}")
    if head in ("ForAll", "Exists"):
        decls, body = s[1], s[2]
        if not decls:
            raise FormulaError("Formula text: binder without variables")
        (name, typ), rest = decls[0], decls[1:]
        inner = [head, rest, body] if rest else body
        if typ == "Set":  # FormulaExtractor's `val A = ...; body`
            if head != "Exists":
                raise FormulaError("Formula text: a Set variable is only bound by a let (Exists)")
            return _let(name, inner, env)
        if typ == "pid":
            v = Var("proc")
            return Quant("forall" if head == "ForAll" else "exists", v, _from_sexp(inner, {**env, name: v}))
        if head == "ForAll":
            raise FormulaError(f"Formula text: ForAll over {typ} cannot be checked (only V.exists)")
        if typ not in ("Int", "Time", "Bool"):
            raise FormulaError(f"Formula text: unknown type {typ}")
        v = Var("bool" if typ == "Bool" else "int")
        return Quant("vbool" if typ == "Bool" else "vint", v, _from_sexp(inner, {**env, name: v}))
    if head == "Comprehension":
        return _comp(s, env)
    if head == "App":
        sym, args = s[1], s[2:]
        a = lambda k: _from_sexp(args[k], env)  # noqa: E731
        if sym in ("And", "Or"):
            out = a(0)
            for k in range(1, len(args)):
                out = Bin(sym.upper(), out, a(k))
            return out
        if sym in _TEXT_BIN:
            if sym == "Minus" and len(args) == 1:
                return Un("NEG", a(0))
            return Bin(_TEXT_BIN[sym], a(0), a(1))
        if sym == "Not":
            return Un("NOT", a(0))
        if sym == "IsDefined":
            return Un("ISDEF", a(0))
        if sym == "IsEmpty":
            return Un("NOT", Un("ISDEF", a(0)))
        if sym in ("Get", "Some", "toInt", "fromInt"):  # Option get / Some; Time <-> Int (ReduceTime)
            return a(0)
        if sym == "Cardinality":
            x = args[0]
            if isinstance(x, list) and x and x[0] == "App" and x[1] == "HO":
                return Field(FIELD_HOSIZE, _from_sexp(x[2], env))
            c = _set(x, env)
            return c.size
        if sym in ("In", "Contains"):
            elem, st = (args[0], args[1]) if sym == "In" else (args[1], args[0])
            return _set(st, env).contains(_from_sexp(elem, env))
        if sym == "coord" and not args:
            return CoordVal()
        tag, base = TAG_CUR, sym
        if sym.startswith("__init__"):
            tag, base = TAG_INIT, sym[len("__init__"):]
        elif sym.startswith("__old__"):
            tag, base = TAG_OLD, sym[len("__old__"):]
        if base in FIELD_NAMES and len(args) == 1:
            return Field(FIELD_NAMES[base], a(0), tag)
        raise FormulaError(f"Formula text: unknown symbol {sym}/{len(args)}")
    raise FormulaError(f"Formula text: unknown form {head}")


def _comp(s, env):
    (name, typ), = s[1]
    if typ != "pid":
        raise FormulaError("Formula text: comprehensions range over processes")
    v = Var("proc")
    return Comprehension(v, _from_sexp(s[2], {**env, name: v}))


def _set(s, env):
    if isinstance(s, list) and s and s[0] == "Comprehension":
        return _comp(s, env)
    if isinstance(s, list) and s and s[0] == "Var" and isinstance(env.get(s[1]), Comprehension):
        return env[s[1]]
    raise FormulaError("Formula text: expected a set of processes")


def _let(name, body, env):
    """Exists A: Set. A == {..} && rest  ->  rest with A := {..}."""
    conj = []

    def flat(x):
        if isinstance(x, list) and len(x) >= 3 and x[0] == "App" and x[1] == "And":
            for y in x[2:]:
                flat(y)
        else:
            conj.append(x)

    flat(body)
    for k, c in enumerate(conj):
        if isinstance(c, list) and len(c) == 4 and c[0] == "App" and c[1] == "Eq":
            for lhs, rhs in ((c[2], c[3]), (c[3], c[2])):
                if lhs == ["Var", name] and isinstance(rhs, list) and rhs and rhs[0] == "Comprehension":
                    rest = conj[:k] + conj[k + 1:]
                    if not rest:
                        return Lit(1)
                    env2 = {**env, name: _comp(rhs, env)}
                    return _from_sexp(rest[0] if len(rest) == 1 else ["App", "And"] + rest, env2)
    raise FormulaError(f"Formula text: Set variable {name} is not defined by a conjunct {name} == {{...}}")


def from_text(text: str) -> Spec:
    """Parse Formula text (the interchange format above) into a Spec."""
    s = _sexp(text)
    if not (isinstance(s, list) and s and s[0] == "Spec"):
        raise FormulaError("Formula text: expected (Spec ...)")
    phase, invs, rinv, props, sp = 1, [], [], [], None
    for part in s[1:]:
        key = part[0]
        if key == "phase":
            phase = int(part[1])
        elif key == "invariants":
            invs = [_from_sexp(f, {}) for f in part[1:]]
        elif key == "roundInvariants":
            rinv = [[_from_sexp(f, {}) for f in l[1:]] for l in part[1:]]
        elif key == "properties":
            props = [(p[1][1], _from_sexp(p[2], {})) for p in part[1:]]
        elif key == "safetyPredicate":
            sp = _from_sexp(part[1], {})
        else:
            raise FormulaError(f"Formula text: unknown Spec part {key}")
    return Spec(invs, rinv, props, safety_predicate=sp, phase_length=phase)


def compile_text(text: str, alg: Optional[int] = None) -> Program:
    """Formula text -> bytecode Program through the C ABI (psg_spec_from_text in libpsg),
    the path the JVM plugin takes; equal to compile_spec(from_text(text), alg)."""
    from . import lib
    return lib.spec_from_text(text, alg or 0)
