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
# The lowering of a Spec to gfx950 code lives in the library, psg_spec_gen.cpp
# (psg_spec_compile_native): ONE generator for this DSL and for the C ABI / JVM route
# (GpuSpec.scala). compile_native writes the Spec as Formula text (to_text below) and has the
# library lower and compile it in-process (hiprtc), cached under build/spec by a hash of the
# source, the kernel headers and the compiler identity. The rewrites it applies are exact for
# every input (psg_spec_rewrite_text exposes them: tests/test_formula.py checks them against
# the Spec as written under the CPU interpreter); DESIGN.md §5 lists them.

# algorithms whose round kernel a fused module instantiates with the Spec as its check hook
FUSED_KERNELS = frozenset({abi.PSG_ALG_OTR, abi.PSG_ALG_OTR2, abi.PSG_ALG_LAST_VOTING, abi.PSG_ALG_FLOODMIN,
                           abi.PSG_ALG_KSET, abi.PSG_ALG_BENOR, abi.PSG_ALG_SLV, abi.PSG_ALG_KSET_ES})

# Generator options, on only for A/B measurements (PSG_SPEC_OPTIONS, include/psg.h): the
# symmetric-check-point lowering (spec::uniform) and the split foralls / hoisted conjuncts.
SYMMETRIC_LOWERING = True
SPLIT_FORALL = True


def compile_native(spec: Spec, alg: Optional[int] = None, cache_dir: str = None, fused: bool = False,
                   n: Optional[int] = None, defines: Sequence[str] = ()) -> Program:
    """Lower `spec` to native gfx950 code and return a Program whose module_path
    psg_run_batch_spec launches instead of the bytecode interpreter (the library's generator,
    psg_spec_compile_native, on the Spec's Formula text).

    fused=True also instantiates the algorithm's round kernel with the Spec as its check hook
    (spec::SpecHook): psg_run_batch_spec then runs ONE launch that executes the rounds and
    evaluates the Spec from registers, with no state trace. `n` (optional) limits the
    instantiations to that group size's wave count. `defines`: preprocessor definitions
    (e.g. "PSG_PHASE_TIMERS=1" for a profiling module; part of the source, so of the cache key)."""
    from . import lib
    if fused and alg not in FUSED_KERNELS:
        raise FormulaError("fused lowering needs one of the integer-state algorithms")
    opts = ([] if SYMMETRIC_LOWERING else ["nosym"]) + ([] if SPLIT_FORALL else ["nosplit"])
    opts += ["D" + d for d in defines]
    return lib.spec_compile_native(to_text(spec), int(alg or 0), fused, int(n or 0), cache_dir, opts)


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
