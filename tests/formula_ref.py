"""Direct recursive evaluation of round_amd.formula trees over a state trace.

Test infrastructure: an independent reading of the Formula semantics (no
bytecode, no finitization: V.exists over Int is brute-forced over every value in
[lo - 2, max(hi, R) + 2] of the instance's trace and rounds plus Int.MinValue / Int.MaxValue), used
to check the compiler and both interpreters on specs the oracle has no
hand-written counterpart for.
"""
from round_amd import formula as F

INT_MIN, INT_MAX = -(1 << 31), (1 << 31) - 1


def _wrap(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


class State:
    def __init__(self, tr, n, R, inst, c):
        self.tr, self.n, self.R, self.c = tr, n, R, c
        self.per = (R + 1) * 9 * n
        self.base = inst * self.per
        vals = [tr[self.base + k] for k in range(self.per)]
        vals = [v for v in vals if v != INT_MIN]
        # every trace value and every round number (terms like r / 4 + 1), +-2, and the extremes
        self.dom = list(range(min(vals + [0]) - 2, max(vals + [0, R]) + 3)) + [INT_MIN, INT_MAX]

    def field(self, f, tag, p):
        if not (0 <= p < self.n):
            return 0
        cc = self.c if tag == F.TAG_CUR else (max(self.c - 1, 0) if tag == F.TAG_OLD else 0)
        return self.tr[self.base + (cc * 9 + f) * self.n + p]


VINT_DOMAIN = None  # optional hook (quant, state, env) -> V.exists-over-Int domain (tests)


def ev(e, st, env):
    if isinstance(e, F.Lit):
        return e.v
    if isinstance(e, F.NVal):
        return st.n
    if isinstance(e, F.RVal):
        return st.c
    if isinstance(e, F.CoordVal):
        return (st.c // 4) % st.n
    if isinstance(e, F.Var):
        return env[e.uid]
    if isinstance(e, F.Field):
        return st.field(e.f, e.tag, ev(e.proc, st, env))
    if isinstance(e, F.Un):
        x = ev(e.x, st, env)
        return {"NOT": int(x == 0), "NEG": _wrap(-x), "ISDEF": int(x != INT_MIN)}[e.op]
    if isinstance(e, F.Bin):
        x, y = ev(e.x, st, env), ev(e.y, st, env)
        op = e.op
        if op == "AND": return int(x != 0 and y != 0)
        if op == "OR": return int(x != 0 or y != 0)
        if op == "IMPL": return int(x == 0 or y != 0)
        if op in ("EQ", "NE", "LT", "LE", "GT", "GE"):
            return int({"EQ": x == y, "NE": x != y, "LT": x < y, "LE": x <= y, "GT": x > y, "GE": x >= y}[op])
        if op == "ADD": return _wrap(x + y)
        if op == "SUB": return _wrap(x - y)
        if op == "MUL": return _wrap(x * y)
        if op == "DIV":
            if y == 0: return 0
            q = abs(x) // abs(y)
            return _wrap(q if (x >= 0) == (y >= 0) else -q)
        if op == "MOD":
            if y in (0, -1): return 0
            m = abs(x) % abs(y)
            return m if x >= 0 else -m
    if isinstance(e, F.Contains):
        env2 = dict(env)
        env2[e.comp.var.uid] = ev(e.e, st, env)
        return ev(e.comp.body, st, env2)
    if isinstance(e, F.Quant):
        dom = range(st.n) if e.kind in ("forall", "exists", "count") else ((0, 1) if e.kind == "vbool" else st.dom)
        if e.kind == "vint" and VINT_DOMAIN is not None:
            dom = VINT_DOMAIN(e, st, env)
        res = []
        for v in dom:
            env2 = dict(env)
            env2[e.var.uid] = v
            res.append(ev(e.body, st, env2) != 0)
        if e.kind == "forall":
            return int(all(res))
        if e.kind == "count":
            return sum(res)
        return int(any(res))
    raise TypeError(type(e))


def evaluate(spec, tr, count, n, R):
    """(first_fail per slot, term_round) per instance, slot layout of compile_spec."""
    prog = F.compile_spec(spec)
    guard = F._rinv_guard(spec)
    invs = [inv if guard is None else (inv & guard) for inv in spec.invariants]
    slots = []
    if invs:
        slots.append((F.Or(*invs), False))
        slots += [(i, False) for i in invs]
    term = None
    for name, f in spec.properties:
        if name == "Termination":
            term = f
        else:
            slots.append((f, F._uses_old(f)))
    if spec.safety_predicate is not None:
        slots.append((spec.safety_predicate, F._uses_old(spec.safety_predicate)))
    out_ff, out_t = [], []
    for i in range(count):
        ff = [255] * len(slots)
        tr_round = 255
        for c in range(R + 1):
            st = State(tr, n, R, i, c)
            for s, (f, rel) in enumerate(slots):
                ok = (c == 0 and rel) or ev(f, st, {}) != 0
                if not ok and ff[s] == 255:
                    ff[s] = c
            if term is not None and tr_round == 255 and ev(term, st, {}) != 0:
                tr_round = c
        out_ff.append(ff)
        out_t.append(tr_round)
    assert len(slots) == len(prog.slot_entry)
    return out_ff, out_t
