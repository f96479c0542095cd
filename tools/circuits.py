"""Circuit compiler for the cooperative (one wavefront per task) kernels.

The tower / curve formulas are written once, in Python, as arithmetic over Fp:
multiplications are nodes, additions / subtractions / small-integer scalings are
kept symbolic as linear combinations (Lin) and folded into the operands of the
multiplications that consume them.  The scheduler levels the DAG (a product's
level = 1 + the deepest product it depends on), packs each level's products into
steps of at most LANES lanes, materialises operands whose linear combination is
too long, allocates frame slots with liveness, and emits the table the device
interpreter (lodestar_amd/csrc/bls/coop.hpp) walks: one 64-byte op per lane per
step.  Step semantics: every lane gathers its operands, the wave synchronises,
every lane writes its result -- so a step may overwrite a slot it also reads.

`simulate()` runs a program on Python integers with exactly those semantics; the
tests check every program against the oracle's math (tests/test_circuits.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
LANES = 64
KMAX = 8          # terms per operand linear combination
CMAX = 32767      # |coefficient| of a term (int16)
OP_NOP, OP_MUL, OP_LIN = 0, 1, 2
ZCHECK = -1       # output "slot" of a zero-check op: ORs is_zero(value) into the task flag


# ----------------------------------------------------------------------------
# symbolic values
# ----------------------------------------------------------------------------
class Lin:
    """sum coef * ref; ref = ('in', slot) | ('n', node_id) | ('c', const_index)."""

    __slots__ = ("t",)

    def __init__(self, terms=None):
        self.t = {}
        if terms:
            for r, c in terms.items():
                if c % P:
                    self.t[r] = c

    def __add__(self, o):
        r = Lin(self.t)
        for k, c in o.t.items():
            r.t[k] = r.t.get(k, 0) + c
            if r.t[k] == 0:
                del r.t[k]
        return r

    def __neg__(self):
        return Lin({k: -c for k, c in self.t.items()})

    def __sub__(self, o):
        return self + (-o)

    def scale(self, s: int):
        return Lin({k: c * s for k, c in self.t.items()})

    def __mul__(self, s: int):
        return self.scale(s)

    __rmul__ = __mul__

    def is_zero(self):
        return not self.t


@dataclass
class Node:
    a: Lin
    b: Lin
    id: int
    kind: int = OP_MUL
    level: int = 0
    depth: int = 0   # LIN nodes: chain depth among LIN nodes of the same level


class ConstBank:
    """Fp constants shared by every program (plain integers; the emitter converts
    them to Montgomery form).  Index 0 is 1."""

    def __init__(self):
        self.vals = [1]
        self._idx = {1: 0}

    def index(self, v: int) -> int:
        v %= P
        if v not in self._idx:
            self._idx[v] = len(self.vals)
            self.vals.append(v)
        return self._idx[v]


class Circuit:
    def __init__(self, name: str, consts: ConstBank):
        self.name = name
        self.nodes: list[Node] = []
        self.consts = consts
        self.outputs: list[tuple[int, Lin]] = []
        self.zchecks: list[Lin] = []
        self.zsets: list[int] = []   # set index of each zero-check (packed multi-set programs)
        self.zset = 0

    @staticmethod
    def inp(slot: int) -> Lin:
        return Lin({("in", slot): 1})

    def const(self, value: int) -> Lin:
        return Lin({("c", self.consts.index(value)): 1})

    def one(self) -> Lin:
        return self.const(1)

    def mul(self, a: Lin, b: Lin) -> Lin:
        if a.is_zero() or b.is_zero():
            return Lin()
        n = Node(a, b, len(self.nodes), OP_MUL)
        self.nodes.append(n)
        return Lin({("n", n.id): 1})

    def mat(self, a: Lin) -> Lin:
        """Materialise a linear combination (a LIN node) so consumers see one term."""
        if len(a.t) <= 1 and all(c == 1 for c in a.t.values()):
            return a
        n = Node(a, Lin(), len(self.nodes), OP_LIN)
        self.nodes.append(n)
        return Lin({("n", n.id): 1})

    def out(self, slot: int, v: Lin):
        self.outputs.append((slot, v))

    def zcheck(self, v: Lin):
        self.zchecks.append(v)
        self.zsets.append(self.zset)


# ----------------------------------------------------------------------------
# scheduled program
# ----------------------------------------------------------------------------
@dataclass
class Op:
    kind: int
    out: int
    a: list  # [(ref, coef)]; ref = slot int or ('c', idx)
    b: list = field(default_factory=list)


@dataclass
class Program:
    name: str
    steps: list          # list[list[Op]]
    n_slots: int
    out_slots: list
    n_mul_steps: int = 0


def _refs(l: Lin):
    return [k for k in l.t if k[0] == "n"]


def schedule(c: Circuit, frame_slots: int, reserved: set, lanes: int = LANES) -> Program:
    """Level-schedule circuit `c` into steps of <= `lanes` ops over a frame of
    `frame_slots` slots; `reserved` slots (the caller's live registers) are never
    used for temporaries.  Both as-soon-as-possible and as-late-as-possible level
    assignments are tried (ALAP keeps values that are consumed late -- e.g. a Miller
    loop's line coefficients -- out of the frame until they are needed); the shorter
    program that fits the frame wins."""
    import copy
    best, err = None, None
    for mode in ("asap", "alap", "list"):
        for hoist in (True, False):
            try:
                pg = _schedule_mode(copy.deepcopy(c), frame_slots, reserved, lanes, mode, hoist)
            except RuntimeError as e:
                err = e
                continue
            if best is None or len(pg.steps) < len(best.steps):
                best = pg
    if best is None:
        raise err
    return best


def _relevel(nodes, roots, mode):
    """Drop dead nodes; recompute levels (ASAP or ALAP) and LIN depths in a
    topological order."""
    byid = {n.id: n for n in nodes}
    order, seen = [], set()
    stack = [r[1] for l in roots for r in _refs(l)]
    # iterative post-order DFS
    for root in list(dict.fromkeys(stack)):
        if root in seen:
            continue
        work = [(root, False)]
        while work:
            nid, done = work.pop()
            if done:
                order.append(byid[nid])
                continue
            if nid in seen:
                continue
            seen.add(nid)
            work.append((nid, True))
            n = byid[nid]
            for l in (n.a, n.b):
                for r in _refs(l):
                    if r[1] not in seen:
                        work.append((r[1], False))
    # ASAP
    for n in order:
        lv = 0
        for l in (n.a, n.b):
            for r in _refs(l):
                lv = max(lv, byid[r[1]].level)
        n.level = lv + 1 if n.kind == OP_MUL else lv
    if mode in ("alap", "list"):
        lmax = max((n.level for n in order), default=0)
        cons = {n.id: [] for n in order}
        for n in order:
            for l in (n.a, n.b):
                for r in _refs(l):
                    cons[r[1]].append(n)
        for n in reversed(order):
            lat = lmax
            for cn in cons[n.id]:
                lat = min(lat, cn.level - 1 if cn.kind == OP_MUL else cn.level)
            n.level = lat
    for n in order:
        d = 0
        if n.kind == OP_LIN:
            for r in _refs(n.a):
                m = byid[r[1]]
                if m.kind == OP_LIN and m.level == n.level:
                    d = max(d, m.depth + 1)
        n.depth = d
    return order


def _schedule_mode(c: Circuit, frame_slots: int, reserved: set, lanes: int, mode: str,
                   hoist: bool = False) -> Program:
    """Level-schedule circuit `c` into steps of <= `lanes` ops over a frame of
    `frame_slots` slots.  `reserved` slots (the caller's live registers) are never
    used for temporaries.  Products of level L run in phase (L, 0); linear
    combinations whose deepest reference has level L run in phases (L, 1, depth).
    hoist: linear combinations and outputs move into earlier steps with spare lanes
    (_hoist_lins, _allocate)."""
    nodes = c.nodes

    def level_of(n: Node):
        lv, dep = 0, 0
        for l in (n.a, n.b):
            for r in _refs(l):
                m = nodes[r[1]]
                lv = max(lv, m.level)
        if n.kind == OP_MUL:
            return lv + 1, 0
        for r in _refs(n.a):
            m = nodes[r[1]]
            if m.kind == OP_LIN and m.level == lv:
                dep = max(dep, m.depth + 1)
        return lv, dep

    def fit(l: Lin) -> Lin:
        for cf in l.t.values():
            if abs(cf) > CMAX:
                raise ValueError(f"{c.name}: coefficient {cf} out of range")
        if len(l.t) <= KMAX:
            return l
        items = list(l.t.items())
        groups = [items[i: i + KMAX] for i in range(0, len(items), KMAX)]
        res = {}
        for g in groups:
            if len(g) == 1:
                res[g[0][0]] = g[0][1]
                continue
            ln = Node(Lin(dict(g)), Lin(), len(nodes), OP_LIN)
            ln.level, ln.depth = level_of(ln)
            nodes.append(ln)
            res[("n", ln.id)] = 1
        return fit(Lin(res))

    i = 0
    while i < len(nodes):   # nodes appended by fit() are already fitted and levelled
        n = nodes[i]
        if n.level == 0 and n.depth == 0 and not getattr(n, "_done", False):
            n.a = fit(n.a)
            n.b = fit(n.b)
            n.level, n.depth = level_of(n)
            n._done = True
        i += 1
    outs = [(slot, fit(v)) for slot, v in c.outputs]
    zchecks = [fit(z) for z in c.zchecks]
    nodes = _relevel(nodes, [v for _, v in outs] + zchecks, mode)

    if mode == "list":
        groups = _list_groups(nodes, lanes)
    else:
        def phase(n: Node):
            return (n.level, 0, 0) if n.kind == OP_MUL else (n.level, 1, n.depth)

        phases: dict = {}
        for n in nodes:
            phases.setdefault(phase(n), []).append(n)
        groups = []
        for ph in sorted(phases):
            ns = phases[ph]
            for k in range(0, len(ns), lanes):
                groups.append((ph[1] == 0, ns[k: k + lanes]))
    if hoist:
        groups = _hoist_lins(groups, lanes)
    return _allocate(c, groups, outs, zchecks, frame_slots, reserved, lanes, hoist)


def _hoist_lins(groups, lanes):
    """Move every linear combination to the earliest step after the steps that produce
    its operands that has a spare lane.  Half of a program's steps were linear-only
    steps, while the product steps of the per-set programs use a quarter of the lanes:
    a LIN op in a product step costs nothing (its lane skips the product), and a LIN
    step that empties disappears."""
    prod = {}
    for r, (_, ns) in enumerate(groups):
        for n in ns:
            prod[n.id] = r
    kinds = [m for m, _ in groups]
    out = [list(ns) for _, ns in groups]
    for r in range(len(out)):
        if kinds[r]:
            continue
        keep = []
        for n in out[r]:
            ready = 1 + max((prod[x[1]] for x in _refs(n.a)), default=-1)
            # (not into a linear-only step that hoisting has emptied: it would survive
            # as a step of its own where the combination could ride in a later product step)
            q = next((g for g in range(ready, r) if 0 < len(out[g]) < lanes), None)
            if q is None:
                keep.append(n)
                continue
            out[q].append(n)
            prod[n.id] = q
        out[r] = keep
    return [(kinds[r], out[r]) for r in range(len(out)) if out[r]]


def _list_groups(nodes, lanes):
    """Slack-driven list scheduling.  Walk the ALAP levels; at each product level
    run every product whose ALAP level it is (mandatory) and fill the spare lanes
    of the last step with ready products that have slack (earliest deadline first);
    then run linear-combination steps until every combination due at this level is
    done, again filling spare lanes with ready ones."""
    byid = {n.id: n for n in nodes}
    done = set()
    todo_mul = [n for n in nodes if n.kind == OP_MUL]
    todo_lin = [n for n in nodes if n.kind == OP_LIN]
    groups = []

    def ready(n):
        return all(r[1] in done for l in (n.a, n.b) for r in _refs(l))

    def run(kind_mul, pool, level):
        rdy = [n for n in pool if ready(n)]
        must = [n for n in rdy if n.level <= level]
        if not must:
            return pool, False
        opt = sorted((n for n in rdy if n.level > level), key=lambda n: n.level)
        nsteps = (len(must) + lanes - 1) // lanes
        take = must + opt[: nsteps * lanes - len(must)]
        for k in range(0, len(take), lanes):
            groups.append((kind_mul, take[k: k + lanes]))
        ids = {n.id for n in take}
        done.update(ids)
        return [n for n in pool if n.id not in ids], True

    lmax = max((n.level for n in nodes), default=0)
    for level in range(0, lmax + 1):
        if level > 0:
            todo_mul, _ = run(True, todo_mul, level)
        while True:
            todo_lin, progressed = run(False, todo_lin, level)
            if not progressed:
                break
    assert not todo_mul and not todo_lin, "list scheduling left nodes behind"
    return groups


def _allocate(c, groups, outs, zchecks, frame_slots, reserved, lanes, hoist=False) -> Program:
    last_use = {}
    tail_rank = len(groups)

    def note(l: Lin, r):
        for x in _refs(l):
            last_use[x[1]] = max(last_use.get(x[1], -1), r)

    for r, (_, ns) in enumerate(groups):
        for n in ns:
            note(n.a, r)
            note(n.b, r)
    # hoisted outputs / zero-checks: into the first step after their operands' steps with
    # a spare lane -- an output only into a reserved slot (never a temporary) and once no
    # later step (and no output) reads the input slot it overwrites (a step gathers
    # before it writes, so its own step may)
    at = {}  # index into outs + zchecks -> group
    if hoist:
        prod = {n.id: r for r, (_, ns) in enumerate(groups) for n in ns}
        last_read = {}
        for r, (_, ns) in enumerate(groups):
            for n in ns:
                for l in (n.a, n.b):
                    for k in l.t:
                        if k[0] == "in":
                            last_read[k[1]] = r
        out_reads = {k[1] for _, v in outs for k in v.t if k[0] == "in"}
        load = [len(ns) for _, ns in groups]
        items = [(slot, v) for slot, v in outs] + [(None, z) for z in zchecks]
        for idx, (slot, v) in enumerate(items):
            # (an output slot outside `reserved` may hold temporaries until the tail)
            if slot is not None and (slot in out_reads or slot not in reserved):
                continue
            ready = 1 + max((prod[x[1]] for x in _refs(v)), default=-1)
            if slot is not None:
                ready = max(ready, last_read.get(slot, -1))
            q = next((g for g in range(ready, len(groups)) if load[g] < lanes), None)
            if q is not None:
                at[idx] = q
                load[q] += 1
    for idx, (_, v) in enumerate(outs):
        note(v, at.get(idx, tail_rank))
    for k, z in enumerate(zchecks):
        note(z, at.get(len(outs) + k, tail_rank))

    free = [s for s in range(frame_slots) if s not in reserved]
    slot_of = {}
    busy_until = {}
    steps = []
    n_mul = 0
    for r, (is_mul, ns) in enumerate(groups):
        for s, until in list(busy_until.items()):
            if until < r:
                del busy_until[s]
                free.append(s)
        free.sort()
        ops = []
        for n in ns:
            if not free:
                raise RuntimeError(f"{c.name}: out of frame slots ({frame_slots})")
            s = free.pop(0)
            slot_of[n.id] = s
            busy_until[s] = last_use.get(n.id, r)
            ops.append(Op(n.kind, s, _emit(n.a, slot_of), _emit(n.b, slot_of)))
        for idx, q in at.items():
            if q == r:
                if idx < len(outs):
                    slot, v = outs[idx]
                    ops.append(Op(OP_LIN, slot, _emit(v, slot_of)))
                else:
                    k = idx - len(outs)
                    ops.append(Op(OP_LIN, ZCHECK - c.zsets[k], _emit(zchecks[k], slot_of)))
        steps.append(ops)
        if is_mul:
            n_mul += 1
    tail = [Op(OP_LIN, slot, _emit(v, slot_of)) for idx, (slot, v) in enumerate(outs) if idx not in at]
    tail += [Op(OP_LIN, ZCHECK - zs, _emit(z, slot_of)) for k, (z, zs) in enumerate(zip(zchecks, c.zsets))
             if len(outs) + k not in at]
    # the outputs land in as few steps as fit the lanes; a later output step may not
    # read a slot an earlier one wrote (outputs are written simultaneously in spirit)
    written = set()
    for k in range(0, len(tail), lanes):
        chunk = tail[k: k + lanes]
        for op in chunk:
            for ref, _ in op.a:
                if not isinstance(ref, tuple) and ref in written:
                    raise RuntimeError(f"{c.name}: output step {k // lanes} reads slot {ref} written before")
        steps.append(chunk)
        written |= {op.out for op in chunk if op.out >= 0}
    return Program(c.name, steps, frame_slots, [s for s, _ in outs], n_mul)


def _emit(l: Lin, slot_of) -> list:
    res = []
    for k, cf in l.t.items():
        if k[0] == "in":
            res.append((k[1], cf))
        elif k[0] == "c":
            res.append((("c", k[1]), cf))
        else:
            res.append((slot_of[k[1]], cf))
    return res


# ----------------------------------------------------------------------------
# simulation (exact device semantics)
# ----------------------------------------------------------------------------
def simulate(prog: Program, frame: list, consts: ConstBank) -> int:
    """Run `prog` in place on `frame` (list of ints mod P); returns the zero-check
    flags (bit s: a zero-check of packed set s saw zero)."""
    flag = 0

    def val(terms):
        s = 0
        for ref, cf in terms:
            v = consts.vals[ref[1]] if isinstance(ref, tuple) else frame[ref]
            s += cf * v
        return s % P

    for step in prog.steps:
        res = []
        for op in step:
            a = val(op.a)
            res.append((op, a * val(op.b) % P if op.kind == OP_MUL else a))
        for op, r in res:
            if op.out <= ZCHECK:
                if r == 0:
                    flag |= 1 << (ZCHECK - op.out)
            else:
                frame[op.out] = r
    return flag
