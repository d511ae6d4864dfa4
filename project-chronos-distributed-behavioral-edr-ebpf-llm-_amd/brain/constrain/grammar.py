"""Byte-level grammars for constrained decoding: a tiny regex algebra -> Thompson NFA -> DFA.

Ollama's ``format`` field (reference chronos_sensor.py:118 sends ``"json"``) is honoured in two forms:

* ``"json"``: any JSON object, nesting depth <= ``depth`` (bounded so the language is regular and the automaton
  finite); strings are printable ASCII plus the JSON escapes.
* a JSON-schema dict (Ollama "structured outputs"): objects with ordered ``properties``, ``string`` (``enum``,
  ``maxLength``), ``integer`` (``minimum``/``maximum``), ``number``, ``boolean``, ``null``, ``array`` (``items``,
  ``maxItems``).  :data:`chronos.sensor.prompt.VERDICT_SCHEMA` - the reply the CHRONOS prompt asks for
  (chronos_sensor.py:113) - compiles to a few hundred states.

The DFA is handed to the C++ token compiler (csrc/constrain/token_dfa.cpp) which lifts it to the vocabulary.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Sequence

import numpy as np

# ---------------------------------------------------------------------------------------------------------------
# regex algebra
# ---------------------------------------------------------------------------------------------------------------


@dataclass(frozen=True)
class Node:
    pass


@dataclass(frozen=True)
class Bytes(Node):
    """One byte from a set."""
    chars: frozenset


@dataclass(frozen=True)
class Seq(Node):
    items: tuple


@dataclass(frozen=True)
class Alt(Node):
    items: tuple


@dataclass(frozen=True)
class Star(Node):
    item: Node


def lit(s: str | bytes) -> Node:
    b = s.encode() if isinstance(s, str) else s
    return Seq(tuple(Bytes(frozenset([c])) for c in b))


def cset(chars: Iterable[int] | str) -> Node:
    if isinstance(chars, str):
        chars = chars.encode()
    return Bytes(frozenset(chars))


def seq(*xs: Node) -> Node:
    return Seq(tuple(xs))


def alt(*xs: Node) -> Node:
    return Alt(tuple(xs))


def opt(x: Node) -> Node:
    return Alt((x, Seq(())))


def star(x: Node) -> Node:
    return Star(x)


def plus(x: Node) -> Node:
    return Seq((x, Star(x)))


def rep(x: Node, lo: int, hi: int) -> Node:
    """x{lo,hi} as nested optionals (keeps the NFA linear in hi)."""
    tail: Node = Seq(())
    for _ in range(hi - lo):
        tail = opt(Seq((x, tail)))
    return Seq(tuple([x] * lo) + (tail,))


# ---------------------------------------------------------------------------------------------------------------
# NFA / DFA
# ---------------------------------------------------------------------------------------------------------------


class _NFA:
    def __init__(self):
        self.eps: list[list[int]] = []
        self.edges: list[list[tuple[frozenset, int]]] = []

    def new(self) -> int:
        self.eps.append([])
        self.edges.append([])
        return len(self.eps) - 1

    def build(self, n: Node, s: int, e: int) -> None:
        if isinstance(n, Bytes):
            self.edges[s].append((n.chars, e))
        elif isinstance(n, Seq):
            cur = s
            for i, it in enumerate(n.items):
                nxt = e if i == len(n.items) - 1 else self.new()
                self.build(it, cur, nxt)
                cur = nxt
            if not n.items:
                self.eps[s].append(e)
        elif isinstance(n, Alt):
            for it in n.items:
                a, b = self.new(), self.new()
                self.eps[s].append(a)
                self.build(it, a, b)
                self.eps[b].append(e)
        elif isinstance(n, Star):
            a, b = self.new(), self.new()
            self.eps[s].append(a)
            self.eps[s].append(e)
            self.build(n.item, a, b)
            self.eps[b].append(a)
            self.eps[b].append(e)
        else:
            raise TypeError(n)


@dataclass
class ByteDFA:
    trans: np.ndarray      # [S, 256] int32, -1 = reject
    accept: list[bool]
    start: int = 0

    @property
    def num_states(self) -> int:
        return self.trans.shape[0]

    def walk(self, data: bytes, state: int | None = None) -> int:
        s = self.start if state is None else state
        for c in data:
            if s < 0:
                return -1
            s = int(self.trans[s, c])
        return s

    def matches(self, data: bytes) -> bool:
        s = self.walk(data)
        return s >= 0 and self.accept[s]


def compile_dfa(node: Node, max_states: int = 30000) -> ByteDFA:
    nfa = _NFA()
    s0, f = nfa.new(), nfa.new()
    nfa.build(node, s0, f)

    def closure(states: Iterable[int]) -> frozenset:
        out = set(states)
        stack = list(out)
        while stack:
            u = stack.pop()
            for v in nfa.eps[u]:
                if v not in out:
                    out.add(v)
                    stack.append(v)
        return frozenset(out)

    start = closure([s0])
    index = {start: 0}
    order = [start]
    rows: list[np.ndarray] = []
    i = 0
    while i < len(order):
        cur = order[i]
        i += 1
        targets: dict[int, set] = {}
        for u in cur:
            for chars, v in nfa.edges[u]:
                for c in chars:
                    targets.setdefault(c, set()).add(v)
        row = np.full(256, -1, dtype=np.int32)
        cache: dict[frozenset, int] = {}
        for c, vs in targets.items():
            key = frozenset(vs)
            if key not in cache:
                cl = closure(vs)
                if cl not in index:
                    if len(order) >= max_states:
                        raise ValueError("grammar automaton too large")
                    index[cl] = len(order)
                    order.append(cl)
                cache[key] = index[cl]
            row[c] = cache[key]
        rows.append(row)
    trans = np.stack(rows) if rows else np.full((1, 256), -1, np.int32)
    accept = [f in st for st in order]
    return _minimize(ByteDFA(trans, accept, 0))


def _minimize(d: ByteDFA) -> ByteDFA:
    """Moore partition refinement (keeps token tables small: one int16 row of V entries per state)."""
    n = d.num_states
    part = np.array([1 if a else 0 for a in d.accept], dtype=np.int64)
    while True:
        tgt = np.where(d.trans >= 0, part[np.clip(d.trans, 0, None)], -1)
        sig = np.concatenate([part[:, None], tgt], axis=1)
        _, newpart = np.unique(sig, axis=0, return_inverse=True)
        newpart = newpart.reshape(-1)
        if len(np.unique(newpart)) == len(np.unique(part)):
            part = newpart
            break
        part = newpart
    # renumber with start = 0, in BFS order
    remap: dict[int, int] = {}
    order = [d.start]
    remap[int(part[d.start])] = 0
    rep_of = {}
    for s in range(n):
        rep_of.setdefault(int(part[s]), s)
    q = [int(part[d.start])]
    while q:
        p = q.pop(0)
        s = rep_of[p]
        for c in range(256):
            t = d.trans[s, c]
            if t >= 0:
                pt = int(part[t])
                if pt not in remap:
                    remap[pt] = len(remap)
                    q.append(pt)
    m = len(remap)
    trans = np.full((m, 256), -1, dtype=np.int32)
    accept = [False] * m
    for p, k in remap.items():
        s = rep_of[p]
        row = d.trans[s]
        ok = row >= 0
        trans[k, ok] = [remap[int(part[t])] for t in row[ok]]
        accept[k] = d.accept[s]
    del order
    return ByteDFA(trans, accept, 0)


# ---------------------------------------------------------------------------------------------------------------
# JSON building blocks
# ---------------------------------------------------------------------------------------------------------------

PRINTABLE = frozenset(range(0x20, 0x7F)) - {ord('"'), ord("\\")}
DIGIT = cset("0123456789")
DIGIT19 = cset("123456789")


def ws(max_ws: int = 1) -> Node:
    return rep(cset(" \n"), 0, max_ws)


def json_string(max_len: int | None = None) -> Node:
    ch = alt(Bytes(PRINTABLE), seq(lit("\\"), cset('"\\/bfnrt')))
    body = star(ch) if max_len is None else rep(ch, 0, max_len)
    return seq(lit('"'), body, lit('"'))


def json_number() -> Node:
    intpart = alt(lit("0"), seq(DIGIT19, rep(DIGIT, 0, 15)))
    frac = opt(seq(lit("."), rep(DIGIT, 1, 15)))
    exp = opt(seq(cset("eE"), opt(cset("+-")), rep(DIGIT, 1, 3)))
    return seq(opt(lit("-")), intpart, frac, exp)


def json_integer(minimum: int | None = None, maximum: int | None = None) -> Node:
    if minimum is not None and maximum is not None and 0 <= maximum - minimum <= 2000:
        return alt(*[lit(str(v)) for v in range(minimum, maximum + 1)])
    nonneg = alt(lit("0"), seq(DIGIT19, rep(DIGIT, 0, 17)))
    if minimum is not None and minimum >= 0:
        return nonneg
    return seq(opt(lit("-")), nonneg)


def json_value(depth: int, max_ws: int = 1) -> Node:
    scalars = [json_string(), json_number(), lit("true"), lit("false"), lit("null")]
    if depth <= 0:
        return alt(*scalars)
    return alt(*scalars, json_object(depth, max_ws), json_array(depth, max_ws))


def json_object(depth: int, max_ws: int = 1) -> Node:
    w = ws(max_ws)
    member = seq(json_string(), w, lit(":"), w, json_value(depth - 1, max_ws), w)
    return seq(lit("{"), w, opt(seq(member, star(seq(lit(","), w, member)))), lit("}"))


def json_array(depth: int, max_ws: int = 1) -> Node:
    w = ws(max_ws)
    item = seq(json_value(depth - 1, max_ws), w)
    return seq(lit("["), w, opt(seq(item, star(seq(lit(","), w, item)))), lit("]"))


def schema_node(schema: dict, max_ws: int = 1, default_max_len: int | None = None) -> Node:
    """JSON schema -> grammar node (Ollama structured outputs subset)."""
    if "enum" in schema:
        import json as _json

        return alt(*[lit(_json.dumps(v)) for v in schema["enum"]])
    if "const" in schema:
        import json as _json

        return lit(_json.dumps(schema["const"]))
    t = schema.get("type")
    if isinstance(t, list):
        return alt(*[schema_node(dict(schema, type=x), max_ws, default_max_len) for x in t])
    w = ws(max_ws)
    if t == "object" or (t is None and "properties" in schema):
        props: dict = schema.get("properties", {})
        if not props:
            return json_object(2, max_ws)
        required = set(schema.get("required", list(props)))
        parts: list[Node] = [lit("{"), w]
        first = True
        for name, sub in props.items():
            import json as _json

            member = seq(lit(_json.dumps(name)), w, lit(":"), w, schema_node(sub, max_ws, default_max_len), w)
            if not first:
                member = seq(lit(","), w, member)
            parts.append(member if name in required else opt(member))
            first = False
        parts.append(lit("}"))
        return seq(*parts)
    if t == "string":
        return json_string(schema.get("maxLength", default_max_len))
    if t == "integer":
        return json_integer(schema.get("minimum"), schema.get("maximum"))
    if t == "number":
        return json_number()
    if t == "boolean":
        return alt(lit("true"), lit("false"))
    if t == "null":
        return lit("null")
    if t == "array":
        item = seq(schema_node(schema.get("items", {"type": "string"}), max_ws, default_max_len), w)
        hi = schema.get("maxItems")
        lo = schema.get("minItems", 0)
        if hi is None:
            body = opt(seq(item, star(seq(lit(","), w, item))))
        else:
            more = rep(seq(lit(","), w, item), max(0, lo - 1), max(0, hi - 1))
            body = seq(item, more) if lo > 0 else opt(seq(item, more)) if hi > 0 else seq()
        return seq(lit("["), w, body, lit("]"))
    return json_value(2, max_ws)


def grammar_for_format(fmt, json_depth: int = 3, max_ws: int = 1, max_string: int | None = None) -> Node | None:
    """Map an Ollama ``format`` value to a grammar (None = unconstrained)."""
    if fmt in (None, "", False):
        return None
    if fmt == "json":
        return seq(ws(max_ws), json_object(json_depth, max_ws), ws(max_ws))
    if isinstance(fmt, dict):
        return seq(ws(max_ws), schema_node(fmt, max_ws, max_string), ws(max_ws))
    raise ValueError(f"unsupported format: {fmt!r}")


def format_key(fmt) -> str:
    import json as _json

    return _json.dumps(fmt, sort_keys=True)


def validate(fmt, text: str) -> bool:
    """Host-side check that `text` is in the language of `fmt` (used by tests and the server's debug mode)."""
    node = grammar_for_format(fmt)
    if node is None:
        return True
    return compile_dfa(node).matches(text.encode())


def walk_all(dfa: ByteDFA, pieces: Sequence[bytes]) -> int:
    s = dfa.start
    for p in pieces:
        s = dfa.walk(p, s)
        if s < 0:
            return -1
    return s
