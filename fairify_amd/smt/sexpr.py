"""Minimal S-expression reader + exact evaluator for the SMT-LIB subset the encoder emits.

Test oracle (the reference has none): an assignment of the integer variables is checked
against every ``assert`` of an encoded query with ``fractions.Fraction`` arithmetic, so the
encoding can be validated without a solver (Z3 is not installed in this environment).
Also parses ``(get-model)`` answers (the role of ``parse_z3Model``,
utils/verif_utils.py:993-1020).
"""
from __future__ import annotations

from fractions import Fraction
from typing import Dict, List, Tuple, Union

Atom = str
SExpr = Union[Atom, List["SExpr"]]


def tokenize(text: str) -> List[str]:
    out: List[str] = []
    i, n = 0, len(text)
    while i < n:
        c = text[i]
        if c == ";":
            while i < n and text[i] != "\n":
                i += 1
        elif c in "()":
            out.append(c)
            i += 1
        elif c.isspace():
            i += 1
        elif c == '"':
            j = text.index('"', i + 1)
            out.append(text[i:j + 1])
            i = j + 1
        else:
            j = i
            while j < n and not text[j].isspace() and text[j] not in "()":
                j += 1
            out.append(text[i:j])
            i = j
    return out


def parse_all(text: str) -> List[SExpr]:
    toks = tokenize(text)
    pos = 0

    def rd() -> SExpr:
        nonlocal pos
        t = toks[pos]
        pos += 1
        if t == "(":
            lst = []
            while toks[pos] != ")":
                lst.append(rd())
            pos += 1
            return lst
        if t == ")":
            raise ValueError("unbalanced )")
        return t

    out = []
    while pos < len(toks):
        out.append(rd())
    return out


def _num(tok: str) -> Fraction:
    return Fraction(tok)


class Evaluator:
    """Evaluate ``define-fun`` / ``assert`` commands under an integer assignment."""

    def __init__(self, script: str):
        self.cmds = parse_all(script)
        self.defs: Dict[str, SExpr] = {}
        self.asserts: List[SExpr] = []
        self.decls: List[str] = []
        for c in self.cmds:
            if not isinstance(c, list) or not c:
                continue
            if c[0] == "define-fun":
                self.defs[c[1]] = c[4]
            elif c[0] == "assert":
                self.asserts.append(c[1])
            elif c[0] == "declare-fun":
                self.decls.append(c[1])

    def value(self, e: SExpr, env: Dict[str, Fraction], cache: Dict[str, object]):
        if isinstance(e, str):
            if e in env:
                return env[e]
            if e in self.defs:
                if e not in cache:
                    cache[e] = self.value(self.defs[e], env, cache)
                return cache[e]
            if e == "true":
                return True
            if e == "false":
                return False
            return _num(e)
        op, args = e[0], e[1:]
        if op == "ite":
            return self.value(args[1], env, cache) if self.value(args[0], env, cache) else self.value(args[2], env, cache)
        v = [self.value(a, env, cache) for a in args]
        if op == "+":
            return sum(v, Fraction(0))
        if op == "-":
            return -v[0] if len(v) == 1 else v[0] - sum(v[1:], Fraction(0))
        if op == "*":
            r = Fraction(1)
            for x in v:
                r *= x
            return r
        if op == "/":
            return v[0] / v[1]
        if op == "to_real":
            return Fraction(v[0])
        if op == "and":
            return all(v)
        if op == "or":
            return any(v)
        if op == "not":
            return not v[0]
        if op == "=":
            return all(x == v[0] for x in v[1:])
        if op == "<":
            return v[0] < v[1]
        if op == "<=":
            return v[0] <= v[1]
        if op == ">":
            return v[0] > v[1]
        if op == ">=":
            return v[0] >= v[1]
        raise ValueError(f"unsupported operator {op}")

    def satisfied(self, assignment: Dict[str, int]) -> bool:
        env = {k: Fraction(int(v)) for k, v in assignment.items()}
        cache: Dict[str, object] = {}
        return all(bool(self.value(a, env, cache)) for a in self.asserts)

    def eval_name(self, name: str, assignment: Dict[str, int]):
        env = {k: Fraction(int(v)) for k, v in assignment.items()}
        return self.value(name, env, {})


def parse_model(text: str) -> Dict[str, int]:
    """``(model (define-fun x0 () Int 5) ...)`` (or the bare list form) -> {name: int}."""
    out: Dict[str, int] = {}

    def walk(e):
        if isinstance(e, list):
            if len(e) == 5 and e[0] == "define-fun" and e[3] == "Int":
                v = e[4]
                if isinstance(v, list) and v[0] == "-":
                    out[e[1]] = -int(v[1])
                else:
                    out[e[1]] = int(v)
            else:
                for x in e:
                    walk(x)

    for c in parse_all(text):
        walk(c)
    return out


def model_to_pair(model: Dict[str, int], n: int) -> Tuple[List[int], List[int]]:
    """Ordered input vectors (x, x') from a model (``parse_z3Model``)."""
    return [model.get(f"x{i}", 0) for i in range(n)], [model.get(f"x_{i}", 0) for i in range(n)]
