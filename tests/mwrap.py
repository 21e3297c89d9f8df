"""TEST INFRASTRUCTURE: run the drop-in MATLAB wrappers (matlab/*.m) without MATLAB.

MATLAB and Octave are absent from this image and the GPU box, so the wrappers' own logic --
argument defaults (lsmr_solver.m's `nargin` / `isempty` lines, the reference's lsmr_solver.m:3,5),
the `nargout <= 4` fast path and the `iscell(DeltaM)` split of the *_bounds wrappers -- would
otherwise never execute.  This module interprets exactly the statement subset those files use:

    function [o1, ...] = name(i1, ...)          (with `...` continuations)
    if COND, STMT; end        if COND ... else ... end        return        end
    x = EXPR;   L = C{1};   [a, b] = f(...);
    EXPR: numbers, 'strings', [], identifiers, calls (nargin, nargout, isempty, iscell, min,
          size, hgmres_mex), cell indexing X{k}, < <= > >= == ~=, ||, &&

and fails loudly on anything else.  hgmres_mex calls go to the mex gateway through the mx API
stand-in (tests/mexmock), i.e. the same compiled C a MATLAB user would load.
"""
import re

import numpy as np

TOKEN = re.compile(r"\s*(?:(?P<num>\d+\.?\d*(?:[eE][-+]?\d+)?)|(?P<str>'[^']*')|(?P<id>[A-Za-z_]\w*)|"
                   r"(?P<op>\|\||&&|<=|>=|==|~=|[<>=(),;{}\[\]]))")


class Cell(list):
    """A MATLAB cell array (1-based {} indexing)."""


class WrapperError(RuntimeError):
    pass


def _tokens(s):
    out, pos = [], 0
    s = s.rstrip()
    while pos < len(s):
        m = TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise WrapperError(f"cannot tokenize {s[pos:]!r}")
        pos = m.end()
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
    return out


class _Expr:
    def __init__(self, toks, env):
        self.t, self.i, self.env = toks, 0, env

    def peek(self):
        return self.t[self.i][1] if self.i < len(self.t) else None

    def take(self, v=None):
        tok = self.t[self.i]
        if v is not None and tok[1] != v:
            raise WrapperError(f"expected {v!r}, got {tok[1]!r}")
        self.i += 1
        return tok

    def parse(self):
        v = self.orexpr()
        return v

    def orexpr(self):
        v = self.andexpr()
        while self.peek() == "||":
            self.take()
            if v:                       # short circuit, as MATLAB
                self._skip_and()
                v = True
            else:
                v = bool(self.andexpr())
        return v

    def _skip_and(self):
        depth = 0
        while self.i < len(self.t):
            p = self.peek()
            if depth == 0 and p in ("||", ",", ";", ")"):
                return
            if p in ("(", "{", "["):
                depth += 1
            if p in (")", "}", "]"):
                depth -= 1
            self.i += 1

    def andexpr(self):
        v = self.cmp()
        while self.peek() == "&&":
            self.take()
            w = self.cmp()
            v = bool(v) and bool(w)
        return v

    def cmp(self):
        a = self.atom()
        op = self.peek()
        if op in ("<", "<=", ">", ">=", "==", "~="):
            self.take()
            b = self.atom()
            return {"<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b, "==": a == b, "~=": a != b}[op]
        return a

    def args(self, close=")"):
        out = []
        if self.peek() == close:
            self.take(close)
            return out
        while True:
            out.append(self.orexpr())
            if self.peek() == ",":
                self.take(",")
                continue
            self.take(close)
            return out

    def atom(self):
        kind, v = self.take()
        if kind == "num":
            return float(v)
        if kind == "str":
            return v[1:-1]
        if v == "[":
            self.take("]")
            return np.zeros((0, 0))
        if kind != "id":
            raise WrapperError(f"unexpected {v!r}")
        if self.peek() == "(":
            self.take("(")
            return self.env.call(v, self.args(")"))
        if self.peek() == "{":
            self.take("{")
            k = self.args("}")
            return self.env.get(v)[int(k[0]) - 1]
        return self.env.get(v)


class Function:
    """One wrapper file, callable as f(nargout, *args)."""

    def __init__(self, path, mex):
        src = open(path).read()
        lines = []
        for raw in src.splitlines():
            s = raw.rstrip()
            if not s.strip() or s.lstrip().startswith("%"):      # blank / comment lines
                continue
            if lines and lines[-1].endswith("..."):
                lines[-1] = lines[-1][:-3] + " " + s.strip()
            else:
                lines.append(s.strip())
        m = re.match(r"function\s+(?:\[(?P<outs>[^\]]*)\]|(?P<out1>\w+))\s*=\s*(?P<name>\w+)\s*\((?P<ins>[^)]*)\)$",
                     lines[0])
        if not m:
            raise WrapperError(f"bad function line {lines[0]!r}")
        self.outs = [o.strip() for o in (m.group("outs") or m.group("out1")).split(",")]
        self.name = m.group("name")
        self.ins = [i.strip() for i in m.group("ins").split(",") if i.strip()]
        if lines[-1] != "end":
            raise WrapperError("function must close with end")
        self.body = lines[1:-1]
        self.mex = mex

    # ---- environment ----
    def get(self, name):
        if name in ("nargin", "nargout") and name not in self.vars:
            return self.call(name, [])
        if name not in self.vars:
            raise WrapperError(f"{self.name}: undefined variable {name}")
        return self.vars[name]

    def call(self, fn, a):
        if fn == "nargin":
            return float(self.nargin)
        if fn == "nargout":
            return float(self.nargout)
        if fn == "isempty":
            return np.size(a[0]) == 0 if not isinstance(a[0], str) else len(a[0]) == 0
        if fn == "iscell":
            return isinstance(a[0], Cell)
        if fn == "min":
            return min(a[0], a[1])
        if fn == "size":
            return float(np.shape(a[0])[int(a[1]) - 1])
        if fn == "hgmres_mex":
            return ("__mex__", a)
        raise WrapperError(f"{self.name}: unsupported function {fn}")

    def _eval(self, toks):
        e = _Expr(toks, self)
        v = e.parse()
        if e.i != len(toks):
            raise WrapperError(f"trailing tokens {toks[e.i:]}")
        return v

    def _assign(self, stmt):
        toks = _tokens(stmt)
        if toks and toks[0][1] == "[":                     # [a, b, ...] = f(...)
            j = [t[1] for t in toks].index("]")
            names = [t[1] for t in toks[1:j] if t[0] == "id"]
            if toks[j + 1][1] != "=":
                raise WrapperError(stmt)
            v = self._eval(toks[j + 2:])
            if not (isinstance(v, tuple) and v[0] == "__mex__"):
                raise WrapperError("multi-assignment only from hgmres_mex")
            outs = self.mex(len(names), *v[1])
            for n_, o in zip(names, outs):
                self.vars[n_] = o
            return
        if len(toks) >= 2 and toks[0][0] == "id" and toks[1][1] == "=":
            v = self._eval(toks[2:])
            if isinstance(v, tuple) and v[0] == "__mex__":
                v = self.mex(1, *v[1])[0]
            self.vars[toks[0][1]] = v
            return
        raise WrapperError(f"unsupported statement {stmt!r}")

    def _run(self, stmts):
        """Execute statements; returns True on `return`."""
        i = 0
        while i < len(stmts):
            s = stmts[i]
            if s == "return":
                return True
            m = re.match(r"if\s+(.*?),\s*(.*?);?\s*end$", s)           # one-line if
            if m:
                if self._eval(_tokens(m.group(1))):
                    for part in [p for p in m.group(2).split(";") if p.strip()]:
                        self._assign(part.strip())
                i += 1
                continue
            if s.startswith("if "):                                   # block if / else / end
                depth, j, els = 1, i + 1, None
                while depth:
                    t = stmts[j]
                    if t.startswith("if ") and not re.match(r"if\s+.*,.*end$", t):
                        depth += 1
                    elif t == "end":
                        depth -= 1
                    elif t == "else" and depth == 1:
                        els = j
                    j += 1
                then = stmts[i + 1:(els if els is not None else j - 1)]
                other = stmts[els + 1:j - 1] if els is not None else []
                branch = then if self._eval(_tokens(s[3:])) else other
                if self._run(branch):
                    return True
                i = j
                continue
            for part in [p for p in s.split(";") if p.strip()]:
                self._assign(part.strip())
            i += 1
        return False

    def __call__(self, nargout, *args):
        if len(args) > len(self.ins):
            raise WrapperError("too many input arguments")
        self.vars = dict(zip(self.ins, args))
        self.nargin, self.nargout = len(args), nargout
        self._run(self.body)
        return [self.get(o) for o in self.outs[:max(nargout, 1)]]
