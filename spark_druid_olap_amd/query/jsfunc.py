"""A tiny JavaScript-function interpreter for Druid ``javascript`` filters / extractions /
aggregators / post-aggregators that arrive as JSON (``ON DRUIDDATASOURCE .. EXECUTE QUERY``).

The reference planner generates such functions (``sd/jscodegen/JSCodeGenerator.scala``) and
Druid runs them per row in Rhino.  Here they are compiled ONCE to a Python closure and then
evaluated over the dictionary domain (filters, extractions: once per distinct value) or
translated to the kernel's expression VM (aggregators: see ``jsagg_to_expr``).

Supported subset: ``function(a, b) { [var x = e;]* return e; }`` with literals, identifiers,
``+ - * / %``, comparisons, ``== === != !==``, ``&& || !``, ``?:``, member calls on strings
(toUpperCase, toLowerCase, substring, substr, indexOf, startsWith, endsWith, trim, charAt,
length, replace), ``Math.*``, ``parseInt``, ``parseFloat``, ``Number``, ``String``.
"""
from __future__ import annotations

import math
import re
from typing import Any, Callable, Dict, List, Tuple

_TOK = re.compile(
    r"\s*(?:(?P<num>\d+\.\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?|\d+(?:[eE][+-]?\d+)?)"
    r"|(?P<str>'(?:[^'\\]|\\.)*'|\"(?:[^\"\\]|\\.)*\")"
    r"|(?P<id>[A-Za-z_$][\w$]*)"
    r"|(?P<op>===|!==|==|!=|<=|>=|&&|\|\||[-+*/%<>!?:(){}\[\],.;=]))"
)


class JSError(ValueError):
    pass


def _tokenize(s: str) -> List[Tuple[str, str]]:
    out, pos = [], 0
    s = s.strip()
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            if s[pos:].strip() == "":
                break
            raise JSError(f"bad javascript near {s[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
    return out


def _unescape(s: str) -> str:
    return bytes(s[1:-1], "utf-8").decode("unicode_escape")


def _js_add(a, b):
    if isinstance(a, str) or isinstance(b, str):
        return _js_str(a) + _js_str(b)
    return (a or 0) + (b or 0)


def _js_str(v):
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return str(v)


def _num(v):
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError:
            return float("nan")
    if v is None:
        return 0.0
    return v


def _cmp(op, a, b):
    if isinstance(a, str) and isinstance(b, str):
        pass
    elif isinstance(a, str) or isinstance(b, str):
        a, b = _num(a), _num(b)
    if a is None or b is None:
        return False
    if op == "<":
        return a < b
    if op == "<=":
        return a <= b
    if op == ">":
        return a > b
    return a >= b


def _div(a, b):
    a, b = _num(a), _num(b)
    if b == 0:
        return float("nan") if a == 0 else math.copysign(float("inf"), a)
    return a / b


_STR_METHODS = {
    "toUpperCase": lambda s: s.upper(),
    "toLowerCase": lambda s: s.lower(),
    "trim": lambda s: s.strip(),
    "substring": lambda s, a, b=None: s[int(min(a, b)) if b is not None else int(a):int(max(a, b)) if b is not None else None],
    "substr": lambda s, a, n=None: s[int(a):(int(a) + int(n)) if n is not None else None],
    "indexOf": lambda s, x: s.find(x),
    "startsWith": lambda s, x: s.startswith(x),
    "endsWith": lambda s, x: s.endswith(x),
    "charAt": lambda s, i: s[int(i)] if 0 <= int(i) < len(s) else "",
    "replace": lambda s, a, b: s.replace(a, b, 1),
    "concat": lambda s, *xs: s + "".join(_js_str(x) for x in xs),
    "toString": lambda s: _js_str(s),
}

_GLOBALS = {
    "Math": {"max": lambda *a: max(_num(x) for x in a), "min": lambda *a: min(_num(x) for x in a),
             "abs": lambda x: abs(_num(x)), "floor": lambda x: float(math.floor(_num(x))),
             "ceil": lambda x: float(math.ceil(_num(x))), "round": lambda x: float(math.floor(_num(x) + 0.5)),
             "sqrt": lambda x: math.sqrt(_num(x)), "pow": lambda a, b: _num(a) ** _num(b),
             "log": lambda x: math.log(_num(x)), "exp": lambda x: math.exp(_num(x)), "PI": math.pi},
    "parseInt": lambda x, *r: float(int(float(x))) if x not in (None, "") else float("nan"),
    "parseFloat": lambda x: _num(x),
    "Number": lambda x: _num(x),
    "String": lambda x: _js_str(x),
    "undefined": None,
    "NaN": float("nan"),
    "Infinity": float("inf"),
}


class _Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else ("eof", "")

    def next(self):
        tok = self.peek()
        self.i += 1
        return tok

    def expect(self, v):
        tok = self.next()
        if tok[1] != v:
            raise JSError(f"expected {v!r}, got {tok[1]!r}")
        return tok

    def accept(self, v):
        if self.peek()[1] == v:
            self.i += 1
            return True
        return False

    # function(params) { body }
    def function(self):
        self.expect("function")
        if self.peek()[0] == "id":
            self.next()
        self.expect("(")
        params = []
        while not self.accept(")"):
            params.append(self.next()[1])
            self.accept(",")
        self.expect("{")
        stmts = []
        while not self.accept("}"):
            stmts.append(self.statement())
        return params, stmts

    def statement(self):
        if self.accept(";"):
            return ("nop",)
        if self.peek()[1] == "var":
            self.next()
            decls = []
            while True:
                name = self.next()[1]
                e = self.expr() if self.accept("=") else (lambda env: None)
                decls.append((name, e))
                if not self.accept(","):
                    break
            self.accept(";")
            return ("var", decls)
        if self.peek()[1] == "return":
            self.next()
            e = self.expr()
            self.accept(";")
            return ("ret", e)
        if self.peek()[1] == "if":
            self.next()
            self.expect("(")
            c = self.expr()
            self.expect(")")
            a = self.block()
            b = self.block() if self.accept("else") else []
            return ("if", c, a, b)
        if self.peek()[0] == "id" and self.peek(1)[1] == "=":
            name = self.next()[1]
            self.next()
            e = self.expr()
            self.accept(";")
            return ("set", name, e)
        e = self.expr()
        self.accept(";")
        return ("expr", e)

    def block(self):
        if self.accept("{"):
            out = []
            while not self.accept("}"):
                out.append(self.statement())
            return out
        return [self.statement()]

    def expr(self):
        c = self.orexpr()
        if self.accept("?"):
            a = self.expr()
            self.expect(":")
            b = self.expr()
            return lambda env: a(env) if c(env) else b(env)
        return c

    def orexpr(self):
        a = self.andexpr()
        while self.accept("||"):
            b = self.andexpr()
            a = (lambda x, y: lambda env: x(env) or y(env))(a, b)
        return a

    def andexpr(self):
        a = self.eqexpr()
        while self.accept("&&"):
            b = self.eqexpr()
            a = (lambda x, y: lambda env: x(env) and y(env))(a, b)
        return a

    def eqexpr(self):
        a = self.relexpr()
        while self.peek()[1] in ("==", "===", "!=", "!=="):
            op = self.next()[1]
            b = self.relexpr()
            if op in ("==", "==="):
                a = (lambda x, y: lambda env: _eq(x(env), y(env)))(a, b)
            else:
                a = (lambda x, y: lambda env: not _eq(x(env), y(env)))(a, b)
        return a

    def relexpr(self):
        a = self.addexpr()
        while self.peek()[1] in ("<", "<=", ">", ">="):
            op = self.next()[1]
            b = self.addexpr()
            a = (lambda x, y, o: lambda env: _cmp(o, x(env), y(env)))(a, b, op)
        return a

    def addexpr(self):
        a = self.mulexpr()
        while self.peek()[1] in ("+", "-"):
            op = self.next()[1]
            b = self.mulexpr()
            if op == "+":
                a = (lambda x, y: lambda env: _js_add(x(env), y(env)))(a, b)
            else:
                a = (lambda x, y: lambda env: _num(x(env)) - _num(y(env)))(a, b)
        return a

    def mulexpr(self):
        a = self.unary()
        while self.peek()[1] in ("*", "/", "%"):
            op = self.next()[1]
            b = self.unary()
            if op == "*":
                a = (lambda x, y: lambda env: _num(x(env)) * _num(y(env)))(a, b)
            elif op == "/":
                a = (lambda x, y: lambda env: _div(x(env), y(env)))(a, b)
            else:
                a = (lambda x, y: lambda env: math.fmod(_num(x(env)), _num(y(env))))(a, b)
        return a

    def unary(self):
        if self.accept("!"):
            a = self.unary()
            return lambda env: not a(env)
        if self.accept("-"):
            a = self.unary()
            return lambda env: -_num(a(env))
        if self.accept("+"):
            a = self.unary()
            return lambda env: _num(a(env))
        return self.postfix()

    def postfix(self):
        a = self.primary()
        while True:
            if self.accept("."):
                name = self.next()[1]
                if self.accept("("):
                    args = self.args()
                    a = (lambda obj, n, ar: lambda env: _call_member(obj(env), n, [x(env) for x in ar]))(a, name, args)
                else:
                    a = (lambda obj, n: lambda env: _member(obj(env), n))(a, name)
            elif self.accept("("):
                args = self.args()
                a = (lambda f, ar: lambda env: f(env)(*[x(env) for x in ar]))(a, args)
            elif self.accept("["):
                idx = self.expr()
                self.expect("]")
                a = (lambda obj, ix: lambda env: _index(obj(env), ix(env)))(a, idx)
            else:
                return a

    def args(self):
        out = []
        while not self.accept(")"):
            out.append(self.expr())
            self.accept(",")
        return out

    def primary(self):
        kind, v = self.next()
        if kind == "num":
            f = float(v)
            return lambda env: f
        if kind == "str":
            s = _unescape(v)
            return lambda env: s
        if kind == "id":
            if v == "true":
                return lambda env: True
            if v == "false":
                return lambda env: False
            if v == "null":
                return lambda env: None
            return lambda env: env[v] if v in env else _GLOBALS[v]
        if v == "(":
            e = self.expr()
            self.expect(")")
            return e
        if v == "[":
            items = []
            while not self.accept("]"):
                items.append(self.expr())
                self.accept(",")
            return lambda env: [x(env) for x in items]
        raise JSError(f"unexpected token {v!r}")


def _eq(a, b):
    if isinstance(a, str) != isinstance(b, str) and a is not None and b is not None:
        return _num(a) == _num(b)
    return a == b


def _member(obj, name):
    if name == "length":
        return float(len(obj))
    if isinstance(obj, dict):
        return obj[name]
    raise JSError(f"unsupported member {name}")


def _index(obj, i):
    if isinstance(obj, (str, list)):
        return obj[int(i)]
    return obj[i]


def _call_member(obj, name, args):
    if isinstance(obj, dict):
        return obj[name](*args)
    if isinstance(obj, str):
        if name not in _STR_METHODS:
            raise JSError(f"unsupported string method {name}")
        return _STR_METHODS[name](obj, *args)
    if name == "toString":
        return _js_str(obj)
    if name == "toFixed":
        return f"{_num(obj):.{int(args[0]) if args else 0}f}"
    raise JSError(f"unsupported call {name} on {type(obj).__name__}")


def _run(stmts, env):
    for st in stmts:
        k = st[0]
        if k == "ret":
            return True, st[1](env)
        if k == "var":
            for name, e in st[1]:
                env[name] = e(env)
        elif k == "set":
            env[st[1]] = st[2](env)
        elif k == "if":
            done, v = _run(st[2] if st[1](env) else st[3], env)
            if done:
                return True, v
        elif k == "expr":
            st[1](env)
    return False, None


def compile_function(src: str) -> Callable[..., Any]:
    """Compile a JS ``function(..){..}`` into a Python callable."""
    p = _Parser(_tokenize(src))
    params, stmts = p.function()

    def fn(*args):
        env: Dict[str, Any] = dict(zip(params, args))
        _, v = _run(stmts, env)
        return v

    fn.params = params  # type: ignore[attr-defined]
    return fn


# ------------------------------------------------------------------------------------------------
# javascript aggregator -> (combine op, expression over fields)
def _strip_parens(e: str) -> str:
    e = e.strip()
    while e.startswith("(") and e.endswith(")"):
        depth = 0
        for i, ch in enumerate(e):
            depth += ch == "("
            depth -= ch == ")"
            if depth == 0 and i < len(e) - 1:
                return e
        e = e[1:-1].strip()
    return e


def jsagg_to_expr(fn_aggregate: str):
    """Recognize ``current + <expr>`` / ``Math.max(current, <expr>)`` aggregate bodies.

    Returns (op in {'sum','max','min'}, param names, expression string) or raises JSError."""
    m = re.match(r"\s*function\s*\w*\s*\((?P<p>[^)]*)\)\s*\{(?P<body>.*)\}\s*$", fn_aggregate, re.S)
    if not m:
        raise JSError("not a javascript function")
    params = [x.strip() for x in m.group("p").split(",") if x.strip()]
    body = m.group("body").strip()
    r = re.match(r"^return\s*(?P<e>.*?)\s*;?\s*$", body, re.S)
    if not r or not params:
        raise JSError("unsupported javascript aggregator body")
    e = _strip_parens(r.group("e"))
    cur = params[0]
    mm = re.match(r"^Math\.(?P<f>max|min)\s*\((?P<rest>.*)\)$", e, re.S)
    if mm:
        rest = mm.group("rest").strip()
        if rest.startswith(cur) and rest[len(cur):].lstrip().startswith(","):
            return (mm.group("f"), params[1:], rest[len(cur):].lstrip()[1:].strip())
    ms = re.match(r"^%s\s*\+\s*(?P<e>.*)$" % re.escape(cur), e, re.S)
    if ms:
        return ("sum", params[1:], ms.group("e").strip())
    raise JSError("unsupported javascript aggregator body")


def parse_expr(src: str):
    """Parse a bare JS expression (no function wrapper) into an AST of tuples for the expr VM."""
    return _ExprAst(_tokenize(src)).expr()


class _ExprAst:
    """Arithmetic-only JS expression -> ('col', name) | ('const', v) | (op, a, b) | ('neg', a)."""

    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else ("eof", "")

    def next(self):
        tok = self.peek()
        self.i += 1
        return tok

    def expr(self):
        a = self.term()
        while self.peek()[1] in ("+", "-"):
            op = self.next()[1]
            a = ("add" if op == "+" else "sub", a, self.term())
        return a

    def term(self):
        a = self.unary()
        while self.peek()[1] in ("*", "/", "%"):
            op = self.next()[1]
            a = ({"*": "mul", "/": "div", "%": "mod"}[op], a, self.unary())
        return a

    def unary(self):
        if self.peek()[1] == "-":
            self.next()
            return ("neg", self.unary())
        if self.peek()[1] == "+":
            self.next()
            return self.unary()
        return self.primary()

    def primary(self):
        kind, v = self.next()
        if kind == "num":
            return ("const", float(v))
        if kind == "id":
            if v == "Math" and self.peek()[1] == ".":
                self.next()
                fn = self.next()[1]
                self.next()  # (
                args = [self.expr()]
                while self.peek()[1] == ",":
                    self.next()
                    args.append(self.expr())
                self.next()  # )
                if fn in ("abs", "floor", "ceil", "sqrt", "log", "exp"):
                    return (fn, args[0])
                if fn in ("pow", "pmod"):  # Math.pmod: Spark pmod (extension used by the SQL planner)
                    return (fn, args[0], args[1])
                if fn in ("max", "min"):
                    out = args[0]
                    for a in args[1:]:
                        out = (fn, out, a)
                    return out
                raise JSError(f"unsupported Math.{fn} in aggregator")
            return ("col", v)
        if v == "(":
            e = self.expr()
            if self.next()[1] != ")":
                raise JSError("missing )")
            return e
        raise JSError(f"unexpected token {v!r} in aggregator expression")
