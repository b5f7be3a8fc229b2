"""Extract the SQL test cases from the reference's ScalaTest sources.

Two source forms are taken:

* ``test("name", "sql" + "sql" ..., <numDruidQueries>, ...)`` / ``cTest("name", druidSql, baseSql)``
  whose SQL is made of plain string literals;
* the spark-datetime DSL form, ``test("name", { val p = dateTime('l_shipdate) <= (dateTime("1997-12-01")
  - 90.day); date\"\"\"... where $p ...\"\"\" }, n, ...)``: every ``$name`` interpolation is resolved to
  the ``val`` visible at that point (lexical brace scoping) and the DSL expression is translated to
  the sparkline date UDFs our SQL layer implements (``dateTime``, ``dateIsBefore...``, ``datePlus``,
  ``period``, ``year(...)``), exactly as the benchmark queries were translated
  (``models/tpch.py``).

Test calls that the reference has commented out are kept (StarSchemaTpchQueriesCTest sstqcT1-T6
are commented out there only because its sample data lacked the rows); the vendored corpus
(``tests/parity/cases.json``, written by ``python tests/parity/extract.py --write``) is what the
test suite runs, so it does not need the reference checkout."""
import json
import os
import re
import sys

REF_TESTS = "/root/reference/src/test/scala/org/sparklinedata/druid/client/test"
VENDORED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cases.json")

_CALL = re.compile(r'\b(test|cTest)\(\s*"([^"]+)"\s*,')
_VAL = re.compile(r'\bval\s+([A-Za-z_][A-Za-z0-9_]*)\s*=\s*([^\n]+)')


# ------------------------------------------------------------------ Scala lexical helpers
def _skip_ws(src, i):
    while i < len(src) and src[i] in " \t\r\n":
        i += 1
    return i


def _string_at(src, i):
    """A plain or triple-quoted literal at i (optionally ``date``-prefixed, optional .stripMargin):
    (text, end) or (None, i)."""
    if src.startswith('date"""', i):
        i += 4
    elif src.startswith('s"""', i):  # the s-interpolator (no substitutions in these tests)
        i += 1
    if src.startswith('"""', i):
        j = src.index('"""', i + 3)
        s = src[i + 3:j]
        i = j + 3
        if src.startswith(".stripMargin", i):
            s = "\n".join(re.sub(r"^\s*\|", "", ln) for ln in s.split("\n"))
            i += len(".stripMargin")
        return s, i
    if i < len(src) and src[i] == '"':
        j = i + 1
        buf = []
        while src[j] != '"':
            if src[j] == "\\":
                buf.append(src[j + 1])
                j += 2
                continue
            buf.append(src[j])
            j += 1
        return "".join(buf), j + 1
    return None, i


def _string_concat(src, i):
    """Parse `"..." + "..." + ...` starting at i."""
    out = []
    while True:
        i = _skip_ws(src, i)
        s, j = _string_at(src, i)
        if s is None:
            return None, i
        out.append(s)
        i = _skip_ws(src, j)
        if i < len(src) and src[i] == "+":
            i += 1
            continue
        return "".join(out), i


def _block_end(src, i):
    """Index just past the ``}`` matching the ``{`` at i (string literals skipped)."""
    depth = 0
    n = len(src)
    while i < n:
        if src.startswith('"""', i):
            i = src.index('"""', i + 3) + 3
            continue
        c = src[i]
        if c == '"':
            _, i = _string_at(src, i)
            continue
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return i + 1
        i += 1
    raise ValueError("unbalanced braces")


def _blocks(src):
    """(start, end) of every brace block, for lexical ``val`` scoping."""
    out, stack = [], []
    i, n = 0, len(src)
    while i < n:
        if src.startswith('"""', i):
            i = src.index('"""', i + 3) + 3
            continue
        c = src[i]
        if c == '"':
            _, i = _string_at(src, i)
            continue
        if c == "{":
            stack.append(i)
        elif c == "}" and stack:
            out.append((stack.pop(), i))
        i += 1
    return out


class _Scope:
    def __init__(self, src):
        self.blocks = _blocks(src)
        self.defs = []  # (pos, name, expr, (block start, block end))
        for m in _VAL.finditer(src):
            enc = min((b for b in self.blocks if b[0] < m.start() < b[1]), key=lambda b: b[1] - b[0],
                      default=(-1, len(src) + 1))
            self.defs.append((m.start(), m.group(1), m.group(2).strip(), enc))

    def lookup(self, name, pos):
        best = None
        for d, nm, expr, (a, b) in self.defs:
            if nm == name and d < pos and a < pos < b and (best is None or d > best[0]):
                best = (d, expr)
        return best[1] if best else None


# ------------------------------------------------------------------ spark-datetime DSL -> SQL
_UNITS = {"day": "D", "days": "D", "week": "W", "weeks": "W", "month": "M", "months": "M", "year": "Y",
          "years": "Y"}
_CMP = {"<": "dateIsBefore", "<=": "dateIsBeforeOrEqual", ">": "dateIsAfter", ">=": "dateIsAfterOrEqual",
        "===": "dateIsEqual"}
_FIELDS = {"year": "year", "monthOfYear": "month", "dayOfMonth": "dayofmonth", "hourOfDay": "hour"}
_TOK = re.compile(r"""\s*(dateTime\('([A-Za-z_][A-Za-z0-9_]*)\)|dateTime\("([^"]*)"\)|(\d+)\.(\w+)|
                       (===|<=|>=|<|>|\+|-|\(|\))|([A-Za-z]+))""", re.X)


def translate_dsl(expr: str) -> str:
    toks = []
    pos = 0
    expr = expr.strip()
    while pos < len(expr):
        m = _TOK.match(expr, pos)
        if not m or m.end() == pos:
            raise ValueError(f"DSL: cannot parse {expr[pos:]!r}")
        pos = m.end()
        if m.group(2):
            toks.append(("e", f"dateTime(`{m.group(2)}`)"))
        elif m.group(3) is not None:
            toks.append(("e", f'dateTime("{m.group(3)}")'))
        elif m.group(4):
            toks.append(("p", f'period("P{m.group(4)}{_UNITS[m.group(5)]}")'))
        elif m.group(6):
            toks.append(("o", m.group(6)))
        else:
            toks.append(("w", m.group(7)))
    i = 0

    def term():
        nonlocal i
        k, v = toks[i]
        if k == "o" and v == "(":
            i += 1
            e = arith()
            assert toks[i] == ("o", ")"), expr
            i += 1
            return e
        assert k == "e", expr
        i += 1
        return v

    def arith():
        nonlocal i
        e = term()
        while i < len(toks) and toks[i][0] == "o" and toks[i][1] in "+-" and toks[i][1] in ("+", "-"):
            op = toks[i][1]
            i += 1
            k, p = toks[i]
            assert k == "p", expr
            i += 1
            e = f"{'datePlus' if op == '+' else 'dateMinus'}({e}, {p})"
        while i < len(toks) and toks[i][0] == "w":
            e = f"{_FIELDS[toks[i][1]]}({e})"
            i += 1
        return e

    left = arith()
    if i < len(toks) and toks[i][0] == "o" and toks[i][1] in _CMP:
        op = toks[i][1]
        i += 1
        right = arith()
        out = f"{_CMP[op]}({left}, {right})"
    else:
        out = left
    if i != len(toks):
        raise ValueError(f"DSL: trailing tokens in {expr!r}")
    return out


_INTERP = re.compile(r"\$([A-Za-z_][A-Za-z0-9_]*)")


def _resolve(sql, scope, pos):
    def sub(m):
        expr = scope.lookup(m.group(1), pos)
        if expr is None:
            raise KeyError(m.group(1))
        return translate_dsl(expr)
    return _INTERP.sub(sub, sql)


def _sql_arg(src, i, scope):
    """One SQL argument at i: string concatenation, a bare date\"\"\"\"\"\" literal, or a ``{ vals;
    date\"\"\"...\"\"\" }`` block. -> (sql or None, end)."""
    i = _skip_ws(src, i)
    if i < len(src) and src[i] == "{":
        end = _block_end(src, i)
        body = src[i + 1:end - 1]
        k = body.find('date"""')
        if k < 0:
            k = body.find('"""')
            if k < 0:
                return None, end
        sql, _ = _string_at(body, k)
        pos = i + 1 + k
    else:
        pos = i
        sql, end = _string_concat(src, i)
        if sql is None:
            return None, i
    try:
        sql = _resolve(sql, scope, pos)
    except (KeyError, ValueError, AssertionError):
        return None, end
    return " ".join(sql.split()), end


def extract_from_reference():
    out = []
    for fn in sorted(os.listdir(REF_TESTS)):
        if not fn.endswith(".scala"):
            continue
        src = open(os.path.join(REF_TESTS, fn)).read()
        scope = _Scope(src)
        for m in _CALL.finditer(src):
            kind, name = m.group(1), m.group(2)
            sql, i = _sql_arg(src, m.end(), scope)
            if not sql:
                continue
            rest = src[i:i + 40]
            if kind == "test":
                mm = re.match(r"\s*,\s*(\d+)", rest)
                if mm:
                    out.append((fn[:-6], name, "shape", sql, int(mm.group(1)), None))
                elif re.match(r"\s*\)", rest):  # numDruidQueries defaults to 1 (tc/AbstractTest.scala:105-106)
                    out.append((fn[:-6], name, "shape", sql, 1, None))
            else:
                mm = re.match(r"\s*,\s*", rest)
                if not mm:
                    continue
                sql2, _ = _sql_arg(src, i + mm.end(), scope)
                if sql2:
                    out.append((fn[:-6], name, "ctest", sql, None, sql2))
    return out


def cases():
    """The vendored corpus (runs without the reference checkout); falls back to live extraction."""
    if os.path.exists(VENDORED):
        with open(VENDORED) as f:
            return [tuple(c) for c in json.load(f)["cases"]]
    if os.path.isdir(REF_TESTS):
        return extract_from_reference()
    return []


if __name__ == "__main__":
    cs = extract_from_reference()
    print(len(cs), "cases;", sum("date" in c[3] for c in cs), "use the date DSL")
    if "--write" in sys.argv:
        with open(VENDORED, "w") as f:
            json.dump({"source": "reference ScalaTest sources (tests/parity/extract.py)", "cases": cs}, f, indent=0)
