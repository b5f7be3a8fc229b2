"""Hand-written lexer + recursive-descent parser for the Spark-SQL subset used by the reference's
tests and benchmarks, plus the Sparkline command grammar.

Parity targets:
  * ``SPLParser`` (``asql/hive/sparklinedata/SparklineDataParser.scala:29-78``): commands are tried
    first, then the SQL grammar; errors from both are merged into one message.
  * Druid commands (same file 85-126): ``CLEAR DRUID CACHE [host]``,
    ``ON DRUIDDATASOURCE <t> [USING HISTORICAL] EXECUTE [QUERY] <json>``,
    ``EXPLAIN DRUID REWRITE <sql>``.
  * DDL: ``CREATE [TEMPORARY] TABLE [IF NOT EXISTS] t [(cols)] USING <provider> OPTIONS (k v, ...)``
    (``sd/DefaultSource.scala:32-194`` consumes the options).
"""
from __future__ import annotations

import re
from typing import List, Optional, Tuple

from . import ast as A


class ParseError(ValueError):
    pass


_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[lLdDsSyY]?(?:BD)?)
  | (?P<bq>`(?:[^`]|``)*`)
  | (?P<sq>'(?:[^'\\]|\\.|'')*')
  | (?P<dq>"(?:[^"\\]|\\.|"")*")
  | (?P<id>[A-Za-z_$][A-Za-z0-9_$]*)
  | (?P<op><=>|<>|!=|>=|<=|==|\|\||&&|[-+*/%=<>(),.;!~&|^\[\]:])
""", re.S | re.X)

_ESC = {"n": "\n", "t": "\t", "r": "\r", "0": "\0", "b": "\b", "Z": "\x1a"}


def _unquote(s: str) -> str:
    q = s[0]
    body = s[1:-1]
    out = []
    i = 0
    while i < len(body):
        c = body[i]
        if c == "\\" and i + 1 < len(body):
            n = body[i + 1]
            out.append(_ESC.get(n, n))
            i += 2
            continue
        if c == q and i + 1 < len(body) and body[i + 1] == q:
            out.append(q)
            i += 2
            continue
        out.append(c)
        i += 1
    return "".join(out)


class Tok:
    __slots__ = ("kind", "text", "pos", "end")

    def __init__(self, kind, text, pos, end):
        self.kind, self.text, self.pos, self.end = kind, text, pos, end

    @property
    def up(self) -> str:
        return self.text.upper() if self.kind == "id" else self.text

    def __repr__(self):
        return f"{self.kind}:{self.text}"


def tokenize(sql: str) -> List[Tok]:
    out = []
    pos = 0
    n = len(sql)
    while pos < n:
        m = _TOKEN_RE.match(sql, pos)
        if not m:  # stray character (e.g. JSON after EXECUTE QUERY): the grammar rejects it later
            out.append(Tok("op", sql[pos], pos, pos + 1))
            pos += 1
            continue
        k = m.lastgroup
        t = m.group(k)
        if k != "ws":
            if k == "bq":
                out.append(Tok("qid", t[1:-1].replace("``", "`"), pos, m.end()))
            elif k in ("sq", "dq"):
                out.append(Tok("str", _unquote(t), pos, m.end()))
            else:
                out.append(Tok(k, t, pos, m.end()))
        pos = m.end()
    out.append(Tok("eof", "", n, n))
    return out


# words that end an expression / cannot be an implicit alias
RESERVED = {
    "SELECT", "FROM", "WHERE", "GROUP", "BY", "HAVING", "ORDER", "SORT", "LIMIT", "UNION", "INTERSECT",
    "EXCEPT", "JOIN", "INNER", "LEFT", "RIGHT", "FULL", "OUTER", "CROSS", "SEMI", "ANTI", "ON", "USING",
    "AS", "AND", "OR", "NOT", "IN", "IS", "LIKE", "RLIKE", "REGEXP", "BETWEEN", "CASE", "WHEN", "THEN",
    "ELSE", "END", "WITH", "DISTINCT", "ALL", "ASC", "DESC", "NULLS", "LATERAL", "WINDOW", "DISTRIBUTE",
    "CLUSTER", "NATURAL", "GROUPING", "CUBE", "ROLLUP", "SETS",
}

TYPE_NAMES = {
    "INT": "int", "INTEGER": "int", "BIGINT": "bigint", "LONG": "bigint", "SMALLINT": "smallint",
    "SHORT": "smallint", "TINYINT": "tinyint", "BYTE": "tinyint", "DOUBLE": "double", "FLOAT": "float",
    "REAL": "float", "DECIMAL": "decimal", "DEC": "decimal", "NUMERIC": "decimal", "STRING": "string",
    "VARCHAR": "string", "CHAR": "string", "TEXT": "string", "DATE": "date", "TIMESTAMP": "timestamp",
    "BOOLEAN": "boolean", "BOOL": "boolean", "BINARY": "binary",
}

_INTERVAL_UNITS = {
    "YEAR": ("m", 12), "YEARS": ("m", 12), "MONTH": ("m", 1), "MONTHS": ("m", 1),
    "WEEK": ("d", 7), "WEEKS": ("d", 7), "DAY": ("d", 1), "DAYS": ("d", 1),
    "HOUR": ("u", 3600 * 10 ** 6), "HOURS": ("u", 3600 * 10 ** 6), "MINUTE": ("u", 60 * 10 ** 6),
    "MINUTES": ("u", 60 * 10 ** 6), "SECOND": ("u", 10 ** 6), "SECONDS": ("u", 10 ** 6),
    "MILLISECOND": ("u", 1000), "MILLISECONDS": ("u", 1000), "MICROSECOND": ("u", 1),
    "MICROSECONDS": ("u", 1),
}


class Parser:
    def __init__(self, sql: str):
        self.src = sql
        self.toks = tokenize(sql)
        self.i = 0

    # -- token helpers -------------------------------------------------------------------------
    def peek(self, k: int = 0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def next(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def at(self, *words) -> bool:
        t = self.peek()
        return (t.kind == "id" and t.up in words) or (t.kind == "op" and t.text in words)

    def at_seq(self, *words) -> bool:
        for k, w in enumerate(words):
            t = self.peek(k)
            if not ((t.kind == "id" and t.up == w) or (t.kind == "op" and t.text == w)):
                return False
        return True

    def accept(self, *words) -> bool:
        if self.at(*words):
            self.i += 1
            return True
        return False

    def expect(self, *words) -> Tok:
        if not self.at(*words):
            t = self.peek()
            raise ParseError(f"expected {' or '.join(words)} but found '{t.text or 'end of input'}' "
                             f"at position {t.pos}")
        return self.next()

    def ident(self) -> str:
        t = self.peek()
        if t.kind == "qid" or (t.kind == "id"):
            self.i += 1
            return t.text
        if t.kind == "str":  # some dialects allow 'name'
            self.i += 1
            return t.text
        raise ParseError(f"expected identifier but found '{t.text or 'end of input'}' at position {t.pos}")

    def qualified_name(self) -> Tuple[str, ...]:
        parts = [self.ident()]
        while self.peek().kind == "op" and self.peek().text == "." and self.peek(1).kind in ("id", "qid"):
            self.i += 1
            parts.append(self.ident())
        return tuple(parts)

    # -- statements ----------------------------------------------------------------------------
    def statement(self):
        st = self._statement()
        self.accept(";")
        if self.peek().kind != "eof":
            t = self.peek()
            raise ParseError(f"unexpected '{t.text}' at position {t.pos}")
        return st

    def _statement(self):
        if self.at_seq("CLEAR", "DRUID", "CACHE"):
            self.i += 3
            host = None
            if self.peek().kind != "eof" and not self.at(";"):
                host = self._rest_text().strip() or None
            return A.ClearDruidCache(host)
        if self.at_seq("ON", "DRUIDDATASOURCE"):
            self.i += 2
            name = self.qualified_name()
            hist = False
            if self.accept("USING"):
                self.expect("HISTORICAL")
                hist = True
            self.expect("EXECUTE")
            self.accept("QUERY")
            return A.ExecuteDruidQuery(name, hist, self._rest_text())
        if self.at_seq("EXPLAIN", "DRUID", "REWRITE"):
            self.i += 3
            return A.ExplainDruidRewrite(self.query())
        if self.accept("EXPLAIN"):
            ext = bool(self.accept("EXTENDED", "CODEGEN", "FORMATTED"))
            return A.Explain(self.query(), ext)
        if self.at("CREATE"):
            return self._create()
        if self.accept("DROP"):
            view = False
            if self.accept("VIEW"):
                view = True
            else:
                self.expect("TABLE")
            ife = False
            if self.accept("IF"):
                self.expect("EXISTS")
                ife = True
            return A.DropTable(self.qualified_name(), ife, view)
        if self.accept("USE"):
            return A.UseDatabase(self.ident())
        if self.accept("SET"):
            rest = self._rest_text().strip().rstrip(";").strip()
            if not rest or rest == "-v":
                return A.SetConf(None, None)
            if "=" in rest:
                k, v = rest.split("=", 1)
                return A.SetConf(k.strip(), v.strip())
            parts = rest.split(None, 1)
            return A.SetConf(parts[0], parts[1].strip() if len(parts) > 1 else None)
        if self.accept("SHOW"):
            self.expect("TABLES")
            db = None
            if self.accept("IN", "FROM"):
                db = self.ident()
            return A.ShowTables(db)
        if self.accept("DESCRIBE", "DESC"):
            self.accept("TABLE", "EXTENDED", "FORMATTED")
            return A.Describe(self.qualified_name())
        if self.accept("CACHE"):
            self.accept("LAZY")
            self.expect("TABLE")
            return A.CacheTable(self.qualified_name())
        if self.accept("UNCACHE"):
            self.expect("TABLE")
            return A.CacheTable(self.qualified_name(), uncache=True)
        return self.query()

    def _rest_text(self) -> str:
        t = self.peek()
        txt = self.src[t.pos:]
        self.i = len(self.toks) - 1
        return txt.rstrip().rstrip(";")

    def _create(self):
        start = self.peek().pos
        self.expect("CREATE")
        replace = False
        if self.accept("OR"):
            self.expect("REPLACE")
            replace = True
        temp = bool(self.accept("TEMPORARY", "TEMP"))
        if self.accept("DATABASE", "SCHEMA"):
            ine = False
            if self.accept("IF"):
                self.expect("NOT")
                self.expect("EXISTS")
                ine = True
            return A.CreateDatabase(self.ident(), ine)
        if self.accept("VIEW"):
            name = self.qualified_name()
            self.expect("AS")
            qpos = self.peek().pos
            q = self.query()
            return A.CreateView(name, q, replace, temp, self.src[qpos:].strip().rstrip(";"))
        self.accept("EXTERNAL")
        self.expect("TABLE")
        ine = False
        if self.accept("IF"):
            self.expect("NOT")
            self.expect("EXISTS")
            ine = True
        name = self.qualified_name()
        cols: List[A.ColumnDef] = []
        if self.accept("("):
            while True:
                cn = self.ident()
                cols.append(A.ColumnDef(cn, self.type_name()))
                while self.peek().kind == "id" and self.peek().up in ("NOT", "NULL", "COMMENT"):
                    if self.accept("COMMENT"):
                        self.next()
                    else:
                        self.next()
                if not self.accept(","):
                    break
            self.expect(")")
        provider = None
        options = {}
        as_query = None
        if self.accept("USING"):
            provider = ".".join(self.qualified_name())
        if self.accept("OPTIONS"):
            self.expect("(")
            while not self.at(")"):
                k = ".".join(self.qualified_name())
                self.accept("=")
                t = self.next()
                if t.kind not in ("str", "num", "id", "qid"):
                    raise ParseError(f"bad option value at position {t.pos}")
                options[k] = t.text
                if not self.accept(","):
                    break
            self.expect(")")
        if self.accept("AS"):
            as_query = self.query()
        _ = start
        return A.CreateTable(name, cols, provider, options, ine, temp, as_query)

    def type_name(self) -> str:
        t = self.ident().upper()
        if t not in TYPE_NAMES:
            raise ParseError(f"unsupported data type {t}")
        ty = TYPE_NAMES[t]
        if self.accept("("):
            args = [self.next().text]
            while self.accept(","):
                args.append(self.next().text)
            self.expect(")")
            if ty == "decimal":
                return f"decimal({','.join(args)})"
        elif ty == "decimal":
            return "decimal(10,0)"
        return ty

    # -- queries -------------------------------------------------------------------------------
    def query(self):
        if self.accept("WITH"):
            ctes = []
            while True:
                n = self.ident()
                self.expect("AS")
                self.expect("(")
                q = self.query()
                self.expect(")")
                ctes.append((n, q))
                if not self.accept(","):
                    break
            return A.With(ctes, self.query())
        q = self._set_term()
        while self.at("UNION", "INTERSECT", "EXCEPT"):
            kind = self.next().up.lower()
            all_ = bool(self.accept("ALL"))
            if not all_:
                self.accept("DISTINCT")
            r = self._set_term()
            q = A.SetOp(kind, all_, q, r)
        if isinstance(q, A.SetOp):
            # ORDER BY / LIMIT written after the last operand bind to the whole set operation
            last = q.right
            if isinstance(last, A.Select) and not getattr(last, "_paren", False) and (last.order_by or
                                                                                       last.limit is not None):
                q.order_by, q.limit = last.order_by, last.limit
                last.order_by, last.limit = [], None
            o, l = self._order_limit()
            if o:
                q.order_by = o
            if l is not None:
                q.limit = l
        return q

    def _set_term(self):
        if self.at("(") and self._paren_is_query():
            self.expect("(")
            q = self.query()
            self.expect(")")
            q._paren = True
            return q
        return self.select()

    def _paren_is_query(self) -> bool:
        k = 0
        while self.peek(k).kind == "op" and self.peek(k).text == "(":
            k += 1
        t = self.peek(k)
        return t.kind == "id" and t.up in ("SELECT", "WITH")

    def _order_limit(self):
        order = []
        if self.at_seq("ORDER", "BY") or self.at_seq("SORT", "BY"):
            self.i += 2
            order = self.sort_items()
        limit = None
        if self.accept("LIMIT"):
            e = self.expr()
            if not isinstance(e, A.Lit):
                raise ParseError("LIMIT expects a literal")
            limit = int(e.value)
        return order, limit

    def sort_items(self) -> List[A.SortOrder]:
        out = []
        while True:
            e = self.expr()
            asc = True
            if self.accept("DESC"):
                asc = False
            else:
                self.accept("ASC")
            nf = None
            if self.accept("NULLS"):
                nf = self.next().up == "FIRST"
            out.append(A.SortOrder(e, asc, nf))
            if not self.accept(","):
                break
        return out

    def select(self) -> A.Select:
        self.expect("SELECT")
        distinct = bool(self.accept("DISTINCT"))
        if not distinct:
            self.accept("ALL")
        items = []
        while True:
            e = self.expr()
            alias = None
            if self.accept("AS"):
                if self.accept("("):  # as (a, b) -- not supported beyond one name
                    alias = self.ident()
                    self.expect(")")
                else:
                    alias = self.ident()
            elif self.peek().kind in ("qid", "str") or (self.peek().kind == "id" and self.peek().up not in RESERVED):
                alias = self.ident()
            items.append(A.SelectItem(e, alias))
            if not self.accept(","):
                break
        sel = A.Select(items, distinct=distinct)
        if self.accept("FROM"):
            sel.from_ = self.relations()
        if self.accept("WHERE"):
            sel.where = self.expr()
        if self.at_seq("GROUP", "BY"):
            self.i += 2
            self._group_by(sel)
        if self.accept("HAVING"):
            sel.having = self.expr()
        sel.order_by, sel.limit = self._order_limit()
        return sel

    def _group_by(self, sel: A.Select):
        if self.at("CUBE", "ROLLUP") and self.peek(1).text == "(":
            kind = self.next().up
            self.expect("(")
            exprs = self.expr_list()
            self.expect(")")
            sel.group_by = exprs
            sel.grouping_sets = _expand_sets(kind, exprs)
            return
        if self.at_seq("GROUPING", "SETS"):
            self.i += 2
            sel.group_by, sel.grouping_sets = self._grouping_sets([])
            return
        exprs = self.expr_list()
        sel.group_by = exprs
        if self.at_seq("WITH", "CUBE") or self.at_seq("WITH", "ROLLUP"):
            self.i += 1
            kind = self.next().up
            sel.grouping_sets = _expand_sets(kind, exprs)
        elif self.at_seq("GROUPING", "SETS"):
            self.i += 2
            _, sel.grouping_sets = self._grouping_sets(exprs)

    def _grouping_sets(self, base: List[A.Expr]):
        self.expect("(")
        sets = []
        allx = list(base)
        keys = [e.key() for e in allx]
        while True:
            if self.accept("("):
                s = [] if self.at(")") else self.expr_list()
                self.expect(")")
            else:
                s = [self.expr()]
            for e in s:
                if e.key() not in keys:
                    keys.append(e.key())
                    allx.append(e)
            sets.append(s)
            if not self.accept(","):
                break
        self.expect(")")
        return allx, sets

    def expr_list(self) -> List[A.Expr]:
        out = [self.expr()]
        while self.accept(","):
            out.append(self.expr())
        return out

    def relations(self):
        rel = self.join_chain()
        while self.accept(","):
            rel = A.JoinRef("cross", rel, self.join_chain())
        return rel

    def join_chain(self):
        rel = self.relation_primary()
        while True:
            kind = None
            if self.accept("JOIN"):
                kind = "inner"
            elif self.at("INNER") and self.peek(1).up == "JOIN":
                self.i += 2
                kind = "inner"
            elif self.at("CROSS"):
                self.i += 1
                self.expect("JOIN")
                kind = "cross"
            elif self.at("LEFT", "RIGHT", "FULL"):
                side = self.next().up.lower()
                if self.accept("SEMI"):
                    kind = "leftsemi"
                elif self.accept("ANTI"):
                    kind = "leftanti"
                else:
                    self.accept("OUTER")
                    kind = side
                self.expect("JOIN")
            else:
                break
            right = self.relation_primary()
            cond = None
            using = None
            if self.accept("ON"):
                cond = self.expr()
            elif self.accept("USING"):
                self.expect("(")
                using = [self.ident()]
                while self.accept(","):
                    using.append(self.ident())
                self.expect(")")
            rel = A.JoinRef(kind, rel, right, cond, using)
        return rel

    def relation_primary(self):
        if self.accept("("):
            if self._paren_is_query() or self.at("SELECT", "WITH"):
                q = self.query()
                self.expect(")")
                return A.SubqueryRef(q, self._alias())
            r = self.relations()
            self.expect(")")
            return r
        name = self.qualified_name()
        return A.TableRef(name, self._alias())

    def _alias(self) -> Optional[str]:
        if self.accept("AS"):
            return self.ident()
        t = self.peek()
        if t.kind == "qid" or (t.kind == "id" and t.up not in RESERVED):
            return self.ident()
        return None

    # -- expressions ---------------------------------------------------------------------------
    def expr(self) -> A.Expr:
        return self._or()

    def _or(self):
        e = self._and()
        while self.accept("OR"):
            e = A.BinOp("or", e, self._and())
        return e

    def _and(self):
        e = self._not()
        while self.accept("AND", "&&"):
            e = A.BinOp("and", e, self._not())
        return e

    def _not(self):
        if self.accept("NOT", "!"):
            return A.UnOp("not", self._not())
        return self._predicate()

    def _predicate(self):
        e = self._bitor()
        while True:
            t = self.peek()
            if t.kind == "op" and t.text in ("=", "==", "<>", "!=", "<", "<=", ">", ">=", "<=>"):
                self.i += 1
                op = {"==": "=", "!=": "<>"}.get(t.text, t.text)
                e = A.BinOp(op, e, self._bitor())
                continue
            neg = False
            save = self.i
            if self.accept("NOT"):
                neg = True
            if self.accept("IN"):
                self.expect("(")
                if self.at("SELECT", "WITH"):
                    q = self.query()
                    self.expect(")")
                    e = A.SubqueryExpr("in", q, e, neg)
                else:
                    items = self.expr_list()
                    self.expect(")")
                    e = A.InList(e, tuple(items), neg)
                continue
            if self.accept("BETWEEN"):
                lo = self._bitor()
                self.expect("AND")
                hi = self._bitor()
                b = A.BinOp("and", A.BinOp(">=", e, lo), A.BinOp("<=", e, hi))
                e = A.UnOp("not", b) if neg else b
                continue
            if self.accept("LIKE"):
                e = A.Like(e, self._bitor(), "like", neg)
                continue
            if self.accept("RLIKE", "REGEXP"):
                e = A.Like(e, self._bitor(), "rlike", neg)
                continue
            if neg:
                self.i = save
                break
            if self.accept("IS"):
                n = bool(self.accept("NOT"))
                if self.accept("NULL"):
                    e = A.IsNull(e, n)
                elif self.accept("TRUE", "FALSE"):
                    v = self.toks[self.i - 1].up == "TRUE"
                    c = A.BinOp("<=>", e, A.Lit(v, "boolean"))
                    e = A.UnOp("not", c) if n else c
                else:
                    raise ParseError(f"bad IS predicate at position {self.peek().pos}")
                continue
            break
        return e

    def _bitor(self):
        e = self._additive()
        while self.peek().kind == "op" and self.peek().text in ("|", "&", "^", "||"):
            op = self.next().text
            r = self._additive()
            e = A.Call("concat", (e, r)) if op == "||" else A.BinOp(op, e, r)
        return e

    def _additive(self):
        e = self._mult()
        while self.peek().kind == "op" and self.peek().text in ("+", "-"):
            op = self.next().text
            e = A.BinOp(op, e, self._mult())
        return e

    def _mult(self):
        e = self._unary()
        while (self.peek().kind == "op" and self.peek().text in ("*", "/", "%")) or self.at("DIV"):
            op = self.next().text
            op = "div" if op.upper() == "DIV" else op
            e = A.BinOp(op, e, self._unary())
        return e

    def _unary(self):
        if self.peek().kind == "op" and self.peek().text in ("-", "+", "~"):
            op = self.next().text
            e = self._unary()
            if op == "+":
                return e
            if op == "-" and isinstance(e, A.Lit) and e.value is not None and e.dtype != "string":
                return A.Lit(-e.value, e.dtype)
            return A.UnOp(op, e)
        return self._postfix()

    def _postfix(self):
        e = self._primary()
        while self.peek().kind == "op" and self.peek().text == "[":
            self.i += 1
            idx = self.expr()
            self.expect("]")
            e = A.Call("element_at", (e, idx))
        return e

    def _primary(self) -> A.Expr:
        t = self.peek()
        if t.kind == "num":
            self.i += 1
            return _num_lit(t.text)
        if t.kind == "str":
            self.i += 1
            s = t.text
            while self.peek().kind == "str":  # adjacent literals concatenate
                s += self.next().text
            return A.Lit(s, "string")
        if t.kind == "op" and t.text == "(":
            self.i += 1
            if self.at("SELECT", "WITH"):
                q = self.query()
                self.expect(")")
                return A.SubqueryExpr("scalar", q)
            e = self.expr()
            self.expect(")")
            return e
        if t.kind == "op" and t.text == "*":
            self.i += 1
            return A.Star()
        if t.kind == "qid":
            return self._column_or_call()
        if t.kind != "id":
            raise ParseError(f"unexpected '{t.text or 'end of input'}' at position {t.pos}")
        u = t.up
        if u == "NULL":
            self.i += 1
            return A.Lit(None, "null")
        if u in ("TRUE", "FALSE"):
            self.i += 1
            return A.Lit(u == "TRUE", "boolean")
        if u == "CASE":
            return self._case()
        if u == "CAST" and self.peek(1).text == "(":
            self.i += 2
            e = self.expr()
            self.expect("AS")
            ty = self.type_name()
            self.expect(")")
            return A.Cast(e, ty)
        if u == "EXISTS" and self.peek(1).text == "(":
            self.i += 2
            q = self.query()
            self.expect(")")
            return A.SubqueryExpr("exists", q)
        if u in ("DATE", "TIMESTAMP") and self.peek(1).kind == "str":
            self.i += 1
            s = self.next().text
            return A.Cast(A.Lit(s, "string"), u.lower())
        if u == "INTERVAL":
            return self._interval()
        return self._column_or_call()

    def _interval(self):
        self.expect("INTERVAL")
        months = days = micros = 0
        got = False
        while True:
            t = self.peek()
            if t.kind == "num" or (t.kind == "str" and re.fullmatch(r"\s*-?\d+\s*", t.text)):
                self.i += 1
                v = int(float(t.text.rstrip("lL")))
                unit = self.ident().upper()
                if unit not in _INTERVAL_UNITS:
                    raise ParseError(f"bad interval unit {unit}")
                k, mult = _INTERVAL_UNITS[unit]
                if k == "m":
                    months += v * mult
                elif k == "d":
                    days += v * mult
                else:
                    micros += v * mult
                got = True
            else:
                break
        if not got:
            raise ParseError("bad interval literal")
        return A.IntervalLit(months, days, micros)

    def _case(self):
        self.expect("CASE")
        base = None
        if not self.at("WHEN"):
            base = self.expr()
        whens = []
        while self.accept("WHEN"):
            c = self.expr()
            self.expect("THEN")
            v = self.expr()
            if base is not None:
                c = A.BinOp("=", base, c)
            whens.append((c, v))
        else_ = None
        if self.accept("ELSE"):
            else_ = self.expr()
        self.expect("END")
        return A.Case(tuple(whens), else_)

    def _over(self, call: A.Call) -> A.WindowExpr:
        """``OVER ( [PARTITION BY e, ..] [ORDER BY o, ..] [ROWS|RANGE frame] )``"""
        self.i += 1
        self.expect("(")
        part: List[A.Expr] = []
        orders: List[A.SortOrder] = []
        frame = None
        if self.at_seq("PARTITION", "BY") or self.at_seq("DISTRIBUTE", "BY"):
            self.i += 2
            part = self.expr_list()
        if self.at_seq("ORDER", "BY") or self.at_seq("SORT", "BY"):
            self.i += 2
            orders = self.sort_items()
        t = self.peek()
        if t.kind == "id" and t.up in ("ROWS", "RANGE"):
            self.i += 1
            kind = t.up.lower()
            if self.accept("BETWEEN"):
                lo = self._frame_bound()
                self.expect("AND")
                hi = self._frame_bound()
            else:  # "ROWS 10 PRECEDING" = BETWEEN 10 PRECEDING AND CURRENT ROW
                lo, hi = self._frame_bound(), 0
            frame = (kind, lo, hi)
        self.expect(")")
        return A.WindowExpr(call, tuple(part), tuple(orders), frame)

    def _frame_bound(self) -> Optional[int]:
        """UNBOUNDED PRECEDING|FOLLOWING -> None, CURRENT ROW -> 0, n PRECEDING -> -n, n FOLLOWING -> n."""
        t = self.next()
        if t.up == "UNBOUNDED":
            self.next()
            return None
        if t.up == "CURRENT":
            self.next()  # ROW
            return 0
        try:
            n = int(t.text)
        except ValueError:
            raise ParseError(f"bad window frame bound {t.text!r}") from None
        side = self.next().up
        if side not in ("PRECEDING", "FOLLOWING"):
            raise ParseError(f"bad window frame bound {t.text} {side}")
        return -n if side == "PRECEDING" else n

    def _column_or_call(self):
        name = self.ident()
        if self.peek().kind == "op" and self.peek().text == "(":
            self.i += 1
            fname = name.lower()
            distinct = False
            args: List[A.Expr] = []
            if self.accept("DISTINCT"):
                distinct = True
            else:
                self.accept("ALL")
            if not self.at(")"):
                args = self.expr_list()
            self.expect(")")
            if fname == "count" and args and isinstance(args[0], A.Star):
                args = []
            call = A.Call(fname, tuple(args), distinct)
            if self.peek().kind == "id" and self.peek().up == "OVER" and self.peek(1).kind == "op" and \
                    self.peek(1).text == "(":
                return self._over(call)
            return call
        parts = [name]
        while self.peek().kind == "op" and self.peek().text == ".":
            if self.peek(1).kind == "op" and self.peek(1).text == "*":
                self.i += 2
                return A.Star(".".join(parts))
            self.i += 1
            parts.append(self.ident())
        return A.Col(tuple(parts))


def _num_lit(s: str) -> A.Lit:
    u = s.upper()
    if u.endswith("BD"):
        return A.Lit(float(s[:-2]), "double")
    if u[-1] == "L":
        return A.Lit(int(s[:-1]), "bigint")
    if u[-1] in "SY":
        return A.Lit(int(s[:-1]), "int")
    if u[-1] == "D":
        return A.Lit(float(s[:-1]), "double")
    if re.fullmatch(r"\d+", s):
        v = int(s)
        return A.Lit(v, "int" if -2 ** 31 <= v < 2 ** 31 else "bigint")
    return A.Lit(float(s), "double")


def _expand_sets(kind: str, exprs: List[A.Expr]) -> List[List[A.Expr]]:
    n = len(exprs)
    if kind == "ROLLUP":
        return [exprs[:k] for k in range(n, -1, -1)]
    sets = []
    for mask in range((1 << n) - 1, -1, -1):
        sets.append([exprs[i] for i in range(n) if mask >> (n - 1 - i) & 1])
    return sets


def parse(sql: str):
    return Parser(sql).statement()


def parse_expr(sql: str) -> A.Expr:
    p = Parser(sql)
    e = p.expr()
    if p.peek().kind != "eof":
        raise ParseError(f"unexpected '{p.peek().text}'")
    return e
