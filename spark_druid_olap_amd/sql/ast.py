"""SQL expression and statement trees.

One expression class hierarchy serves both the parser (unresolved ``Col`` names) and the analyzer
(resolved ``Ref`` attributes with a unique id and a SQL type), the way Catalyst expressions do for
the reference (which inherits Spark's; the rewrite rules that consume them are
``asd/ProjectFilterTransfom.scala`` / ``asd/AggregateTransform.scala``).  Expressions are immutable;
``key()`` gives a structural hash used to match GROUP BY expressions inside SELECT items.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from typing import Any, List, Optional, Sequence, Tuple

_ids = itertools.count(1)


def new_id() -> int:
    return next(_ids)


class Expr:
    __slots__ = ()

    @property
    def children(self) -> Tuple["Expr", ...]:
        return ()

    def with_children(self, ch: Sequence["Expr"]) -> "Expr":
        return self

    def key(self):
        return (type(self).__name__,) + tuple(c.key() for c in self.children)

    def transform(self, fn) -> "Expr":
        """Bottom-up rewrite."""
        ch = self.children
        e = self
        if ch:
            nch = [c.transform(fn) for c in ch]
            if any(a is not b for a, b in zip(nch, ch)):
                e = self.with_children(nch)
        r = fn(e)
        return e if r is None else r

    def walk(self):
        yield self
        for c in self.children:
            yield from c.walk()

    def refs(self) -> List["Ref"]:
        return [e for e in self.walk() if isinstance(e, Ref)]

    def __repr__(self) -> str:
        return self.sql()

    def sql(self) -> str:
        return type(self).__name__


@dataclass(frozen=True, repr=False)
class Lit(Expr):
    value: Any
    dtype: str  # int bigint double string boolean date timestamp null decimal

    def key(self):
        return ("Lit", repr(self.value), self.dtype)

    def sql(self):
        if self.value is None:
            return "NULL"
        if self.dtype == "string":
            return "'" + str(self.value).replace("'", "\\'") + "'"
        return str(self.value)


@dataclass(frozen=True, repr=False)
class Col(Expr):
    parts: Tuple[str, ...]

    def key(self):
        return ("Col",) + tuple(p.lower() for p in self.parts)

    def sql(self):
        return ".".join(self.parts)

    @property
    def name(self):
        return self.parts[-1]


@dataclass(frozen=True, repr=False, eq=False)
class Ref(Expr):
    rid: int
    name: str
    dtype: str
    qualifier: Optional[str] = None

    def key(self):
        return ("Ref", self.rid)

    def sql(self):
        return f"{self.name}#{self.rid}"

    def __eq__(self, o):
        return isinstance(o, Ref) and o.rid == self.rid

    def __hash__(self):
        return hash(self.rid)


@dataclass(frozen=True, repr=False)
class Star(Expr):
    qualifier: Optional[str] = None

    def sql(self):
        return (self.qualifier + ".*") if self.qualifier else "*"


@dataclass(frozen=True, repr=False, eq=False)
class Alias(Expr):
    child: Expr
    name: str
    rid: int = field(default_factory=new_id)

    @property
    def children(self):
        return (self.child,)

    def with_children(self, ch):
        return Alias(ch[0], self.name, self.rid)

    def key(self):
        return self.child.key()

    def to_ref(self, dtype: str) -> Ref:
        return Ref(self.rid, self.name, dtype)

    def sql(self):
        return f"{self.child.sql()} AS {self.name}"


AGG_FUNCS = {"count", "sum", "min", "max", "avg", "mean", "approx_count_distinct", "first", "last",
             "stddev", "stddev_samp", "stddev_pop", "variance", "var_samp", "var_pop", "collect_set",
             "collect_list", "grouping", "grouping_id"}


@dataclass(frozen=True, repr=False)
class Call(Expr):
    name: str
    args: Tuple[Expr, ...]
    distinct: bool = False

    @property
    def children(self):
        return self.args

    def with_children(self, ch):
        return Call(self.name, tuple(ch), self.distinct)

    def key(self):
        return ("Call", self.name, self.distinct) + tuple(a.key() for a in self.args)

    @property
    def is_agg(self) -> bool:
        return self.name in AGG_FUNCS

    def sql(self):
        d = "DISTINCT " if self.distinct else ""
        return f"{self.name}({d}{', '.join(a.sql() for a in self.args)})"


@dataclass(frozen=True, repr=False)
class BinOp(Expr):
    op: str  # + - * / % = <> < <= > >= <=> and or ||
    l: Expr
    r: Expr

    @property
    def children(self):
        return (self.l, self.r)

    def with_children(self, ch):
        return BinOp(self.op, ch[0], ch[1])

    def key(self):
        return ("BinOp", self.op, self.l.key(), self.r.key())

    def sql(self):
        return f"({self.l.sql()} {self.op.upper()} {self.r.sql()})"


@dataclass(frozen=True, repr=False)
class UnOp(Expr):
    op: str  # - not ~
    child: Expr

    @property
    def children(self):
        return (self.child,)

    def with_children(self, ch):
        return UnOp(self.op, ch[0])

    def key(self):
        return ("UnOp", self.op, self.child.key())

    def sql(self):
        return f"({self.op.upper()} {self.child.sql()})"


@dataclass(frozen=True, repr=False)
class Case(Expr):
    whens: Tuple[Tuple[Expr, Expr], ...]
    else_: Optional[Expr]

    @property
    def children(self):
        out = []
        for c, v in self.whens:
            out += [c, v]
        if self.else_ is not None:
            out.append(self.else_)
        return tuple(out)

    def with_children(self, ch):
        n = len(self.whens)
        whens = tuple((ch[2 * i], ch[2 * i + 1]) for i in range(n))
        return Case(whens, ch[2 * n] if self.else_ is not None else None)

    def sql(self):
        s = " ".join(f"WHEN {c.sql()} THEN {v.sql()}" for c, v in self.whens)
        e = f" ELSE {self.else_.sql()}" if self.else_ is not None else ""
        return f"CASE {s}{e} END"


@dataclass(frozen=True, repr=False)
class Cast(Expr):
    child: Expr
    to: str

    @property
    def children(self):
        return (self.child,)

    def with_children(self, ch):
        return Cast(ch[0], self.to)

    def key(self):
        return ("Cast", self.to, self.child.key())

    def sql(self):
        return f"CAST({self.child.sql()} AS {self.to.upper()})"


@dataclass(frozen=True, repr=False)
class InList(Expr):
    child: Expr
    items: Tuple[Expr, ...]
    negated: bool = False

    @property
    def children(self):
        return (self.child,) + self.items

    def with_children(self, ch):
        return InList(ch[0], tuple(ch[1:]), self.negated)

    def key(self):
        return ("In", self.negated) + tuple(c.key() for c in self.children)

    def sql(self):
        n = "NOT " if self.negated else ""
        return f"({self.child.sql()} {n}IN ({', '.join(i.sql() for i in self.items)}))"


@dataclass(frozen=True, repr=False)
class Like(Expr):
    child: Expr
    pattern: Expr
    kind: str = "like"  # like | rlike
    negated: bool = False

    @property
    def children(self):
        return (self.child, self.pattern)

    def with_children(self, ch):
        return Like(ch[0], ch[1], self.kind, self.negated)

    def key(self):
        return ("Like", self.kind, self.negated, self.child.key(), self.pattern.key())

    def sql(self):
        n = "NOT " if self.negated else ""
        return f"({self.child.sql()} {n}{self.kind.upper()} {self.pattern.sql()})"


@dataclass(frozen=True, repr=False)
class IsNull(Expr):
    child: Expr
    negated: bool = False

    @property
    def children(self):
        return (self.child,)

    def with_children(self, ch):
        return IsNull(ch[0], self.negated)

    def key(self):
        return ("IsNull", self.negated, self.child.key())

    def sql(self):
        return f"({self.child.sql()} IS {'NOT ' if self.negated else ''}NULL)"


@dataclass(frozen=True, repr=False)
class IntervalLit(Expr):
    """``interval 90 days`` -> (months, days, microseconds)."""
    months: int = 0
    days: int = 0
    micros: int = 0

    def key(self):
        return ("Interval", self.months, self.days, self.micros)

    def sql(self):
        return f"INTERVAL {self.months} MONTHS {self.days} DAYS {self.micros} MICROSECONDS"


@dataclass(frozen=True, repr=False, eq=False)
class SubqueryExpr(Expr):
    """Scalar subquery / IN (subquery) / EXISTS.  ``query`` is a statement AST before analysis and
    a logical plan after."""
    kind: str  # scalar | in | exists
    query: Any
    child: Optional[Expr] = None
    negated: bool = False

    @property
    def children(self):
        return (self.child,) if self.child is not None else ()

    def with_children(self, ch):
        return SubqueryExpr(self.kind, self.query, ch[0] if ch else None, self.negated)

    def key(self):
        return ("Subquery", id(self.query))

    def sql(self):
        return f"{self.kind}(subquery)"


@dataclass(frozen=True, repr=False)
class SortOrder:
    expr: Expr
    ascending: bool = True
    nulls_first: Optional[bool] = None

    def sql(self):
        return f"{self.expr.sql()} {'ASC' if self.ascending else 'DESC'}"


# functions that only exist over a window (Spark's ranking / offset functions); the aggregates of
# AGG_FUNCS may also be used over a window
WINDOW_FUNCS = {"rank", "dense_rank", "row_number", "percent_rank", "cume_dist", "ntile", "lag", "lead",
                "first_value", "last_value"}


@dataclass(frozen=True, repr=False)
class WindowExpr(Expr):
    """``func(args) OVER (PARTITION BY .. ORDER BY .. [ROWS|RANGE frame])``.  ``frame`` is
    (kind, lo, hi) with row offsets relative to the current row (negative = preceding, None =
    unbounded); None = Spark's default frame (RANGE UNBOUNDED PRECEDING .. CURRENT ROW with an
    ORDER BY, the whole partition without one).  Evaluated on the host over the (aggregated) rows
    below it (``sql/window.py``), like Spark's WindowExec above the reference's pushed Druid
    aggregate (the BI workload's windowed templates, docs/bi-benchmark/snap-sales-demo.jmx)."""
    func: Call
    partition: Tuple[Expr, ...] = ()
    orders: Tuple[SortOrder, ...] = ()
    frame: Optional[Tuple[str, Optional[int], Optional[int]]] = None

    @property
    def children(self):
        return (self.func,) + tuple(self.partition) + tuple(o.expr for o in self.orders)

    def with_children(self, ch):
        np_ = len(self.partition)
        f = ch[0]
        orders = tuple(SortOrder(c, o.ascending, o.nulls_first) for c, o in zip(ch[1 + np_:], self.orders))
        return WindowExpr(f, tuple(ch[1:1 + np_]), orders, self.frame)

    def key(self):
        return ("Window", self.func.key(), tuple(p.key() for p in self.partition),
                tuple((o.expr.key(), o.ascending, o.nulls_first) for o in self.orders), self.frame)

    def sql(self):
        parts = []
        if self.partition:
            parts.append("PARTITION BY " + ", ".join(p.sql() for p in self.partition))
        if self.orders:
            parts.append("ORDER BY " + ", ".join(o.sql() for o in self.orders))
        if self.frame is not None:
            k, lo, hi = self.frame
            b = lambda v, side: ("UNBOUNDED " + side) if v is None else (  # noqa: E731
                "CURRENT ROW" if v == 0 else f"{abs(v)} {'PRECEDING' if v < 0 else 'FOLLOWING'}")
            parts.append(f"{k.upper()} BETWEEN {b(lo, 'PRECEDING')} AND {b(hi, 'FOLLOWING')}")
        return f"{self.func.sql()} OVER ({' '.join(parts)})"


def conjuncts(e: Optional[Expr]) -> List[Expr]:
    if e is None:
        return []
    if isinstance(e, BinOp) and e.op == "and":
        return conjuncts(e.l) + conjuncts(e.r)
    return [e]


def disjuncts(e: Expr) -> List[Expr]:
    if isinstance(e, BinOp) and e.op == "or":
        return disjuncts(e.l) + disjuncts(e.r)
    return [e]


def and_all(es: Sequence[Expr]) -> Optional[Expr]:
    es = list(es)
    if not es:
        return None
    out = es[0]
    for e in es[1:]:
        out = BinOp("and", out, e)
    return out


def or_all(es: Sequence[Expr]) -> Expr:
    es = list(es)
    out = es[0]
    for e in es[1:]:
        out = BinOp("or", out, e)
    return out


# ------------------------------------------------------------------------------------------------
# statements
@dataclass
class TableRef:
    name: Tuple[str, ...]
    alias: Optional[str] = None


@dataclass
class SubqueryRef:
    query: Any
    alias: Optional[str] = None


@dataclass
class JoinRef:
    kind: str  # inner left right full cross leftsemi leftanti
    left: Any
    right: Any
    cond: Optional[Expr] = None
    using: Optional[List[str]] = None


@dataclass
class SelectItem:
    expr: Expr
    alias: Optional[str] = None


@dataclass
class Select:
    items: List[SelectItem]
    from_: Any = None
    where: Optional[Expr] = None
    group_by: List[Expr] = field(default_factory=list)
    grouping_sets: Optional[List[List[Expr]]] = None  # explicit sets (cube/rollup expanded)
    having: Optional[Expr] = None
    order_by: List[SortOrder] = field(default_factory=list)
    limit: Optional[int] = None
    distinct: bool = False


@dataclass
class SetOp:
    kind: str  # union | intersect | except
    all: bool
    left: Any
    right: Any
    order_by: List[SortOrder] = field(default_factory=list)
    limit: Optional[int] = None


@dataclass
class With:
    ctes: List[Tuple[str, Any]]
    query: Any


@dataclass
class ColumnDef:
    name: str
    dtype: str


@dataclass
class CreateTable:
    name: Tuple[str, ...]
    columns: List[ColumnDef]
    provider: Optional[str]
    options: dict
    if_not_exists: bool = False
    temporary: bool = False
    as_query: Any = None


@dataclass
class CreateView:
    name: Tuple[str, ...]
    query: Any
    replace: bool = False
    temporary: bool = False
    text: str = ""


@dataclass
class DropTable:
    name: Tuple[str, ...]
    if_exists: bool = False
    view: bool = False


@dataclass
class CreateDatabase:
    name: str
    if_not_exists: bool = False


@dataclass
class UseDatabase:
    name: str


@dataclass
class SetConf:
    key: Optional[str]
    value: Optional[str]


@dataclass
class ShowTables:
    db: Optional[str] = None


@dataclass
class Describe:
    name: Tuple[str, ...]


@dataclass
class CacheTable:
    name: Tuple[str, ...]
    uncache: bool = False


@dataclass
class ClearDruidCache:
    host: Optional[str] = None


@dataclass
class ExecuteDruidQuery:
    table: Tuple[str, ...]
    historical: bool
    json_text: str


@dataclass
class ExplainDruidRewrite:
    query: Any


@dataclass
class Explain:
    query: Any
    extended: bool = False
