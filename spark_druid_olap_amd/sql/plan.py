"""Logical plan nodes.

The analyzer produces these; the optimizer and the Druid rewrite (``sql/druid_rewrite.py``) rewrite
them; the host executor (``sql/execute.py``) runs what is left.  Aggregates are kept in a normal
form that makes the reference's ``AggregateTransform`` pattern easy to match
(``asd/AggregateTransform.scala:170-329``):

    Project(select items over group/agg refs)
      Filter(HAVING over group/agg refs)
        Sort(ORDER BY over group/agg refs)
          Aggregate(groups: [Alias], aggs: [Alias(agg call)], child)
"""
from __future__ import annotations

from typing import Any, List, Optional, Sequence

from . import ast as A
from .functions import typeof


class Plan:
    children: Sequence["Plan"] = ()

    @property
    def output(self) -> List[A.Ref]:
        raise NotImplementedError

    def with_children(self, ch: Sequence["Plan"]) -> "Plan":
        return self

    def transform_up(self, fn) -> "Plan":
        ch = [c.transform_up(fn) for c in self.children]
        p = self.with_children(ch) if any(a is not b for a, b in zip(ch, self.children)) else self
        r = fn(p)
        return p if r is None else r

    def walk(self):
        yield self
        for c in self.children:
            yield from c.walk()

    def describe(self) -> str:
        return type(self).__name__

    def tree_string(self, indent: int = 0) -> str:
        s = "  " * indent + self.describe() + "\n"
        for c in self.children:
            s += c.tree_string(indent + 1)
        return s

    def __repr__(self):
        return self.tree_string()


def out_ref(e: A.Expr) -> A.Ref:
    if isinstance(e, A.Ref):
        return e
    if isinstance(e, A.Alias):
        return e.to_ref(typeof(e.child))
    raise TypeError(f"not a named expression: {e!r}")


class TableScan(Plan):
    """Scan of a catalog table (base table or Druid relation)."""

    def __init__(self, table, refs: List[A.Ref]):
        self.table = table
        self.refs = refs

    @property
    def output(self):
        return self.refs

    def describe(self):
        return f"Relation[{self.table.qualified_name}] ({', '.join(r.sql() for r in self.refs[:8])}" \
               f"{', ...' if len(self.refs) > 8 else ''})"


class LocalRelation(Plan):
    """In-memory rows (command results, VALUES, the one-row relation of ``SELECT 1``)."""

    def __init__(self, refs: List[A.Ref], data: Optional[dict] = None, nrows: int = 1):
        self.refs = refs
        self.data = data or {}
        self.nrows = nrows

    @property
    def output(self):
        return self.refs

    def describe(self):
        return f"LocalRelation ({', '.join(r.sql() for r in self.refs)}) rows={self.nrows}"


class Filter(Plan):
    def __init__(self, cond: A.Expr, child: Plan):
        self.cond = cond
        self.child = child
        self.children = (child,)

    @property
    def output(self):
        return self.child.output

    def with_children(self, ch):
        return Filter(self.cond, ch[0])

    def describe(self):
        return f"Filter {self.cond.sql()}"


class Project(Plan):
    def __init__(self, exprs: List[A.Expr], child: Plan):
        self.exprs = exprs  # Ref or Alias
        self.child = child
        self.children = (child,)

    @property
    def output(self):
        return [out_ref(e) for e in self.exprs]

    def with_children(self, ch):
        return Project(self.exprs, ch[0])

    def describe(self):
        return "Project [" + ", ".join(e.sql() for e in self.exprs) + "]"


class Aggregate(Plan):
    """groups / aggs are Aliases; output = group refs + agg refs (+ grouping-id ref for sets)."""

    def __init__(self, groups: List[A.Alias], aggs: List[A.Alias], child: Plan,
                 grouping_sets: Optional[List[List[int]]] = None, gid: Optional[A.Alias] = None):
        self.groups = groups
        self.aggs = aggs
        self.child = child
        self.children = (child,)
        self.grouping_sets = grouping_sets
        self.gid = gid

    @property
    def output(self):
        out = [out_ref(g) for g in self.groups] + [out_ref(a) for a in self.aggs]
        if self.gid is not None:
            out.append(self.gid.to_ref("int"))
        return out

    def with_children(self, ch):
        return Aggregate(self.groups, self.aggs, ch[0], self.grouping_sets, self.gid)

    def describe(self):
        gs = f" sets={self.grouping_sets}" if self.grouping_sets is not None else ""
        return ("Aggregate [" + ", ".join(g.sql() for g in self.groups) + "] [" +
                ", ".join(a.sql() for a in self.aggs) + "]" + gs)


class Window(Plan):
    """Window expressions (``A.WindowExpr`` under Aliases) evaluated over the child's rows on the
    host (``sql/window.py``); output = the child's columns + one column per expression."""

    def __init__(self, exprs: List[A.Alias], child: Plan):
        self.exprs = exprs
        self.child = child
        self.children = (child,)

    @property
    def output(self):
        return list(self.child.output) + [out_ref(e) for e in self.exprs]

    def with_children(self, ch):
        return Window(self.exprs, ch[0])

    def describe(self):
        return "Window [" + ", ".join(e.sql() for e in self.exprs) + "]"


class Sort(Plan):
    def __init__(self, orders: List[A.SortOrder], child: Plan):
        self.orders = orders
        self.child = child
        self.children = (child,)

    @property
    def output(self):
        return self.child.output

    def with_children(self, ch):
        return Sort(self.orders, ch[0])

    def describe(self):
        return "Sort [" + ", ".join(o.sql() for o in self.orders) + "]"


class Limit(Plan):
    def __init__(self, n: int, child: Plan):
        self.n = n
        self.child = child
        self.children = (child,)

    @property
    def output(self):
        return self.child.output

    def with_children(self, ch):
        return Limit(self.n, ch[0])

    def describe(self):
        return f"Limit {self.n}"


class Join(Plan):
    def __init__(self, kind: str, left: Plan, right: Plan, cond: Optional[A.Expr]):
        self.kind = kind
        self.left = left
        self.right = right
        self.cond = cond
        self.children = (left, right)

    @property
    def output(self):
        if self.kind in ("leftsemi", "leftanti"):
            return self.left.output
        return self.left.output + self.right.output

    def with_children(self, ch):
        return Join(self.kind, ch[0], ch[1], self.cond)

    def describe(self):
        return f"Join {self.kind}" + (f" {self.cond.sql()}" if self.cond is not None else "")


class Union(Plan):
    def __init__(self, children: List[Plan], refs: List[A.Ref], distinct: bool = False):
        self.children = tuple(children)
        self.refs = refs
        self.distinct = distinct

    @property
    def output(self):
        return self.refs

    def with_children(self, ch):
        return Union(list(ch), self.refs, self.distinct)

    def describe(self):
        return "Union" + (" distinct" if self.distinct else " all")


class SetOperation(Plan):
    """INTERSECT / EXCEPT (distinct semantics)."""

    def __init__(self, kind: str, left: Plan, right: Plan, all_: bool = False):
        self.kind = kind
        self.left = left
        self.right = right
        self.all = all_
        self.children = (left, right)

    @property
    def output(self):
        return self.left.output

    def with_children(self, ch):
        return SetOperation(self.kind, ch[0], ch[1], self.all)

    def describe(self):
        return self.kind.capitalize()


class DruidQuery(Plan):
    """A QuerySpec pushed to the GPU engine (the reference's DruidRelation-with-DruidQuery scan,
    ``sd/DruidRelation.scala:30-126``).  ``columns`` maps each output ref to the Druid result
    column that carries it and the SQL type to convert to."""

    def __init__(self, relation, spec, columns: List[tuple], refs: List[A.Ref],
                 builder_info: Optional[dict] = None):
        self.relation = relation        # catalog DruidTable
        self.spec = spec                # QuerySpec
        self.columns = columns          # [(druid output name, sql dtype, kind)] aligned with refs
        self.refs = refs
        self.info = builder_info or {}

    @property
    def output(self):
        return self.refs

    def describe(self):
        import json

        h = self.info.get("historical")
        mode = f" queryHistorical=true numSegmentsPerQuery={h}" if h else ""
        return (f"DruidQuery[{self.relation.qualified_name}]{mode} {type(self.spec).__name__} -> "
                f"({', '.join(r.sql() for r in self.refs)})\n      "
                + json.dumps(self.spec.to_json(), sort_keys=False)[:2000])


def find_all(plan: Plan, cls) -> List[Any]:
    return [p for p in plan.walk() if isinstance(p, cls)]


def node_exprs(p: Plan) -> List[A.Expr]:
    """Every expression a plan node holds (conditions, projections, groupings, sort keys)."""
    out: List[A.Expr] = []

    def add(v):
        if isinstance(v, A.Expr):
            out.append(v)
        elif isinstance(v, A.SortOrder):
            out.append(v.expr)
        elif isinstance(v, (list, tuple)):
            for x in v:
                add(x)

    for k, v in vars(p).items():
        if k != "children":
            add(v)
    return out


def subquery_exprs(plan: Plan) -> List[A.SubqueryExpr]:
    """Subquery expressions of a plan (not descending into the subqueries themselves)."""
    seen, out = set(), []
    for p in plan.walk():
        for e in node_exprs(p):
            for x in e.walk():
                if isinstance(x, A.SubqueryExpr) and id(x) not in seen:
                    seen.add(id(x))
                    out.append(x)
    return out


def find_all_deep(plan: Plan, cls) -> List[Any]:
    """find_all, also inside the plans of subquery expressions."""
    from ..query.spec import find_deferred

    out = find_all(plan, cls)
    sqs = list(subquery_exprs(plan))
    for dq in find_all(plan, DruidQuery):  # subqueries parameterising pushed filters / having
        for d in find_deferred(dq.spec):
            sqs.extend(d.subqueries)
    seen = set()
    for sq in sqs:
        if isinstance(sq.query, Plan) and id(sq.query) not in seen:
            seen.add(id(sq.query))
            out.extend(find_all_deep(sq.query, cls))
    return out
