"""Analyzer: statement AST -> resolved logical plan.

Resolves names against the catalog and FROM-clause scopes, expands ``*``, types expressions,
extracts aggregates into the ``Aggregate`` normal form (see ``sql/plan.py``), supports GROUP BY
ordinals/aliases, HAVING / ORDER BY over aggregates not in the select list, grouping sets / CUBE /
ROLLUP with ``grouping_id()``, set operations, CTEs, views and uncorrelated subqueries.  This is the
part of Spark's Catalyst analyzer the reference relies on (its planner matches on analyzed plans:
``asd/DruidPlanner.scala:29-50``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from . import ast as A
from . import plan as P
from .functions import constant_fold, has_function, typeof
from .types import AnalysisError, wider


class Scope:
    def __init__(self, refs: List[A.Ref], outer: Optional["Scope"] = None):
        self.refs = refs
        self.outer = outer
        self._by_name: Optional[Dict[str, List[A.Ref]]] = None

    def resolve(self, parts: Tuple[str, ...]) -> Optional[A.Ref]:
        name = parts[-1].lower()
        qual = [p.lower() for p in parts[:-1]]
        if self._by_name is None:  # (a wide view resolves thousands of names per statement)
            idx: Dict[str, List[A.Ref]] = {}
            for r in self.refs:
                idx.setdefault(r.name.lower(), []).append(r)
            self._by_name = idx
        hits = []
        for r in self._by_name.get(name, ()):
            if qual:
                q = (r.qualifier or "").lower()
                # qualifier may be "alias", "table" or "db.table"
                if not (q == ".".join(qual) or q.split(".")[-1] == qual[-1] and (len(qual) == 1 or q == ".".join(qual))):
                    continue
            hits.append(r)
        uniq = {h.rid: h for h in hits}
        if len(uniq) > 1:
            raise AnalysisError(f"Reference '{'.'.join(parts)}' is ambiguous, could be: "
                                f"{', '.join(sorted(f'{h.qualifier}.{h.name}' for h in uniq.values()))}")
        if uniq:
            return next(iter(uniq.values()))
        if len(parts) > 1 and not qual:
            return None
        return None


def requalify(refs: List[A.Ref], q: Optional[str]) -> List[A.Ref]:
    return [A.Ref(r.rid, r.name, r.dtype, q) for r in refs]


def auto_name(e: A.Expr) -> str:
    if isinstance(e, A.Col):
        return e.parts[-1]
    if isinstance(e, A.Ref):
        return e.name
    if isinstance(e, A.Call):
        if e.name == "count" and not e.args:
            return "count(1)"
        d = "DISTINCT " if e.distinct else ""
        return f"{e.name}({d}{', '.join(auto_name(a) for a in e.args)})"
    if isinstance(e, A.Lit):
        return "NULL" if e.value is None else str(e.value)
    if isinstance(e, A.Cast):
        return f"CAST({auto_name(e.child)} AS {e.to.upper()})"
    if isinstance(e, A.BinOp):
        return f"({auto_name(e.l)} {e.op.upper() if e.op.isalpha() else e.op} {auto_name(e.r)})"
    if isinstance(e, A.UnOp):
        return f"(- {auto_name(e.child)})" if e.op == "-" else f"(NOT {auto_name(e.child)})"
    return e.sql()


class Analyzer:
    def __init__(self, catalog, session=None):
        self.catalog = catalog
        self.session = session
        self.ctes: List[Dict[str, object]] = []
        self._view_depth = 0

    # -------------------------------------------------------------------------------- queries
    def analyze(self, q, outer: Optional[Scope] = None) -> P.Plan:
        if isinstance(q, A.With):
            self.ctes.append({n.lower(): cq for n, cq in q.ctes})
            try:
                return self.analyze(q.query, outer)
            finally:
                self.ctes.pop()
        if isinstance(q, A.SetOp):
            return self._setop(q, outer)
        if isinstance(q, A.Select):
            return self._select(q, outer)
        raise AnalysisError(f"not a query: {type(q).__name__}")

    def _setop(self, q: A.SetOp, outer) -> P.Plan:
        l = self.analyze(q.left, outer)
        r = self.analyze(q.right, outer)
        lo, ro = l.output, r.output
        if len(lo) != len(ro):
            raise AnalysisError(f"{q.kind.upper()} can only be performed on tables with the same number of columns")
        types = [wider(a.dtype, b.dtype) for a, b in zip(lo, ro)]

        def conform(p, outs):
            if all(o.dtype == t for o, t in zip(outs, types)):
                return p
            return P.Project([o if o.dtype == t else A.Alias(A.Cast(o, t), o.name) for o, t in zip(outs, types)], p)

        l, r = conform(l, lo), conform(r, ro)
        if q.kind == "union":
            refs = [A.Ref(A.new_id(), o.name, t) for o, t in zip(lo, types)]
            # flatten nested unions of the same kind
            kids = []
            for c in (l, r):
                if isinstance(c, P.Union) and c.distinct == (not q.all):
                    kids += list(c.children)
                else:
                    kids.append(c)
            plan: P.Plan = P.Union(kids, refs, distinct=not q.all)
        else:
            plan = P.SetOperation(q.kind, l, r, q.all)
        if q.order_by:
            scope = Scope(plan.output)
            orders = []
            for o in q.order_by:
                e = o.expr
                if isinstance(e, A.Lit) and isinstance(e.value, int):
                    e = plan.output[e.value - 1]
                else:
                    e = self.resolve(e, scope)
                orders.append(A.SortOrder(e, o.ascending, o.nulls_first))
            plan = P.Sort(orders, plan)
        if q.limit is not None:
            plan = P.Limit(q.limit, plan)
        return plan

    # -------------------------------------------------------------------------------- FROM
    def relation(self, rel, outer) -> Tuple[P.Plan, List[A.Ref]]:
        if rel is None:
            return P.LocalRelation([], {}, 1), []
        if isinstance(rel, A.TableRef):
            return self._table(rel)
        if isinstance(rel, A.SubqueryRef):
            p = self.analyze(rel.query, outer)
            return p, requalify(p.output, rel.alias)
        if isinstance(rel, A.JoinRef):
            lp, lr = self.relation(rel.left, outer)
            rp, rr = self.relation(rel.right, outer)
            scope = Scope(lr + rr, outer)
            cond = None
            kind = rel.kind
            if rel.using:
                conds = []
                for c in rel.using:
                    a = Scope(lr).resolve((c,))
                    b = Scope(rr).resolve((c,))
                    if a is None or b is None:
                        raise AnalysisError(f"USING column {c} not found on both sides")
                    conds.append(A.BinOp("=", a, b))
                cond = A.and_all(conds)
            elif rel.cond is not None:
                cond = self.resolve(rel.cond, scope)
            if kind == "cross" and cond is not None:
                kind = "inner"
            p = P.Join(kind, lp, rp, cond)
            refs = lr if kind in ("leftsemi", "leftanti") else lr + rr
            return p, refs
        raise AnalysisError(f"bad relation {rel!r}")

    def _table(self, rel: A.TableRef):
        name = rel.name
        if len(name) == 1:
            for frame in reversed(self.ctes):
                if name[0].lower() in frame:
                    p = self.analyze(frame[name[0].lower()])
                    return p, requalify(p.output, rel.alias or name[0])
        t = self.session.lookup_table(name) if self.session is not None else self.catalog.get(name)
        q = rel.alias or t.name
        if t.kind == "view":
            if self._view_depth > 32:
                raise AnalysisError("view nesting too deep")
            self._view_depth += 1
            try:
                saved = self.ctes
                self.ctes = []
                p = self.analyze(t.query)
                self.ctes = saved
            finally:
                self._view_depth -= 1
            return p, requalify(p.output, q)
        refs = [A.Ref(A.new_id(), c, ty, q) for c, ty in t.schema]
        return P.TableScan(t, refs), refs

    # -------------------------------------------------------------------------------- SELECT
    def _select(self, s: A.Select, outer) -> P.Plan:
        plan, refs = self.relation(s.from_, outer)
        scope = Scope(refs, outer)
        if s.where is not None:
            cond = self.resolve(s.where, scope)
            if _has_agg(cond):
                raise AnalysisError("aggregate functions are not allowed in WHERE")
            if _has_window(cond):
                raise AnalysisError("window functions are not allowed in WHERE")
            plan = P.Filter(cond, plan)
        # expand stars
        items: List[Tuple[A.Expr, Optional[str]]] = []
        for it in s.items:
            if isinstance(it.expr, A.Star):
                q = it.expr.qualifier
                for r in refs:
                    if q is None or (r.qualifier or "").lower().split(".")[-1] == q.lower().split(".")[-1]:
                        items.append((r, r.name))
                if q is not None and not any((r.qualifier or "").lower().split(".")[-1] == q.lower().split(".")[-1]
                                             for r in refs):
                    raise AnalysisError(f"cannot resolve '{q}.*'")
            else:
                items.append((it.expr, it.alias or auto_name(it.expr)))
        resolved_items = [(self.resolve(e, scope) if not isinstance(e, A.Ref) else e, n) for e, n in items]
        is_agg = bool(s.group_by) or s.grouping_sets is not None or any(_has_agg(e) for e, _ in resolved_items) \
            or (s.having is not None)
        if not is_agg:
            return self._select_plain(s, plan, scope, resolved_items)
        return self._select_agg(s, plan, scope, items, resolved_items)

    def _select_plain(self, s, plan, scope, items):
        proj = []
        for e, n in items:
            if isinstance(e, A.Ref) and e.name == n:
                proj.append(e)
            else:
                proj.append(A.Alias(e, n))
        alias_map = {n.lower(): e for e, n in items}
        if s.distinct:
            plan, proj, _ = _with_windows(plan, proj, [])
            plan = P.Project(proj, plan)
            outs = plan.output
            groups = [A.Alias(o, o.name) for o in outs]
            plan = P.Aggregate(groups, [], plan)
            plan = P.Project([A.Alias(g.to_ref(g.child.dtype), g.name) for g in groups], plan)
            if s.order_by:
                oscope = Scope(requalify(plan.output, None))
                orders = []
                for o in s.order_by:
                    e = o.expr
                    if isinstance(e, A.Lit) and isinstance(e.value, int) and e.dtype in ("int", "bigint"):
                        e = plan.output[e.value - 1]
                    else:
                        e = self.resolve(e, oscope)
                    orders.append(A.SortOrder(e, o.ascending, o.nulls_first))
                plan = P.Sort(orders, plan)
        else:
            orders = []
            for o in s.order_by:
                orders.append(A.SortOrder(self._order_expr(o.expr, items, alias_map, scope), o.ascending,
                                          o.nulls_first))
            plan, proj, orders = _with_windows(plan, proj, orders)
            if orders:
                plan = P.Sort(orders, plan)
            plan = P.Project(proj, plan)
        if s.limit is not None:
            plan = P.Limit(s.limit, plan)
        return plan

    def _order_expr(self, e, items, alias_map, scope):
        if isinstance(e, A.Lit) and isinstance(e.value, int) and e.dtype in ("int", "bigint"):
            if not 1 <= e.value <= len(items):
                raise AnalysisError(f"ORDER BY position {e.value} is not in select list")
            return items[e.value - 1][0]
        if isinstance(e, A.Col) and len(e.parts) == 1 and e.parts[0].lower() in alias_map:
            r = scope.resolve(e.parts)
            ae = alias_map[e.parts[0].lower()]
            if r is None or (isinstance(ae, A.Ref) and ae.rid == r.rid) or not isinstance(ae, A.Ref):
                return ae
        return self.resolve(e, scope)

    def _select_agg(self, s, plan, scope, raw_items, items):
        alias_map = {n.lower(): e for e, n in items}
        # group expressions (ordinals and select aliases allowed)
        gexprs: List[A.Expr] = []
        for g in s.group_by:
            if isinstance(g, A.Lit) and isinstance(g.value, int) and g.dtype in ("int", "bigint"):
                if not 1 <= g.value <= len(items):
                    raise AnalysisError(f"GROUP BY position {g.value} is not in select list")
                ge = items[g.value - 1][0]
            else:
                ge = self._resolve_or_alias(g, scope, alias_map)
            if _has_agg(ge):
                raise AnalysisError(f"aggregate functions are not allowed in GROUP BY: {ge.sql()}")
            gexprs.append(ge)
        sets = None
        if s.grouping_sets is not None:
            keys = [g.key() for g in gexprs]
            sets = []
            for st in s.grouping_sets:
                idx = []
                for e in st:
                    re_ = self._resolve_or_alias(e, scope, alias_map)
                    k = re_.key()
                    if k not in keys:
                        keys.append(k)
                        gexprs.append(re_)
                    idx.append(keys.index(k))
                sets.append(sorted(set(idx)))
        groups = [A.Alias(g, g.name if isinstance(g, A.Ref) else auto_name(g)) for g in gexprs]
        gkeys = {g.child.key(): g for g in groups}
        aggs: List[A.Alias] = []
        akeys: Dict[tuple, A.Alias] = {}
        gid = A.Alias(A.Lit(0, "int"), "grouping__id") if sets is not None else None

        def rw(e: A.Expr) -> A.Expr:
            if isinstance(e, A.WindowExpr):
                # the window runs over the aggregated rows: its arguments, partition and order
                # expressions are rewritten to group / aggregate references, the function stays
                f = e.func
                return A.WindowExpr(A.Call(f.name, tuple(rw(a) for a in f.args), f.distinct),
                                    tuple(rw(p) for p in e.partition),
                                    tuple(A.SortOrder(rw(o.expr), o.ascending, o.nulls_first) for o in e.orders),
                                    e.frame)
            k = e.key()
            if k in gkeys and not isinstance(e, A.Lit):
                g = gkeys[k]
                return g.to_ref(typeof(g.child))
            if isinstance(e, A.Call) and e.name in ("grouping_id", "grouping__id") and not e.args:
                if gid is None:
                    raise AnalysisError("grouping_id() requires GROUPING SETS / CUBE / ROLLUP")
                return gid.to_ref("int")
            if isinstance(e, A.Call) and e.name == "grouping":
                if gid is None:
                    raise AnalysisError("grouping() requires GROUPING SETS / CUBE / ROLLUP")
                ak = e.args[0].key()
                if ak not in gkeys:
                    raise AnalysisError(f"grouping() argument must be a grouping column: {e.args[0].sql()}")
                pos = list(gkeys).index(ak)
                n = len(groups)
                return A.Cast(A.BinOp("%", A.BinOp("div", gid.to_ref("int"), A.Lit(1 << (n - 1 - pos), "int")),
                                      A.Lit(2, "int")), "tinyint")
            if isinstance(e, A.Call) and e.is_agg:
                if any(_has_agg(a) for a in e.args):
                    raise AnalysisError("nested aggregate functions are not allowed")
                if k not in akeys:
                    a = A.Alias(e, auto_name(e))
                    akeys[k] = a
                    aggs.append(a)
                a = akeys[k]
                return a.to_ref(typeof(e))
            if isinstance(e, A.Ref):
                raise AnalysisError(f"expression '{e.name}' is neither present in the group by, nor is it an "
                                    f"aggregate function. Add to group by or wrap in first() if you don't care "
                                    f"which value you get.")
            if isinstance(e, (A.Lit, A.IntervalLit, A.SubqueryExpr)) or not e.children:
                return e
            return e.with_children([rw(c) for c in e.children])

        proj = []
        for e, n in items:
            x = rw(e)
            proj.append(x if isinstance(x, A.Ref) and x.name == n else A.Alias(x, n))
        having = None
        if s.having is not None:
            he = self._resolve_with_aliases(s.having, scope, alias_map)
            having = rw(he)
        orders = []
        for o in s.order_by:
            oe = o.expr
            if isinstance(oe, A.Lit) and isinstance(oe.value, int) and oe.dtype in ("int", "bigint"):
                ex = items[oe.value - 1][0]
            elif isinstance(oe, A.Col) and len(oe.parts) == 1 and oe.parts[0].lower() in alias_map:
                # Spark resolves ORDER BY of an aggregate against the SELECT output first: an alias
                # shadows an input column of the same name (SSB Q3.1 "sum(lo_revenue) as lo_revenue")
                ex = alias_map[oe.parts[0].lower()]
            else:
                ex = self._resolve_with_aliases(oe, scope, alias_map)
            orders.append(A.SortOrder(rw(ex), o.ascending, o.nulls_first))
        plan = P.Aggregate(groups, aggs, plan, sets, gid)
        if having is not None:
            if _has_window(having):
                raise AnalysisError("window functions are not allowed in HAVING")
            plan = P.Filter(having, plan)
        plan, proj, orders = _with_windows(plan, proj, orders)
        if orders:
            plan = P.Sort(orders, plan)
        plan = P.Project(proj, plan)
        if s.distinct:
            outs = plan.output
            g2 = [A.Alias(o, o.name) for o in outs]
            plan = P.Project([A.Alias(g.to_ref(g.child.dtype), g.name) for g in g2], P.Aggregate(g2, [], plan))
        if s.limit is not None:
            plan = P.Limit(s.limit, plan)
        return plan

    def _resolve_or_alias(self, e, scope, alias_map):
        if isinstance(e, A.Col) and len(e.parts) == 1:
            r = scope.resolve(e.parts)
            if r is None and e.parts[0].lower() in alias_map:
                return alias_map[e.parts[0].lower()]
        return self.resolve(e, scope)

    def _resolve_with_aliases(self, e, scope, alias_map):
        def sub(x):
            if isinstance(x, A.Col) and len(x.parts) == 1 and scope.resolve(x.parts) is None \
                    and x.parts[0].lower() in alias_map:
                return alias_map[x.parts[0].lower()]
            return None
        return self.resolve(e, scope, substitute=sub)

    # -------------------------------------------------------------------------------- expressions
    def resolve(self, e: A.Expr, scope: Scope, substitute=None) -> A.Expr:
        def go(x: A.Expr) -> A.Expr:
            if substitute is not None:
                s = substitute(x)
                if s is not None:
                    return s
            if isinstance(x, A.Col):
                s = scope
                while s is not None:
                    r = s.resolve(x.parts)
                    if r is not None:
                        if s is not scope:
                            raise AnalysisError(f"correlated reference {x.sql()} is not supported")
                        return r
                    s = s.outer
                raise AnalysisError(f"cannot resolve '`{x.sql()}`' given input columns: "
                                    f"[{', '.join(sorted({r.name for r in scope.refs}))}]")
            if isinstance(x, (A.Ref, A.Lit, A.IntervalLit)):
                return x
            if isinstance(x, A.Star):
                raise AnalysisError("'*' is only allowed in the select list or count(*)")
            if isinstance(x, A.SubqueryExpr):
                p = self.analyze(x.query, scope)
                child = go(x.child) if x.child is not None else None
                if x.kind in ("scalar", "in") and len(p.output) != 1:
                    raise AnalysisError("subquery must return exactly one column")
                return A.SubqueryExpr(x.kind, p, child, x.negated)
            if isinstance(x, A.WindowExpr):
                f = x.func
                if not (f.is_agg or f.name in A.WINDOW_FUNCS):
                    raise AnalysisError(f"{f.name} is not a window function")
                fargs = tuple(go(a) for a in f.args)
                if f.name == "count" and fargs and all(isinstance(a, A.Lit) and a.value is not None for a in fargs) \
                        and not f.distinct:
                    fargs = ()
                return A.WindowExpr(A.Call(f.name, fargs, f.distinct), tuple(go(p) for p in x.partition),
                                    tuple(A.SortOrder(go(o.expr), o.ascending, o.nulls_first) for o in x.orders),
                                    x.frame)
            if isinstance(x, A.Call):
                if not has_function(x.name):
                    raise AnalysisError(f"Undefined function: '{x.name}'. This function is neither a registered "
                                        f"temporary function nor a permanent function registered in the database "
                                        f"'{self.catalog.current_db}'.")
                if x.name == "count" and x.args and all(isinstance(a, A.Lit) and a.value is not None for a in x.args) \
                        and not x.distinct:
                    return A.Call("count", ())
            ch = x.children
            if ch:
                x = x.with_children([go(c) for c in ch])
            return x

        out = go(e)
        typeof(out)  # type check
        return constant_fold(out)


def _has_agg(e: A.Expr) -> bool:
    """An aggregate of the enclosing GROUP BY inside ``e`` (a window function itself is not one:
    ``sum(x) OVER (..)`` aggregates over the window, ``avg(sum(x)) OVER (..)`` holds one)."""
    if isinstance(e, A.WindowExpr):
        return any(_has_agg(c) for c in e.func.args) or any(_has_agg(c) for c in e.children[1:])
    if isinstance(e, A.Call) and e.is_agg:
        return True
    return any(_has_agg(c) for c in e.children)


def _has_window(e: A.Expr) -> bool:
    return any(isinstance(x, A.WindowExpr) for x in e.walk())


def _extract_windows(exprs: List[A.Expr], windows: List[A.Alias], wkeys: Dict[tuple, A.Alias]) -> List[A.Expr]:
    """Replace every window expression by a reference to the column a ``Window`` node computes."""
    def ex(e):
        if isinstance(e, A.WindowExpr):
            k = e.key()
            a = wkeys.get(k)
            if a is None:
                a = wkeys[k] = A.Alias(e, auto_name(e))
                windows.append(a)
            return a.to_ref(typeof(e))
        return None
    return [e.transform(ex) for e in exprs]


def _with_windows(plan: P.Plan, proj: List[A.Expr], orders: List[A.SortOrder]):
    """(plan with a Window node on top if any select item / ORDER BY uses one, proj, orders)."""
    if not any(_has_window(e) for e in proj) and not any(_has_window(o.expr) for o in orders):
        return plan, proj, orders
    windows: List[A.Alias] = []
    wkeys: Dict[tuple, A.Alias] = {}
    proj = _extract_windows(proj, windows, wkeys)
    oex = _extract_windows([o.expr for o in orders], windows, wkeys)
    orders = [A.SortOrder(e, o.ascending, o.nulls_first) for e, o in zip(oex, orders)]
    return P.Window(windows, plan), proj, orders
