"""Logical optimizer: the Catalyst rules the Druid rewrite depends on, plus the reference's own.

  * predicate pushdown through projections and into join inputs; comma joins with WHERE equalities
    become inner equi-joins (Spark's PushPredicateThroughJoin / ReorderJoin), which is what lets the
    star-join elimination see ``lineitem ⋈ orders ⋈ customer`` trees (``tc/StarSchemaBaseTest.scala:46-60``);
  * filter simplification / NULL scans (``asql/util/ExprUtil.scala:156-183``);
  * ``PullVColsIntoAgg`` (``DruidLogicalOptimizer.scala:304-329``): computed projection columns
    are inlined into the Aggregate above them;
  * ``SumOfLiteralRewrite`` (``asql/planner/logical/DruidLogicalOptimizer.scala:245-302``):
    ``sum(lit)`` -> ``count(1) * lit``;
  * exact ``COUNT(DISTINCT)`` rewrite (``SPLRewriteDistinctAggregates.scala:37-205``): the distinct
    aggregate becomes a two-level aggregation (inner GROUP BY adds the distinct column); mixed with
    regular aggregates the two halves are joined on the grouping keys -- two Druid queries, as the
    reference's ``basicAgg`` plan-shape test expects (``tc/DruidRewritesTest.scala:45-52``).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Set

from . import ast as A
from . import plan as P
from .functions import constant_fold, is_deterministic, typeof


def optimize(plan: P.Plan, conf=None) -> P.Plan:
    approx = bool(conf.typed("spark.sparklinedata.druid.approxCountDistinct")) if conf is not None else False
    p = plan.transform_up(_simplify_filter)
    p = p.transform_up(_sum_of_literal)
    if not approx:
        p = p.transform_up(_distinct_rewrite)
    p = _push_down_all(p)
    p = _push_down_all(_reorder_joins(p))
    q = p.transform_up(_push_gb)
    if q is not p:
        p = _push_down_all(q)
    return p.transform_up(_pull_vcols_into_agg)


def _push_down_all(p: P.Plan) -> P.Plan:
    for _ in range(64):
        q = _push_down(p)
        if q is p:
            break
        p = q
    return p


# ------------------------------------------------------------------------------------------------
def _simplify_filter(p: P.Plan):
    if isinstance(p, P.Filter):
        c = constant_fold(p.cond)
        cs = [x for x in A.conjuncts(c) if not (isinstance(x, A.Lit) and x.value is True)]
        if not cs:
            return p.child
        if isinstance(p.child, P.Filter):
            return P.Filter(A.and_all(A.conjuncts(p.child.cond) + cs), p.child.child)
        if len(cs) != len(A.conjuncts(p.cond)) or c is not p.cond:
            return P.Filter(A.and_all(cs), p.child)
    return None


def _sum_of_literal(p: P.Plan):
    if not isinstance(p, P.Aggregate):
        return None
    changed = False
    aggs = []
    for a in p.aggs:
        c = a.child
        if c.name == "sum" and not c.distinct and len(c.args) == 1 and isinstance(c.args[0], A.Lit) \
                and isinstance(c.args[0].value, (int, float)) and not isinstance(c.args[0].value, bool):
            changed = True
            aggs.append((a, c))
        else:
            aggs.append((a, None))
    if not changed:
        return None
    # sum(lit) = count(*) * lit: aggregate count and multiply in a projection above
    new_aggs = []
    post: Dict[int, A.Expr] = {}
    for a, lit_sum in aggs:
        if lit_sum is None:
            new_aggs.append(a)
            continue
        cnt = A.Alias(A.Call("count", ()), "count(1)")
        new_aggs.append(cnt)
        lit = lit_sum.args[0]
        post[a.rid] = A.Cast(A.BinOp("*", cnt.to_ref("bigint"), lit), typeof(lit_sum))
    agg = P.Aggregate(p.groups, new_aggs, p.child, p.grouping_sets, p.gid)
    exprs = []
    for r in p.output:
        if r.rid in post:
            exprs.append(A.Alias(post[r.rid], r.name, r.rid))
        else:
            exprs.append(r)
    return P.Project(exprs, agg)


def _has_druid(p: P.Plan) -> bool:
    return any(isinstance(x, P.TableScan) and x.table.kind == "druid" for x in p.walk())


def _distinct_rewrite(p: P.Plan):
    if not isinstance(p, P.Aggregate) or p.grouping_sets is not None:
        return None
    dist = [a for a in p.aggs if a.child.name == "count" and a.child.distinct]
    if not dist or not _has_druid(p.child):
        return None
    regular = [a for a in p.aggs if not (a.child.name == "count" and a.child.distinct)]
    if any(a.child.distinct for a in regular):
        return None
    outs = p.output
    ng = len(p.groups)
    parts = []  # (plan, {orig rid -> ref in plan})
    if regular:
        gs = [A.Alias(g.child, g.name) for g in p.groups]
        ags = [A.Alias(a.child, a.name) for a in regular]
        sub = P.Aggregate(gs, ags, p.child)
        so = sub.output
        m = {outs[i].rid: so[i] for i in range(ng)}
        for a, r in zip(regular, so[ng:]):
            m[a.rid] = r
        parts.append((sub, m))
    by_args: "OrderedDict[tuple, List[A.Alias]]" = OrderedDict()
    for a in dist:
        by_args.setdefault(tuple(x.key() for x in a.child.args), []).append(a)
    for _, aliases in by_args.items():
        args = aliases[0].child.args
        gs = [A.Alias(g.child, g.name) for g in p.groups]
        xs = [A.Alias(x, f"_distinct_{i}") for i, x in enumerate(args)]
        inner = P.Aggregate(gs + xs, [], p.child)
        io = inner.output
        og = [A.Alias(io[i], p.groups[i].name) for i in range(ng)]
        xrefs = io[ng:]
        oa = [A.Alias(A.Call("count", tuple(xrefs)), a.name) for a in aliases]
        outer = P.Aggregate(og, oa, inner)
        oo = outer.output
        m = {outs[i].rid: oo[i] for i in range(ng)}
        for a, r in zip(aliases, oo[ng:]):
            m[a.rid] = r
        parts.append((outer, m))
    plan, m = parts[0]
    for sub, m2 in parts[1:]:
        conds = [A.BinOp("<=>", m[outs[i].rid], m2[outs[i].rid]) for i in range(ng)]
        plan = P.Join("inner" if conds else "cross", plan, sub, A.and_all(conds))
        for k, v in m2.items():
            if k not in m:
                m[k] = v
    exprs = [A.Alias(m[r.rid], r.name, r.rid) for r in outs]
    return P.Project(exprs, plan)


# ------------------------------------------------------------------------------------------------
def _max_card_one(p: P.Plan) -> bool:
    """At most one row: a global (no GROUP BY) aggregate under filters / projections / LIMIT 1
    (``PlanUtil.maxCardinalityIsOne``, ``asql/util/PlanUtil.scala``)."""
    if isinstance(p, P.Aggregate):
        return not p.groups and p.grouping_sets is None
    if isinstance(p, (P.Filter, P.Project, P.Sort)):
        return _max_card_one(p.child)
    if isinstance(p, P.Limit):
        return p.n <= 1 or _max_card_one(p.child)
    return False


def _has_aggregate(p: P.Plan) -> bool:
    return any(isinstance(x, P.Aggregate) for x in p.walk())


def _push_gb(p: P.Plan):
    """PushGB (``asql/planner/logical/DruidLogicalOptimizer.scala:60-243``): an Aggregate over a
    cross product whose other side has at most one row (typically a scalar aggregate subquery)
    aggregates the big side first and joins the single row afterwards:

        Aggregate(g_big, g_one, aggs(big)) (Join cross (big, one))
          -> Project(..., g_one re-evaluated) (Join cross (Aggregate(g_big, aggs)(big), one))

    which turns the big side into a pushable Druid GroupBy (the one-row side is its own query)."""
    if not isinstance(p, P.Aggregate) or p.grouping_sets is not None or p.gid is not None:
        return None
    child = p.child
    subst: Dict[int, A.Expr] = {}
    if isinstance(child, P.Project) and isinstance(child.child, P.Join):
        if not all(_pushable(e.child) for e in child.exprs if isinstance(e, A.Alias)) or \
                any(_has_agg_or_window(e) for e in child.exprs):
            return None
        subst = {e.rid: e.child for e in child.exprs if isinstance(e, A.Alias)}
        j = child.child
    elif isinstance(child, P.Join):
        j = child
    else:
        return None
    if j.kind not in ("inner", "cross") or j.cond is not None:
        return None

    def inline(e: A.Expr) -> A.Expr:
        return e.transform(lambda x: subst[x.rid] if isinstance(x, A.Ref) and x.rid in subst else None)

    groups = [inline(g.child) for g in p.groups]
    aggs = [inline(a.child) for a in p.aggs]
    l_big = not _has_aggregate(j.left) and _max_card_one(j.right)
    r_big = not _has_aggregate(j.right) and _max_card_one(j.left)
    if l_big == r_big:
        return None
    big, one = (j.left, j.right) if l_big else (j.right, j.left)
    big_ids = {r.rid for r in big.output}
    one_ids = {r.rid for r in one.output}
    if not all(is_deterministic(e) for e in groups + aggs):
        return None
    if any(not (_refs_of(a) <= big_ids) for a in aggs):
        return None
    big_groups = []
    for gi, g in enumerate(groups):
        rs = _refs_of(g)
        if rs and rs <= one_ids:
            continue
        if not (rs <= big_ids):
            return None
        big_groups.append(gi)
    if not big_groups:
        return None
    new_groups = [A.Alias(groups[gi], p.groups[gi].name) for gi in big_groups]
    new_aggs = [A.Alias(a, p.aggs[i].name) for i, a in enumerate(aggs)]
    inner = P.Aggregate(new_groups, new_aggs, big)
    io = inner.output
    nj = P.Join("cross", inner, one, None) if l_big else P.Join("cross", one, inner, None)
    exprs: List[A.Expr] = []
    gpos = {gi: k for k, gi in enumerate(big_groups)}
    for gi, g in enumerate(p.groups):
        src = io[gpos[gi]] if gi in gpos else groups[gi]
        exprs.append(A.Alias(src, g.name, g.rid))
    for i, a in enumerate(p.aggs):
        exprs.append(A.Alias(io[len(new_groups) + i], a.name, a.rid))
    return P.Project(exprs, nj)


def _pull_vcols_into_agg(p: P.Plan):
    """PullVColsIntoAgg (``asql/planner/logical/DruidLogicalOptimizer.scala:304-329``): an Aggregate
    over a Project that computes virtual columns (aliases of expressions over several inputs) gets
    those expressions inlined into its grouping / aggregate expressions; the Project below keeps
    only the plain columns they reference.  Grouping by ``(a + b)`` then appears to the Druid
    rewrite as an expression over index columns instead of an opaque projected column."""
    if not isinstance(p, P.Aggregate) or not isinstance(p.child, P.Project):
        return None
    proj = p.child
    if not all(is_deterministic(e) for e in proj.exprs) or any(_has_agg_or_window(e) for e in proj.exprs) or \
            any(isinstance(x, A.SubqueryExpr) for e in proj.exprs for x in e.walk()):
        return None
    aliases = {e.rid: e.child for e in proj.exprs if isinstance(e, A.Alias)}
    if not any(len(list(c.refs())) > 1 or (not isinstance(c, A.Ref) and c.children)
               for c in aliases.values() if not isinstance(c, A.Ref)):
        return None

    def inline(e: A.Expr) -> A.Expr:
        return e.transform(lambda x: aliases[x.rid] if isinstance(x, A.Ref) and x.rid in aliases else None)

    groups = [A.Alias(inline(g.child), g.name, g.rid) for g in p.groups]
    aggs = [A.Alias(inline(a.child), a.name, a.rid) for a in p.aggs]
    gid = p.gid
    need: Dict[int, A.Ref] = {}
    for e in groups + aggs:
        for r in e.refs():
            need.setdefault(r.rid, r)
    child_out = {r.rid for r in proj.child.output}
    if not set(need) <= child_out:
        return None
    keep = [r for r in proj.child.output if r.rid in need]
    return P.Aggregate(groups, aggs, P.Project(keep, proj.child), p.grouping_sets, gid)


def _refs_of(e: A.Expr) -> Set[int]:
    return {r.rid for r in e.refs()}


def _pushable(e: A.Expr) -> bool:
    return is_deterministic(e) and not any(isinstance(x, A.SubqueryExpr) for x in e.walk())


def _push_down(p: P.Plan) -> P.Plan:
    """One top-down pass of predicate pushdown; returns p itself when nothing changed."""
    if isinstance(p, P.Filter):
        child = p.child
        conds = A.conjuncts(p.cond)
        if isinstance(child, P.Filter):
            return P.Filter(A.and_all(A.conjuncts(child.cond) + conds), child.child)
        if isinstance(child, P.Project):
            subst = {e.rid: e.child for e in child.exprs if isinstance(e, A.Alias)}
            if all(_pushable(e.child) for e in child.exprs if isinstance(e, A.Alias)) and \
                    not any(_has_agg_or_window(e) for e in child.exprs):
                down, keep = [], []
                for c in conds:
                    if _pushable(c):
                        down.append(c.transform(lambda x: subst[x.rid] if isinstance(x, A.Ref) and x.rid in subst
                                                else None))
                    else:
                        keep.append(c)
                if down:
                    np_ = P.Project(child.exprs, P.Filter(A.and_all(down), child.child))
                    return P.Filter(A.and_all(keep), np_) if keep else np_
        if isinstance(child, P.Join) and child.kind in ("inner", "cross"):
            lids = {r.rid for r in child.left.output}
            rids = {r.rid for r in child.right.output}
            lc, rc, jc, keep = [], [], [], []
            for c in conds:
                rs = _refs_of(c)
                if not _pushable(c):
                    keep.append(c)
                elif rs and rs <= lids:
                    lc.append(c)
                elif rs and rs <= rids:
                    rc.append(c)
                elif rs <= (lids | rids):
                    jc.append(c)
                else:
                    keep.append(c)
            if lc or rc or jc:
                left = P.Filter(A.and_all(lc), child.left) if lc else child.left
                right = P.Filter(A.and_all(rc), child.right) if rc else child.right
                cond = A.and_all(A.conjuncts(child.cond) + jc)
                kind = "inner" if cond is not None else child.kind
                j = P.Join(kind, left, right, cond)
                return P.Filter(A.and_all(keep), j) if keep else j
        if isinstance(child, P.Sort):
            return P.Sort(child.orders, P.Filter(p.cond, child.child))
    if isinstance(p, P.Join) and p.kind == "inner" and p.cond is not None:
        lids = {r.rid for r in p.left.output}
        rids = {r.rid for r in p.right.output}
        lc, rc, jc = [], [], []
        for c in A.conjuncts(p.cond):
            rs = _refs_of(c)
            if _pushable(c) and rs and rs <= lids:
                lc.append(c)
            elif _pushable(c) and rs and rs <= rids:
                rc.append(c)
            else:
                jc.append(c)
        if lc or rc:
            left = P.Filter(A.and_all(lc), p.left) if lc else p.left
            right = P.Filter(A.and_all(rc), p.right) if rc else p.right
            return P.Join("inner", left, right, A.and_all(jc))
    ch = [_push_down(c) for c in p.children]
    if any(a is not b for a, b in zip(ch, p.children)):
        return p.with_children(ch)
    return p


def _flatten_joins(p: P.Plan, items: List[P.Plan], conds: List[A.Expr]) -> bool:
    """Leaves and conjuncts of a tree of inner/cross joins; True if any join in it is a cross join."""
    if isinstance(p, P.Join) and p.kind in ("inner", "cross"):
        a = _flatten_joins(p.left, items, conds)
        b = _flatten_joins(p.right, items, conds)
        if p.cond is not None:
            conds.extend(A.conjuncts(p.cond))
        return a or b or p.cond is None
    items.append(p)
    return False


def _reorder_joins(p: P.Plan) -> P.Plan:
    """Spark's ReorderJoin: a FROM list ``a, b, c`` with the join predicates in WHERE becomes a
    left-deep tree of cross joins with the conditions pushed to the top.  Re-build it so each
    leaf joins to the leaves before it through a condition (keeping the written order otherwise),
    which is the shape the star-join elimination (asd/JoinTransform.scala) walks.  SSB Q4.x list
    the fact table last: ``dwdate, customer, supplier, part, lineorder``."""
    if isinstance(p, P.Join) and p.kind in ("inner", "cross"):
        items: List[P.Plan] = []
        conds: List[A.Expr] = []
        has_cross = _flatten_joins(p, items, conds)
        if has_cross and len(items) > 2 and conds:
            items = [_reorder_joins(i) for i in items]
            ids = [{r.rid for r in i.output} for i in items]
            cur, cur_ids = items[0], set(ids[0])
            rest = list(range(1, len(items)))
            pending = list(conds)
            while rest:
                pick = None
                for k in rest:
                    both = cur_ids | ids[k]
                    if any((_refs_of(c) & ids[k]) and (_refs_of(c) & cur_ids) and _refs_of(c) <= both
                           for c in pending):
                        pick = k
                        break
                if pick is None:
                    pick = rest[0]
                rest.remove(pick)
                cur_ids |= ids[pick]
                use = [c for c in pending if _refs_of(c) <= cur_ids]
                pending = [c for c in pending if not _refs_of(c) <= cur_ids]
                cond = A.and_all(use)
                cur = P.Join("inner" if cond is not None else "cross", cur, items[pick], cond)
            return P.Filter(A.and_all(pending), cur) if pending else cur
    ch = [_reorder_joins(c) for c in p.children]
    if any(a is not b for a, b in zip(ch, p.children)):
        return p.with_children(ch)
    return p


def _has_agg_or_window(e: A.Expr) -> bool:
    return any(isinstance(x, A.Call) and x.is_agg for x in e.walk())
