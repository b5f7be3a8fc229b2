"""Druid rewrite: replace plan fragments over Druid-backed relations with GPU QuerySpecs.

Parity map (reference -> here):
  * ``ProjectFilterTransfom`` (``asd/ProjectFilterTransfom.scala:32-417``): Project/Filter chains over
    a Druid relation -> ``_collect``; time predicates -> query intervals
    (``sd/QueryIntervals.scala:96-130``, ``sd/DateTimeExtractor.scala:374-436``); dimension predicates
    -> selector / bound / IN(extraction-lookup) / isNull / not / and / or / spatial filters
    (``dimFilterExpression`` 321-416); anything else over one dimension -> a JavaScript filter, which
    here carries a vectorised dictionary-domain evaluator (``_pyvec``) instead of running JS per row.
  * ``JoinTransform`` (``asd/JoinTransform.scala:238-385``): inner equi-join trees that follow the
    declared star schema collapse onto the single denormalized index.
  * ``AggregateTransform`` (``asd/AggregateTransform.scala:48-543``): grouping expressions ->
    default / time-format / time-parsing / JavaScript(dictionary-domain) dimension specs; aggregates
    -> count / long|double Sum|Min|Max / cardinality / hyperUnique / JavaScript (metric expression
    VM); ``avg`` -> sum + count with the division on the host; grouping sets -> one query per set.
  * ``LimitTransfom`` (``asd/DruidTransforms.scala:26-98``): Sort / Limit over a pushed aggregate ->
    ``LimitSpec``.
  * ``DruidStrategy.selectPlan`` (``asd/DruidStrategy.scala:86-282``): non-aggregate scans -> Select
    with paging when ``nonAggregateQueryHandling`` allows it.
  * ``QuerySpecTransforms`` (search / timeseries / topN / between / spatial) run on the result.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Set, Tuple

import numpy as np
import pandas as pd

from ..query import spec as S
from ..query import transforms as QT
from ..query.intervals import fmt_iso
from . import ast as A
from . import plan as P
from .functions import Frame, Period, constant_fold, evaluate, is_deterministic, typeof
from .jscodegen import JSGenError, js_aggregator, js_expr, js_single_column_fn, vm_compatible
from .types import AnalysisError, base, is_vec, to_series

DAY_MS = 86_400_000
MIN_MS = -(2 ** 62)
MAX_MS = 2 ** 62



def _is_day_expr(e: A.Expr) -> bool:
    """to_date(x) / cast(x as date): a value that is already a whole day."""
    return (isinstance(e, A.Call) and e.name == "to_date" and len(e.args) == 1) or \
        (isinstance(e, A.Cast) and e.to == "date")

class NotPushable(Exception):
    pass


# ------------------------------------------------------------------------------------------------
@dataclass
class PF:
    """A Project/Filter(/star-join) fragment over one Druid relation, in terms of base columns."""
    table: object                                 # DruidTable (None while only dimension tables seen)
    cols: Dict[int, object] = field(default_factory=dict)   # base ref id -> DruidRelationColumn | None
    refs: Dict[int, A.Ref] = field(default_factory=dict)    # base ref id -> Ref
    tables: Dict[int, str] = field(default_factory=dict)     # base ref id -> star table short name
    subst: Dict[int, A.Expr] = field(default_factory=dict)   # projected alias id -> expr over base refs
    conds: List[A.Expr] = field(default_factory=list)
    noop_conds: List[A.Expr] = field(default_factory=list)
    dim_scans: List[Tuple[str, List[A.Ref]]] = field(default_factory=list)
    pairs: List[Tuple[Tuple[str, str], List[Tuple[str, str]]]] = field(default_factory=list)

    def sub(self, e: A.Expr) -> A.Expr:
        if not self.subst:
            return e

        def f(x):
            if isinstance(x, A.Ref) and x.rid in self.subst:
                return self.subst[x.rid]
            return None
        return e.transform(f)


def _numeric_dimension(c) -> bool:
    """A dimension whose SQL type is numeric: row expressions read it through its dictionary
    (engine E_LUT: one f64 per dictionary entry)."""
    return c.kind == "dimension" and not c.is_time and \
        base(c.sql_type) in ("tinyint", "smallint", "int", "integer", "bigint", "float", "double", "decimal")


def _short(n: str) -> str:
    return n.split(".")[-1].lower()


class DruidRewriter:
    def __init__(self, session):
        self.session = session
        self.conf = session.conf
        self.approx_distinct = bool(self.conf.typed("spark.sparklinedata.druid.approxCountDistinct"))
        self.log: List[str] = []

    # ============================================================================== driver
    def rewrite(self, plan: P.Plan) -> P.Plan:
        p = self._top_down(plan)
        return p.transform_up(self._finalize)

    def _try(self, fn, p):
        try:
            return fn(p)
        except NotPushable as ex:
            self.log.append(f"{type(p).__name__}: not pushed ({ex})")
            return None

    def _top_down(self, p: P.Plan) -> P.Plan:
        # structural rules first: they need the original Project/Filter/Join chains below them
        if isinstance(p, P.Aggregate):
            r = self._try(self._aggregate, p)
            if r is not None:
                return r
        elif isinstance(p, (P.Project, P.Filter)):
            r = self._try(self._select, p)
            if r is not None:
                return r
        ch = [self._top_down(c) for c in p.children]
        if any(a is not b for a, b in zip(ch, p.children)):
            p = p.with_children(ch)
        if isinstance(p, P.Aggregate):
            r = self._try(self._nested_aggregate, p)
            if r is not None:
                return r
        if isinstance(p, P.Sort):
            r = self._try(self._sort, p)
            if r is not None:
                p = r
        elif isinstance(p, P.Limit):
            self._try(self._limit, p)
        elif isinstance(p, P.Filter):
            self._try(self._having, p)
        return p

    # ============================================================================== fragments
    def _collect(self, p: P.Plan) -> PF:
        if isinstance(p, P.TableScan):
            t = p.table
            if t.kind == "druid":
                info = t.info
                pf = PF(t)
                fact = info.star.fact.name
                for r in p.refs:
                    pf.cols[r.rid] = info.column(r.name)
                    pf.refs[r.rid] = r
                    pf.tables[r.rid] = fact
                return pf
            pf = PF(None)
            pf.dim_scans.append((_short(t.name), p.refs))
            for r in p.refs:
                pf.refs[r.rid] = r
                pf.tables[r.rid] = _short(t.name)
            return pf
        if isinstance(p, P.Filter):
            pf = self._collect(p.child)
            pf.conds.extend(A.conjuncts(pf.sub(p.cond)))
            return pf
        if isinstance(p, P.Project):
            pf = self._collect(p.child)
            new = {}
            for e in p.exprs:
                if isinstance(e, A.Alias):
                    new[e.rid] = pf.sub(e.child)
            pf.subst.update(new)
            return pf
        if isinstance(p, P.Join) and p.kind in ("inner", "cross"):
            return self._join(p)
        raise NotPushable(f"{type(p).__name__} is not a project/filter/star-join over a Druid relation")

    def _join(self, p: P.Join) -> PF:
        l = self._collect(p.left)
        r = self._collect(p.right)
        if l.table is not None and r.table is not None:
            raise NotPushable("join of two Druid relations")
        if l.table is None and r.table is None:
            pf = PF(None)
        else:
            pf = PF(l.table or r.table)
        for x in (l, r):
            pf.cols.update(x.cols)
            pf.refs.update(x.refs)
            pf.tables.update(x.tables)
            pf.subst.update(x.subst)
            pf.conds += x.conds
            pf.noop_conds += x.noop_conds
            pf.dim_scans += x.dim_scans
        cond = pf.sub(p.cond) if p.cond is not None else None
        pairs: Dict[Tuple[str, str], List[Tuple[str, str]]] = {}
        lt = set(l.tables.values())
        rt = set(r.tables.values())
        for c in A.conjuncts(cond):
            if isinstance(c, A.BinOp) and c.op == "=" and isinstance(c.l, A.Ref) and isinstance(c.r, A.Ref):
                a, b = c.l, c.r
                ta, tb = pf.tables.get(a.rid), pf.tables.get(b.rid)
                if ta is not None and tb is not None and ta != tb and \
                        ((ta in lt and tb in rt) or (ta in rt and tb in lt)):
                    if ta in rt:
                        a, b, ta, tb = b, a, tb, ta
                    pairs.setdefault((ta, tb), []).append((a.name, b.name))
                    continue
            pf.conds.append(c)
        if not pairs:
            raise NotPushable("join without equi-join keys (cross product)")
        pf.pairs = l.pairs + r.pairs + list(pairs.items())
        return pf

    def _finish_pf(self, pf: PF) -> PF:
        """Bind dimension-table columns to the Druid relation and validate the star joins."""
        if pf.table is None:
            raise NotPushable("no Druid relation in fragment")
        info = pf.table.info
        star = info.star
        for tname, refs in pf.dim_scans:
            if tname not in star.table_map:
                raise NotPushable(f"table {tname} is not in the star schema of {pf.table.name}")
            for r in refs:
                pf.cols[r.rid] = info.column(r.name)
        for (ta, tb), keys in pf.pairs:
            lcols = [k[0] for k in keys]
            rcols = [k[1] for k in keys]
            if star.is_star_join(lcols, rcols) is None:
                raise NotPushable(f"join {ta}-{tb} on {keys} is not a star-schema join")
        if pf.dim_scans:
            joined = {t for (ta, tb), _ in pf.pairs for t in (ta, tb)}
            for tname, _ in pf.dim_scans:
                if tname not in joined:
                    raise NotPushable(f"table {tname} is not joined")
        # IsNotNull on a star-join column that is not in the index: always true for the index
        # (ProjectFilterTransfom.scala:383-388)
        keep = []
        for c in pf.conds:
            if isinstance(c, A.IsNull) and c.negated and isinstance(c.child, A.Ref):
                col = pf.cols.get(c.child.rid)
                if col is None and star.is_joining_column(None, c.child.name):
                    pf.noop_conds.append(c)
                    continue
            keep.append(c)
        pf.conds = keep
        return pf

    def _column(self, pf: PF, r: A.Ref):
        c = pf.cols.get(r.rid)
        if c is None:
            raise NotPushable(f"column {r.name} is not mapped to the Druid index")
        return c

    # ============================================================================== filters
    def _filters(self, pf: PF) -> Tuple[List[str], Optional[object]]:
        ds = pf.table.info.datasource
        lo, hi = data_interval(ds)
        specs = []
        for c in pf.conds:
            iv = self._time_interval(pf, c)
            if iv is not None:
                lo, hi = max(lo, iv[0]), min(hi, iv[1])
                continue
            f = self._filter(pf, c)
            if f is not None:
                specs.append(f)
        if hi <= lo:
            hi = lo  # empty interval -> empty result (NULL scan)
        intervals = [f"{fmt_iso(lo)}/{fmt_iso(hi)}"]
        filt = None
        if len(specs) == 1:
            filt = specs[0]
        elif specs:
            filt = S.LogicalFilterSpec("and", specs)
        return intervals, filt

    # -- time ---------------------------------------------------------------------------------
    def _time_ref(self, pf: PF, e: A.Expr) -> Optional[Tuple[object, bool]]:
        """(column, truncates_to_day) if e is a reference to the time column (optionally wrapped in
        dateTime / to_date / cast)."""
        trunc = False
        while True:
            if isinstance(e, A.Call) and e.name in ("datetime", "datetimewithtz") and len(e.args) == 1:
                e = e.args[0]
            elif isinstance(e, A.Call) and e.name == "to_date" and len(e.args) == 1:
                e, trunc = e.args[0], True
            elif isinstance(e, A.Call) and e.name == "concat" and len(e.args) == 2 and \
                    isinstance(e.args[1], A.Lit) and isinstance(e.args[1].value, str) and \
                    re.fullmatch(r"[ T]00:00:00(\.0+)?Z?", e.args[1].value) and _is_day_expr(e.args[0]):
                # Cast(Concat(To_date(t), ' 00:00:00') AS TIMESTAMP): midnight of t's day (the BI-tool
                # spelling the reference's SparkIntervalConditionExtractor folds, DateTimeExtractor.scala:374-436)
                e, trunc = e.args[0], True
            elif isinstance(e, A.Cast) and e.to in ("date", "timestamp"):
                trunc = trunc or e.to == "date"
                e = e.child
            else:
                break
        if isinstance(e, A.Ref):
            c = pf.cols.get(e.rid)
            if c is not None and c.is_time:
                return c, trunc or base(c.sql_type) in ("date", "string")
        return None

    def _time_interval(self, pf: PF, c: A.Expr) -> Optional[Tuple[int, int]]:
        cmp = _as_comparison(c)
        if cmp is None:
            return None
        op, l, r = cmp
        tr = self._time_ref(pf, l)
        if tr is None:
            tr = self._time_ref(pf, r)
            if tr is None:
                return None
            op = _FLIP[op]
            l, r = r, l
        if not isinstance(r, A.Lit):
            return None
        ms = _lit_ms(r)
        if ms is None:
            return None
        _, day = tr
        unit = DAY_MS if day else 1
        if day and ms % DAY_MS != 0:
            # a day-valued column compared with a timestamp inside a day
            if op in ("<", "<="):
                return (MIN_MS, (ms // DAY_MS + 1) * DAY_MS)
            if op in (">", ">="):
                return ((ms // DAY_MS + 1) * DAY_MS, MAX_MS)
            return (0, 0)
        if op == "<":
            return (MIN_MS, ms)
        if op == "<=":
            return (MIN_MS, ms + unit)
        if op == ">":
            return (ms + unit, MAX_MS)
        if op == ">=":
            return (ms, MAX_MS)
        if op == "=":
            return (ms, ms + unit)
        return None

    # -- dimension / metric predicates ----------------------------------------------------------
    def _filter(self, pf: PF, e: A.Expr):
        if not is_deterministic(e):
            raise NotPushable(f"non-deterministic predicate {e.sql()}")
        sqs = [x for x in e.walk() if isinstance(x, A.SubqueryExpr)]
        if sqs:
            return self._deferred_filter(pf, e, sqs)
        nn = self._null_test_constant(pf, e)
        if nn is not None:
            return None if nn else S.SelectorFilterSpec("__time", "")
        f = self._native_filter(pf, e)
        if f is not None:
            return f
        return self._expr_filter(pf, e)

    def _deferred_filter(self, pf: PF, e: A.Expr, sqs: List[A.SubqueryExpr]):
        """Predicate over uncorrelated scalar subqueries: pushed as a DeferredFilterSpec whose
        concrete filter is built from the subquery values at execution time.  A trial build with
        placeholder values decides pushability now (the value never changes the filter's shape,
        only its constants)."""
        if any(x.kind not in ("scalar", "in") for x in sqs):
            raise NotPushable("EXISTS subquery in predicate")

        def build(values, _e=e, _pf=pf):
            def sub(x):
                if isinstance(x, A.SubqueryExpr):
                    v = values[id(x.query)]
                    if x.kind == "scalar":
                        return A.Lit(v, typeof(x))
                    # IN (subquery) -> IN list of the subquery's distinct values (semi-join pushdown)
                    vals, has_null = v
                    if not vals:
                        return A.Lit(bool(x.negated) and not has_null, "boolean")
                    if x.negated and has_null:
                        return A.Lit(False, "boolean")  # NOT IN over a NULL-containing set: never true
                    t = typeof(x.child)
                    return A.InList(x.child, tuple(A.Lit(u, t) for u in vals), x.negated)
                return None

            f = self._filter(_pf, constant_fold(_e.transform(sub)))
            # trivially true -> NOT(NULL scan), so the filter tree keeps its shape
            return f if f is not None else S.NotFilterSpec(S.SelectorFilterSpec("__time", ""))

        probe = {}
        for x in sqs:
            t = base(typeof(x) if x.kind == "scalar" else typeof(x.child))
            pv = "x" if t == "string" else (0.5 if t in ("double", "float", "decimal") else 1)
            probe[id(x.query)] = pv if x.kind == "scalar" else ([pv], False)
        build(probe)  # raises NotPushable when the predicate shape is not pushable
        d = S.DeferredFilterSpec(e.sql())
        d.subqueries = sqs
        d.build = build
        return d

    def _native_filter(self, pf: PF, e: A.Expr):
        if isinstance(e, A.Lit):
            if e.value is True:
                return None
            return S.SelectorFilterSpec("__time", "")  # NULL scan (ProjectFilterTransfom.scala:402-404)
        if isinstance(e, A.BinOp) and e.op in ("and", "or"):
            a = self._filter(pf, e.l)
            b = self._filter(pf, e.r)
            fields = [x for x in (a, b) if x is not None]
            if not fields:
                return None
            if len(fields) == 1:
                return fields[0] if e.op == "and" else None
            return S.LogicalFilterSpec(e.op, fields)
        if isinstance(e, A.UnOp) and e.op == "not":
            inner = self._filter(pf, e.child)
            if inner is None:
                raise NotPushable("NOT over a trivially-true predicate")
            if isinstance(inner, S.JavascriptFilterSpec):
                # NOT(expr) must exclude the values where expr is NULL (SQL three-valued logic):
                # evaluate the negated expression itself instead of complementing its TRUE set
                return self._expr_filter(pf, e)
            return S.NotFilterSpec(inner)
        if isinstance(e, A.IsNull) and isinstance(e.child, A.Ref):
            c = pf.cols.get(e.child.rid)
            if c is not None and c.kind == "dimension":
                sel = S.SelectorFilterSpec(c.druid_column, "")
                return S.NotFilterSpec(sel) if e.negated else sel
            if c is not None and (c.is_metric or c.is_time):
                if e.negated:
                    return None
                return S.SelectorFilterSpec("__time", "")
        if isinstance(e, A.InList) and isinstance(e.child, A.Ref) and all(isinstance(i, A.Lit) for i in e.items):
            c = pf.cols.get(e.child.rid)
            if c is not None and c.kind == "dimension" and _same_domain(c, e.child):
                vals = [_druid_str(i.value) for i in e.items if i.value is not None]
                f = S.ExtractionFilterSpec(c.druid_column, "true", S.InExtractionFnSpec.for_values(vals))
                return S.NotFilterSpec(f) if e.negated else f
            if c is not None and c.kind == "metric" and e.items and \
                    all(isinstance(i.value, (int, float)) and not isinstance(i.value, bool) for i in e.items):
                # metric IN (v1, v2, ...) -> OR of metric equalities (TPC-H Q16 p_size IN (...))
                f = S.LogicalFilterSpec("or", [_metric_compare(c, "=", i.value) for i in e.items])
                return S.NotFilterSpec(f) if e.negated else f
        cmp = _as_comparison(e)
        if cmp is not None:
            op, l, r = cmp
            if isinstance(l, A.Lit) and isinstance(r, A.Ref):
                op, l, r = _FLIP[op], r, l
            if isinstance(l, A.Ref) and isinstance(r, A.Lit) and r.value is not None:
                c = pf.cols.get(l.rid)
                if c is not None:
                    if c.spatial is not None and c.kind is None and op in ("<", "<=", ">", ">="):
                        return self._spatial(pf, c, op, r.value)
                    if c.kind == "dimension" and _same_domain(c, l, r):
                        return _dim_compare(c, op, r.value, l.dtype)
                    if c.kind == "metric" and isinstance(r.value, (int, float)) and not isinstance(r.value, bool):
                        return _metric_compare(c, op, r.value)
                    if c.is_time:
                        iv = self._time_interval(pf, e)
                        if iv is not None:
                            return S.IntervalFilterSpec("__time", [f"{fmt_iso(max(iv[0], 0))}/{fmt_iso(iv[1])}"])
            # date comparisons on a date-string dimension: ISO dates order lexicographically
            df = self._date_dim_compare(pf, op, l, r)
            if df is not None:
                return df
        return None

    def _null_test_constant(self, pf: PF, e: A.Expr) -> Optional[bool]:
        """IS [NOT] NULL over metric / spatial-axis expressions: those columns are never NULL in the
        index, so the test folds to a constant when the expression cannot introduce a NULL."""
        if not isinstance(e, A.IsNull):
            return None
        refs = e.child.refs()
        if not refs:
            return None
        for r in refs:
            c = pf.cols.get(r.rid)
            if c is None or not (c.is_metric or (c.kind is None and c.spatial is not None)):
                return None
        for x in e.child.walk():
            if isinstance(x, A.BinOp) and x.op in ("/", "div") or (isinstance(x, A.BinOp) and x.op == "%" and
                                                                   not isinstance(x.r, A.Lit)):
                return None
            if isinstance(x, A.Call) and x.name not in ("abs", "floor", "ceil", "round", "greatest", "least"):
                return None
            if isinstance(x, A.Cast) and x.to not in ("double", "float", "bigint", "int") and \
                    not x.to.startswith("decimal"):
                return None
        return bool(e.negated)  # NOT NULL -> always true ; IS NULL -> always false

    def _date_dim_compare(self, pf, op, l, r):
        if isinstance(l, A.Lit):
            op, l, r = _FLIP[op], r, l
        if not isinstance(r, A.Lit):
            return None
        inner = l
        wrapped = False
        while isinstance(inner, (A.Call, A.Cast)):
            if isinstance(inner, A.Call) and inner.name in ("datetime", "to_date") and len(inner.args) == 1:
                inner = inner.args[0]
                wrapped = True
            elif isinstance(inner, A.Cast) and inner.to in ("date", "timestamp"):
                inner = inner.child
                wrapped = True
            else:
                break
        if not wrapped or not isinstance(inner, A.Ref):
            return None
        c = pf.cols.get(inner.rid)
        if c is None or c.kind != "dimension" or base(c.sql_type) != "string":
            return None
        if not _iso_date_dictionary(pf.table.info.datasource, c.druid_column):
            return None
        ms = _lit_ms(r)
        if ms is None:
            return None
        if ms % DAY_MS == 0:
            v = fmt_iso(ms)[:10]
            strict_hi = op == "<"
            strict_lo = op == ">"
        else:
            v = fmt_iso((ms // DAY_MS) * DAY_MS)[:10]
            strict_hi = False
            strict_lo = True
        if op in ("<", "<="):
            return S.BoundFilterSpec(c.druid_column, None, v, False, strict_hi)
        if op in (">", ">="):
            return S.BoundFilterSpec(c.druid_column, v, None, strict_lo, False)
        if op == "=":
            return S.SelectorFilterSpec(c.druid_column, v) if ms % DAY_MS == 0 else S.SelectorFilterSpec("__time", "")
        return None

    def _spatial(self, pf, c, op, value):
        idx = pf.table.info.spatial_indexes()[c.spatial.druid_column]
        mins = [x.spatial.min_value if x.spatial.min_value is not None else -1.7976931348623157e308 for x in idx]
        maxs = [x.spatial.max_value if x.spatial.max_value is not None else 1.7976931348623157e308 for x in idx]
        pos = [x.column for x in idx].index(c.column)
        v = float(value)
        if op in (">", ">="):
            mins[pos] = v if op == ">=" else np.nextafter(v, np.inf)
        else:
            maxs[pos] = v if op == "<=" else np.nextafter(v, -np.inf)
        return S.SpatialFilterSpec(c.spatial.druid_column, {"type": "rectangular", "minCoords": mins,
                                                            "maxCoords": maxs})

    def _multi_column_filter(self, pf: PF, e: A.Expr, refs: Dict[int, A.Ref]):
        """``a <cmp> b`` over several index columns -> an expression filter evaluated per row in the
        scan kernel's expression VM (string dimensions compared as bare columns only)."""
        if not (isinstance(e, A.BinOp) and e.op in ("=", "<>", "<", "<=", ">", ">=")):
            raise NotPushable(f"predicate over {len(refs)} columns: {e.sql()}")
        names = {}
        strings = set()
        times = set()
        ds = pf.table.info.datasource
        for rid, r in refs.items():
            c = self._column(pf, r)
            if c.is_time:
                names[rid] = "__time"
                times.add(rid)
                continue
            if c.kind not in ("dimension", "metric"):
                raise NotPushable(f"predicate over {len(refs)} columns: {e.sql()}")
            names[rid] = c.druid_column
            if c.kind == "dimension" and base(c.sql_type) == "string":
                strings.add(rid)
        sides = (e.l, e.r)
        if times:
            # time column vs an ISO-date dimension (TPC-H Q12 l_shipdate < l_commitdate): both
            # compared as epoch ms in the kernel (day-grain dates order like their strings)
            if not all(isinstance(x, A.Ref) and (x.rid in times or
                                                 (x.rid in strings and _iso_date_dictionary(ds, names[x.rid])))
                       for x in sides):
                raise NotPushable(f"predicate over {len(refs)} columns: {e.sql()}")
        elif strings:
            # string comparison: both sides bare string columns (rank-compared in the kernel)
            if not all(isinstance(x, A.Ref) and x.rid in strings for x in sides):
                raise NotPushable(f"predicate over {len(refs)} columns: {e.sql()}")
        elif not all(vm_compatible(x) for x in sides):
            raise NotPushable(f"predicate over {len(refs)} columns: {e.sql()}")
        try:
            lhs, rhs = js_expr(e.l, names), js_expr(e.r, names)
        except JSGenError as ex:
            raise NotPushable(str(ex))
        op = {"=": "==", "<>": "!="}.get(e.op, e.op)
        return S.ExpressionFilterSpec(f"{lhs} {op} {rhs}")

    def _expr_filter(self, pf: PF, e: A.Expr):
        refs = {r.rid: r for r in e.refs()}
        if len(refs) > 1 and not any(isinstance(x, A.SubqueryExpr) for x in e.walk()):
            return self._multi_column_filter(pf, e, refs)
        if len(refs) != 1:
            raise NotPushable(f"predicate over {len(refs)} columns: {e.sql()}")
        r = next(iter(refs.values()))
        c = self._column(pf, r)
        if any(isinstance(x, A.SubqueryExpr) for x in e.walk()):
            raise NotPushable("subquery in predicate")
        if c.kind == "dimension":
            js = js_single_column_fn(e, r, c.druid_column)
            f = S.JavascriptFilterSpec(c.druid_column, js)
            f._pyvec = _dict_predicate(e, r, c)  # type: ignore[attr-defined]
            lk = _bare_like(e, r)
            if lk is not None:
                f._pylike = lk  # type: ignore[attr-defined]
            return f
        if c.is_time:
            js = js_single_column_fn(e, r, "__time")
            f = S.JavascriptFilterSpec("__time", js)
            f._pyfn = _time_predicate(e, r, c)  # type: ignore[attr-defined]
            f._pyvec = _time_predicate_vec(e, r, c)  # type: ignore[attr-defined]
            return f
        raise NotPushable(f"predicate over metric {c.column}: {e.sql()}")

    # ============================================================================== aggregate
    def _aggregate(self, agg: P.Aggregate) -> Optional[P.Plan]:
        pf = self._finish_pf(self._collect(agg.child))
        if agg.grouping_sets is not None:
            return self._grouping_sets(agg, pf)
        return self._groupby(agg, pf, list(range(len(agg.groups))), None)

    def _grouping_sets(self, agg: P.Aggregate, pf: PF) -> P.Plan:
        outs = agg.output
        kids = []
        ngr = len(agg.groups)
        for st in agg.grouping_sets:
            sub = self._groupby(agg, pf, st, None)
            # sub outputs agg.output rids; give each branch fresh ids for union
            refs = sub.output
            exprs = []
            for i, r in enumerate(outs):
                if i < ngr and i not in st:
                    exprs.append(A.Alias(A.Lit(None, r.dtype) if r.dtype != "null" else A.Lit(None, "null"), r.name))
                elif agg.gid is not None and i == len(outs) - 1:
                    gid = 0
                    for j in range(ngr):
                        if j not in st:
                            gid |= 1 << (ngr - 1 - j)
                    exprs.append(A.Alias(A.Lit(gid, "int"), r.name))
                else:
                    src = [x for x in refs if x.rid == r.rid][0]
                    exprs.append(A.Alias(src, r.name))
            kids.append(P.Project(exprs, sub))
        return P.Union(kids, outs, distinct=False)

    def _groupby(self, agg: P.Aggregate, pf: PF, gset: List[int], _unused) -> P.Plan:
        info = pf.table.info
        ds = info.datasource
        intervals, filt = self._filters(pf)
        names = _Names()
        dims = []
        columns = []   # (druid out name, sql type, kind)
        drefs = []     # DruidQuery output refs
        final = {}     # agg.output rid -> expr over drefs
        outs = agg.output
        for i in gset:
            g = agg.groups[i]
            e = pf.sub(g.child)
            if not is_deterministic(e):
                raise NotPushable(f"non-deterministic grouping expression {e.sql()}")
            if not e.refs():
                final[outs[i].rid] = e  # grouping by a constant does not split groups
                continue
            spec, kind = self._dim_spec(pf, e, names.dim(g.name))
            dims.append(spec)
            t = typeof(e)
            r = A.Ref(A.new_id(), g.name, t)
            drefs.append(r)
            columns.append((spec.outputName, t, kind))
            final[outs[i].rid] = r
        aggs = []
        for j, a in enumerate(agg.aggs):
            call = a.child
            call = A.Call(call.name, tuple(pf.sub(x) for x in call.args), call.distinct)
            if not is_deterministic(call):
                raise NotPushable(f"non-deterministic aggregate {call.sql()}")
            parts, combine = self._agg_spec(pf, call, names)
            prefs = []
            for part in parts:
                spec_, t = part[0], part[1]
                aggs.append(spec_)
                r = A.Ref(A.new_id(), spec_.name, t)
                drefs.append(r)
                columns.append((spec_.name, t, part[2] if len(part) > 2 else "value"))
                prefs.append(r)
            out_t = outs[len(agg.groups) + j].dtype
            ex = combine(prefs)
            if typeof(ex) != out_t:
                ex = A.Cast(ex, out_t)
            final[outs[len(agg.groups) + j].rid] = ex
        if not dims and agg.aggs and any(a.child.name not in ("count", "approx_count_distinct") for a in agg.aggs):
            # global aggregate: SQL returns one row with NULL sum/min/max/avg over no input rows
            cref = None
            for a_, r_ in zip(aggs, drefs[len(dims):]):
                if isinstance(a_, S.FunctionAggregationSpec) and a_.type == "count" and r_.name == a_.name:
                    cref = r_
                    break
            if cref is None:
                cname = names.agg()
                aggs.append(S.FunctionAggregationSpec("count", cname, "count"))
                cref = A.Ref(A.new_id(), cname, "bigint")
                drefs.append(cref)
                columns.append((cname, "bigint", "value"))
            for j, a in enumerate(agg.aggs):
                if a.child.name in ("count", "approx_count_distinct"):
                    continue
                rid = outs[len(agg.groups) + j].rid
                final[rid] = A.Case(((A.BinOp("=", cref, A.Lit(0, "int")), A.Lit(None, typeof(final[rid]))),),
                                    final[rid])
        q = S.GroupByQuerySpec(info.ds_name, dims, None, None, S.Granularity.parse("all"), filt, aggs, None,
                               intervals)
        method = {}
        dq = P.DruidQuery(pf.table, q, columns, drefs, {"groupby": True, "noop_conds": pf.noop_conds,
                                                         "historical": self._historical(pf, q, method)})
        dq.info.update(method)
        exprs = []
        for r in outs:
            if r.rid in final:
                exprs.append(A.Alias(final[r.rid], r.name, r.rid))
        return P.Project(exprs, dq)

    def _historical(self, pf: PF, q, out: Optional[dict] = None) -> Optional[int]:
        """Broker vs historical execution (``asd/DruidStrategy.scala:324-332``).  With the cost model
        on, the GPU cost model decides between broker and every segments-per-query up to the limit
        (planner/cost.py ``choose_method_costed``, ``asd/DruidQueryCostModel.scala:343-413``); with
        it off, the relation's ``queryHistoricalServers`` / ``numSegmentsPerHistoricalQuery`` options
        (and their ``spark.sparklinedata.druid.option.*`` session overrides) decide.  Returns
        segments per historical query, or None for broker execution; ``out`` receives the priced
        alternatives and the reason (EXPLAIN DRUID REWRITE prints them)."""
        from ..planner.cost import choose_method_costed

        out = out if out is not None else {}
        opts = pf.table.info.options
        wanted = opts.query_historical(self.conf)
        nseg = max(1, min(opts.num_segments_per_query(self.conf), 1 << 30))
        if bool(self.conf.typed("spark.sparklinedata.druid.querycostmodel.enabled")):
            mc = choose_method_costed(pf.table.info.datasource, q, self.conf, pf.table.info,
                                      self.session.engine.world.size)
            out["method_costs"] = mc.costs
            out["method_reason"] = (f"cost model (queryHistoricalServers={str(wanted).lower()}, "
                                    f"numSegmentsPerHistoricalQuery={nseg} in the DDL)")
            return mc.segments_per_query
        out["method_reason"] = f"relation options queryHistoricalServers={str(wanted).lower()}"
        if not wanted:
            return None
        return nseg

    # -- grouping expressions ------------------------------------------------------------------
    def _dim_spec(self, pf: PF, e: A.Expr, out: str):
        if isinstance(e, A.Ref):
            c = self._column(pf, e)
            if c.kind == "dimension":
                return S.DefaultDimensionSpec(c.druid_column, out), "value"
            if c.is_time:
                fmt = _time_format_for(c.sql_type, pf.table.info.datasource)
                return S.ExtractionDimensionSpec("__time", out, S.TimeFormatExtractionFunctionSpec(fmt)), "string"
            if c.is_metric and c.metric_kind == "long":
                # integral metric with a bounded value range: the engine keys it directly (K_INT;
                # TPC-H Q17 groups lineitems by l_quantity), beyond what a Druid broker can do
                return S.DefaultDimensionSpec(c.druid_column, out), "value"
            raise NotPushable(f"cannot group by metric {c.column}")
        te = self._time_element(pf, e)
        if te is not None:
            col, fmt = te
            if col.is_time:
                return S.ExtractionDimensionSpec("__time", out, S.TimeFormatExtractionFunctionSpec(fmt)), "string"
            return (S.ExtractionDimensionSpec(col.druid_column, out,
                                              S.TimeParsingExtractionFunctionSpec("yyyy-MM-dd", fmt)), "string")
        refs = {r.rid: r for r in e.refs()}
        if len(refs) == 0:
            raise NotPushable("constant grouping expression")
        if len(refs) > 1:
            raise NotPushable(f"grouping expression over {len(refs)} columns: {e.sql()}")
        r = next(iter(refs.values()))
        c = self._column(pf, r)
        if c.kind == "dimension":
            fn = S.JavaScriptExtractionFunctionSpec(js_single_column_fn(e, r, c.druid_column))
            fn._pyvec = _dict_extraction(e, r, c)  # type: ignore[attr-defined]
            return S.ExtractionDimensionSpec(c.druid_column, out, fn), "value"
        if c.is_time:
            fn = S.JavaScriptExtractionFunctionSpec(js_single_column_fn(e, r, "__time"))
            fn._pyfn = _time_extraction(e, r, c)  # type: ignore[attr-defined]
            return S.ExtractionDimensionSpec("__time", out, fn), "value"
        raise NotPushable(f"cannot group by an expression over metric {c.column}")

    def _time_element(self, pf: PF, e: A.Expr):
        """year(dateTime(col)) / month(col) / date_format(col, fmt) / to_date(col) ... ->
        (column, Joda format) when col is the time column or an ISO-date string dimension."""
        fmt = None
        arg = None
        if isinstance(e, A.Call):
            n = e.name
            if n in _TIME_FIELD_FMT and len(e.args) == 1:
                fmt, arg = _TIME_FIELD_FMT[n], e.args[0]
            elif n == "date_format" and len(e.args) == 2 and isinstance(e.args[1], A.Lit):
                fmt, arg = str(e.args[1].value), e.args[0]
            elif n == "to_date" and len(e.args) == 1:
                fmt, arg = "yyyy-MM-dd", e.args[0]
        elif isinstance(e, A.Cast) and e.to == "date":
            fmt, arg = "yyyy-MM-dd", e.child
        if fmt is None:
            return None
        while True:
            if isinstance(arg, A.Call) and arg.name in ("datetime", "to_date") and len(arg.args) == 1:
                arg = arg.args[0]
            elif isinstance(arg, A.Cast) and arg.to in ("date", "timestamp"):
                arg = arg.child
            else:
                break
        if not isinstance(arg, A.Ref):
            return None
        c = pf.cols.get(arg.rid)
        if c is None:
            return None
        if c.is_time:
            return c, fmt
        if c.kind == "dimension" and base(c.sql_type) == "string" and \
                _iso_date_dictionary(pf.table.info.datasource, c.druid_column):
            return c, fmt
        return None

    # -- aggregates ------------------------------------------------------------------------------
    def _agg_spec(self, pf: PF, call: A.Call, names: "_Names"):
        info = pf.table.info
        ds = info.datasource
        n = call.name
        rolled = "count" in ds.metrics and getattr(ds, "rollup", False)

        def count_spec():
            nm = names.agg()
            if rolled:
                return S.FunctionAggregationSpec("longSum", nm, "count"), "bigint"
            return S.FunctionAggregationSpec("count", nm, "count"), "bigint"

        if n == "count" and not call.args:
            return [count_spec()], lambda rs: rs[0]
        if n == "count" and not call.distinct:
            if len(call.args) != 1 or not isinstance(call.args[0], A.Ref):
                raise NotPushable("count over an expression")
            c = self._column(pf, call.args[0])
            if c.kind == "dimension":
                cs, t = count_spec()
                f = S.FilteredAggregationSpec(S.NotFilterSpec(S.SelectorFilterSpec(c.druid_column, "")), cs, cs.name)
                return [(f, t)], lambda rs: rs[0]
            return [count_spec()], lambda rs: rs[0]
        if (n == "count" and call.distinct) or n == "approx_count_distinct":
            if n == "count" and not self.approx_distinct:
                raise NotPushable("exact COUNT(DISTINCT) (rewritten to a two-level aggregate)")
            if not info.options.pushHLLTODruid:
                raise NotPushable("pushHLLTODruid is false")
            if len(call.args) != 1 or not isinstance(call.args[0], A.Ref):
                raise NotPushable("distinct count over an expression")
            c = self._column(pf, call.args[0])
            nm = names.agg()
            if c.hll_metric is not None:
                return [(S.HyperUniqueAggregationSpec(nm, c.hll_metric), "double")], \
                    lambda rs: A.Call("round", (rs[0],))
            if c.kind != "dimension":
                raise NotPushable(f"cardinality over non-dimension {c.column}")
            return [(S.CardinalityAggregationSpec(nm, [c.druid_column], True), "double")], \
                lambda rs: A.Call("round", (rs[0],))
        if n in ("sum", "min", "max", "avg", "mean"):
            if call.distinct:
                raise NotPushable(f"{n}(DISTINCT)")
            x = call.args[0]
            fa = self._filtered_agg(pf, n, x, names, count_spec) if n == "sum" else None
            if fa is not None:
                return [fa], lambda rs: rs[0]
            kind = "sum" if n in ("avg", "mean") else n
            null_t = typeof(x) if n in ("min", "max") else "double"
            if kind in ("min", "max"):
                tv = self._time_valued_agg(pf, kind, x, names)
                if tv is None and base(typeof(x)) in ("timestamp", "date"):
                    tv = self._dim_expr_agg(pf, kind, x, names)
                if tv == "null":
                    return [count_spec()], lambda rs: A.Cast(A.Lit(None, "null"), null_t)
                if tv is not None:
                    return [tv], lambda rs: rs[0]
            try:
                spec_, t = self._numeric_agg(pf, kind, x, names)
            except NotPushable:
                de = self._dim_expr_agg(pf, kind, x, names) if base(typeof(x)) not in ("timestamp", "date") else None
                if de is None:
                    raise
                if de == "null":
                    return [count_spec()], lambda rs: A.Cast(A.Lit(None, "null"), null_t)
                spec_, t = de[0], de[1]
            if n in ("avg", "mean"):
                cnt, ct = count_spec()
                return [(spec_, t), (cnt, ct)], \
                    lambda rs: A.BinOp("/", A.Cast(rs[0], "double"), rs[1])
            return [(spec_, t)], lambda rs: rs[0]
        raise NotPushable(f"aggregate {n} is not pushable")

    def _filtered_agg(self, pf: PF, n: str, x: A.Expr, names: "_Names", count_spec):
        """``sum(CASE WHEN p THEN v ELSE 0 END)`` -> Druid filtered aggregator (filter p over sum(v),
        or count for ``THEN 1``): TPC-H Q8 / Q12 / Q14 market-share and line-count ratios."""
        if not (isinstance(x, A.Case) and len(x.whens) == 1):
            return None
        cond, val = x.whens[0]
        el = x.else_
        if not (el is None or (isinstance(el, A.Lit) and el.value in (0, 0.0) and not isinstance(el.value, bool))):
            return None
        f = self._filter(pf, cond)
        if isinstance(val, A.Lit) and val.value == 1 and not isinstance(val.value, bool):
            inner, t = count_spec()
        else:
            inner, t = self._numeric_agg(pf, "sum", val, names)
        if f is None:
            return inner, t
        return S.FilteredAggregationSpec(f, inner, inner.name), t

    def _time_valued_agg(self, pf: PF, kind: str, x: A.Expr, names: "_Names"):
        """MIN/MAX of a timestamp/date-valued column: the time column (``longMin``/``longMax`` over
        ``__time``) or an ISO-date string dimension cast to a timestamp/date (javascript aggregator
        over the dimension: its dictionary entries as epoch ms).  The Druid output is epoch ms,
        converted back like a time column (kind "time")."""
        e, casted = x, False
        while True:
            if isinstance(e, A.Cast) and e.to in ("timestamp", "date"):
                e, casted = e.child, True
            elif isinstance(e, A.Call) and e.name in ("datetime", "to_date", "to_timestamp") and len(e.args) == 1:
                e, casted = e.args[0], True
            else:
                break
        if not isinstance(e, A.Ref):
            return None
        c = pf.cols.get(e.rid)
        if c is None:
            return None
        op = "Min" if kind == "min" else "Max"
        if c.is_time and (casted or base(typeof(e)) in ("date", "timestamp")):
            return S.FunctionAggregationSpec("long" + op, names.agg(), "__time"), "timestamp", "time"
        if casted and c.kind == "dimension" and base(c.sql_type) == "string" and \
                _iso_date_dictionary(pf.table.info.datasource, c.druid_column):
            p = _js_ident(c.druid_column)
            agg, comb, reset = js_aggregator(kind, A.Ref(e.rid, p, "double"), {e.rid: p}, [p])
            return S.JavascriptAggregationSpec(names.agg(), [c.druid_column], agg, comb, reset), "timestamp", "time"
        return None

    def _dim_expr_agg(self, pf: PF, kind: str, x: A.Expr, names: "_Names"):
        """SUM / MIN / MAX of an expression over ONE dimension (or the day-grained time column) that
        the scan VM cannot evaluate per row -- ``unix_timestamp(l_shipdate) * 1000``, nested
        to_date / concat / cast chains (tc/CodeGenTest.scala:417-482): the expression is evaluated
        once per dictionary entry (per day) with the SQL function library, exactly as the base-table
        plan would, and the aggregator reads that table by the row's id (engine E_LUT) -- the
        reference sends these as JavaScript aggregators.  Returns (spec, SQL type, kind) or None."""
        import hashlib

        refs = {r.rid: r for r in x.refs()}
        if len(refs) != 1:
            return None
        r = next(iter(refs.values()))
        c = pf.cols.get(r.rid)
        if c is None or c.is_metric:
            return None
        ds = pf.table.info.datasource
        if c.is_time:
            if ds.time_unit_ms != DAY_MS:
                return None
            gi = getattr(ds, "global_interval_ms", None)
            hi_ms = gi[1] if gi is not None else data_interval(ds)[1]
            ndays = int(hi_ms // DAY_MS) + 1
            if ndays > (1 << 20):
                return None
            values = [_time_value(d * DAY_MS, c) for d in range(ndays)]
            column = "__time"
        else:
            dc = ds.dims.get(c.druid_column) if hasattr(ds, "dims") else None
            if dc is None or len(dc.dictionary) > (1 << 22):
                return None
            values = list(dc.dictionary.all_values())
            column = c.druid_column
        try:
            v = evaluate(x, _dict_frame(values, r, c))
        except Exception:  # noqa: BLE001  (an expression the host library cannot evaluate)
            return None
        if not is_vec(v):
            return None
        timed = v.dtype.kind == "M"
        if timed:
            arr = np.where(v.isna().to_numpy(), np.nan, v.astype("int64").to_numpy() / 1e6)
        elif v.dtype.kind in "iufb" or str(v.dtype) in ("Int64", "Float64", "boolean"):
            arr = v.astype("Float64").to_numpy(dtype="float64", na_value=np.nan)
        else:
            return None
        if np.isnan(arr).all():
            return "null"  # every value NULL (e.g. unix_timestamp of a date-only string): SQL NULL
        if np.isnan(arr).any():
            return None  # some NULL values: the aggregator would have to skip them
        name = "__vx_" + hashlib.sha1(f"{column}|{x.sql()}".encode()).hexdigest()[:12]
        ds.__dict__.setdefault("_virtual_luts", {})[name] = (column, np.ascontiguousarray(arr, dtype=np.float64))
        p = _js_ident(name)
        rid = A.new_id()
        try:
            agg, comb, reset = js_aggregator(kind, A.Ref(rid, p, "double"), {rid: p}, [p])
        except JSGenError:
            return None
        spec = S.JavascriptAggregationSpec(names.agg(), [name], agg, comb, reset)
        return (spec, "timestamp", "time") if timed else (spec, "double", None)

    def _numeric_agg(self, pf: PF, kind: str, x: A.Expr, names: "_Names"):
        if isinstance(x, A.Cast) and (x.to in ("double", "float") or x.to.startswith("decimal")):
            x = x.child
        nm = names.agg()
        if isinstance(x, A.Ref):
            c = self._column(pf, x)
            if c.is_metric:
                integral = c.metric_kind == "long"
                prefix = "long" if integral else "double"
                op = {"sum": "Sum", "min": "Min", "max": "Max"}[kind]
                return S.FunctionAggregationSpec(prefix + op, nm, c.druid_column), ("bigint" if integral else "double")
            if not _numeric_dimension(c):
                raise NotPushable(f"{kind} over non-metric column {c.column}")
        refs = {r.rid: r for r in x.refs()}
        if not refs:
            raise NotPushable("aggregate of a constant")
        cols = []
        for r in refs.values():
            c = self._column(pf, r)
            if not c.is_metric and not _numeric_dimension(c):
                raise NotPushable(f"aggregate expression over non-metric {c.column}")
            cols.append((r, c))
        if not vm_compatible(x):
            raise NotPushable(f"aggregate expression not supported by the scan VM: {x.sql()}")
        stripped = x.transform(lambda e: e.child if isinstance(e, A.Cast) else None)
        params = []
        pnames = {}
        for r, c in cols:
            p = _js_ident(c.druid_column)
            if p in params:
                continue
            params.append(p)
            pnames[r.rid] = p
        try:
            agg, comb, reset = js_aggregator(kind, stripped, pnames, params)
        except JSGenError as ex:
            raise NotPushable(str(ex))
        fields = []
        seen = set()
        for r, c in cols:
            if c.druid_column not in seen:
                seen.add(c.druid_column)
                fields.append(c.druid_column)
        return S.JavascriptAggregationSpec(nm, fields, agg, comb, reset), "double"

    # ============================================================================== sort / limit
    def _druid_below(self, p: P.Plan):
        """Follow row-preserving Projects down to a DruidQuery groupBy; returns (dq, ref map) where
        ref map sends each visible ref id to the DruidQuery output ref it is a plain copy of."""
        m: Dict[int, int] = {}
        chain = []
        while isinstance(p, P.Project) or (isinstance(p, P.Filter) and p.__dict__.get("_absorbed")):
            # (a HAVING absorbed into the groupBy's havingSpec: the engine applies it before the
            # limitSpec, so ORDER BY / LIMIT above it push down too -- the host Filter re-applies it)
            if isinstance(p, P.Project):
                chain.append(p)
            p = p.child
        if not isinstance(p, P.DruidQuery) or not p.info.get("groupby"):
            return None, None
        ids = {r.rid for r in p.refs}
        ident = {rid: rid for rid in ids}
        for proj in reversed(chain):
            nxt = {}
            for e, r in zip(proj.exprs, proj.output):
                src = e.child if isinstance(e, A.Alias) else e
                while isinstance(src, A.Cast):
                    src = src.child
                if isinstance(src, A.Ref) and src.rid in ident:
                    nxt[r.rid] = ident[src.rid]
            ident = nxt
        return p, ident

    def _sort(self, s: P.Sort) -> Optional[P.Plan]:
        dq, m = self._druid_below(s.child)
        if dq is None:
            return None
        q = dq.spec
        if q.limitSpec is not None and (q.limitSpec.columns or q.limitSpec.limit is not None):
            return None
        cols = []
        names = {r.rid: c[0] for r, c in zip(dq.refs, dq.columns)}
        for o in s.orders:
            if not isinstance(o.expr, A.Ref) or o.expr.rid not in m:
                raise NotPushable("ORDER BY expression is not a pushed column")
            if o.nulls_first is not None and o.nulls_first != o.ascending:
                raise NotPushable("non-default NULLS ordering")
            cols.append(S.OrderByColumnSpec(names[m[o.expr.rid]], "ascending" if o.ascending else "descending"))
        dq.spec = q.copy(limitSpec=S.LimitSpec(None, cols))
        return s.child

    def _nested_aggregate(self, agg: P.Aggregate) -> Optional[P.Plan]:
        """Aggregate over a pushed groupBy -> nested groupBy over a query data source, executed on
        the device (engine/nested.py): COUNT(DISTINCT) rewritten as two aggregation levels (TPC-H
        Q16), orders per customer then customers per order count (Q13), orders with a late line
        per priority (Q4).  Outer keys and aggregate inputs must be plain inner output columns;
        count(*) / count(agg) / sum / min / max aggregate."""
        if agg.grouping_sets is not None:
            return None
        dq, m = self._druid_below(agg.child)
        if dq is None or not isinstance(dq.spec, S.GroupByQuerySpec):
            return None
        q = dq.spec
        if q.limitSpec is not None or q.having is not None or q.postAggregations:
            raise NotPushable("nested aggregate over a limited / filtered inner groupBy")
        names = {r.rid: c for r, c in zip(dq.refs, dq.columns)}   # inner ref -> (name, type, kind)
        inner_aggs = {a.name for a in (q.aggregations or [])}
        used = {d.outputName for d in q.dimensions} | inner_aggs
        nm = _Names()
        dims, columns, drefs, final = [], [], [], {}
        outs = agg.output

        def inner_col(e):
            if not (isinstance(e, A.Ref) and e.rid in m):
                raise NotPushable(f"nested aggregate over expression {e.sql()}")
            return names[m[e.rid]]

        for i, g in enumerate(agg.groups):
            name, t, kind = inner_col(g.child)
            out = nm.dim(g.name)
            while out in used:
                out = out + "_"
            dims.append(S.DefaultDimensionSpec(name, out))
            r = A.Ref(A.new_id(), g.name, typeof(g.child))
            drefs.append(r)
            columns.append((out, typeof(g.child), kind))
            final[outs[i].rid] = r
        aggs = []
        for j, a in enumerate(agg.aggs):
            call = a.child
            if call.distinct:
                raise NotPushable("nested DISTINCT aggregate")
            n = call.name
            out_t = outs[len(agg.groups) + j].dtype
            aname = nm.agg()
            while aname in used:
                aname = aname + "_"
            if n == "count" and not call.args:
                spec_ = S.FunctionAggregationSpec("count", aname, "count")
            elif n == "count" and len(call.args) == 1 and (inner_col(call.args[0])[0] in inner_aggs or
                                                           _non_null_dim(q, inner_col(call.args[0])[0],
                                                                         dq.relation.info.datasource)):
                # inner aggregates / NULL-free dimensions: count(x) == count(*)
                spec_ = S.FunctionAggregationSpec("count", aname, "count")
            elif n in ("sum", "min", "max") and len(call.args) == 1 and isinstance(call.args[0], A.Ref):
                name, t, kind = inner_col(call.args[0])
                if name not in inner_aggs:
                    raise NotPushable(f"nested {n} over a dimension")
                pre = "long" if base(t) in ("tinyint", "smallint", "int", "bigint") else "double"
                spec_ = S.FunctionAggregationSpec(pre + n.capitalize(), aname, name)
            elif n in ("sum", "min", "max") and len(call.args) == 1 and vm_compatible(call.args[0]):
                # arithmetic over inner aggregates (TPC-H Q17 sum(qty * n)): javascript aggregator
                # over the inner columns, evaluated with device tensor ops in the nested engine
                x = call.args[0]
                jn: Dict[int, str] = {}
                fields: List[str] = []
                for r_ in x.refs():
                    name, t, kind = inner_col(r_)
                    if name not in inner_aggs and kind != "value":
                        raise NotPushable(f"nested expression over dimension {name}")
                    if r_.rid not in jn:
                        jn[r_.rid] = f"p{len(fields)}"
                        fields.append(name)
                try:
                    fa, fc, fr = js_aggregator(n, x, jn, [f"p{i}" for i in range(len(fields))])
                except JSGenError as ex:
                    raise NotPushable(str(ex))
                spec_ = S.JavascriptAggregationSpec(aname, fields, fa, fc, fr)
            else:
                raise NotPushable(f"nested aggregate {call.sql()}")
            aggs.append(spec_)
            rt = "bigint" if getattr(spec_, "type", "") in ("count", "longSum", "longMin", "longMax") else "double"
            r = A.Ref(A.new_id(), aname, rt)
            drefs.append(r)
            columns.append((aname, rt, "value"))
            ex = r if rt == out_t else A.Cast(r, out_t)
            final[outs[len(agg.groups) + j].rid] = ex
        outer = S.GroupByQuerySpec(S.QueryDataSourceSpec(q), dims, None, None, S.Granularity.parse("all"), None,
                                   aggs, None, q.intervals)
        info = {"groupby": True, "nested": True, "historical": dq.info.get("historical")}
        if not dims:
            # global aggregate over a groupBy (TPC-H Q15's max(total_revenue) over 1M supplier
            # groups): one device reduction instead of shipping every group to the host; SQL's
            # one-row answer over an empty input is filled in by the executor (count 0, else NULL)
            info["global_counts"] = [a.name for a in aggs if getattr(a, "type", "") == "count"]
        nq = P.DruidQuery(dq.relation, outer, columns, drefs, info)
        exprs = [A.Alias(final[r.rid], r.name, r.rid) for r in outs if r.rid in final]
        return P.Project(exprs, nq)

    def _having(self, f: P.Filter) -> None:
        """HAVING over a pushed groupBy -> Druid ``havingSpec`` (comparisons of aggregate outputs
        with numeric literals under AND / OR / NOT).  The engine evaluates it on the device before
        any group is shipped; the host Filter stays for exact SQL semantics over the survivors."""
        dq, m = self._druid_below(f.child)
        if dq is None or not isinstance(dq.spec, S.GroupByQuerySpec):
            return None
        q = dq.spec
        if q.having is not None or (q.limitSpec is not None and q.limitSpec.limit is not None):
            return None
        names = {r.rid: c[0] for r, c in zip(dq.refs, dq.columns)}
        aggs = {a.name for a in (q.aggregations or [])}
        flip = {"<": ">", ">": "<", "<=": ">=", ">=": "<=", "=": "=", "<>": "<>"}

        def conv(e):
            if isinstance(e, A.BinOp) and e.op in ("and", "or"):
                return S.LogicalHavingSpec(e.op, [conv(e.l), conv(e.r)])
            if isinstance(e, A.UnOp) and e.op == "not":
                return S.NotHavingSpec(conv(e.child))
            if isinstance(e, A.BinOp) and e.op in flip:
                l, r, op = e.l, e.r, e.op
                if isinstance(l, A.Lit):
                    l, r, op = r, l, flip[op]
                if not (isinstance(l, A.Ref) and l.rid in m and isinstance(r, A.Lit) and
                        isinstance(r.value, (int, float)) and not isinstance(r.value, bool)):
                    raise NotPushable(f"HAVING term {e.sql()}")
                name = names[m[l.rid]]
                if name not in aggs:
                    raise NotPushable(f"HAVING over non-aggregate {e.sql()}")
                v = float(r.value)

                def cmp(t):
                    return S.ComparisonHavingSpec(t, name, v)
                return {">": cmp("greaterThan"), "<": cmp("lessThan"), "=": cmp("equalTo"),
                        ">=": S.NotHavingSpec(cmp("lessThan")), "<=": S.NotHavingSpec(cmp("greaterThan")),
                        "<>": S.NotHavingSpec(cmp("equalTo"))}[op]
            raise NotPushable(f"HAVING term {e.sql()}")

        sqs = [x for x in f.cond.walk() if isinstance(x, A.SubqueryExpr)]
        if sqs:
            # HAVING against scalar subqueries (TPC-H Q11): resolved when the subqueries have run
            if any(x.kind != "scalar" for x in sqs):
                raise NotPushable("IN / EXISTS subquery in HAVING")

            def build(values, _c=f.cond):
                def sub(x):
                    if isinstance(x, A.SubqueryExpr):
                        return A.Lit(values[id(x.query)], typeof(x))
                    return None
                return conv(constant_fold(_c.transform(sub)))

            build({id(x.query): 1.5 for x in sqs})  # shape check with placeholder values
            d = S.DeferredFilterSpec(f.cond.sql())
            d.subqueries, d.build = sqs, build
            dq.spec = q.copy(having=d)
            dq.__dict__.pop("_deferred", None)
            return None
        dq.spec = q.copy(having=conv(f.cond))
        f._absorbed = True
        return None

    def _limit(self, l: P.Limit) -> Optional[P.Plan]:
        dq, m = self._druid_below(l.child)
        if dq is None:
            return None
        q = dq.spec
        ls = q.limitSpec
        if ls is None:
            dq.spec = q.copy(limitSpec=S.LimitSpec(l.n, []))
        else:
            lim = l.n if ls.limit is None else min(ls.limit, l.n)
            dq.spec = q.copy(limitSpec=S.LimitSpec(lim, ls.columns))
        return None

    # ============================================================================== select
    def _select(self, p: P.Plan) -> Optional[P.Plan]:
        """Non-aggregate Project/Filter over a Druid relation -> Select query (paged)."""
        chain = p
        try:
            pf = self._collect(chain)
        except NotPushable:
            return None
        if pf.table is None:
            return None
        pf = self._finish_pf(pf)
        info = pf.table.info
        mode = info.options.nonAggQueryHandling
        src = self.session.catalog.lookup(info.source_name)
        has_src = src is not None and getattr(src, "has_data", False)
        if mode == "push_none" and has_src:
            return None
        if mode == "push_filters" and not pf.conds and has_src:
            return None
        # only fire at the top of a maximal Project/Filter chain: the parent rule sees it otherwise
        intervals, filt = self._filters(pf)
        outs = p.output
        needed: Dict[int, A.Ref] = {}
        exprs = []
        for r in outs:
            e = pf.sub(r) if r.rid in pf.subst else r
            for x in e.refs():
                needed[x.rid] = x
            exprs.append((r, e))
        dims, mets = [], []
        columns = []
        drefs = []
        rmap = {}
        for rid, x in needed.items():
            c = self._column(pf, x)
            if c.is_time:
                name = "timestamp"
                kind = "time"
            elif c.kind == "dimension":
                name = c.druid_column
                dims.append(name) if name not in dims else None
                kind = "value"
            elif c.is_metric:
                name = c.druid_column
                mets.append(name) if name not in mets else None
                kind = "value"
            elif c.spatial is not None and f"{c.spatial.druid_column}.{c.spatial.position}" in \
                    pf.table.info.datasource.metrics:
                # a spatial axis: the point's component column (DruidValTransform "dimN")
                name = f"{c.spatial.druid_column}.{c.spatial.position}"
                mets.append(name) if name not in mets else None
                kind = "value"
            else:
                raise NotPushable(f"column {c.column} has no direct Druid column")
            nr = A.Ref(A.new_id(), x.name, x.dtype)
            drefs.append(nr)
            columns.append((name, x.dtype, kind))
            rmap[rid] = nr
        page = int(self.conf.typed("spark.sparklinedata.druid.selectquery.pagesize"))
        q = S.SelectSpec(info.ds_name, dims, mets, filt, S.PagingSpec({}, page), intervals)
        dq = P.DruidQuery(pf.table, q, columns, drefs, {"select": True})

        def remap(e):
            return e.transform(lambda x: rmap[x.rid] if isinstance(x, A.Ref) and x.rid in rmap else None)
        proj = [A.Alias(remap(e), r.name, r.rid) for r, e in exprs]
        return P.Project(proj, dq)

    # ============================================================================== finalize
    def _finalize(self, p: P.Plan) -> Optional[P.Plan]:
        if not isinstance(p, P.DruidQuery) or not p.info.get("groupby"):
            return None
        info = p.relation.info
        ds = info.datasource
        q = p.spec
        lo, hi = data_interval(ds)
        whole = f"{fmt_iso(lo)}/{fmt_iso(hi)}"
        ctx = QT.TransformContext(
            allow_topn=info.options.allow_topn(self.conf),
            topn_max=info.options.topn_max_threshold(self.conf),
            covers_all=lambda qq: list(qq.intervals) == [whole],
            metric_is_numeric=lambda m: True)
        nq = QT.transform(q, ctx)
        if isinstance(nq, S.SearchQuerySpec):
            cols = [("value", t, k) for (_, t, k) in p.columns]
            p.columns = cols
            p.info["search"] = True
        p.spec = nq
        return None


# ------------------------------------------------------------------------------------------------
def _non_null_dim(q, out_name: str, ds) -> bool:
    for d in q.dimensions:
        if d.outputName == out_name and isinstance(d, S.DefaultDimensionSpec):
            dc = ds.dims.get(d.dimension) if ds is not None else None
            return dc is not None and not dc.dictionary.has_null
    return False


class _Names:
    def __init__(self):
        self.n = 0
        self.used: Set[str] = set()

    def agg(self) -> str:
        self.n += 1
        nm = f"alias-{self.n}"
        self.used.add(nm)
        return nm

    def dim(self, base_: str) -> str:
        nm = base_
        k = 1
        while nm in self.used:
            nm = f"{base_}_{k}"
            k += 1
        self.used.add(nm)
        return nm


_FLIP = {"<": ">", "<=": ">=", ">": "<", ">=": "<=", "=": "=", "<>": "<>"}
_DATE_CMP = {"dateisbefore": "<", "dateisafter": ">", "dateisbeforeorequal": "<=", "dateisafterorequal": ">=",
             "dateisequal": "="}

_TIME_FIELD_FMT = {
    "year": "yyyy", "month": "MM", "monthofyear": "MM", "dayofmonth": "dd", "day": "dd", "hour": "HH",
    "hourofday": "HH", "minute": "mm", "minuteofhour": "mm", "second": "ss", "secondofminute": "ss",
    "weekofyear": "ww", "weekofweekyear": "ww", "dayofyear": "DDD", "monthofyearname": "MMMM",
    "dayofweekname": "EEEE", "weekyear": "xxxx", "yearofcentury": "yy", "yearofera": "YYYY",
}


def _as_comparison(e: A.Expr):
    if isinstance(e, A.BinOp) and e.op in ("=", "<", "<=", ">", ">="):
        return e.op, e.l, e.r
    if isinstance(e, A.Call) and e.name in _DATE_CMP and len(e.args) == 2:
        return _DATE_CMP[e.name], e.args[0], e.args[1]
    return None


def _lit_ms(l: A.Lit) -> Optional[int]:
    v = l.value
    if v is None:
        return None
    if isinstance(v, pd.Timestamp):
        return int(v.value // 10 ** 6)
    if isinstance(v, str):
        s = v.strip()
        if not re.match(r"^\d{4}-\d{2}-\d{2}", s):
            return None
        try:
            return int(pd.Timestamp(s.replace("Z", "")).value // 10 ** 6)
        except ValueError:
            return None
    return None


def data_interval(ds) -> Tuple[int, int]:
    gi = getattr(ds, "global_interval_ms", None)
    if gi is not None:
        return gi
    segs = getattr(ds, "segments", None)
    if segs:
        return min(s.interval_lo_ms for s in segs), max(s.interval_hi_ms for s in segs)
    return ds.min_time_ms(), ds.max_time_ms() + ds.time_unit_ms


def _druid_str(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v == int(v):
        return str(int(v))
    if isinstance(v, pd.Timestamp):
        return v.strftime("%Y-%m-%d")
    return str(v)


def _same_domain(c, ref: A.Ref, lit: Optional[A.Lit] = None) -> bool:
    """Comparisons on the raw dimension values only mean the same thing when the SQL column type
    and the literal agree with the dictionary's domain (DruidDataType.sparkDataType == dT)."""
    if lit is None:
        return True
    st = base(ref.dtype)
    if st == "string":
        return isinstance(lit.value, str)
    if st in ("tinyint", "smallint", "int", "bigint", "double", "float", "decimal"):
        return isinstance(lit.value, (int, float)) and not isinstance(lit.value, bool)
    return False


def _dim_compare(c, op, value, sqlt):
    d = c.druid_column
    numeric = base(sqlt) in ("tinyint", "smallint", "int", "bigint", "double", "float", "decimal")
    v = _druid_str(value)
    if op == "=":
        return S.SelectorFilterSpec(d, v)
    if op == "<":
        return S.BoundFilterSpec(d, None, v, False, True, numeric)
    if op == "<=":
        return S.BoundFilterSpec(d, None, v, False, False, numeric)
    if op == ">":
        return S.BoundFilterSpec(d, v, None, True, False, numeric)
    if op == ">=":
        return S.BoundFilterSpec(d, v, None, False, False, numeric)
    return None


def _metric_compare(c, op, value):
    d = c.druid_column
    v = str(value)
    if op == "=":
        return S.BoundFilterSpec(d, v, v, False, False, True)
    if op == "<":
        return S.BoundFilterSpec(d, None, v, False, True, True)
    if op == "<=":
        return S.BoundFilterSpec(d, None, v, False, False, True)
    if op == ">":
        return S.BoundFilterSpec(d, v, None, True, False, True)
    return S.BoundFilterSpec(d, v, None, False, False, True)


def _iso_date_dictionary(ds, dim: str) -> bool:
    dc = ds.dims.get(dim) if hasattr(ds, "dims") else None
    if dc is None:
        return False
    d = dc.dictionary
    n = len(d)
    if n == 0:
        return False
    probe = [d.value(i) for i in sorted({0, n // 2, n - 1})]
    return all(isinstance(v, str) and re.match(r"^\d{4}-\d{2}-\d{2}$", v) for v in probe if v is not None)


def _time_format_for(sqlt: str, ds) -> str:
    if base(sqlt) in ("string", "date"):
        return "yyyy-MM-dd" if ds.time_unit_ms >= DAY_MS else "yyyy-MM-dd'T'HH:mm:ss.SSS'Z'"
    return "yyyy-MM-dd'T'HH:mm:ss.SSS'Z'"


def _js_ident(name: str) -> str:
    s = re.sub(r"[^A-Za-z0-9_$]", "_", name)
    return s if not s[0].isdigit() else "_" + s


# -- dictionary-domain evaluators ------------------------------------------------------------------
def _dict_frame(values, r: A.Ref, c) -> Frame:
    s = to_series(pd.Series(np.asarray(values, dtype=object)), c.sql_type)
    return Frame({r.rid: s}, len(s))


def _bare_like(e: A.Expr, r: A.Ref) -> Optional[Tuple[str, bool]]:
    """(pattern, negated) when e is ``r [NOT] LIKE '<literal>'`` over the bare column."""
    neg = False
    if isinstance(e, A.UnOp) and e.op == "not":
        e, neg = e.child, True
    if isinstance(e, A.Like) and e.kind == "like" and isinstance(e.child, A.Ref) and e.child.rid == r.rid and \
            isinstance(e.pattern, A.Lit) and isinstance(e.pattern.value, str):
        return e.pattern.value, neg != e.negated
    return None


def _dict_predicate(e: A.Expr, r: A.Ref, c) -> Callable:
    def fn(values):
        fr = _dict_frame(values, r, c)
        v = evaluate(e, fr)
        if is_vec(v):
            return v.fillna(False).to_numpy(dtype=bool)
        return np.full(fr.n, bool(v), dtype=bool)
    return fn


def _dict_extraction(e: A.Expr, r: A.Ref, c) -> Callable:
    def fn(values):
        fr = _dict_frame(values, r, c)
        v = evaluate(e, fr)
        if not is_vec(v):
            v = pd.Series([v] * fr.n)
        return np.array([None if (x is pd.NA or x is pd.NaT or x is None or (isinstance(x, float) and x != x))
                         else (x.item() if isinstance(x, np.generic) else x) for x in v], dtype=object)
    return fn


def _time_value(ms: int, c):
    ts = pd.Timestamp(int(ms) * 10 ** 6)
    t = base(c.sql_type)
    if t == "string":
        return ts.strftime("%Y-%m-%d") if ms % DAY_MS == 0 else ts.strftime("%Y-%m-%dT%H:%M:%S.%f")[:-3] + "Z"
    if t == "date":
        return ts.normalize()
    if t in ("bigint", "int"):
        return int(ms)
    return ts


def _time_values_vec(ms: np.ndarray, c) -> pd.Series:
    """``_time_value`` over an array of epoch milliseconds (one evaluation per distinct time value
    of the shard, vectorised: the BI templates' ``substr(l_shipdate, 1, 4) = '1995'`` over ~2,500
    days costs one pandas expression instead of 2,500 interpreted ones)."""
    ms = np.asarray(ms, dtype=np.int64)
    idx = pd.to_datetime(ms, unit="ms")
    t = base(c.sql_type)
    if t == "string":
        if len(ms) and (ms % DAY_MS == 0).all():
            return pd.Series(idx.strftime("%Y-%m-%d"), dtype=object)
        return pd.Series([_time_value(int(x), c) for x in ms], dtype=object)
    if t == "date":
        return pd.Series(idx.normalize())
    if t in ("bigint", "int"):
        return pd.Series(ms)
    return pd.Series(idx)


def _time_predicate_vec(e: A.Expr, r: A.Ref, c) -> Callable:
    def fn(ms):
        s = to_series(_time_values_vec(ms, c), c.sql_type) if base(c.sql_type) == "string" else _time_values_vec(ms, c)
        v = evaluate(e, Frame({r.rid: s}, len(s)))
        if not is_vec(v):
            return np.full(len(s), bool(v) if v is not None else False)
        return v.fillna(False).to_numpy(dtype=bool)
    return fn


def _time_predicate(e: A.Expr, r: A.Ref, c) -> Callable:
    def fn(ms):
        v = evaluate(e, Frame({r.rid: _time_value(ms, c)}, 1))
        return bool(v) if v is not None else False
    return fn


def _time_extraction(e: A.Expr, r: A.Ref, c) -> Callable:
    def fn(ms):
        if ms is None:
            return None
        v = evaluate(e, Frame({r.rid: _time_value(ms, c)}, 1))
        return v.item() if isinstance(v, np.generic) else v
    return fn
