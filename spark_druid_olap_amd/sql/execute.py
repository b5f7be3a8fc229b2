"""Host executor for logical plans.

Runs whatever the Druid rewrite left on the host: residual projections (``avg = sum / count``,
casts, expressions over aggregates), HAVING filters, sorts/limits the GPU did not absorb, joins
with non-star tables, unions, and plain (non-Druid) tables -- the roles Spark's physical operators
play around ``DruidRDD`` in the reference (``asd/DruidStrategy.scala:368-461``).  ``DruidQuery``
leaves execute on the GPU engine (one fused scan kernel per shard + RCCL merge) and come back as
typed columns.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import pandas as pd

from ..query import spec as S
from . import ast as A
from . import plan as P
from .functions import Frame, eval_series, evaluate, typeof
from .types import AnalysisError, base, broadcast, fast_series, is_vec, pandas_dtype, to_series


def take_series(v: pd.Series, idx: np.ndarray) -> pd.Series:
    """``v.iloc[idx].reset_index(drop=True)`` for in-range int64 positions, without pandas'
    per-call index validation (joins gather 500K-row columns: TPC-H Q17)."""
    try:
        arr = v.array if not isinstance(v.dtype, np.dtype) else v.to_numpy(copy=False)
        out = fast_series(arr[idx] if isinstance(arr, np.ndarray) else arr.take(idx))
        out._name = v.name
        return out
    except Exception:  # noqa: BLE001  (exotic extension arrays)
        return v.iloc[idx].reset_index(drop=True)


class LazySeries:
    """A result column whose values are final (typed numpy values, or dictionary codes over cached
    categories) but whose pandas wrapper is built on first access.  Numeric columns carry their
    array (``arr``), so compiled projections and the serving encoder read it without a Series:
    a small query's result costs no pandas constructions unless a caller asks for pandas."""

    __slots__ = ("_make", "arr", "dc")

    def __init__(self, make, arr: Optional[np.ndarray] = None, dc=None):
        # dc: (dictionary-coded column, SQL type) when the values are a dictionary decode -- a
        # gather then moves codes and decodes only the rows it keeps.  make None: the Series is
        # built from ``arr`` / ``dc`` (no closure per result column)
        self._make, self.arr, self.dc = make, arr, dc

    def make(self):
        if self._make is not None:
            return self._make()
        if self.arr is not None:
            return fast_series(self.arr)
        return _dict_series(*self.dc)


class LazyGather(LazySeries):
    """A row gather (join pairing, filter, sort, limit) deferred until the column is read: an
    operator above that never reads a column -- the join keys and payloads a later projection or
    aggregate drops (TPC-H Q17 pairs 450K rows x 6 columns and sums one) -- never gathers it.
    ``DataFrame.run`` materializes the ones that reach the statement's result."""

    __slots__ = ()


def _lazy_take(v, idx: np.ndarray) -> LazyGather:
    if isinstance(v, LazySeries) and v.arr is not None:
        arr = v.arr
        return LazyGather(lambda: fast_series(arr[idx]))
    if isinstance(v, LazySeries) and v.dc is not None:
        # a dictionary column: gather the codes, decode the kept rows only (a window or filter over
        # 300K groups that keeps 5 decodes 5 names, not 300K)
        col, sqlt = v.dc
        sub = type(col)(np.asarray(col.codes)[idx], col.dictionary)
        return LazyGather(lambda: _dict_series(sub, sqlt), dc=(sub, sqlt))
    return LazyGather(lambda: take_series(v.make() if isinstance(v, LazySeries) else v, idx))


class Cols(dict):
    """Batch columns by attribute id; ``LazySeries`` entries become Series when read through the
    mapping interface (``raw`` returns an entry as stored)."""

    __slots__ = ()

    def __getitem__(self, k):
        v = dict.__getitem__(self, k)
        if type(v) is LazySeries or type(v) is LazyGather:
            v = v.make()
            dict.__setitem__(self, k, v)
        return v

    def get(self, k, default=None):
        return self[k] if k in self else default

    def items(self):
        return [(k, self[k]) for k in self]

    def values(self):
        return [self[k] for k in self]

    def raw(self, k):
        return dict.get(self, k)

    def array(self, k) -> Optional[np.ndarray]:
        """The numeric numpy values of column ``k`` when available without building pandas
        objects (a lazy numeric column, or a Series over a plain numeric numpy dtype)."""
        v = dict.get(self, k)
        if type(v) is LazySeries:
            return v.arr
        if type(v) is LazyGather:
            v = self[k]
        if v is not None:
            dt = v.dtype
            if isinstance(dt, np.dtype) and dt.kind in "iuf":
                return v.to_numpy()
        return None


def lazy_series(arr: np.ndarray) -> LazySeries:
    return LazySeries(None, arr)


class Batch:
    """Columns (by attribute id) of equal length, in ``refs`` order."""

    def __init__(self, refs: List[A.Ref], cols: Dict[int, pd.Series], n: int):
        self.refs = refs
        self.cols = cols if type(cols) is Cols else Cols(cols)
        self.n = n

    def frame(self, subq=None) -> Frame:
        return Frame(self.cols, self.n, subq)

    def take(self, idx: np.ndarray) -> "Batch":
        idx = np.asarray(idx, dtype=np.int64)
        raw = self.cols
        return Batch(self.refs, {k: _lazy_take(dict.__getitem__(raw, k), idx) for k in raw}, len(idx))

    def materialize_gathers(self) -> "Batch":
        """Force the deferred gathers (``LazyGather``) still held by this batch's columns."""
        for k in list(self.cols):
            if type(dict.__getitem__(self.cols, k)) is LazyGather:
                self.cols[k]
        return self

    def to_pandas(self, names: Optional[List[str]] = None) -> pd.DataFrame:
        names = names or [r.name for r in self.refs]
        data = {}
        for i, (r, nm) in enumerate(zip(self.refs, names)):
            key = nm if nm not in data else f"{nm}_{i}"
            data[key] = self.cols[r.rid].reset_index(drop=True)
        return pd.DataFrame(data)


class Executor:
    def __init__(self, session, token=None):
        self.session = session
        self.token = token
        # host-side checks between operators only on one rank: across ranks the engine's pre-scan
        # checkpoint (agreed inside the merge collective) is the only place a query may stop
        self._host_checks = token is not None and not session.engine.world.distributed
        self.druid_stats: List[dict] = []
        self._subq_cache: Dict[int, object] = {}
        self._druid_results: Dict[str, object] = {}

    # ----------------------------------------------------------------------------------------
    def run(self, plan: P.Plan) -> Batch:
        if self._host_checks:
            self.token.check()
        m = getattr(self, "_" + type(plan).__name__, None)
        if m is None:
            raise AnalysisError(f"cannot execute {type(plan).__name__}")
        return m(plan)

    def _subquery(self, e: A.SubqueryExpr, fr: Frame):
        key = id(e.query)
        if key not in self._subq_cache:
            b = self.run(e.query)
            self._subq_cache[key] = b
        b = self._subq_cache[key]
        if e.kind == "scalar":
            if b.n > 1:
                raise AnalysisError("more than one row returned by a subquery used as an expression")
            if b.n == 0:
                return None
            v = b.cols[b.refs[0].rid].iloc[0]
            return None if v is pd.NA or v is pd.NaT else (v.item() if isinstance(v, np.generic) else v)
        if e.kind == "exists":
            r = b.n > 0
            return (not r) if e.negated else r
        # IN (subquery)
        vals = b.cols[b.refs[0].rid]
        v = evaluate(e.child, fr)
        has_null = bool(vals.isna().any())
        vset = vals.dropna()
        if not is_vec(v):
            if v is None:
                return None
            hit = bool((vset == v).any())
            r = True if hit else (None if has_null else False)
            return (None if r is None else not r) if e.negated else r
        res = v.isin(vset.tolist()).astype("boolean")
        res = res.mask(v.isna().to_numpy(), pd.NA)
        if has_null:
            res = res.mask(~res.fillna(False).to_numpy(dtype=bool), pd.NA)
        return ~res if e.negated else res

    def _subquery_param(self, e: A.SubqueryExpr):
        """Value a deferred filter needs from a subquery: the scalar, or for IN (subquery) the
        distinct non-NULL values plus whether a NULL was among them.

        The value becomes a literal of the outer pushed query, whose resolved plan is cached per
        value: the subquery's own pushed queries sum exactly (deterministic float sums,
        engine/lower.py fixed_sum), so a repeated statement resolves to the same plan every time --
        a float sum's last bits vary with the device's atomic order, which re-planned the outer
        query on every run (the BI plan's SmallQuantityOrdersRevenue under 64 clients)."""
        for dq in P.find_all_deep(e.query, P.DruidQuery):
            dq.info["deterministic"] = True
        if e.kind == "scalar":
            return self._subquery(e, None)
        key = id(e.query)
        if key not in self._subq_cache:
            self._subq_cache[key] = self.run(e.query)
        b = self._subq_cache[key]
        col = b.cols[b.refs[0].rid]
        has_null = bool(col.isna().any())
        vals = []
        for v in pd.unique(col.dropna()):
            vals.append(v.item() if isinstance(v, np.generic) else v)
        return vals, has_null

    # ----------------------------------------------------------------------------------------
    def _TableScan(self, p: P.TableScan) -> Batch:
        t = p.table
        if t.kind == "druid":
            src = self.session.catalog.get(t.info.source_name)
            df = src.frame()
        else:
            df = t.frame()
        cols = {}
        for r, (c, _) in zip(p.refs, t.schema):
            cols[r.rid] = df[c].reset_index(drop=True)
        return Batch(p.refs, cols, len(df))

    def _LocalRelation(self, p: P.LocalRelation) -> Batch:
        cols = {}
        for r in p.refs:
            v = p.data.get(r.rid)
            cols[r.rid] = v if isinstance(v, pd.Series) else to_series(pd.Series(v if v is not None else [],
                                                                                 dtype=object), r.dtype)
        return Batch(p.refs, cols, p.nrows)

    def _Filter(self, p: P.Filter) -> Batch:
        b = self.run(p.child)
        m = evaluate(p.cond, b.frame(self._subquery))
        if not is_vec(m):
            return b if m else b.take(np.zeros(0, dtype=np.int64))
        mask = m.fillna(False).to_numpy(dtype=bool)
        if mask.all():
            return b
        return b.take(np.nonzero(mask)[0])

    def _Project(self, p: P.Project, b: Optional[Batch] = None) -> Batch:
        if b is None:
            b = self.run(p.child)
        prog = p.__dict__.get("_proj")
        if prog is None:
            # compiled once per plan node: column passthroughs and numpy closures for the
            # arithmetic over Druid results (no per-run expression-tree dispatch)
            p._out = list(p.output)
            prog = p._proj = [_compile_proj(e, r) for e, r in zip(p.exprs, p._out)]
        fr = None
        cols = {}
        refs = p._out
        bcols = b.cols
        for (kind, x), e, r in zip(prog, p.exprs, refs):
            if kind == "ref":
                v = bcols.raw(x)
                cols[r.rid] = v if v is not None else bcols[x]
                continue
            if x is not None and b.n <= _NP_FAST_MAX_ROWS:
                try:
                    a = x(bcols)
                except _NoFast:
                    a = None
                if a is not None:
                    cols[r.rid] = lazy_series(a)
                    continue
            if fr is None:
                fr = b.frame(self._subquery)
            cols[r.rid] = _conform(eval_series(e, fr), r.dtype)
        return Batch(refs, cols, b.n)

    def _Window(self, p: P.Window) -> Batch:
        from .window import evaluate_window

        b = self.run(p.child)
        fr = b.frame(self._subquery)
        cols = {r.rid: dict.__getitem__(b.cols, r.rid) for r in b.refs if r.rid in b.cols}
        layouts: dict = {}  # one sort per distinct (PARTITION BY, ORDER BY) spec
        outs = p.output[len(b.refs):]
        for a, r in zip(p.exprs, outs):
            cols[r.rid] = _conform(evaluate_window(a.child, fr, layouts), r.dtype)
        return Batch(list(b.refs) + list(outs), cols, b.n)

    def _Sort(self, p: P.Sort) -> Batch:
        b = self.run(p.child)
        if b.n <= 1:
            return b
        fr = b.frame(self._subquery)
        keys = []
        for o in p.orders:
            s = eval_series(o.expr, fr)
            keys.append((s, o.ascending, o.nulls_first))
        idx = sort_indices(keys, b.n)
        return b.take(idx)

    def _Limit(self, p: P.Limit) -> Batch:
        node, projs = p.child, []
        while isinstance(node, P.Project):  # row-wise projections commute with the top-k gather
            projs.append(node)
            node = node.child
        if isinstance(node, P.Sort):
            # ORDER BY ... LIMIT k: sort only the top-k candidates, gather k rows, then project them
            b = self.run(node.child)
            if b.n > 1:
                fr = b.frame(self._subquery)
                keys = [(eval_series(o.expr, fr), o.ascending, o.nulls_first) for o in node.orders]
                b = b.take(sort_indices(keys, b.n, limit=p.n)[:p.n])
            elif b.n > p.n:
                b = b.take(np.arange(p.n))
            for pr in reversed(projs):
                b = self._Project(pr, b)
            return b
        b = self.run(p.child)
        if b.n <= p.n:
            return b
        return b.take(np.arange(p.n))

    def _Aggregate(self, p: P.Aggregate) -> Batch:
        b = self.run(p.child)
        return aggregate(p, b, self._subquery)

    def _Join(self, p: P.Join) -> Batch:
        lb = self.run(p.left)
        rb = self.run(p.right)
        return join(p, lb, rb, self._subquery)

    def _Union(self, p: P.Union) -> Batch:
        self._fuse_grouping_sets(p)
        parts = [self.run(c) for c in p.children]
        cols = {}
        n = sum(b.n for b in parts)
        for i, r in enumerate(p.refs):
            ss = [_conform(b.cols[b.refs[i].rid], r.dtype).reset_index(drop=True) for b in parts]
            cols[r.rid] = pd.concat(ss, ignore_index=True) if ss else to_series([], r.dtype)
        out = Batch(p.refs, cols, n)
        if p.distinct:
            out = distinct(out)
        return out

    def _SetOperation(self, p: P.SetOperation) -> Batch:
        lb = distinct(self.run(p.left)) if not p.all else self.run(p.left)
        rb = self.run(p.right)
        ldf = lb.to_pandas([f"c{i}" for i in range(len(lb.refs))])
        rdf = rb.to_pandas([f"c{i}" for i in range(len(rb.refs))])
        keys = list(ldf.columns)
        ltag = ldf.astype(object).where(ldf.notna(), None)
        rtag = rdf.astype(object).where(rdf.notna(), None).drop_duplicates()
        m = ltag.merge(rtag, on=keys, how="left", indicator=True)
        keep = (m["_merge"] == "both") if p.kind == "intersect" else (m["_merge"] == "left_only")
        idx = np.nonzero(keep.to_numpy())[0]
        return lb.take(idx)

    def _fuse_grouping_sets(self, p: P.Union) -> None:
        """A UNION of pushed groupBys that differ only in their dimensions (CUBE / ROLLUP / GROUPING
        SETS, one Druid query per set as the reference plans them) executes as ONE scan on the
        engine; each branch then finds its result already computed."""
        dqs = []
        for c in p.children:
            node = c.child if isinstance(c, P.Project) else c
            if not isinstance(node, P.DruidQuery) or not isinstance(node.spec, S.GroupByQuerySpec) or \
                    node.info.get("historical") or S.find_deferred(node.spec):
                return
            dqs.append(node)
        if len({id(d.relation.info.datasource) for d in dqs}) != 1 or \
                any(share_key(d) in self._druid_results for d in dqs):
            return
        res = self.session.run_druid_sets(dqs)
        if res is not None:
            for d, r in zip(dqs, res):
                self._druid_results[share_key(d)] = r

    def preload(self, p: P.DruidQuery, res) -> None:
        """Use ``res`` as the result of pushed query ``p`` (a streamed Select page)."""
        self._druid_results[share_key(p)] = res

    def _DruidQuery(self, p: P.DruidQuery) -> Batch:
        t0 = time.perf_counter()
        if self._host_checks:
            self.token.check()
        deferred = getattr(p, "_deferred", None)
        if deferred is None:
            deferred = p._deferred = S.find_deferred(p.spec)
        if deferred:
            # scalar subqueries first (pushed queries themselves), then the filter they parameterise;
            # the resolved query (and its lowered program) is cached per subquery-value tuple
            vals = {id(sq.query): self._subquery_param(sq) for d in deferred for sq in d.subqueries}
            key = tuple(repr(vals[k]) for k in sorted(vals))
            cache = p.__dict__.setdefault("_resolved", {})
            q = cache.get(key)
            if q is None:
                if len(cache) > 16:
                    cache.clear()
                q = cache[key] = P.DruidQuery(p.relation, S.resolve_deferred(p.spec, vals), p.columns, p.refs,
                                              p.info)
            p = q
        # identical pushed queries within one statement (a CTE referenced twice, TPC-H Q15) run once
        key = share_key(p)
        res = self._druid_results.get(key)
        if res is None:
            res = self._druid_results[key] = self.session.run_druid(p)
        cols = {}
        n = res.num_rows
        gc = p.info.get("global_counts")
        if gc is not None and n == 0:
            # a global aggregate answers one row over an empty input: count 0, everything else NULL
            n = 1
            for r, (name, sqlt, kind) in zip(p.refs, p.columns):
                v = np.zeros(1, dtype=np.int64) if name in gc else (
                    np.full(1, np.nan) if base(sqlt) in ("double", "float", "decimal") else np.array([None], dtype=object))
                cols[r.rid] = druid_value_series(v, sqlt, kind, 1)
            self.druid_stats.append({"spec": p.spec, "ms": (time.perf_counter() - t0) * 1e3, "rows": 1})
            return Batch(p.refs, cols, 1)
        for r, (name, sqlt, kind) in zip(p.refs, p.columns):
            cols[r.rid] = druid_value_lazy(res.data[name], sqlt, kind, n)
        self.druid_stats.append({"spec": p.spec, "ms": (time.perf_counter() - t0) * 1e3, "rows": n,
                                 "stats": getattr(res, "stats", None)})
        return Batch(p.refs, cols, n)


class FastStatement:
    """A repeated statement of the dashboard shape -- projections over ONE pushed query (the
    reference's benchmark suite, ``TpchBenchMark.scala:137-291``, is all of this form) -- run without
    the general operator dispatch: the pushed query's result columns become the batch directly and
    each projection applies its compiled numpy closures (``_compile_proj``).  Built once per plan
    (``compile``); ``run`` returns None whenever the general executor must answer instead (a
    projection that needs the full evaluator for this result, an empty global aggregate), so the
    answer is always the general executor's.  Saves the per-statement interpreter overhead that
    dominates small queries' host latency (``tools/host_floor.py``)."""

    __slots__ = ("dq", "projs", "colspec")

    def __init__(self, dq, projs, colspec):
        self.dq, self.projs, self.colspec = dq, projs, colspec

    @staticmethod
    def compile(plan) -> Optional["FastStatement"]:
        projs = []
        node = plan
        while isinstance(node, P.Project):
            projs.append(node)
            node = node.child
        if not isinstance(node, P.DruidQuery) or node.info.get("historical") or S.find_deferred(node.spec):
            return None
        if not isinstance(node.spec, (S.GroupByQuerySpec, S.TimeSeriesQuerySpec, S.TopNQuerySpec)):
            return None
        out = []
        for pr in reversed(projs):  # innermost first
            prog = pr.__dict__.get("_proj")
            if prog is None:
                pr._out = list(pr.output)
                prog = pr._proj = [_compile_proj(e, r) for e, r in zip(pr.exprs, pr._out)]
            if any(kind == "expr" and x is None for kind, x in prog):
                return None
            out.append((pr._out, [(kind, x, r.rid) for (kind, x), r in zip(prog, pr._out)]))
        colspec = [(r.rid, name, sqlt, kind) for r, (name, sqlt, kind) in zip(node.refs, node.columns)]
        return FastStatement(node, out, colspec)

    def run(self, session):
        """(batch, pushed query's result, druid stats); batch None = let the general executor
        finish (it is handed the result: the pushed query does not run twice)."""
        dq = self.dq
        t0 = time.perf_counter()
        res = session.run_druid(dq)
        n = res.num_rows
        stats = [{"spec": dq.spec, "ms": (time.perf_counter() - t0) * 1e3, "rows": n, "stats": res.stats}]
        if n == 0 and dq.info.get("global_counts") is not None:
            return None, res, stats
        data = res.data
        cols = Cols()
        for rid, name, sqlt, kind in self.colspec:
            dict.__setitem__(cols, rid, druid_value_lazy(data[name], sqlt, kind, n))
        refs = dq.refs
        if n > _NP_FAST_MAX_ROWS and any(kind != "ref" for _, prog in self.projs for kind, _, _ in prog):
            return None, res, stats
        for out_refs, prog in self.projs:
            nc = Cols()
            for kind, x, rid in prog:
                if kind == "ref":
                    v = dict.get(cols, x)
                    if v is None:
                        return None, res, stats
                    dict.__setitem__(nc, rid, v)
                    continue
                try:
                    a = x(cols)
                except _NoFast:
                    return None, res, stats
                dict.__setitem__(nc, rid, lazy_series(a))
            cols, refs = nc, out_refs
        return Batch(refs, cols, n), res, stats


def share_key(p: P.DruidQuery) -> str:
    key = p.__dict__.get("_share_key")
    if key is None:
        import json

        key = p._share_key = json.dumps(p.spec.to_json(), sort_keys=True, default=str) + \
            str(id(p.relation.info.datasource)) + repr(p.info.get("historical")) + \
            repr(p.info.get("partition_extreme"))
    return key


# ------------------------------------------------------------------------------------------------
_NP_FAST_MAX_ROWS = 1 << 16
_INT_T = ("tinyint", "smallint", "int", "bigint")


def _np_eval(e: A.Expr, b: Batch) -> Optional[np.ndarray]:
    """numpy evaluation of the arithmetic projections that sit on top of Druid results (AVG =
    sum / count, CAST(round(cardinality) AS BIGINT), ...) when every input column is a NULL-free
    numpy column (floats: NaN is NULL and propagates).  Each pandas nullable-array op costs tens of
    microseconds of interpreter time -- most of a small query's host latency -- while these numpy
    ops cost a few.  Returns None for anything else (the general evaluator handles it)."""
    try:
        v = _np_rec(e, b)
    except _NoFast:
        return None
    if not isinstance(v, np.ndarray):
        return None
    t = base(typeof(e))
    if t in ("double", "float") and v.dtype.kind == "f":
        return v
    if t in _INT_T and v.dtype.kind in "iu":
        return v.astype(np.int64, copy=False)
    return None


class _NoFast(Exception):
    pass


def _np_rec(e: A.Expr, b: Batch):
    if isinstance(e, A.Alias):
        return _np_rec(e.child, b)
    if isinstance(e, A.Ref):
        s = b.cols.get(e.rid)
        if s is None or not isinstance(s.dtype, np.dtype) or s.dtype.kind not in "iuf":
            raise _NoFast
        return s.to_numpy()
    if isinstance(e, A.Lit):
        if isinstance(e.value, bool) or not isinstance(e.value, (int, float)):
            raise _NoFast
        return e.value
    if isinstance(e, A.Cast):
        x = _np_rec(e.child, b)
        to = base(e.to)
        if to in ("double", "float"):
            return np.asarray(x, dtype=np.float64) if isinstance(x, np.ndarray) else float(x)
        if to in _INT_T and isinstance(x, np.ndarray):
            if x.dtype.kind == "f":
                if not np.isfinite(x).all():
                    raise _NoFast
                return np.trunc(x).astype(np.int64)
            return x.astype(np.int64, copy=False)
        raise _NoFast
    if isinstance(e, A.UnOp) and e.op == "-":
        return -_np_rec(e.child, b)
    if isinstance(e, A.BinOp) and e.op in ("+", "-", "*", "/"):
        l, r = _np_rec(e.l, b), _np_rec(e.r, b)
        if e.op == "/":
            lf = np.asarray(l, dtype=np.float64)
            rf = np.asarray(r, dtype=np.float64)
            with np.errstate(divide="ignore", invalid="ignore"):
                out = lf / rf
            return np.where(rf == 0, np.nan, out)      # x / 0 is NULL in Spark SQL
        if base(typeof(e)) in _INT_T:
            if (isinstance(l, np.ndarray) and l.dtype.kind == "f") or (isinstance(r, np.ndarray) and r.dtype.kind == "f"):
                raise _NoFast
        elif base(typeof(e)) not in ("double", "float"):
            raise _NoFast
        return {"+": np.add, "-": np.subtract, "*": np.multiply}[e.op](l, r)
    if isinstance(e, A.Call) and e.name in ("round", "bround") and not e.is_agg and e.name == "round":
        x = _np_rec(e.args[0], b)
        d = 0
        if len(e.args) > 1:
            dv = _np_rec(e.args[1], b)
            if isinstance(dv, np.ndarray):
                raise _NoFast
            d = int(dv)
        if not isinstance(x, np.ndarray):
            raise _NoFast
        if x.dtype.kind in "iu":
            if d >= 0:
                return x
            raise _NoFast
        from .functions import _half_up_np

        return _half_up_np(x, d)
    raise _NoFast


def _compile_proj(e: A.Expr, r: A.Ref):
    """("ref", rid) for a passthrough, else ("expr", closure | None): the closure evaluates ``e``
    over NULL-free numpy input columns (same semantics as ``_np_rec``; raises _NoFast otherwise)."""
    if isinstance(e, A.Ref):
        return ("ref", e.rid)
    if isinstance(e, A.Alias) and isinstance(e.child, A.Ref) and e.child.dtype == r.dtype:
        return ("ref", e.child.rid)
    try:
        f = _np_compile(e)
    except _NoFast:
        return ("expr", None)
    t = base(typeof(e))

    def run(cols, f=f, t=t):
        v = f(cols)
        if not isinstance(v, np.ndarray):
            raise _NoFast
        if t in ("double", "float") and v.dtype.kind == "f":
            return v
        if t in _INT_T and v.dtype.kind in "iu":
            return v.astype(np.int64, copy=False)
        raise _NoFast
    return ("expr", run)


def _np_compile(e: A.Expr):
    """Closure form of ``_np_rec`` (type decisions taken at compile time)."""
    if isinstance(e, A.Alias):
        return _np_compile(e.child)
    if isinstance(e, A.Ref):
        rid = e.rid

        def ref(cols):
            a = cols.array(rid)
            if a is None:
                raise _NoFast
            return a
        return ref
    if isinstance(e, A.Lit):
        if isinstance(e.value, bool) or not isinstance(e.value, (int, float)):
            raise _NoFast
        v = e.value
        return lambda cols: v
    if isinstance(e, A.Cast):
        f = _np_compile(e.child)
        to = base(e.to)
        if to in ("double", "float"):
            def cast_f(cols):
                x = f(cols)
                return np.asarray(x, dtype=np.float64) if isinstance(x, np.ndarray) else float(x)
            return cast_f
        if to in _INT_T:
            def cast_int(cols):
                x = f(cols)
                if not isinstance(x, np.ndarray):
                    raise _NoFast
                if x.dtype.kind == "f":
                    if not np.isfinite(x).all():
                        raise _NoFast
                    return np.trunc(x).astype(np.int64)
                return x.astype(np.int64, copy=False)
            return cast_int
        raise _NoFast
    if isinstance(e, A.UnOp) and e.op == "-":
        f = _np_compile(e.child)
        return lambda cols: -f(cols)
    if isinstance(e, A.BinOp) and e.op in ("+", "-", "*", "/"):
        fl, fr_ = _np_compile(e.l), _np_compile(e.r)
        if e.op == "/":
            def div(cols):
                lf = np.asarray(fl(cols), dtype=np.float64)
                rf = np.asarray(fr_(cols), dtype=np.float64)
                # x / 0 is NULL in Spark SQL (NaN here); no floating-point state switch per call
                out = np.full(np.broadcast(lf, rf).shape, np.nan)
                return np.divide(lf, rf, out=out, where=rf != 0)
            return div
        t = base(typeof(e))
        if t not in _INT_T and t not in ("double", "float"):
            raise _NoFast
        op = {"+": np.add, "-": np.subtract, "*": np.multiply}[e.op]
        is_int = t in _INT_T

        def arith(cols):
            l, r = fl(cols), fr_(cols)
            if is_int and ((isinstance(l, np.ndarray) and l.dtype.kind == "f") or
                           (isinstance(r, np.ndarray) and r.dtype.kind == "f")):
                raise _NoFast
            return op(l, r)
        return arith
    if isinstance(e, A.Call) and e.name == "round" and not e.is_agg:
        f = _np_compile(e.args[0])
        d = 0
        if len(e.args) > 1:
            a1 = e.args[1]
            a1 = a1.child if isinstance(a1, A.Alias) else a1
            if not isinstance(a1, A.Lit) or isinstance(a1.value, bool) or not isinstance(a1.value, (int, float)):
                raise _NoFast
            d = int(a1.value)
        from .functions import _half_up_np

        def rnd(cols):
            x = f(cols)
            if not isinstance(x, np.ndarray):
                raise _NoFast
            if x.dtype.kind in "iu":
                if d >= 0:
                    return x
                raise _NoFast
            return _half_up_np(x, d)
        return rnd
    raise _NoFast


def _conform(s: pd.Series, t: str) -> pd.Series:
    want = pandas_dtype(t)
    if want == "string" and isinstance(s.dtype, pd.CategoricalDtype):
        return s  # dictionary-encoded strings stay encoded until something needs the values
    if str(s.dtype) == want or (want == "datetime64[ns]" and s.dtype.kind == "M"):
        return s
    # plain numpy numerics (no NULLs, NaN == NULL for floats) are accepted as-is
    if (want == "Float64" and s.dtype.kind == "f") or (want == "Int64" and s.dtype.kind in "iu"):
        return s
    if want == "object":
        return s
    return to_series(s, t)


def druid_value_series(col, sqlt: str, kind: str, n: int) -> pd.Series:
    """Druid result column -> typed Series (``DruidValTransform``, ``sd/DruidRDD.scala:285-418``)."""
    from ..engine.columns import DictColumn, materialize

    if isinstance(col, DictColumn):
        return _dict_series(col, sqlt)
    arr = np.asarray(col)
    if kind == "time":
        if arr.dtype.kind in "iu":
            ts = pd.Series(pd.to_datetime(arr.astype(np.int64), unit="ms"))
        elif arr.dtype.kind == "f":  # epoch ms from a f64 aggregator (NaN / inf = NULL)
            ts = pd.Series(pd.to_datetime(np.where(np.isfinite(arr), arr, np.nan), unit="ms"))
        else:
            ts = pd.Series(pd.to_datetime(pd.Series(arr).astype(str).str.replace("Z", "", regex=False)))
        if base(sqlt) in ("date", "timestamp"):
            return to_series(ts, sqlt)
        if base(sqlt) == "string":
            midnight = bool((ts.dt.normalize() == ts).all())
            fmt = "%Y-%m-%d" if midnight else "%Y-%m-%dT%H:%M:%S.000Z"
            return pd.Series(ts.dt.strftime(fmt), dtype="string")
        return to_series(ts, sqlt)
    bt = base(sqlt)
    if arr.dtype.kind in "fiu" and bt in ("double", "float", "decimal"):
        return fast_series(arr.astype(np.float64, copy=False))       # numpy float64: NaN == NULL
    if arr.dtype.kind in "iu" and bt in ("tinyint", "smallint", "int", "bigint"):
        if arr.dtype == np.int32 and bt != "bigint":
            return fast_series(arr)  # 32-bit SQL ints stay 32-bit (no widening pass)
        return fast_series(arr.astype(np.int64, copy=False))
    if arr.dtype.kind == "f" and bt in ("tinyint", "smallint", "int", "bigint"):
        if not np.isnan(arr).any():
            return pd.Series(np.rint(arr).astype(np.int64))
        return to_series(pd.Series(arr), sqlt)
    if arr.dtype.kind == "O" and bt in ("tinyint", "smallint", "int", "bigint") and len(arr):
        try:  # digit strings of a numeric time format (year(...) -> 'yyyy'): one numpy cast
            return fast_series(arr.astype(np.int64))
        except (TypeError, ValueError):
            pass
    if arr.dtype.kind == "O" and base(sqlt) != "string":
        return to_series(pd.Series(arr), sqlt)
    return to_series(pd.Series(arr), sqlt)


_DictColumn = None


def druid_value_lazy(col, sqlt: str, kind: str, n: int):
    """``druid_value_series`` with the pandas wrapper deferred (``LazySeries``) for the common
    result columns: numeric aggregates / integer keys (their final numpy values are computed here)
    and dictionary-coded strings (codes over cached categories)."""
    global _DictColumn
    if _DictColumn is None:
        from ..engine.columns import DictColumn as _DC

        _DictColumn = _DC
    if type(col) is _DictColumn:
        return LazySeries(None, None, (col, sqlt))
    if kind != "time":
        if type(col) is np.ndarray:
            # (the common numeric result columns: already at their final numpy dtype)
            conv = _LAZY_CONV.get((col.dtype, sqlt))
            if conv is not None:
                return LazySeries(None, col if conv is True else col.astype(conv))
        arr = np.asarray(col)
        bt = base(sqlt)
        if arr.dtype.kind in "fiu" and bt in ("double", "float", "decimal"):
            _LAZY_CONV[(arr.dtype, sqlt)] = True if arr.dtype == np.float64 else np.float64
            return lazy_series(arr.astype(np.float64, copy=False))
        if arr.dtype.kind in "iu" and bt in ("tinyint", "smallint", "int", "bigint"):
            keep = arr.dtype == np.int64 or (arr.dtype == np.int32 and bt != "bigint")
            _LAZY_CONV[(arr.dtype, sqlt)] = True if keep else np.int64
            return lazy_series(arr if keep else arr.astype(np.int64))
    return druid_value_series(col, sqlt, kind, n)


_LAZY_CONV: Dict[tuple, object] = {}  # (numpy dtype, SQL type) -> True (as is) | target dtype


def _categorical(codes: np.ndarray, dtype) -> pd.Categorical:
    """A Categorical over validated codes of a cached dtype (pandas' internal constructor: the
    public ``from_codes`` re-derives the code width and checks every code on each call)."""
    try:
        from pandas.core.dtypes.cast import coerce_indexer_dtype

        return pd.Categorical._simple_new(coerce_indexer_dtype(codes, dtype.categories), dtype=dtype)
    except Exception:  # noqa: BLE001  (pandas internals moved)
        return pd.Categorical.from_codes(codes, dtype=dtype, validate=False)


_FULL_DICT_MAX = 1 << 20
_LAZY_DICT_MAX = 1 << 22


def _dict_series(col, sqlt: str) -> pd.Series:
    """Typed values of a dictionary-coded result column.  Small dictionaries are converted once and
    cached on the (immutable) dictionary; large ones (e.g. o_orderkey) decode only the distinct
    codes present in the result."""
    d = col.dictionary
    codes = np.asarray(col.codes)
    nd = len(d)
    lazy_ok = getattr(d, "lazy", False) and nd <= _LAZY_DICT_MAX and base(sqlt) == "string"
    if (nd <= _FULL_DICT_MAX and (nd <= 65536 or nd <= 2 * len(codes))) or lazy_ok:
        # (lazy synthetic dictionaries up to a few million entries are materialised once, like the
        # string dictionaries a Druid historical keeps in memory; per query only codes move)
        cache = d.__dict__.setdefault("_sql_typed", {})
        key = sqlt if base(sqlt) != "string" else "__categories__"
        full = cache.get(key)
        bt = base(sqlt)
        if full is None:
            if bt == "string":
                # zero-copy dictionary encoding: a pandas Categorical over the (sorted, unique) values
                vals = d.all_values()
                has_null = bool(getattr(d, "has_null", False))
                cats = pd.Index(np.asarray(vals[1:] if has_null else vals, dtype=object).astype(str), dtype=object)
                full = (cats, has_null)
            else:
                typed = to_series(_raw(d.all_values()), sqlt)
                if typed.isna().any() or bt not in ("tinyint", "smallint", "int", "bigint", "double", "float"):
                    full = ("typed", typed)
                else:
                    full = ("numpy", typed.to_numpy(dtype=np.int64 if bt in ("tinyint", "smallint", "int", "bigint")
                                                    else np.float64))
            cache[key] = full
        if bt == "string":
            cats, has_null = full
            c = codes.astype(np.int32, copy=False) - (1 if has_null else 0) if has_null else codes
            cdt = cache.get("__cdtype__")
            if cdt is None:
                cdt = cache["__cdtype__"] = pd.CategoricalDtype(cats)
            return fast_series(_categorical(c, cdt))
        if full[0] == "numpy":
            return fast_series(full[1][codes])
        return pd.Series(full[1].array.take(codes))
    if hasattr(d, "start") and not getattr(d, "has_null", False) and not hasattr(d, "prefix"):
        # integer range dictionary: value = start + code
        vals = d.decode(codes)
        if base(sqlt) in ("tinyint", "smallint", "int", "bigint"):
            return fast_series(vals.astype(np.int64, copy=False))
        return to_series(pd.Series(vals), sqlt)
    inv, uniq = pd.factorize(codes)
    typed = to_series(_raw(d.decode(np.asarray(uniq, dtype=np.int64))), sqlt)
    return pd.Series(typed.array.take(inv))


def _raw(vals) -> pd.Series:
    a = np.asarray(vals)
    if a.dtype != object:
        return pd.Series(a)
    return pd.Series(a, dtype=object)


def _sort_key(s: pd.Series, asc: bool):
    """(null mask, order-preserving numeric key with DESC folded in) of one ORDER BY column."""
    isna = s.isna().to_numpy()
    if s.dtype.kind == "M":
        arr = np.where(isna, 0, s.astype("int64").to_numpy())
    elif isinstance(s.dtype, np.dtype) and s.dtype.kind in "iuf":
        arr = s.to_numpy()
        arr = np.where(isna, 0.0, arr) if arr.dtype.kind == "f" else arr.astype(np.int64, copy=False)
    elif str(s.dtype) in ("Int64", "Float64", "boolean") or s.dtype.kind in "iufb":
        arr = s.astype("Float64").to_numpy(dtype="float64", na_value=0.0) if str(s.dtype) != "Int64" else \
            s.to_numpy(dtype="int64", na_value=0)
        if arr.dtype.kind == "f":
            arr = np.where(isna, 0.0, arr)
    elif isinstance(s.dtype, pd.CategoricalDtype) and s.cat.categories.is_monotonic_increasing:
        # dictionary-coded strings: categories are the sorted dictionary, so codes order like values
        arr = s.cat.codes.to_numpy().astype(np.int64)
    else:
        arr = np.asarray(pd.factorize(s, sort=True)[0], dtype=np.int64)
    if not asc:
        arr = -arr if arr.dtype.kind == "f" else ~arr.astype(np.int64)  # ~x: order-reversing, no overflow
    return isna, arr


def sort_indices(keys, n: int, limit: Optional[int] = None) -> np.ndarray:
    """Stable multi-key sort (one ``np.lexsort``); Spark default null ordering: NULLS FIRST for
    ASC, NULLS LAST for DESC.  With ``limit`` (ORDER BY ... LIMIT k) only the rows whose leading
    key is within the k smallest (ties included) are sorted -- TPC-H Q2 keeps 100 of ~50K join
    rows; the returned indices then cover at least the first ``limit`` positions."""
    if n == 0:
        return np.arange(0)
    cols = [(_sort_key(s.reset_index(drop=True), asc), asc if nf is None else nf) for s, asc, nf in keys]
    cand = None
    (na0, v0), _ = cols[0]
    if limit is not None and 0 < limit < n // 2 and not na0.any():
        kth = np.partition(v0, limit - 1)[limit - 1]
        cand = np.nonzero(v0 <= kth)[0]
    lex = []
    for (isna, arr), nf in reversed(cols):
        if cand is not None:
            isna, arr = isna[cand], arr[cand]
        lex.append(arr)
        if isna.any():
            lex.append(~isna if nf else isna)  # primary over this key's values
    m = n if cand is None else len(cand)
    if lex and m >= GPU_SORT_MIN_ROWS and _gpu_sort_ok():
        order = _lexsort_device(lex)
    else:
        order = np.lexsort(lex) if lex else np.arange(m)
    return order if cand is None else cand[order]


GPU_SORT_MIN_ROWS = 1 << 16  # host rows above which an ORDER BY / window sort runs on the GPU
_GPU_SORT: list = []


def _gpu_sort_ok() -> bool:
    if not _GPU_SORT:
        import torch

        _GPU_SORT.append(bool(torch.cuda.is_available()))
    return _GPU_SORT[0]


def _lexsort_device(lex) -> np.ndarray:
    """``np.lexsort(lex)`` (last key primary, stable) as chained stable device sorts, least
    significant key first: a 300K-row window partition sort takes ~1 ms instead of ~27 ms."""
    import torch

    dev = torch.device("cuda", torch.cuda.current_device())
    keys = [torch.from_numpy(np.ascontiguousarray(k)).to(dev, non_blocking=True) for k in lex]
    idx = torch.arange(keys[0].numel(), device=dev)
    for k in keys:
        kk = k[idx]
        if kk.dtype == torch.bool:
            kk = kk.to(torch.uint8)
        idx = idx[torch.sort(kk, stable=True).indices]
    return idx.cpu().numpy()


def _neg(arr):
    if arr.dtype.kind == "f":
        return -arr
    return -(arr.astype(np.int64))


def distinct(b: Batch) -> Batch:
    if b.n == 0:
        return b
    df = b.to_pandas([f"c{i}" for i in range(len(b.refs))])
    dup = df.astype(object).where(df.notna(), None).duplicated()
    idx = np.nonzero(~dup.to_numpy())[0]
    return b.take(idx)


# ------------------------------------------------------------------------------------------------
# aggregation
def _group_codes(keys: List[pd.Series], n: int):
    keys = [k.cat.codes if isinstance(k.dtype, pd.CategoricalDtype) else k for k in keys]
    if not keys:
        return np.zeros(n, dtype=np.int64), 1, np.zeros(1 if n else 0, dtype=np.int64)
    if len(keys) == 1:
        codes, uniq = pd.factorize(keys[0], use_na_sentinel=False)
        codes = np.asarray(codes, dtype=np.int64)
    else:
        df = pd.DataFrame({i: k.reset_index(drop=True) for i, k in enumerate(keys)})
        codes = df.groupby(list(range(len(keys))), dropna=False, sort=False).ngroup().to_numpy().astype(np.int64)
    ng = int(codes.max()) + 1 if n else 0
    first = np.full(ng, n, dtype=np.int64)
    np.minimum.at(first, codes, np.arange(n, dtype=np.int64))
    return codes, ng, first


_GLOBAL_AGG = {
    "sum": lambda x: x.sum(min_count=1),
    "avg": lambda x: x.mean(),
    "mean": lambda x: x.mean(),
    "min": lambda x: x.min(),
    "max": lambda x: x.max(),
}


def _agg_one(call: A.Call, fr: Frame, codes: np.ndarray, ng: int, n: int, out_t: str) -> pd.Series:
    name = call.name
    if name == "count" and not call.args:
        cnt = np.bincount(codes, minlength=ng) if n else np.zeros(ng, dtype=np.int64)
        return pd.Series(cnt.astype(np.int64), dtype="Int64")
    args = [eval_series(a, fr) for a in call.args]
    x = args[0] if args else None
    if name == "count":
        valid = np.ones(n, dtype=bool)
        for a in args:
            valid &= ~a.isna().to_numpy()
        if call.distinct:
            if len(args) == 1:
                s = x[valid]
                r = s.groupby(codes[valid]).nunique(dropna=True)
            else:
                df = pd.DataFrame({i: a[valid].astype(object) for i, a in enumerate(args)})
                df["_g"] = codes[valid]
                r = df.drop_duplicates().groupby("_g").size()
            return pd.Series(r.reindex(range(ng), fill_value=0).to_numpy().astype(np.int64), dtype="Int64")
        cnt = np.bincount(codes[valid], minlength=ng) if n else np.zeros(ng, dtype=np.int64)
        return pd.Series(cnt.astype(np.int64), dtype="Int64")
    if name == "approx_count_distinct":
        valid = ~x.isna().to_numpy()
        r = x[valid].groupby(codes[valid]).nunique()
        return pd.Series(r.reindex(range(ng), fill_value=0).to_numpy().astype(np.int64), dtype="Int64")
    xt = typeof(call.args[0]) if call.args else "null"
    if ng == 1 and not call.distinct and name in _GLOBAL_AGG and x is not None and n and \
            pd.api.types.is_numeric_dtype(x.dtype) and not pd.api.types.is_bool_dtype(x.dtype) and \
            (not len(codes) or not codes.any()):
        # a global aggregate (no GROUP BY) over a numeric column: the Series reduction itself, not a
        # one-group groupby (TPC-H Q17's sum over the joined rows: 0.65 -> ~0.05 ms)
        v = _GLOBAL_AGG[name](x)
        return to_series(pd.Series([None if v is pd.NA or (isinstance(v, float) and v != v) else v]), out_t)
    if name in ("sum", "avg", "mean", "stddev", "stddev_samp", "stddev_pop", "variance", "var_samp", "var_pop"):
        if base(xt) == "string":
            x = to_series(x, "double")
        if call.distinct:
            df = pd.DataFrame({"v": x, "g": codes}).dropna().drop_duplicates()
            x, codes_ = df["v"].reset_index(drop=True), df["g"].to_numpy()
        else:
            codes_ = codes
        g = x.groupby(codes_)
        if name == "sum":
            r = g.sum(min_count=1)
        elif name in ("avg", "mean"):
            r = g.mean()
        elif name in ("stddev", "stddev_samp"):
            r = g.std(ddof=1)
        elif name == "stddev_pop":
            r = g.std(ddof=0)
        elif name in ("variance", "var_samp"):
            r = g.var(ddof=1)
        else:
            r = g.var(ddof=0)
        r = r.reindex(range(ng))
        return to_series(r, out_t)
    if name in ("min", "max"):
        valid = ~x.isna().to_numpy()
        g = x[valid].groupby(codes[valid])
        r = (g.min() if name == "min" else g.max()).reindex(range(ng))
        return to_series(r, out_t)
    if name in ("first", "last"):
        g = x.groupby(codes)
        r = (g.first() if name == "first" else g.last()).reindex(range(ng))
        return to_series(r, out_t)
    if name in ("collect_list", "collect_set"):
        valid = ~x.isna().to_numpy()
        g = x[valid].astype(object).groupby(codes[valid])
        r = g.agg(lambda v: list(v) if name == "collect_list" else sorted(set(v), key=str)).reindex(range(ng))
        return pd.Series(r.to_numpy(), dtype=object)
    raise AnalysisError(f"unsupported aggregate {name}")


def aggregate(p: P.Aggregate, b: Batch, subq=None) -> Batch:
    fr = b.frame(subq)
    outs = p.output
    gkeys = [eval_series(g.child, fr) for g in p.groups]
    sets = p.grouping_sets if p.grouping_sets is not None else [list(range(len(p.groups)))]
    results = []
    ngr = len(p.groups)
    for st in sets:
        keys = [gkeys[i] for i in st]
        codes, ng, first = _group_codes(keys, b.n)
        if not p.groups and p.grouping_sets is None:
            ng = 1
            first = np.zeros(1, dtype=np.int64)
        cols = {}
        for i, g in enumerate(p.groups):
            r = outs[i]
            if i in st:
                cols[r.rid] = gkeys[i].iloc[first].reset_index(drop=True) if b.n else to_series([], r.dtype)
            else:
                cols[r.rid] = broadcast(None, ng, r.dtype)
        for j, a in enumerate(p.aggs):
            r = outs[ngr + j]
            cols[r.rid] = _agg_one(a.child, fr, codes, ng, b.n, r.dtype).reset_index(drop=True)
        if p.gid is not None:
            gid = 0
            for i in range(ngr):
                if i not in st:
                    gid |= 1 << (ngr - 1 - i)
            cols[outs[-1].rid] = pd.Series([gid] * ng, dtype="Int64")
        results.append((cols, ng))
    if len(results) == 1:
        cols, ng = results[0]
        return Batch(outs, cols, ng)
    cols = {r.rid: pd.concat([c[r.rid] for c, _ in results], ignore_index=True) for r in outs}
    return Batch(outs, cols, sum(n for _, n in results))


# ------------------------------------------------------------------------------------------------
# joins
def _equi_keys(cond: Optional[A.Expr], lrefs, rrefs):
    lids = {r.rid for r in lrefs}
    rids = {r.rid for r in rrefs}
    keys = []
    rest = []
    for c in A.conjuncts(cond):
        if isinstance(c, A.BinOp) and c.op in ("=", "<=>"):
            lr = {x.rid for x in c.l.refs()}
            rr = {x.rid for x in c.r.refs()}
            if lr and rr and lr <= lids and rr <= rids:
                keys.append((c.l, c.r, c.op == "<=>"))
                continue
            if lr and rr and lr <= rids and rr <= lids:
                keys.append((c.r, c.l, c.op == "<=>"))
                continue
        rest.append(c)
    return keys, rest


def _key_series(exprs, b: Batch, subq) -> List[pd.Series]:
    fr = b.frame(subq)
    return [eval_series(e, fr) for e in exprs]


def _key_frame_of(series: List[pd.Series]) -> pd.DataFrame:
    d = {}
    for i, s in enumerate(series):
        d[f"k{i}"] = s.astype(object).where(s.notna(), None) if s.dtype.kind != "M" else s
    return pd.DataFrame(d)


def _key_frame(exprs, b: Batch, subq, null_safe):
    return _key_frame_of(_key_series(exprs, b, subq))


def join(p: P.Join, lb: Batch, rb: Batch, subq=None) -> Batch:
    keys, rest = _equi_keys(p.cond, lb.refs, rb.refs)
    kind = p.kind
    if keys:
        lks = _key_series([k[0] for k in keys], lb, subq)
        rks = _key_series([k[1] for k in keys], rb, subq)
        # SQL: NULL keys never match (unless <=>)
        lnull = np.zeros(lb.n, dtype=bool)
        rnull = np.zeros(rb.n, dtype=bool)
        for i, (_, _, ns) in enumerate(keys):
            if not ns:
                lnull |= lks[i].isna().to_numpy()
                rnull |= rks[i].isna().to_numpy()
        cols = [f"k{i}" for i in range(len(keys))]
        null_safe = any(ns for _, _, ns in keys)
        fast = None if null_safe else _numeric_key_join(lks, rks, ~lnull, ~rnull)
        if fast is not None:
            li, ri = fast
        else:
            lkf, rkf = _key_frame_of(lks), _key_frame_of(rks)
            lkf["_li"] = np.arange(lb.n)
            rkf["_ri"] = np.arange(rb.n)
            m = lkf[~lnull].merge(rkf[~rnull], on=cols, how="inner")
            li = m["_li"].to_numpy(dtype=np.int64)
            ri = m["_ri"].to_numpy(dtype=np.int64)
    else:
        li = np.repeat(np.arange(lb.n), rb.n)
        ri = np.tile(np.arange(rb.n), lb.n)
    if rest:
        both = _pair_batch(lb, rb, li, ri)
        m = evaluate(A.and_all(rest), both.frame(subq))
        ok = m.fillna(False).to_numpy(dtype=bool) if is_vec(m) else np.full(len(li), bool(m))
        li, ri = li[ok], ri[ok]
    if kind in ("inner", "cross"):
        return _pair_batch(lb, rb, li, ri)
    if kind == "leftsemi":
        return lb.take(np.unique(li))
    if kind == "leftanti":
        keep = np.ones(lb.n, dtype=bool)
        keep[li] = False
        return lb.take(np.nonzero(keep)[0])
    # outer joins: matched pairs + unmatched rows padded with NULL
    extra_l = np.setdiff1d(np.arange(lb.n), li) if kind in ("left", "full") else np.zeros(0, dtype=np.int64)
    extra_r = np.setdiff1d(np.arange(rb.n), ri) if kind in ("right", "full") else np.zeros(0, dtype=np.int64)
    out = _pair_batch(lb, rb, li, ri)
    parts = [out]
    if len(extra_l):
        parts.append(_pair_batch(lb, rb, extra_l, None))
    if len(extra_r):
        parts.append(_pair_batch(lb, rb, None, extra_r))
    refs = lb.refs + rb.refs
    cols = {r.rid: pd.concat([pb.cols[r.rid] for pb in parts], ignore_index=True) for r in refs}
    return Batch(refs, cols, sum(pb.n for pb in parts))


def _numeric_key_join(lks, rks, lok: np.ndarray, rok: np.ndarray):
    """Inner equi-join indices for numpy-numeric key columns (the aggregated Druid results joined
    on the host: TPC-H Q2 part x min-cost, Q17 part x avg-quantity): keys are factorized jointly
    into one int64 code, the right side is sorted once and every left row finds its match range
    with a binary search.  Output pairs are in left-row order (like pandas' inner merge).  None
    when a key is not a plain numeric column."""
    def plain(x: pd.Series):
        dt = x.dtype
        if isinstance(dt, np.dtype):
            return x.to_numpy() if dt.kind in "iuf" else None
        kind = getattr(getattr(dt, "numpy_dtype", None), "kind", "")
        if kind in "iu" and kind:  # nullable Int64 (NULL rows are masked out by the caller)
            return x.to_numpy(dtype=np.int64, na_value=0)
        if kind == "f":
            return x.to_numpy(dtype=np.float64, na_value=np.nan)
        return None

    arrs = []
    for a, b in zip(lks, rks):
        x, y = plain(a), plain(b)
        if x is None or y is None:
            return None
        arrs.append((x, y))
    li_all = np.nonzero(lok)[0]
    ri_all = np.nonzero(rok)[0]
    if len(li_all) + len(ri_all) >= _DEVICE_JOIN_MIN:
        out = _numeric_key_join_device(arrs, li_all, ri_all)
        if out is not None:
            return out
    lc = np.zeros(len(li_all), dtype=np.int64)
    rc = np.zeros(len(ri_all), dtype=np.int64)
    span = 1
    for a, b in arrs:
        x, y = a[li_all], b[ri_all]
        if x.dtype.kind == "f" or y.dtype.kind == "f":
            x, y = x.astype(np.float64), y.astype(np.float64)
        else:
            x, y = x.astype(np.int64), y.astype(np.int64)
        u, inv = np.unique(np.concatenate([x, y]), return_inverse=True)
        if span * max(1, len(u)) >= 2 ** 62:
            return None
        lc += inv[:len(x)] * span
        rc += inv[len(x):] * span
        span *= max(1, len(u))
    order = np.argsort(rc, kind="stable")
    rs = rc[order]
    lo = np.searchsorted(rs, lc, "left")
    cnt = np.searchsorted(rs, lc, "right") - lo
    tot = int(cnt.sum())
    li = np.repeat(li_all, cnt)
    start = np.repeat(lo - (np.cumsum(cnt) - cnt), cnt)
    ri = ri_all[order[start + np.arange(tot)]]
    return li, ri


_DEVICE_JOIN_MIN = 1 << 16


def _numeric_key_join_device(arrs, li_all: np.ndarray, ri_all: np.ndarray):
    """The same join on the GPU (torch radix sorts instead of numpy's single-threaded ones: TPC-H
    Q2 / Q17 join ~0.5M aggregated rows, 15 ms on the host).  None without a GPU."""
    import torch

    if not torch.cuda.is_available():
        return None
    dev = torch.device("cuda", torch.cuda.current_device())
    if len(arrs) == 1:
        out = _unique_right_join_device(arrs[0], li_all, ri_all, dev)
        if out is not None:
            return out
    nl = len(li_all)
    lc = torch.zeros(nl, dtype=torch.int64, device=dev)
    rc = torch.zeros(len(ri_all), dtype=torch.int64, device=dev)
    span = 1
    for a, b in arrs:
        x, y = a[li_all], b[ri_all]
        if x.dtype.kind == "f" or y.dtype.kind == "f":
            t = torch.from_numpy(np.concatenate([x.astype(np.float64), y.astype(np.float64)])).to(dev)
        else:
            t = torch.from_numpy(np.concatenate([x.astype(np.int64), y.astype(np.int64)])).to(dev)
        u, inv = torch.unique(t, return_inverse=True)
        if span * max(1, int(u.numel())) >= 2 ** 62:
            return None
        lc += inv[:nl] * span
        rc += inv[nl:] * span
        span *= max(1, int(u.numel()))
    rs, order = torch.sort(rc, stable=True)
    lo = torch.searchsorted(rs, lc, right=False)
    cnt = torch.searchsorted(rs, lc, right=True) - lo
    tot = int(cnt.sum())
    li_t = torch.from_numpy(li_all).to(dev)
    ri_t = torch.from_numpy(ri_all).to(dev)
    li = torch.repeat_interleave(li_t, cnt)
    start = torch.repeat_interleave(lo - (torch.cumsum(cnt, 0) - cnt), cnt)
    ri = ri_t[order[start + torch.arange(tot, device=dev)]]
    return li.cpu().numpy(), ri.cpu().numpy()


_DIRECT_JOIN_SPAN = 1 << 26


def _unique_right_join_device(arr, li_all: np.ndarray, ri_all: np.ndarray, dev):
    """One integer key, unique on the right (a pushed group-by's result joined on its own key: TPC-H
    Q17's part x avg-quantity): a direct-address table over the key range instead of sorts -- one
    scatter of the right rows' positions, one gather per left row.  None when the keys are not
    integers, their range exceeds _DIRECT_JOIN_SPAN, or the right keys repeat."""
    import torch

    a, b = arr
    if a.dtype.kind not in "iu" or b.dtype.kind not in "iu" or not len(ri_all) or not len(li_all):
        return None
    x = torch.from_numpy(np.ascontiguousarray(a[li_all], dtype=np.int64)).to(dev)
    y = torch.from_numpy(np.ascontiguousarray(b[ri_all], dtype=np.int64)).to(dev)
    lo, hi, ylo, yhi = (int(v) for v in torch.stack([x.min(), x.max(), y.min(), y.max()]).tolist())
    lo, hi = min(lo, ylo), max(hi, yhi)
    span = hi - lo + 1
    if span > _DIRECT_JOIN_SPAN:
        return None
    pos = torch.full((span,), -1, dtype=torch.int64, device=dev)
    cnt = torch.zeros(span, dtype=torch.int32, device=dev)
    cnt.index_add_(0, y - lo, torch.ones_like(y, dtype=torch.int32))
    pos.index_copy_(0, y - lo, torch.arange(len(y), dtype=torch.int64, device=dev))
    r = pos.index_select(0, x - lo)
    hit = r >= 0
    li = torch.nonzero(hit).flatten()
    ri = r.index_select(0, li)
    if int(cnt.max()) > 1:
        return None  # (repeated right keys: the general join pairs them all)
    return li_all[li.cpu().numpy()], ri_all[ri.cpu().numpy()]


def _pair_batch(lb: Batch, rb: Batch, li, ri) -> Batch:
    n = len(li) if li is not None else len(ri)
    li = np.asarray(li, dtype=np.int64) if li is not None else None
    ri = np.asarray(ri, dtype=np.int64) if ri is not None else None
    cols = {}
    for r in lb.refs:
        cols[r.rid] = _lazy_take(lb.cols.raw(r.rid), li) if li is not None else broadcast(None, n, r.dtype)
    for r in rb.refs:
        cols[r.rid] = _lazy_take(rb.cols.raw(r.rid), ri) if ri is not None else broadcast(None, n, r.dtype)
    return Batch(lb.refs + rb.refs, cols, n)
