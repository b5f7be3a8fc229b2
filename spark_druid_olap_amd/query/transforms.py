"""QuerySpec-to-QuerySpec rewrites run after planning (fixed-point batches).

Parity with ``sd/query/QuerySpecTransforms.scala:29-344``:
  * dimensionQueries: GroupBy on one dimension with no aggregates over the whole datasource ->
    Search (optionally lexicographically sorted + limited); add a ``count`` aggregate to metric-less
    GroupBys; merge ``lower`` and ``upper`` bounds on one dimension into a single between-bound.
  * combineSpatialFilters: AND-ed rectangular filters on one spatial dimension intersect.
  * timeseries: GroupBy with no dimensions, no having, no limit -> Timeseries(granularity all).
  * topN: one default dimension + a single order-by on a metric + limit below
    ``topNMaxThreshold`` (when ``allowTopNRewrite``) -> TopN with ``minTopNThreshold`` in context.
"""
from __future__ import annotations

from typing import Callable, List, Optional

from . import spec as S


def _merge_between(f):
    """AND of a lower and an upper bound on one dimension -> one between-bound.  The reference only
    merges 2-element ANDs; any such pair inside an AND is merged here."""
    if isinstance(f, S.LogicalFilterSpec):
        fields = [_merge_between(x) for x in f.fields]
        if f.type == "and":
            out = []
            for x in fields:
                merged = False
                if isinstance(x, S.BoundFilterSpec):
                    for i, y in enumerate(out):
                        if isinstance(y, S.BoundFilterSpec) and y.dimension == x.dimension and \
                                y.alphaNumeric == x.alphaNumeric:
                            lo, hi = (y, x) if y.lower is not None and y.upper is None else (x, y)
                            if lo.lower is not None and lo.upper is None and hi.upper is not None and hi.lower is None:
                                out[i] = S.BoundFilterSpec(lo.dimension, lo.lower, hi.upper, lo.lowerStrict,
                                                           hi.upperStrict, lo.alphaNumeric)
                                merged = True
                                break
                if not merged:
                    out.append(x)
            if len(out) == 1:
                return out[0]
            return S.LogicalFilterSpec("and", out)
        return S.LogicalFilterSpec(f.type, fields)
    if isinstance(f, S.NotFilterSpec):
        return S.NotFilterSpec(_merge_between(f.field))
    return f


def _combine_spatial(f):
    if isinstance(f, S.LogicalFilterSpec):
        fields = [_combine_spatial(x) for x in f.fields]
        if f.type == "and":
            flat = []
            for x in fields:
                if isinstance(x, S.LogicalFilterSpec) and x.type == "and":
                    flat += x.fields
                else:
                    flat.append(x)
            spatial = {}
            rest = []
            for x in flat:
                if isinstance(x, S.SpatialFilterSpec):
                    if x.dimension in spatial:
                        spatial[x.dimension] = _intersect_rect(spatial[x.dimension], x)
                    else:
                        spatial[x.dimension] = x
                else:
                    rest.append(x)
            out = list(spatial.values()) + rest
            if len(out) == 1:
                return out[0]
            return S.LogicalFilterSpec("and", out)
        return S.LogicalFilterSpec(f.type, fields)
    if isinstance(f, S.NotFilterSpec):
        return S.NotFilterSpec(_combine_spatial(f.field))
    return f


def _intersect_rect(a: S.SpatialFilterSpec, b: S.SpatialFilterSpec) -> S.SpatialFilterSpec:
    amin, amax = a.bound["minCoords"], a.bound["maxCoords"]
    bmin, bmax = b.bound["minCoords"], b.bound["maxCoords"]
    mn = [max(x, y) for x, y in zip(amin, bmin)]
    mx = [min(x, y) for x, y in zip(amax, bmax)]
    return S.SpatialFilterSpec(a.dimension, {"type": "rectangular", "minCoords": mn, "maxCoords": mx})


class TransformContext:
    def __init__(self, allow_topn: bool = False, topn_max: int = 100000,
                 covers_all: Optional[Callable[[S.QuerySpec], bool]] = None,
                 metric_is_numeric: Optional[Callable[[str], bool]] = None):
        self.allow_topn = allow_topn
        self.topn_max = topn_max
        self.covers_all = covers_all or (lambda q: False)
        self.metric_is_numeric = metric_is_numeric or (lambda m: True)


def search_transform(q, ctx: TransformContext):
    if not isinstance(q, S.GroupByQuerySpec) or q.aggregations or q.having is not None or q.postAggregations:
        return q
    if len(q.dimensions) != 1 or not isinstance(q.dimensions[0], S.DefaultDimensionSpec):
        return q
    d = q.dimensions[0]
    if d.dimension != d.outputName or not ctx.covers_all(q):
        return q
    ls = q.limitSpec
    if ls is None:
        return S.SearchQuerySpec(q.dataSource, q.intervals, q.granularity, q.filter, [d.dimension],
                                 S.SearchQueryQuerySpec("insensitive_contains", ""), 2 ** 31 - 1, None, q.context)
    cols = ls.columns or []
    if len(cols) == 1 and cols[0].dimension == d.dimension and cols[0].direction == "ascending":
        return S.SearchQuerySpec(q.dataSource, q.intervals, q.granularity, q.filter, [d.dimension],
                                 S.SearchQueryQuerySpec("insensitive_contains", ""), ls.limit,
                                 {"type": "lexicographic"}, q.context)
    return q


def add_count(q, ctx):
    if isinstance(q, S.GroupByQuerySpec) and not q.aggregations:
        return q.copy(aggregations=[S.FunctionAggregationSpec("count", "addCountAggForNoMetricQuery", "count")])
    return q


def between(q, ctx):
    f = getattr(q, "filter", None)
    if f is None:
        return q
    return q.setFilter(_merge_between(f))


def spatial(q, ctx):
    f = getattr(q, "filter", None)
    if f is None:
        return q
    return q.setFilter(_combine_spatial(f))


def timeseries(q, ctx):
    if isinstance(q, S.GroupByQuerySpec) and not q.dimensions and q.having is None and q.limitSpec is None \
            and not isinstance(q.dataSource, S.QueryDataSourceSpec):  # nested levels stay groupBys
        return S.TimeSeriesQuerySpec(q.dataSource, q.intervals, False, S.Granularity.parse("all"), q.filter,
                                     q.aggregations, q.postAggregations, q.context)
    return q


def topn(q, ctx):
    if not isinstance(q, S.GroupByQuerySpec) or not ctx.allow_topn or q.having is not None:
        return q
    if len(q.dimensions) != 1 or not isinstance(q.dimensions[0], S.DefaultDimensionSpec):
        return q
    ls = q.limitSpec
    if ls is None or ls.limit is None or len(ls.columns or []) != 1 or ls.limit >= ctx.topn_max:
        return q
    d = q.dimensions[0]
    oc = ls.columns[0]
    if oc.dimension == d.outputName:
        return q
    numeric = ctx.metric_is_numeric(oc.dimension)
    if numeric:
        m = S.NumericTopNMetricSpec(oc.dimension)
    else:
        m = S.LexiCographicTopNMetricSpec(oc.dimension)
    if oc.direction == "ascending":
        m = S.InvertedTopNMetricSpec(m)
    ctx_ = q.context.copy(minTopNThreshold=ls.limit) if q.context is not None else \
        S.QuerySpecContext(minTopNThreshold=ls.limit)
    return S.TopNQuerySpec(q.dataSource, d, m, ls.limit, q.intervals, q.granularity, q.filter, q.aggregations,
                           q.postAggregations, ctx_)


BATCHES = [
    ("dimensionQueries", 100, [search_transform, add_count, between]),
    ("combineSpatialFilters", 100, [spatial]),
    ("timeseries", 1, [timeseries]),
    ("topN", 1, [topn]),
]


def transform(q: S.QuerySpec, ctx: TransformContext) -> S.QuerySpec:
    for _name, max_iter, fns in BATCHES:
        for _ in range(max_iter):
            before = q
            for fn in fns:
                q = fn(q, ctx)
            # fixpoint: rules return their input when they do not apply; otherwise compare the
            # specs field by field (dataclass equality -- no JSON rendering per iteration)
            if q is before or q == before:
                break
    return q
