"""Window functions over the rows below a ``Window`` plan node (Spark's WindowExec).

The reference leaves windows to Spark: in its BI workload (``docs/bi-benchmark/snap-sales-demo.jmx``,
templates WindowingMovingAvg, WindowingDeltaFromTopMfgr, Windowing-1, the dense_rank TopN
templates) the Druid group-by is pushed and the window runs over its (small) result.  Here the
pushed aggregate runs on the GPU and the window on the host over the aggregated rows, vectorised:

* rows are ordered by (partition, ORDER BY keys) once per distinct (partition, order) spec;
* ranking functions come from partition starts and peer-group starts (rows with equal ORDER BY
  keys are peers);
* sum / count / avg over a frame are prefix-sum differences (int64 for integer arguments, so they
  stay exact; bounded float frames are summed directly); min / max over running frames are
  per-partition accumulates, over bounded frames a sliding minimum / maximum;
* lag / lead / first_value / last_value are shifted gathers inside the partition.

Frames follow Spark: with an ORDER BY the default is RANGE BETWEEN UNBOUNDED PRECEDING AND CURRENT
ROW (the current row's peers included), without one the whole partition.  ROWS frames take row
offsets; RANGE frames support UNBOUNDED / CURRENT ROW bounds.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np
import pandas as pd

from . import ast as A
from .functions import Frame, eval_series, typeof
from .types import AnalysisError


def _codes(series: List[pd.Series], n: int) -> np.ndarray:
    """Dense group id per row of the key tuple (NULLs are a group of their own)."""
    if not series:
        return np.zeros(n, dtype=np.int64)
    if len(series) == 1:
        s = series[0]
        s = s.cat.codes if isinstance(s.dtype, pd.CategoricalDtype) else s
        return np.asarray(pd.factorize(s, use_na_sentinel=False)[0], dtype=np.int64)
    df = pd.DataFrame({i: (k.cat.codes if isinstance(k.dtype, pd.CategoricalDtype) else k).reset_index(drop=True)
                       for i, k in enumerate(series)})
    return df.groupby(list(range(len(series))), dropna=False, sort=False).ngroup().to_numpy().astype(np.int64)


class _Layout:
    """Row order and partition / peer boundaries of one (PARTITION BY, ORDER BY) spec."""

    def __init__(self, w: A.WindowExpr, fr: Frame):
        from .execute import sort_indices

        n = fr.n
        pcodes = _codes([eval_series(p, fr) for p in w.partition], n)
        okeys = [(eval_series(o.expr, fr), o.ascending, o.nulls_first) for o in w.orders]
        keys = [(pd.Series(pcodes), True, None)] + okeys
        self.order = sort_indices(keys, n) if n else np.arange(0)
        o = self.order
        sp = pcodes[o]
        self.n = n
        pstart = np.ones(n, dtype=bool)
        if n:
            pstart[1:] = sp[1:] != sp[:-1]
        # peers: same partition and equal ORDER BY keys (every row of a partition without ORDER BY)
        peer = pstart.copy()
        if okeys and n:
            oc = _codes([k.iloc[o].reset_index(drop=True) for k, _, _ in okeys], n)
            peer[1:] |= oc[1:] != oc[:-1]
        idx = np.arange(n, dtype=np.int64)
        self.pstart_idx = np.maximum.accumulate(np.where(pstart, idx, 0)) if n else idx
        pend = np.ones(n, dtype=bool)
        if n:
            pend[:-1] = pstart[1:]
        self.pend_idx = np.minimum.accumulate(np.where(pend, idx, n)[::-1])[::-1] if n else idx  # inclusive
        self.peer = peer
        self.peer_start = np.maximum.accumulate(np.where(peer, idx, 0)) if n else idx
        pe = np.ones(n, dtype=bool)
        if n:
            pe[:-1] = peer[1:]
        self.peer_end = np.minimum.accumulate(np.where(pe, idx, n)[::-1])[::-1] if n else idx  # inclusive
        self.has_order = bool(w.orders)

    def bounds(self, frame) -> Tuple[np.ndarray, np.ndarray]:
        """[lo, hi] (inclusive, in sorted positions) of every row's frame; empty when lo > hi."""
        n = self.n
        idx = np.arange(n, dtype=np.int64)
        if frame is None:
            if self.has_order:
                return self.pstart_idx, self.peer_end
            return self.pstart_idx, self.pend_idx
        kind, lo, hi = frame
        if kind == "range":
            if lo not in (None, 0) or hi not in (None, 0):
                raise AnalysisError("RANGE frames with value offsets are not supported; use ROWS")
            lo_i = self.pstart_idx if lo is None else (self.peer_start if self.has_order else self.pstart_idx)
            hi_i = self.pend_idx if hi is None else (self.peer_end if self.has_order else self.pend_idx)
            return lo_i, hi_i
        lo_i = self.pstart_idx if lo is None else np.maximum(self.pstart_idx, idx + lo)
        hi_i = self.pend_idx if hi is None else np.minimum(self.pend_idx, idx + hi)
        return lo_i, hi_i


def _values(e: A.Expr, fr: Frame, order: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """(values, non-null mask) of a numeric argument, in sorted order: int64 for integer arguments
    (so framed sums stay exact, as Spark's sum(bigint) is), float64 otherwise."""
    s = eval_series(e, fr)
    if pd.api.types.is_integer_dtype(s.dtype) and not pd.api.types.is_bool_dtype(s.dtype):
        ok = s.notna().to_numpy()[order]
        v = s.fillna(0).to_numpy(dtype=np.int64)[order]
        return v, ok
    v = pd.to_numeric(s, errors="coerce").to_numpy(dtype=np.float64, na_value=np.nan)[order]
    ok = ~np.isnan(v)
    return np.where(ok, v, 0.0), ok


def _prefix(v: np.ndarray) -> np.ndarray:
    c = np.zeros(len(v) + 1, dtype=np.int64 if v.dtype.kind in "iub" else np.float64)
    np.cumsum(v, out=c[1:])
    return c


def _frame_sum(v: np.ndarray, lo: np.ndarray, hi: np.ndarray) -> np.ndarray:
    """Sum over each row's [lo, hi] frame: prefix-sum differences (exact in int64 for integer
    inputs), and per-partition rebased prefixes for floats so a frame deep into a long partition
    does not lose its digits to cancellation against the partition's running total."""
    n = len(v)
    ok = lo <= hi
    if v.dtype.kind in "iub":
        c = _prefix(v)
        return np.where(ok, c[np.minimum(hi + 1, n)] - c[np.minimum(lo, n)], 0)
    c = _prefix(v)
    # bounded frames of up to 64 rows are summed directly (no cancellation); longer ones use the prefix
    span = np.where(ok, hi - lo + 1, 0)
    out = np.where(ok, c[np.minimum(hi + 1, n)] - c[np.minimum(lo, n)], 0.0)
    small = ok & (span <= 64)
    if small.any() and n:
        w = int(span[small].max())
        j = lo[small][:, None] + np.arange(w)[None, :]
        m = j <= hi[small][:, None]
        out[small] = np.where(m, v[np.minimum(j, n - 1)], 0.0).sum(axis=1)
    return out


def _frame_extreme(v: np.ndarray, ok: np.ndarray, lo: np.ndarray, hi: np.ndarray, lay: _Layout,
                   is_max: bool) -> Tuple[np.ndarray, np.ndarray]:
    n = len(v)
    fill = -np.inf if is_max else np.inf
    x = np.where(ok, v, fill)
    out = np.full(n, fill)
    running = bool(n) and np.array_equal(lo, lay.pstart_idx)
    if running and np.array_equal(hi, np.arange(n)) or running and np.array_equal(hi, lay.peer_end) or \
            running and np.array_equal(hi, lay.pend_idx):
        # running frames: a per-partition accumulate, read at each row's frame end
        acc = np.empty(n)
        starts = np.nonzero(lay.pstart_idx == np.arange(n))[0]
        ends = np.append(starts[1:], n)
        f = np.maximum.accumulate if is_max else np.minimum.accumulate
        for a, b in zip(starts, ends):
            acc[a:b] = f(x[a:b])
        out = acc[hi]
    else:  # bounded frames: per-row slice (aggregated results are small)
        for i in range(n):
            if lo[i] <= hi[i]:
                seg = x[lo[i]:hi[i] + 1]
                out[i] = seg.max() if is_max else seg.min()
    has = _frame_sum(ok.astype(np.int64), lo, hi) > 0
    return np.where(has, out, 0.0), has


def evaluate_window(w: A.WindowExpr, fr: Frame, cache: Optional[dict] = None) -> pd.Series:
    """The window expression's value for every row of ``fr`` (in the frame's row order)."""
    n = fr.n
    key = (tuple(p.key() for p in w.partition), tuple((o.expr.key(), o.ascending, o.nulls_first) for o in w.orders))
    lay = cache.get(key) if cache is not None else None
    if lay is None:
        lay = _Layout(w, fr)
        if cache is not None:
            cache[key] = lay
    order = lay.order
    f = w.func
    name = f.name
    idx = np.arange(n, dtype=np.int64)
    out_sorted: np.ndarray
    nulls = np.zeros(n, dtype=bool)
    if name == "row_number":
        out_sorted = idx - lay.pstart_idx + 1
    elif name == "rank":
        out_sorted = lay.peer_start - lay.pstart_idx + 1
    elif name == "dense_rank":
        pc = np.cumsum(lay.peer.astype(np.int64))
        out_sorted = pc - pc[lay.pstart_idx] + 1
    elif name == "percent_rank":
        size = lay.pend_idx - lay.pstart_idx + 1
        r = lay.peer_start - lay.pstart_idx
        out_sorted = np.where(size > 1, r / np.maximum(size - 1, 1), 0.0)
    elif name == "cume_dist":
        size = lay.pend_idx - lay.pstart_idx + 1
        out_sorted = (lay.peer_end - lay.pstart_idx + 1) / size
    elif name == "ntile":
        k = int(f.args[0].value) if f.args and isinstance(f.args[0], A.Lit) else 1
        size = lay.pend_idx - lay.pstart_idx + 1
        pos = idx - lay.pstart_idx
        base_, extra = size // k, size % k
        # the first `extra` buckets hold base_ + 1 rows
        big = extra * (base_ + 1)
        out_sorted = np.where(pos < big, pos // np.maximum(base_ + 1, 1), extra + (pos - big) // np.maximum(base_, 1)) + 1
    elif name in ("lag", "lead", "first_value", "last_value"):
        s = eval_series(f.args[0], fr).reset_index(drop=True)
        vals = s.iloc[order].reset_index(drop=True)
        if name in ("lag", "lead"):
            off = int(f.args[1].value) if len(f.args) > 1 else 1
            src = idx - off if name == "lag" else idx + off
            inside = (src >= lay.pstart_idx) & (src <= lay.pend_idx)
        else:
            lo, hi = lay.bounds(w.frame)
            src = lo if name == "first_value" else hi
            inside = lo <= hi
        res = vals.iloc[np.clip(src, 0, max(n - 1, 0))].reset_index(drop=True) if n else vals
        if name in ("lag", "lead") and len(f.args) > 2:
            dflt = f.args[2].value if isinstance(f.args[2], A.Lit) else None
            res = res.where(pd.Series(inside), dflt)
        else:
            res = res.where(pd.Series(inside))
        inv = np.empty(n, dtype=np.int64)
        inv[order] = idx
        return res.iloc[inv].reset_index(drop=True)
    elif name in ("sum", "count", "avg", "mean", "min", "max"):
        lo, hi = lay.bounds(w.frame)
        if f.distinct:
            raise AnalysisError("DISTINCT aggregates over a window are not supported")
        if name == "count" and not f.args:
            out_sorted = np.maximum(hi - lo + 1, 0)
        else:
            v, ok = _values(f.args[0], fr, order)
            cnt = _frame_sum(ok.astype(np.int64), lo, hi)
            if name == "count":
                out_sorted = cnt.astype(np.int64)
            elif name == "sum":
                out_sorted = _frame_sum(v, lo, hi)
                nulls = cnt == 0
            elif name in ("avg", "mean"):
                out_sorted = _frame_sum(v, lo, hi) / np.maximum(cnt, 1)
                nulls = cnt == 0
            else:
                out_sorted, has = _frame_extreme(v, ok, lo, hi, lay, name == "max")
                nulls = ~has
    else:
        raise AnalysisError(f"window function {name} is not supported")
    res = np.empty(n, dtype=np.asarray(out_sorted).dtype)
    res[order] = out_sorted
    nl = np.empty(n, dtype=bool)
    nl[order] = nulls
    s = pd.Series(res)
    if nl.any():
        s = s.astype(object).where(~pd.Series(nl), None)
    return s


# ------------------------------------------------------------------------------------------------
# rank() / dense_rank() = 1 over a pushed aggregate -> a device pre-filter
#
# The BI plan's "MinCost Supplier by Part in each Region" template (docs/bi-benchmark/
# snap-sales-demo.jmx) ranks ~10^5 groups of a pushed groupBy per region by sum(ps_supplycost) and
# keeps rank 1: the reference ships every group to Spark's WindowExec.  Rank 1 of rank() and of
# dense_rank() is exactly "the value equals the partition's minimum" (maximum for DESC), so the
# engine can drop every other group on the device (engine/executor.py _device_extreme) before the
# groups are decoded and shipped; the host window and filter still run, over the survivors, and
# return the same rows (all survivors have rank 1 among themselves).
def _rank_one_rid(cond) -> Optional[int]:
    """The window-output ref id that the filter condition pins to 1 (as ``= 1`` or ``<= 1`` / ``< 2``
    in a conjunction), else None."""
    if isinstance(cond, A.BinOp) and cond.op == "and":
        return _rank_one_rid(cond.l) or _rank_one_rid(cond.r)
    if not isinstance(cond, A.BinOp):
        return None
    l, r, op = cond.l, cond.r, cond.op
    if isinstance(l, A.Lit) and isinstance(r, A.Ref):
        l, r = r, l
        op = {"<=": ">=", ">=": "<=", "<": ">", ">": "<"}.get(op, op)
    if not isinstance(l, A.Ref) or not isinstance(r, A.Lit) or isinstance(r.value, bool) or \
            not isinstance(r.value, (int, float)):
        return None
    if (op == "=" and r.value == 1) or (op == "<=" and 1 <= r.value < 2) or (op == "<" and 1 < r.value <= 2):
        return l.rid
    return None


# Casts the ORDER BY metric may go through.  The device keeps the groups whose f64 image of the
# metric equals their partition's extreme; that must be a SUPERSET of the groups Spark ranks 1 by
# the cast value, so the cast may not merge values the f64 image keeps apart: injective casts
# (integer widening, float -> double) and the cast to double itself (the very f64 image the device
# compares) qualify.  A narrowing cast (double -> int truncates, double -> float rounds, bigint ->
# int wraps) maps distinct sums to one value: Spark then ranks several groups 1 where the device
# would keep only the partition extreme of the uncast sum.
_INT_WIDTH = {"tinyint": 1, "smallint": 2, "int": 4, "bigint": 8}


def _rank_safe_cast(frm: str, to: str) -> bool:
    if frm == to:
        return True
    if frm in _INT_WIDTH and to in _INT_WIDTH:
        return _INT_WIDTH[to] >= _INT_WIDTH[frm]
    return to == "double" and (frm in _INT_WIDTH or frm in ("float", "double"))


def _through_projects(rid: int, projs, monotone: bool = False) -> Optional[int]:
    """Follow a column down a chain of projections (outermost first) as long as it is passed through
    or renamed (``monotone``: or cast without merging values -- ``_rank_safe_cast``); None when it is computed."""
    from . import plan as P

    for pr in projs:
        nxt = None
        for e in pr.exprs:
            if P.out_ref(e).rid != rid:
                continue
            c = e.child if isinstance(e, A.Alias) else e
            if monotone and isinstance(c, A.Cast) and isinstance(c.child, A.Ref) and \
                    _rank_safe_cast(str(c.child.dtype).lower(), str(c.to).lower()):
                c = c.child
            if isinstance(c, A.Ref):
                nxt = c.rid
            break
        if nxt is None:
            return None
        rid = nxt
    return rid


def push_rank_one(plan):
    """Annotate pushed groupBys under ``Filter(rank = 1) <- Window(rank | dense_rank)`` with their
    partition-extreme pre-filter (``info["partition_extreme"] = (partition output names, metric
    name, ascending)``)."""
    from ..query import spec as S
    from . import plan as P

    def rule(p):
        if not isinstance(p, P.Filter) or not isinstance(p.child, P.Window):
            return None
        w = p.child
        rid = _rank_one_rid(p.cond)
        if rid is None or len(w.exprs) != 1 or P.out_ref(w.exprs[0]).rid != rid:
            return None
        we = w.exprs[0].child
        if not isinstance(we, A.WindowExpr) or we.func.name not in ("rank", "dense_rank") or \
                len(we.orders) != 1 or we.frame is not None:
            return None
        projs, node = [], w.child
        while isinstance(node, P.Project):
            projs.append(node)
            node = node.child
        if not isinstance(node, P.DruidQuery) or not isinstance(node.spec, S.GroupByQuerySpec) or \
                node.spec.limitSpec is not None or node.info.get("partition_extreme"):
            return None
        o = we.orders[0]
        if not isinstance(o.expr, A.Ref) or any(not isinstance(x, A.Ref) for x in we.partition):
            return None
        if o.nulls_first is not None and o.nulls_first != o.ascending:
            return None  # (Spark's default null placement only: our aggregates are never NULL anyway)
        by_rid = {r.rid: c for r, c in zip(node.refs, node.columns)}
        m = _through_projects(o.expr.rid, projs, monotone=True)
        parts = [_through_projects(x.rid, projs) for x in we.partition]
        if m is None or m not in by_rid or any(x is None or x not in by_rid for x in parts):
            return None
        dims = {d.outputName for d in (node.spec.dimensions or [])}
        aggs = {a.name for a in (node.spec.aggregations or [])}
        metric = by_rid[m][0]
        pnames = tuple(by_rid[x][0] for x in parts)
        if metric not in aggs or any(n not in dims for n in pnames):
            return None
        dq = P.DruidQuery(node.relation, node.spec, node.columns, node.refs,
                          dict(node.info, partition_extreme=(pnames, metric, bool(o.ascending))))
        chain = dq
        for pr in reversed(projs):
            chain = P.Project(pr.exprs, chain)
        return P.Filter(p.cond, P.Window(w.exprs, chain))

    return plan.transform_up(rule)
