"""Nested groupBy (Druid query data source) executed on the device.

The outer groupBy of ``{"dataSource": {"type": "query", "query": <inner groupBy>}}`` aggregates the
inner query's result rows.  Druid brokers run the outer level over the merged inner results; the
reference never issues nested queries (its Spark plans aggregate the Druid rows again on the
executors, ``asd/PostAggregate.scala``).  Here the inner query's merged partials never leave HBM:
key components are decoded to dictionary ids on the device, the outer keys are packed and
grouped with ``torch.unique``, and the outer aggregates reduce with scatter ops -- TPC-H Q13's
150M (customer, order) groups at SF100 collapse to ~40 rows before anything is copied to the host.

Outer dimensions name inner output columns (inner dimensions, or inner aggregates used as keys:
Q13 groups customers by their order count); outer aggregators are count / long|double
Sum|Min|Max over inner columns.  Outer having / limitSpec / postAggregations run like any other
query's (executor._post).
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ops import desc as D

from ..query import spec as S
from ..segment.datasource import DataSource
from .lower import LoweringError


_TRACE = False  # (tools: print the nested-level plans)


class DeviceColumn:
    """One inner output column on the device.  ``ids`` (int64) for dimensions with ``decode``
    (ids -> values); ``vals`` (int64 with decimal ``scale``, or float64) for aggregates."""

    def __init__(self, name: str, t: torch.Tensor, decode: Optional[Callable] = None, scale: int = 0,
                 card: Optional[int] = None):
        self.name = name
        self.t = t
        self.decode = decode
        self.scale = scale
        self.card = card  # key ids are known to lie in [0, card) (no min/max pass needed)
        self.num: Optional[Tuple[int, int]] = None  # integral key: value = (id + base) / 10^scale

    @property
    def is_float(self) -> bool:
        return self.t.dtype == torch.float64

    def as_float(self) -> torch.Tensor:
        if self.is_float:
            return self.t
        v = self.t.to(torch.float64)
        return v / (10.0 ** self.scale) if self.scale else v

    def host_values(self, t: torch.Tensor) -> np.ndarray:
        h = t.cpu().numpy()
        if self.decode is not None:
            return self.decode(h)
        if self.is_float:
            return h
        return h / (10.0 ** self.scale) if self.scale else h


def device_columns(pq) -> Tuple[Dict[str, DeviceColumn], int]:
    """Run a (non-nested) groupBy PreparedQuery up to its merged partials and expose every output
    column as a device tensor.  Returns (columns, row count)."""
    t0 = time.perf_counter()
    prog, part, _ = pq.run_partials(t0)
    if _TRACE:
        torch.cuda.synchronize()
        print(f"[nested] inner scan+merge {(time.perf_counter() - t0) * 1e3:.2f} ms mode="
              f"{getattr(pq.scans[0][2], 'mode', None)} G={prog.G} rows={part.rows}", flush=True)
    if prog.thetas or any(kc.collapse for kc in prog.keys):
        raise LoweringError("nested query over theta sketches / non-injective keys")
    if part.kind == "dense":
        part = part.compact()
    g = part.keys
    dev = part.acc.device
    cols: Dict[str, DeviceColumn] = {}
    ids_of = []
    G = int(prog.G)
    for kc in prog.keys:
        # (150M-group inner levels: each elementwise pass over the keys is ~0.4 ms -- skip the
        # divide / remainder a key's position in the packed key does not need)
        if kc.stride == 1 and kc.card >= G:
            ids = g  # the only (or a G-spanning lowest) key: the packed key is its id
        elif kc.stride * max(1, kc.card) >= G:
            ids = torch.div(g, kc.stride, rounding_mode="floor")  # the leading key: no wrap-around
        else:
            ids = torch.remainder(torch.div(g, kc.stride, rounding_mode="floor"), max(1, kc.card))
        ids_of.append(ids)
        cols[kc.name] = DeviceColumn(kc.name, ids, kc.decoder if kc.decoder is not None else (lambda x: x),
                                     card=max(1, kc.card))
        if kc.kind == D.K_INT and kc.col in pq.ds.metrics:
            m = pq.ds.metrics[kc.col]
            cols[kc.name].num = (int(kc.base), m.scale if m.kind == "decimal" else 0)
    for kc, det, lut in getattr(prog, "derived", ()):
        did = ids_of[det]
        orig = prog.keys[det].orig
        if orig is not None:
            did = torch.from_numpy(orig).to(dev)[did]
        ids = lut.to(dev)[did].to(torch.int64)
        cols[kc.name] = DeviceColumn(kc.name, ids, kc.decoder if kc.decoder is not None else (lambda x: x),
                                     card=max(1, kc.card))
    for a, det, lut in getattr(prog, "derived_aggs", ()):
        did = ids_of[det]
        orig = prog.keys[det].orig
        if orig is not None:
            did = torch.from_numpy(orig).to(dev)[did]
        cols[a.name] = DeviceColumn(a.name, lut.to(dev)[did], scale=a.scale)
    for a in prog.aggs:
        if a.name in cols:
            continue
        col = part.acc[:, a.slot] if a.slot >= 0 else None
        if a.kind in ("count", "min_i", "max_i"):
            cols[a.name] = DeviceColumn(a.name, col, scale=a.scale)
        elif a.kind == "sum_i":
            cols[a.name] = DeviceColumn(a.name, col, scale=a.scale)
        elif a.kind == "sum_f":
            cols[a.name] = DeviceColumn(a.name, col.contiguous().view(torch.float64))
        elif a.kind == "sum_fx":
            from .lower import fixed_value

            cols[a.name] = DeviceColumn(a.name, fixed_value(col, part.acc[:, a.slot2]))
        elif a.kind in ("min_f", "max_f"):
            cols[a.name] = DeviceColumn(a.name, torch.where(col >= 0, col, col ^ 0x7FFFFFFFFFFFFFFF).view(torch.float64))
        else:
            raise LoweringError(f"nested query over a {a.kind} aggregate")
    return cols, int(part.acc.shape[0])


def _torch_eval(n, pmap: Dict[str, str], cols: Dict[str, DeviceColumn]) -> torch.Tensor:
    """f64 value per inner row of a javascript-aggregator expression AST (query/jsfunc.parse_expr)."""
    k = n[0]
    if k == "const":
        return torch.tensor(float(n[1]), dtype=torch.float64)
    if k == "col":
        c = cols.get(pmap.get(n[1], n[1]))
        if c is None:
            raise LoweringError(f"nested expression over unknown column {n[1]!r}")
        if c.num is not None:  # grouped integral metric: key id -> stored value
            v = (c.t + c.num[0]).to(torch.float64)
            return v / (10.0 ** c.num[1]) if c.num[1] else v
        return c.as_float() if c.decode is None else c.t.to(torch.float64)
    if k in ("neg", "abs", "floor", "ceil", "sqrt", "log", "exp"):
        a = _torch_eval(n[1], pmap, cols)
        return {"neg": torch.neg, "abs": torch.abs, "floor": torch.floor, "ceil": torch.ceil, "sqrt": torch.sqrt,
                "log": torch.log, "exp": torch.exp}[k](a)
    a, b = _torch_eval(n[1], pmap, cols), _torch_eval(n[2], pmap, cols)
    if a.device != b.device:
        a, b = a.to(b.device) if a.dim() == 0 else a, b.to(a.device) if b.dim() == 0 else b
    fns = {"add": torch.add, "sub": torch.sub, "mul": torch.mul, "div": torch.div, "min": torch.minimum,
           "max": torch.maximum, "mod": torch.fmod, "pow": torch.pow}
    if k not in fns:
        raise LoweringError(f"nested expression operator {k}")
    return fns[k](a, b)


def _nonzero(t: torch.Tensor) -> torch.Tensor:
    """Indices of the non-zero entries (native ballot + compaction kernels on the GPU)."""
    if t.is_cuda and t.dtype == torch.int64:
        from ..ops import native

        return native.nonzero_rows(t)
    return torch.nonzero(t).flatten()


def _histogram(keys: torch.Tensor, nbins: int) -> torch.Tensor:
    """Per-bin counts (native 32-bit-atomic histogram kernel on the GPU)."""
    if keys.is_cuda:
        from ..ops import native

        return native.histogram(keys.contiguous(), nbins)
    return torch.bincount(keys, minlength=nbins)


def _group_sum(R: int, inv: Optional[torch.Tensor], src: torch.Tensor, deterministic: bool) -> torch.Tensor:
    """Per-group sum of ``src`` rows (group ``inv``; None = one global group, reduced with a tree
    reduction instead of a million atomics on one address).  Deterministic float sums go through
    the same 64.32 fixed point as the scan (engine/lower.py fixed_sum): integer sums are
    order-free."""
    if inv is None:
        if not deterministic or src.dtype != torch.float64:
            return src.sum().reshape(1).to(src.dtype)
        from .lower import FIX_ONE, fixed_value

        fl = torch.floor(src)
        return fixed_value(fl.to(torch.int64).sum().reshape(1),
                           torch.round((src - fl) * FIX_ONE).to(torch.int64).sum().reshape(1))
    if not deterministic or src.dtype != torch.float64:
        return torch.zeros(R, dtype=src.dtype, device=src.device).index_add_(0, inv, src)
    from .lower import FIX_ONE, fixed_value

    fl = torch.floor(src)
    hi = torch.zeros(R, dtype=torch.int64, device=src.device).index_add_(0, inv, fl.to(torch.int64))
    lo = torch.zeros(R, dtype=torch.int64, device=src.device).index_add_(
        0, inv, torch.round((src - fl) * FIX_ONE).to(torch.int64))
    return fixed_value(hi, lo)


class NestedPreparedQuery:
    """groupBy over a query data source (see module doc)."""

    def __init__(self, engine, qs: S.GroupByQuerySpec, ds: DataSource, segments_per_query: Optional[int] = None):
        if qs.queryType != "groupBy":
            raise LoweringError("only groupBy runs over a query data source")
        if qs.filter is not None and not isinstance(qs.filter, S.NoopFilterSpec):
            raise LoweringError("filters on a nested groupBy are not supported")
        self.engine = engine
        self.qs = qs
        self.ds = ds
        self.world = engine.world
        inner_q = qs.dataSource.query
        if isinstance(inner_q, S.GroupByQuerySpec) and not isinstance(inner_q.dataSource, S.QueryDataSourceSpec):
            # inner aggregates the outer level never reads are not computed; with none left the
            # inner scan only records which groups exist (Q13: 600M lines -> order existence)
            used = {d.dimension for d in qs.dimensions}
            for a in qs.aggregations:
                used.add(getattr(a, "fieldName", None))
                used.update(getattr(a, "fieldNames", None) or [])
            keep = [a for a in (inner_q.aggregations or []) if a.name in used]
            if len(keep) != len(inner_q.aggregations or []) and not inner_q.postAggregations and \
                    inner_q.having is None and inner_q.limitSpec is None:
                inner_q = inner_q.copy(aggregations=keep)
        ctx = getattr(qs, "context", None)
        self.deterministic = bool(engine.deterministic or (ctx is not None and getattr(ctx, "deterministic", None)))
        if self.deterministic and not engine.deterministic:
            ictx = getattr(inner_q, "context", None)
            inner_q = inner_q.copy(context=ictx.copy(deterministic=True) if ictx is not None
                                   else S.QuerySpecContext(deterministic=True))
        self.inner = engine.prepare(inner_q, ds, segments_per_query, key_passes=False)
        for d in qs.dimensions:
            if not isinstance(d, S.DefaultDimensionSpec):
                raise LoweringError("nested groupBy dimensions must be default dimension specs")
        self._js = {}
        for a in qs.aggregations:
            if isinstance(a, S.JavascriptAggregationSpec):
                from ..query.jsfunc import JSError, jsagg_to_expr, parse_expr

                try:
                    op, params, expr = jsagg_to_expr(a.fnAggregate)
                    self._js[a.name] = (op, dict(zip(params, a.fieldNames)), parse_expr(expr))
                except JSError as e:
                    raise LoweringError(f"nested javascript aggregator not translatable: {e}")
                continue
            if not (isinstance(a, S.FunctionAggregationSpec) and
                    a.type in ("count", "longSum", "doubleSum", "longMin", "longMax", "doubleMin", "doubleMax")):
                raise LoweringError(f"nested groupBy aggregator {type(a).__name__}")

    # ------------------------------------------------------------------ run
    def _compute(self) -> Tuple[Dict[str, DeviceColumn], int, float]:
        """Outer groups on the device: (columns by output name, row count, inner time ms)."""
        t0 = time.perf_counter()
        inner = self.inner
        if isinstance(inner, NestedPreparedQuery):
            cols, n = inner.device_result()
        else:
            cols, n = device_columns(inner)
        if _TRACE:
            torch.cuda.synchronize()
        inner_ms = (time.perf_counter() - t0) * 1e3
        qs = self.qs
        dev = next(iter(cols.values())).t.device if cols else self.ds.device
        # ---- outer keys: pack inner columns (ids / integral values) into one int64
        keycols = []
        for d in qs.dimensions:
            c = cols.get(d.dimension)
            if c is None:
                raise LoweringError(f"nested dimension {d.dimension!r} is not an inner output")
            if c.is_float:
                raise LoweringError(f"nested dimension {d.dimension!r} is floating point")
            keycols.append((d, c))
        dense_counts = None
        if n == 0:
            inv = torch.zeros(0, dtype=torch.int64, device=dev)
            R = 0
            firsts = torch.zeros(0, dtype=torch.int64, device=dev)
        elif keycols:
            packed = None
            span = 1
            radix = []  # (lo, card, stride) per key column
            for _, c in reversed(keycols):
                if c.card is not None:
                    lo, card = 0, c.card
                else:
                    mm = torch.aminmax(c.t)
                    lo, hi = int(mm.min.item()), int(mm.max.item())
                    card = hi - lo + 1
                if span * card >= 2 ** 62:
                    raise LoweringError("nested group key space exceeds 64 bits")
                term = c.t if lo == 0 else c.t - lo
                if span != 1:
                    term = term * span
                if packed is None:  # (one key column: its ids are the packed key, no extra passes)
                    packed = term if term.dtype == torch.int64 else term.to(torch.int64)
                else:
                    packed = packed + term
                radix.append((lo, card, span))
                span *= card
            radix.reverse()
            count_only = bool(qs.aggregations) and not self._js and all(
                getattr(a, "type", None) == "count" for a in qs.aggregations)
            if span <= max(1 << 26, 4 * n) and count_only:
                # dense key space, counts only (Q13's orders per customer): one histogram pass +
                # compaction of the non-empty bins -- no per-row group index at all
                counts = _histogram(packed, span)
                slots = _nonzero(counts)
                R = int(slots.numel())
                inv = None
                dense_counts = counts.index_select(0, slots)
                firsts = None
            elif span <= max(1 << 26, 4 * n):
                # dense key space: presence bitmap + prefix ranks, no sort (Q13: 15M customers)
                present = torch.zeros(span, dtype=torch.bool, device=dev)
                present[packed] = True
                rank = torch.cumsum(present, 0, dtype=torch.int64) - 1
                inv = rank[packed]
                slots = torch.nonzero(present).flatten()
                R = int(slots.numel())
                firsts = None
            else:
                uk, inv = torch.unique(packed, return_inverse=True)
                R = int(uk.numel())
                slots = uk
                firsts = None
        else:
            # global aggregate (no outer keys): whole-column reductions, no scatter
            inv = None
            R = 1
            firsts = torch.zeros(1, dtype=torch.int64, device=dev)
        if _TRACE:
            torch.cuda.synchronize()
            print(f"[nested] inner {inner_ms:.2f} ms rows={n}; grouping {(time.perf_counter() - t0) * 1e3 - inner_ms:.2f}"
                  f" ms -> {R} groups", flush=True)
        out: Dict[str, DeviceColumn] = {}
        for j, (d, c) in enumerate(keycols):
            if n == 0:
                t = c.t[:0]
            else:
                lo, card, stride = radix[j]
                # key components straight from the packed group key
                t = torch.remainder(torch.div(slots, stride, rounding_mode="floor"), card) + lo
            out[d.outputName] = DeviceColumn(d.outputName, t, c.decode, c.scale, c.card)
        for a in qs.aggregations:
            if a.name in self._js:
                op, pmap, ast = self._js[a.name]
                src = _torch_eval(ast, pmap, cols)
                if src.dim() == 0:
                    src = src.expand(n).contiguous()
                if op == "sum":
                    acc = _group_sum(R, inv, src, self.deterministic)
                elif inv is None:
                    acc = (src.amin() if op == "min" else src.amax()).reshape(1).to(torch.float64)
                else:
                    acc = torch.full((R,), float("inf") if op == "min" else float("-inf"), dtype=torch.float64,
                                     device=dev)
                    acc.scatter_reduce_(0, inv, src, reduce="amin" if op == "min" else "amax")
                out[a.name] = DeviceColumn(a.name, acc)
                continue
            if a.type == "count":
                if dense_counts is not None:
                    v = dense_counts
                elif inv is None:
                    v = torch.full((R,), n, dtype=torch.int64, device=dev)
                else:
                    v = torch.zeros(R, dtype=torch.int64, device=dev).index_add_(0, inv, torch.ones_like(inv))
                out[a.name] = DeviceColumn(a.name, v)
                continue
            c = cols.get(a.fieldName)
            if c is None:
                raise LoweringError(f"nested aggregator over unknown column {a.fieldName!r}")
            op = a.type[4:].lower() if a.type.startswith("long") else a.type[6:].lower()
            exact = not c.is_float and c.decode is None  # integral (scaled) values stay int64
            src = c.t if exact else (c.t.to(torch.float64) if c.decode is not None else c.as_float())
            if op == "sum":
                acc = _group_sum(R, inv, src, self.deterministic)
            elif inv is None:
                acc = (src.amin() if op == "min" else src.amax()).reshape(1)
            else:
                if src.dtype == torch.int64:
                    init = torch.iinfo(torch.int64).max if op == "min" else torch.iinfo(torch.int64).min
                else:
                    init = float("inf") if op == "min" else float("-inf")
                acc = torch.full((R,), init, dtype=src.dtype, device=dev)
                acc.scatter_reduce_(0, inv, src, reduce="amin" if op == "min" else "amax")
            if a.type.startswith("long") and not exact:
                acc = acc.to(torch.int64)
            out[a.name] = DeviceColumn(a.name, acc, scale=c.scale if exact else 0)
        if _TRACE:
            torch.cuda.synchronize()
            print(f"[nested] done {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
        return out, R, inner_ms

    def device_result(self) -> Tuple[Dict[str, DeviceColumn], int]:
        """This nested query's groups as device columns (input of a further nesting level)."""
        qs = self.qs
        if qs.having is not None or qs.limitSpec is not None or qs.postAggregations:
            raise LoweringError("having / limit / post-aggregations on an inner nested groupBy")
        cols, R, _ = self._compute()
        return cols, R

    def _host_inner(self):
        """Fallback: the inner result on the host (non-injective keys, sketches): numpy columns."""
        from .executor import materialize

        res = self.inner.run()
        return {c: materialize(res.data[c]) for c in res.columns}, res.num_rows

    def _host_compute(self):
        """Outer aggregation over host columns (pandas), same semantics as ``_compute``."""
        import pandas as pd

        qs = self.qs
        if self._js:
            raise LoweringError("javascript aggregators of a nested groupBy need the device path")
        t0 = time.perf_counter()
        cols, n = self._host_inner()
        inner_ms = (time.perf_counter() - t0) * 1e3
        df = pd.DataFrame({k: pd.Series(v) for k, v in cols.items()})
        keys = [d.dimension for d in qs.dimensions]
        df["__one__"] = 1
        spec = {}
        for a in qs.aggregations:
            if a.type == "count":
                spec[a.name] = ("__one__", "sum")
            else:
                op = a.type[4:].lower() if a.type.startswith("long") else a.type[6:].lower()
                spec[a.name] = (a.fieldName, op)
        if n and not keys:  # global aggregate: one row
            g = pd.DataFrame({name: [df[col].agg(op)] for name, (col, op) in spec.items()})
        else:
            g = df.groupby(keys, dropna=False, sort=False).agg(**spec).reset_index() if n else \
                pd.DataFrame({**{k: [] for k in keys}, **{a.name: [] for a in qs.aggregations}})
        out = {}
        for d in qs.dimensions:
            out[d.outputName] = np.asarray(g[d.dimension].to_numpy(), dtype=object)
        for a in qs.aggregations:
            v = g[a.name].to_numpy()
            out[a.name] = v.astype(np.int64) if (a.type == "count" or a.type.startswith("long")) else \
                v.astype(np.float64)
        return out, len(g), inner_ms

    def run(self):
        t0 = time.perf_counter()
        qs = self.qs
        try:
            dcols, R, inner_ms = self._compute()
        except LoweringError:
            if isinstance(self.inner, NestedPreparedQuery):
                raise
            out, R, inner_ms = self._host_compute()
            return self._finish(out, R, inner_ms, t0)
        out: Dict[str, np.ndarray] = {}
        names: List[str] = []
        for d in qs.dimensions:
            c = dcols[d.outputName]
            out[d.outputName] = c.host_values(c.t)
            names.append(d.outputName)
        for a in qs.aggregations:
            c = dcols[a.name]
            h = c.host_values(c.t)
            t_ = getattr(a, "type", "")
            out[a.name] = np.asarray(h, dtype=np.int64) if ((t_ == "count" or t_.startswith("long")) and not c.scale) \
                else np.asarray(h, dtype=np.float64)
            names.append(a.name)
        return self._finish(out, R, inner_ms, t0)

    def _finish(self, out, R, inner_ms, t0):
        from .executor import QueryResult, eval_having, eval_postagg, order_and_limit, take

        qs = self.qs
        names = [d.outputName for d in qs.dimensions] + [a.name for a in qs.aggregations]
        for pa in (getattr(qs, "postAggregations", None) or []):
            out[pa.name] = np.asarray(eval_postagg(pa, out, R), dtype=np.float64) * np.ones(R)
            names.append(pa.name)
        idx = np.arange(R)
        if qs.having is not None:
            idx = idx[eval_having(qs.having, out)[idx]]
        if qs.limitSpec is not None:
            idx = order_and_limit(out, idx, qs.limitSpec.columns, qs.limitSpec.limit)
        data = {k: take(out[k], idx) for k in names}
        res = QueryResult(names, data, "groupBy", {"groups": R})
        res.stats.update(inner_ms=inner_ms, exec_ms=(time.perf_counter() - t0) * 1e3)
        return res
