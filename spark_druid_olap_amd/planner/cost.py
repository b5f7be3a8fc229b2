"""GPU query cost model.

The reference's ``DruidQueryCostModel`` (``asd/DruidQueryCostModel.scala:32-872``) chooses between
broker and historical execution and the number of segments per historical query by comparing
estimated merge/shuffle/scheduling costs.  On MI355X every GPU scans its own shard in one fused
kernel, so the decisions are different, but the estimation machinery is the same:

  * input rows: rows inside the query intervals x filter selectivity (selector 1/card,
    IN n/card, AND product, OR sum, NOT complement, anything else 1/3; ``estimateInput`` 660-677);
  * output rows: product of grouping cardinalities with functional-dependency pruning, capped by
    input rows (``estimateOutputCardinality`` 691-716);
  * scan time: bytes streamed from HBM / bandwidth + launch overhead;
  * group-by table choice: dense LDS (fits the per-block LDS budget), dense global, or hash;
  * merge: one-shot all_gather for small partials, per-op all_reduce for large dense ones, varlen
    all_gather by key for sparse (hash) partials; priced by the xGMI ring model (7 links x ~153 GB/s).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

from ..query import spec as S
from ..query.intervals import Interval

HBM_BW = 5.0e12         # achievable streaming bandwidth per MI355X (bytes/s)
LAUNCH_S = 12e-6        # kernel launch + host overhead per scan
XGMI_LINK_BW = 153e9    # per direction per link
COLL_LAT_S = 25e-6      # small-message RCCL latency
LDS_BUDGET = 64 * 1024
DENSE_GLOBAL_MAX = 1 << 24


@dataclass
class CostEstimate:
    rows_in_interval: int
    selectivity: float
    input_rows: float
    output_rows: float
    bytes_scanned: int
    groupby_mode: str
    merge: str
    scan_ms: float
    merge_ms: float

    @property
    def total_ms(self) -> float:
        return self.scan_ms + self.merge_ms


def _card(ds, dim: str) -> int:
    if dim in ds.dims:
        return max(len(ds.dims[dim].dictionary), 1)
    return 1000


def selectivity(ds, f) -> float:
    if f is None:
        return 1.0
    if isinstance(f, S.SelectorFilterSpec):
        return 1.0 / _card(ds, f.dimension)
    if isinstance(f, S.InFilterSpec):
        return min(1.0, len(f.values) / _card(ds, f.dimension))
    if isinstance(f, S.ExtractionFilterSpec) and isinstance(f.extractionFn, S.InExtractionFnSpec):
        return min(1.0, len(f.extractionFn.lookup.get("map", {})) / _card(ds, f.dimension))
    if isinstance(f, S.LogicalFilterSpec):
        parts = [selectivity(ds, x) for x in f.fields]
        if f.type == "and":
            return math.prod(parts)
        return min(1.0, sum(parts))
    if isinstance(f, S.NotFilterSpec):
        return 1.0 - selectivity(ds, f.field)
    return 1.0 / 3.0


def rows_in_intervals(ds, intervals: List[str]) -> int:
    total = 0
    for s in intervals:
        iv = Interval.parse(s)
        a, b = ds.rows_for_interval(iv.lo, iv.hi)
        total += max(0, b - a)
    return total


def output_cardinality(ds, spec, info=None) -> float:
    dims = []
    if isinstance(spec, S.GroupByQuerySpec):
        dims = spec.dimensions
    elif isinstance(spec, S.TopNQuerySpec):
        return float(spec.threshold)
    elif isinstance(spec, S.TimeSeriesQuerySpec):
        return 1.0
    names = []
    prod = 1.0
    for d in dims:
        dim = d.dimension if hasattr(d, "dimension") else str(d)
        if dim == "__time":
            prod *= 366
            continue
        names.append(dim)
    if info is not None and names:
        prod *= info.estimate_cardinality(names)
    else:
        for n in names:
            prod *= _card(ds, n)
    return prod


def _col_bytes(ds, name: str) -> int:
    if name in ds.dims:
        return ds.dims[name].ids.element_size()
    if name in ds.metrics:
        return ds.metrics[name].data.element_size()
    return 0


def referenced_columns(spec) -> List[str]:
    cols = set()

    def walk(x):
        if isinstance(x, S.Spec):
            for k, v in vars(x).items():
                if k in ("dimension", "fieldName") and isinstance(v, str):
                    cols.add(v)
                elif k in ("fieldNames", "fields") and isinstance(v, list) and v and isinstance(v[0], str):
                    cols.update(v)
                else:
                    walk(v)
        elif isinstance(x, (list, tuple)):
            for y in x:
                walk(y)
    walk(spec)
    return sorted(cols)


def estimate(ds, spec, info=None, world_size: int = 1) -> CostEstimate:
    rows = rows_in_intervals(ds, spec.intervals) if getattr(spec, "intervals", None) else ds.num_rows
    sel = selectivity(ds, getattr(spec, "filter", None))
    inp = rows * sel
    out = min(output_cardinality(ds, spec, info), max(inp, 1.0))
    cols = referenced_columns(spec)
    nbytes = int(rows * sum(_col_bytes(ds, c) for c in cols)) + int(rows * ds.time.element_size())
    aggs = len(spec.aggregation_specs) + 1
    acc_bytes = out * aggs * 8
    if out * aggs * 8 <= LDS_BUDGET:
        mode = "dense-lds"
    elif out <= DENSE_GLOBAL_MAX:
        mode = "dense-global"
    else:
        mode = "hash"
    scan_s = nbytes / HBM_BW + LAUNCH_S
    if world_size <= 1:
        merge, merge_s = "none", 0.0
    elif mode == "hash":
        merge = "varlen-allgather(keys)"
        merge_s = COLL_LAT_S * 2 + acc_bytes * (world_size - 1) / (7 * XGMI_LINK_BW)
    elif acc_bytes <= 4 << 20:
        merge = "oneshot-allgather"
        merge_s = COLL_LAT_S + acc_bytes * (world_size - 1) / (7 * XGMI_LINK_BW)
    else:
        merge = "ring-allreduce"
        merge_s = COLL_LAT_S + 2 * acc_bytes * (world_size - 1) / world_size / XGMI_LINK_BW
    return CostEstimate(rows, sel, inp, out, nbytes, mode, merge, scan_s * 1e3, merge_s * 1e3)


def explain_cost(session, dq) -> str:
    ds = dq.relation.info.datasource
    c = estimate(ds, dq.spec, dq.relation.info, session.engine.world.size)
    return "\n".join([
        "DruidQuery cost ::",
        f"  rowsInInterval={c.rows_in_interval}  selectivity={c.selectivity:.4g}  inputRows={c.input_rows:.4g}",
        f"  outputRows={c.output_rows:.4g}  bytesScanned={c.bytes_scanned}  groupBy={c.groupby_mode}",
        f"  merge={c.merge}  estScanMs={c.scan_ms:.4f}  estMergeMs={c.merge_ms:.4f}  gpus={session.engine.world.size}",
    ])


def historical_cost_ms(ds, spec, segments_per_query: int, info=None) -> float:
    """Segment-batched ("historical") execution: one scan launch + partial compaction per batch of
    segments, then a merge of the partials (the reference's historical waves + Spark shuffle/agg,
    ``asd/DruidQueryCostModel.scala:505-547``)."""
    c = estimate(ds, spec, info)
    nseg = max(1, sum(1 for _ in ds.segments))
    batches = math.ceil(nseg / max(1, segments_per_query))
    per_batch_out = min(c.output_rows, c.input_rows / batches if batches else c.input_rows)
    merge_bytes = batches * per_batch_out * (len(spec.aggregation_specs) + 2) * 8
    return c.scan_ms + batches * LAUNCH_S * 1e3 + merge_bytes / HBM_BW * 1e3 * 4


def choose_method(ds, spec, conf=None, info=None):
    """Broker (None) or historical (segments per query).  On one MI355X the broker plan -- one
    fused scan over every resident segment with the partials merged in LDS/HBM -- is never more
    expensive than batching segments into several launches plus a merge, so the GPU cost model
    picks broker unless the batched plan is estimated cheaper (it is not, for any batch count)."""
    limit = 5
    if conf is not None:
        try:
            limit = int(conf.typed("spark.sparklinedata.druid.querycostmodel.histSegsPerQueryLimit"))
        except Exception:  # noqa: BLE001
            pass
    broker = estimate(ds, spec, info).total_ms
    best = None
    for n in range(1, max(1, limit) + 1):
        h = historical_cost_ms(ds, spec, n, info)
        if h < broker and (best is None or h < best[0]):
            best = (h, n)
    return None if best is None else best[1]
