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
  * merge: one-shot all_gather for small partials, per-op all_reduce for large dense ones, a
    hash-partitioned all-to-all plus a gather to rank 0 for sparse (hash) partials; priced by the
    xGMI model (7 point-to-point links x ~153 GB/s per direction).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..query import spec as S
from ..query.intervals import Interval

HBM_BW = 6.1e12         # measured streaming bandwidth per MI355X (tools/stream_probe.py: 5.55 GB in 0.91 ms)
LAUNCH_S = 12e-6        # kernel launch + host overhead per scan
XGMI_LINK_BW = 153e9    # per direction per link
COLL_LAT_S = 25e-6      # small-message RCCL latency
LDS_PER_CU = 160 * 1024  # CDNA4 (gfx950) LDS per CU
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
    if out * aggs * 8 <= PLAN_LDS_BUDGET:
        mode = "dense-lds"
    elif out <= DENSE_GLOBAL_MAX:
        mode = "dense-global"
    else:
        mode = "hash"
    scan_s = nbytes / HBM_BW + LAUNCH_S
    merge, merge_s = merge_cost_s(mode, acc_bytes, world_size)
    return CostEstimate(rows, sel, inp, out, nbytes, mode, merge, scan_s * 1e3, merge_s * 1e3)


def merge_cost_s(mode: str, state_bytes: float, world_size: int):
    """(merge path, seconds) of one cross-rank merge of a state of ``state_bytes`` per rank -- the
    paths parallel/merge.py takes: sparse states go through one hash-partitioned all-to-all (each
    rank sends (N-1)/N of its rows, each peer over its own xGMI link) and the merged slices to rank
    0; small dense states one all-gather; large dense states a ring all-reduce."""
    n = world_size
    if n <= 1:
        return "none", 0.0
    links = min(7, n - 1)
    if mode == "hash":
        shuffle = state_bytes * (n - 1) / n / (links * XGMI_LINK_BW)
        gather = state_bytes / (links * XGMI_LINK_BW)  # rank 0 takes in ~one state's worth of groups
        return "alltoall-shuffle+gather-to-root", 4 * COLL_LAT_S + shuffle + gather
    if state_bytes * n <= ONESHOT_MAX_BYTES:
        return "oneshot-allgather", COLL_LAT_S + state_bytes * (n - 1) / (links * XGMI_LINK_BW)
    return "ring-allreduce", 3 * COLL_LAT_S + 2 * state_bytes * (n - 1) / n / XGMI_LINK_BW


def explain_cost(session, dq) -> str:
    ds = dq.relation.info.datasource
    c = estimate(ds, dq.spec, dq.relation.info, session.engine.world.size)
    lines = [
        "DruidQuery cost ::",
        f"  rowsInInterval={c.rows_in_interval}  selectivity={c.selectivity:.4g}  inputRows={c.input_rows:.4g}",
        f"  outputRows={c.output_rows:.4g}  bytesScanned={c.bytes_scanned}",
        f"  estScanMs={c.scan_ms:.4f}  estMergeMs={c.merge_ms:.4f}  merge={c.merge}  gpus={session.engine.world.size}",
    ]
    h = dq.info.get("historical")
    lines.append(f"  method: {'broker' if not h else f'historical(segmentsPerQuery={h})'}"
                 f"  [{dq.info.get('method_reason', '')}]")
    mc = dq.info.get("method_costs")
    if mc:
        lines.append("  method costs: " + "  ".join(f"{k}={v:.4f}ms" for k, v in sorted(mc.items(), key=lambda kv: kv[1])))
    prep = getattr(dq, "_prepared", None)
    if prep is None:
        try:  # plan it now (EXPLAIN before the first execution)
            prep = session.engine.prepare(dq.spec, ds, dq.info.get("historical"))
        except Exception:  # noqa: BLE001
            prep = None
    w = session.engine.world
    for _, prog, ps in getattr(prep, "scans", []) or []:
        gp = getattr(ps, "plan", None)
        if gp is None and hasattr(prog, "nslots"):
            gp = plan_groupby(prog, True, not w.distributed)
        if gp is not None:
            lines.append(f"  execution: groupBy={gp.describe()}")
            if w.distributed:
                dense = gp.mode != "hash" and not gp.touch and not gp.presence_bytes
                mp = plan_merge(dense, prog.G * prog.nslots * 8 + prog.nhll * prog.G * (8 << prog.hll_p), w.size)
                lines.append(f"  execution: merge={mp.describe()}")
    return "\n".join(lines)


def broker_cost_ms(ds, spec, info=None, world_size: int = 1, est: Optional[CostEstimate] = None) -> float:
    """One fused scan over every resident segment of the shard, then ONE cross-rank merge of the
    whole state (not overlapped with anything)."""
    return (est or estimate(ds, spec, info, world_size)).total_ms


def historical_cost_ms(ds, spec, segments_per_query: int, info=None, world_size: int = 1,
                       est: Optional[CostEstimate] = None) -> float:
    """Segment-batched ("historical") execution (the reference's historical waves + Spark
    shuffle/agg, ``asd/DruidQueryCostModel.scala:505-547``): B = segments / n scans, each followed
    by a merge of that batch's partials that runs while the next batch scans
    (``engine/executor.py _run_pipelined``), then a local combine of the B merged states.  The
    executor merges every batch in the full dense layout, so each batch's merge moves the whole
    state: pipelining pays only when one merge is shorter than one batch's scan, and even then
    the last merge and B launches remain -- except when the time bucket leads the group key: then
    a batch's groups are one slice of the table, each batch merges only its slice, and the merge
    of a large time-bucketed state hides behind the scans (historical wins across ranks)."""
    c = est or estimate(ds, spec, info, world_size)
    nseg = max(1, sum(1 for _ in ds.segments))
    batches = max(1, math.ceil(nseg / max(1, segments_per_query)))
    s_b = c.scan_ms / batches + LAUNCH_S * 1e3
    g = getattr(spec, "granularity", None)
    time_leading = g is not None and not getattr(g, "is_all", True) and spec.queryType in ("groupBy", "timeseries")
    if time_leading and world_size > 1 and c.merge_ms > 0:
        # the time bucket is the leading group key: a batch of segments covers a time range, so
        # its groups are one slice of the table and only that slice crosses the wire
        # (engine/executor.py _batch_key_slices) -- Druid's interval-partitioned historicals
        lat = COLL_LAT_S * 1e3
        m_b = lat + max(0.0, c.merge_ms - lat) / batches
        combine = c.output_rows * (len(spec.aggregation_specs) + 2) * 8 / HBM_BW * 1e3
    else:
        m_b = c.merge_ms
        combine = batches * c.output_rows * (len(spec.aggregation_specs) + 2) * 8 / HBM_BW * 1e3
    pipelined = s_b + (batches - 1) * max(s_b, m_b) + m_b
    return pipelined + combine


@dataclass
class MethodChoice:
    segments_per_query: Optional[int]          # None = broker
    costs: Dict[str, float] = field(default_factory=dict)

    def describe(self) -> str:
        alts = "  ".join(f"{k}={v:.4f}ms" for k, v in sorted(self.costs.items(), key=lambda kv: kv[1]))
        m = "broker" if self.segments_per_query is None else f"historical(segmentsPerQuery={self.segments_per_query})"
        return f"{m} {alts}"


def choose_method_costed(ds, spec, conf=None, info=None, world_size: int = 1) -> MethodChoice:
    """Broker vs historical and the segments per historical query, by the cheaper estimate
    (``DruidQueryCostModel.druidQueryMethod``, ``asd/DruidQueryCostModel.scala:343-413``): the
    broker plan against every n in 1..histSegsPerQueryLimit."""
    limit = 5
    if conf is not None:
        try:
            limit = int(conf.typed("spark.sparklinedata.druid.querycostmodel.histSegsPerQueryLimit"))
        except Exception:  # noqa: BLE001
            pass
    est = estimate(ds, spec, info, world_size)  # one estimate prices every alternative
    costs = {"broker": broker_cost_ms(ds, spec, info, world_size, est)}
    best, best_n = costs["broker"], None
    for n in range(1, max(1, limit) + 1):
        h = historical_cost_ms(ds, spec, n, info, world_size, est)
        costs[f"historical(n={n})"] = h
        if h < best:
            best, best_n = h, n
    return MethodChoice(best_n, costs)


def choose_method(ds, spec, conf=None, info=None, world_size: int = 1):
    """Segments per historical query, or None for broker (``choose_method_costed``)."""
    return choose_method_costed(ds, spec, conf, info, world_size).segments_per_query


# ================================================================================================
# Execution planning: the decisions the engine takes per prepared query come from here (the GPU
# analogue of the reference's broker-vs-historical / segments-per-query choice,
# ``asd/DruidQueryCostModel.scala:343-413, 724-829``).  Feasibility limits are device facts (LDS per
# CU, table budgets); between feasible alternatives the cheaper estimate wins.
# ------------------------------------------------------------------------------------------------
BLOCK_WAVES = 8                                             # 512-thread workgroups
# per-wave accumulator copies + HLL registers of one workgroup: 64 KiB leaves room for the staging
# planes and keeps 2 workgroups (16 waves) resident in a CU's 160 KiB (LDS_PER_CU); the scan is
# latency-bound below 8 waves per CU
PLAN_LDS_BUDGET = 64 * 1024
SHARED_LDS_MAX = 112 * 1024
SHARED_MIN_GROUPS = 512
DENSE_MAX_MULTI = 128 << 20       # dense partials merged whole
DENSE_MAX_SPARSE_MULTI = 4 << 30  # touched rows only
DENSE_MAX_1GPU = 16 << 30
TOUCH_MIN_G = 1 << 20
PROBE_S = 1.0e-9        # hash-table insert (CAS probe + key compare) per qualifying row
# Random read-modify-write atomics into a table beyond the L2: ~16-20 G updates/s on MI355X whether
# the table sits in HBM or in the Infinity Cache (TPC-H Q18 at SF100: 600M updates, 29 ms; see the
# KEY_PASSES note below) -- each update is its own cache-line transaction.
ATOMIC_RATE = 18e9
L2_TABLE_BYTES = 4 << 20   # one XCD's L2: tables this small take their atomics in cache
PARTITIONED = True
FORCE_PARTITIONED = False  # (tests: any eligible HBM-table plan)
ONESHOT_MAX_BYTES = 256 << 20   # gather buffer (world x state) ceiling for the one-shot merge


@dataclass
class GroupByPlan:
    mode: str                      # dense-lds | dense-global | partitioned | hash
    shared: bool = False           # one LDS table per workgroup (else one copy per wave)
    hll_lds: bool = False          # HLL registers in LDS
    touch: bool = False            # first-touch byte table (dense-global)
    presence_bytes: bool = False   # existence-only byte table (dense-global)
    costs: Dict[str, float] = field(default_factory=dict)   # priced alternatives, ms
    reason: str = ""

    def describe(self) -> str:
        extra = [k for k in ("shared", "hll_lds", "touch", "presence_bytes") if getattr(self, k)]
        alts = "  ".join(f"{k}={v:.3f}ms" for k, v in sorted(self.costs.items(), key=lambda kv: kv[1]))
        return f"{self.mode}{'(' + ','.join(extra) + ')' if extra else ''} [{self.reason}] {alts}"


def plan_groupby(prog, jit: bool, local: bool) -> GroupByPlan:
    """Group-by table for one lowered program on one shard.

    ``local``: the partials stay on this GPU (one rank, or a shard-local key window), so a dense HBM
    table may be as large as ``DENSE_MAX_1GPU``.  Across ranks dense partials that are merged whole
    are capped at ``DENSE_MAX_MULTI``; tables whose partials come back sparse (first-touch /
    presence byte tables) at ``DENSE_MAX_SPARSE_MULTI``."""
    G, ns = prog.G, prog.nslots
    m = 1 << prog.hll_p
    per_wave = G * ns * 8 * BLOCK_WAVES
    hll_bytes = prog.nhll * G * m * 4
    shared_bytes = G * ns * 8
    empty = bool(prog.empty)
    if jit and not empty and G > SHARED_MIN_GROUPS and shared_bytes <= SHARED_LDS_MAX and not prog.nhll:
        return GroupByPlan("dense-lds", shared=True, reason=f"{G} groups: one LDS table per workgroup")
    if per_wave + hll_bytes <= PLAN_LDS_BUDGET:
        return GroupByPlan("dense-lds", hll_lds=bool(prog.nhll), reason="per-wave LDS copies")
    if per_wave <= PLAN_LDS_BUDGET // 2 and hll_bytes <= DENSE_MAX_MULTI:
        return GroupByPlan("dense-lds", reason="per-wave LDS copies, HLL registers in HBM")
    if jit and not empty and shared_bytes <= SHARED_LDS_MAX and hll_bytes <= DENSE_MAX_MULTI:
        return GroupByPlan("dense-lds", shared=True, reason="shared LDS table")
    # HBM table vs hash table: priced
    presence = bool(jit and local and getattr(prog, "presence_only", False) and ns == 1 and not prog.nhll
                    and not empty)
    touch = bool(jit and not presence and not prog.nhll and not empty and G >= TOUCH_MIN_G
                 )
    table = G * ns * 8 + hll_bytes
    est_rows = max(1.0, float(getattr(prog, "est_rows", G)))
    if touch and local and est_rows >= G:
        # one GPU: a first-touch byte per group pays off only when groups go untouched -- every
        # qualifying row also stores its group's byte.  With at least as many qualifying rows as
        # groups (TPC-H Q18: 600M lines over 150M orders) the byte table is pure overhead
        # (45 -> 36 ms without it); selective scans keep it (Q3: 1.0 vs 1.4 ms)
        touch = False
    if local:
        limit = DENSE_MAX_1GPU
    else:
        limit = DENSE_MAX_SPARSE_MULTI if (touch or presence) else DENSE_MAX_MULTI
    costs = {}
    if table <= limit:
        if presence:
            dense = 2 * G / HBM_BW
        elif touch:
            touched = min(G, est_rows)
            dense = (2 * G + touched * ns * 8 * 2) / HBM_BW
        else:
            dense = 2 * table / HBM_BW
        if not presence:
            # one random atomic per qualifying row and slot (and HLL register: a byte CAS)
            dense += est_rows * (ns + prog.nhll) / (ATOMIC_RATE * (8 if table <= L2_TABLE_BYTES else 1))
        costs["dense-global"] = dense * 1e3
        part = partitioned_cost_s(prog, est_rows) if (jit and PARTITIONED and not presence and not empty) else None
        if part is not None:
            costs["partitioned"] = part * 1e3
    if table > limit and jit and PARTITIONED and not empty:
        # beyond any dense table (TPC-H Q16: 1.7e11 keys): hash-partitioned records, sparse output
        part = partitioned_cost_s(prog, est_rows)
        if part is not None:
            costs["partitioned"] = part * 1e3
    cap = 1 << max(10, math.ceil(math.log2(max(2.0, 2 * (min(G, est_rows * 1.2) + 1024)))))
    costs["hash"] = (2 * cap * (8 + ns * 8) / HBM_BW + est_rows * PROBE_S) * 1e3
    if "partitioned" in costs and (FORCE_PARTITIONED or costs["partitioned"] <= min(costs.get("dense-global", math.inf),
                                                                                    costs["hash"])):
        return GroupByPlan("partitioned", costs=costs,
                           reason="radix-partitioned records aggregated in LDS (no random HBM atomics)")
    if "dense-global" in costs and costs["dense-global"] <= costs["hash"]:
        return GroupByPlan("dense-global", touch=touch, presence_bytes=presence, costs=costs,
                           reason="HBM table indexed by the packed key")
    why = "table over budget" if "dense-global" not in costs else "few qualifying rows for the key space"
    return GroupByPlan("hash", costs=costs, reason=why)


def partitioned_cost_s(prog, est_rows: float) -> Optional[float]:
    """Radix-partitioned group-by (ops/csrc/partition.hip): one producer scan appending records,
    a count + tile-sorted scatter pass per level, the LDS aggregation, the dense table written once."""
    from ..ops import jit

    if not jit.part_eligible(prog):
        return None
    if jit.part_hashed(prog):
        from ..engine.device_exec import part_hash_layout

        L = part_hash_layout(prog)
        rec = 4 * L["rw"]
        passes = 1 + 3 * L["levels"] + 1
        groups = min(float(prog.G), est_rows)
        return (est_rows * rec * passes + groups * (1 + max(1, prog.nslots)) * 8) / HBM_BW + \
            (3 + 4 * L["levels"]) * LAUNCH_S
    if est_rows < prog.G / 4:
        # few updates per group: the touched lines are sparse (TPC-H Q3 touches ~1M of 150M orders)
        # and stay cached; the atomic table wins and a full-table write would be waste
        return None
    from ..engine.device_exec import part_layout

    try:
        L = part_layout(prog)
    except ValueError:
        return None
    rec = 4 * L["rw"]
    # producer write, per level a count read + a scatter read and write, the aggregation read, the
    # table (and the HLL register tables) written once
    passes = 1 + 3 * L["levels"] + 1
    traffic = est_rows * rec * passes + prog.G * (max(1, prog.nslots) * 8 + L.get("nhll", 0) * (1 << prog.hll_p))
    return traffic / HBM_BW + (2 + 4 * L["levels"]) * LAUNCH_S


@dataclass
class MergePlan:
    kind: str                      # none | oneshot-allgather | bucketed-allreduce | alltoall-shuffle | disjoint-concat
    costs: Dict[str, float] = field(default_factory=dict)

    def describe(self) -> str:
        alts = "  ".join(f"{k}={v:.3f}ms" for k, v in sorted(self.costs.items(), key=lambda kv: kv[1]))
        return f"{self.kind} {alts}"


MALL_BYTES = 256 << 20  # MI355X Infinity Cache (last level, shared by the XCDs)
PASS_TABLE_BYTES = 96 << 20
# Measured on MI355X (tools/sql_probe.py, TPC-H Q18 at SF100): 12 cache-sized passes run 2.9 ms of
# scan each -- the random-atomic rate into a 100 MB Infinity-Cache-resident table (~17 G/s) is no
# better than into the 1.2 GB HBM table (~16 G/s), and every pass repeats compaction / HAVING /
# key decoding: 130 ms vs 41 ms single-pass.  Kept as an opt-in plan (KEY_PASSES = True).
KEY_PASSES = False
FORCE_KEY_PASSES = 0  # (tests: this many passes for any groupBy)


def plan_key_passes(prep) -> int:
    """Key-range passes for a dense HBM group table far larger than the Infinity Cache (TPC-H Q18:
    150M orders x 8 B = 1.2 GB): every row is an HBM read-modify-write atomic on a random line of the
    table, so split the key space into P ranges whose tables (<= PASS_TABLE_BYTES) stay
    cache-resident.  Each pass re-reads only the key and payload columns (a few bytes per row at
    streaming bandwidth) and its atomics hit the 256 MB Infinity Cache.  Returns P (1 = no split)."""
    from ..ops import desc as D

    forced = FORCE_KEY_PASSES  # (tests: split any groupBy)
    if forced > 1:
        return forced
    if not KEY_PASSES or prep is None or getattr(prep, "mode", None) != D.M_DENSE_GLOBAL:
        return 1
    if getattr(prep, "pres_bytes", False):
        return 1
    prog = prep.prog
    if prog.est_rows < prog.G / 4:
        return 1  # few groups touched (first-touch table, TPC-H Q3): the atomics are sparse anyway
    table = prog.G * max(1, prog.nslots) * 8
    if table <= 2 * MALL_BYTES or prog.nhll or prog.thetas or getattr(prog, "stored_hll", None):
        return 1
    return int(math.ceil(table / PASS_TABLE_BYTES))


def plan_merge(dense: bool, state_bytes: int, world_size: int, disjoint: bool = False) -> MergePlan:
    """Cross-GPU merge of one query's partials.  Inputs must be identical on every rank (layout
    sizes, never local row counts) so every rank takes the same collective path.

    * dense state: one all-gather of the whole state + local reduction (latency-bound, every peer
      read over its own xGMI link) vs a bucketed ring all-reduce (bandwidth-optimal, three
      collectives); the one-shot gather buffer is capped at ``ONESHOT_MAX_BYTES``;
    * sparse state: concatenation when the groups are disjoint across ranks (grouped on the shard
      key), else the hash-partitioned all-to-all shuffle."""
    n = world_size
    if n <= 1:
        return MergePlan("none")
    if not dense:
        return MergePlan("disjoint-concat" if disjoint else "alltoall-shuffle")
    b = float(state_bytes)
    costs = {}
    if b * n <= ONESHOT_MAX_BYTES:
        costs["oneshot-allgather"] = (COLL_LAT_S + b * (n - 1) / (min(7, n - 1) * XGMI_LINK_BW) + n * b / HBM_BW) * 1e3
    costs["bucketed-allreduce"] = (3 * COLL_LAT_S + 2 * b * (n - 1) / n / XGMI_LINK_BW) * 1e3
    return MergePlan(min(costs, key=costs.get), costs)


# Segment-batch pipelining (engine/executor.py _auto_batches / _run_pipelined): batch j's merge of its
# time slice runs on the process group's stream while batch j+1 scans.  With B batches of a scan
# taking S and a merge taking M (each slice 1/B of the state):
#     one merge:  S + M
#     pipelined:  S/B + (B - 1) * max(S/B, M/B) + M/B + (B - 1) * overhead
# where every extra batch re-initialises and combines its table (two passes over the state at HBM
# speed) and pays a few launches.  On xGMI a dense state's all-reduce is fast (2 x 4 MB x 7/8 over
# 153 GB/s links: ~50 us), so the split pays only for states of tens of MB and more.  Host-staged
# collectives (gloo: the one-card rehearsal) copy to the host synchronously inside the collective
# call -- the next batch cannot even be launched before the copy returns -- so they never overlap:
# measured, 3 batches 4.28 ms against one merge 2.81 ms (profiles/r5/rehearsal_auto_pipeline_sf10.txt).
BATCH_LAUNCHES = 4


def plan_pipeline(state_bytes: int, scan_bytes: int, world_size: int, host_staged: bool,
                  max_batches: int) -> int:
    """Batches for a pipelined multi-rank scan (1: scan once, merge once).  Inputs are layout sizes
    -- identical on every rank."""
    if host_staged or world_size <= 1 or max_batches <= 1:
        return 1
    S = scan_bytes / HBM_BW + LAUNCH_S

    def merge_s(b):
        return min(plan_merge(True, int(b), world_size).costs.values()) / 1e3

    best_b, best_t = 1, S + merge_s(state_bytes)
    for B in range(2, max_batches + 1):
        m = merge_s(state_bytes / B)
        over = BATCH_LAUNCHES * LAUNCH_S + 2 * state_bytes / HBM_BW
        t = S / B + (B - 1) * max(S / B, m) + m + (B - 1) * over
        if t < best_t:
            best_b, best_t = B, t
    return best_b
