"""Lower a Druid QuerySpec into a kernel ``ScanProgram`` for one datasource shard.

This is where Druid's per-segment engine semantics are re-designed for the GPU:

* filters  -> dictionary-domain evaluation of every leaf (selector / in / bound / regex /
  search / javascript / extraction; reference ``sd/DruidQuerySpec.scala:152-281``) into an id
  set, then the cheapest device encoding: inverted-bitmap words (<= 4 id runs on an indexed
  dimension), an id range, or an id bitset; time leaves become row ranges;
* dimensions -> mixed-radix key components: dictionary ids, dictionary-domain remaps
  (extraction functions, evaluated once per distinct value) or in-register time buckets;
* aggregators -> accumulator slots (exact int64 for integral/decimal metrics, f64 otherwise),
  HLL registers, and a float expression VM for javascript aggregators.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import desc as D
from ..query import joda
from ..query import spec as S
from ..query.granularity import Granularity, bucket_start_from_value, bucket_value
from ..query.intervals import Interval, parse_iso_ms
from ..query.jsfunc import JSError, compile_function, jsagg_to_expr, parse_expr
from ..segment.datasource import CHUNK_ROWS, DataSource, dtype_code
from ..segment.dictionary import Dictionary
from .columns import DictColumn

FD_KEYS = True    # (tests / tools: False keeps functionally dependent keys in the scan)
FOLD_PRESENCE = True  # (tests: False keeps the separate presence-count slot)
TRACE_FD = False  # (tools: print every functional-dependency decision)

TIME = "__time"
HLL_P = 11  # 2048 registers, the precision of Druid's HyperUnique


class LoweringError(ValueError):
    pass


# =================================================================================== boolean IR
# ('true',) ('false',) ('and', [..]) ('or', [..]) ('not', x)
# ('ids', dim, mask)                       dictionary-domain id set (np.bool_[card])
# ('time', lo_ms, hi_ms)                   half open
# ('int', col, lo, hi)                     inclusive, integer domain (scaled decimals)
# ('flt', col, lo, hi, flags)              flags bit0 lo strict, bit1 hi strict
TRUE = ("true",)
FALSE = ("false",)


def _is(x, k):
    return x[0] == k


def b_and(xs):
    out = []
    for x in xs:
        if _is(x, "false"):
            return FALSE
        if _is(x, "true"):
            continue
        out.extend(x[1] if _is(x, "and") else [x])
    # merge id-set leaves on the same dimension
    merged: Dict[str, np.ndarray] = {}
    rest = []
    for x in out:
        if _is(x, "ids"):
            merged[x[1]] = merged[x[1]] & x[2] if x[1] in merged else x[2].copy()
        else:
            rest.append(x)
    leaves = [("ids", k, v) for k, v in merged.items()]
    for lf in leaves:
        if not lf[2].any():
            return FALSE
    out = [lf for lf in leaves if not lf[2].all()] + rest
    if not out:
        return TRUE
    return out[0] if len(out) == 1 else ("and", out)


def b_or(xs):
    out = []
    for x in xs:
        if _is(x, "true"):
            return TRUE
        if _is(x, "false"):
            continue
        out.extend(x[1] if _is(x, "or") else [x])
    merged: Dict[str, np.ndarray] = {}
    rest = []
    for x in out:
        if _is(x, "ids"):
            merged[x[1]] = merged[x[1]] | x[2] if x[1] in merged else x[2].copy()
        else:
            rest.append(x)
    leaves = [("ids", k, v) for k, v in merged.items()]
    for lf in leaves:
        if lf[2].all():
            return TRUE
    out = [lf for lf in leaves if lf[2].any()] + rest
    if not out:
        return FALSE
    return out[0] if len(out) == 1 else ("or", out)


_PRE_OPS = (D.F_TRUE, D.F_FALSE, D.F_BITMAP, D.F_BITMAP_OR, D.F_AND, D.F_OR, D.F_NOT)  # chunk-level evaluable
IMPLY_OR = True  # AND the id sets every disjunct of an OR implies (imply_or_conjuncts)


def _or_implied(x) -> list:
    """Per dimension constrained by an id set in EVERY disjunct of OR ``x``: the union of those
    sets -- a necessary condition of the OR."""
    per = None
    for d in x[1]:
        m: Dict[str, np.ndarray] = {}
        for c in (d[1] if _is(d, "and") else [d]):
            if _is(c, "ids"):
                m[c[1]] = m[c[1]] & c[2] if c[1] in m else c[2].copy()
        per = m if per is None else {k: per[k] | m[k] for k in per if k in m}
        if not per:
            return []
    return [("ids", k, v) for k, v in (per or {}).items() if not v.all()]


def imply_or_conjuncts(x):
    """``OR_i (A_i and ...)`` whose disjuncts all constrain dimension d implies ``d in U_i A_i(d)``:
    those implied id sets become top-level conjuncts next to the OR (semantics unchanged).  They are
    what the scan can use -- bitmap pre-filter leaves, zones, word skipping -- where the OR alone is
    evaluated row by row: TPC-H Q19's three (brand, containers, sizes, ship mode, instruction,
    quantity) disjuncts imply ship mode in (AIR, AIR REG), DELIVER IN PERSON and 3 of 25 brands."""
    if not IMPLY_OR:
        return x

    def split(o):
        """(implied conjuncts, the OR without the disjuncts' conjuncts that equal them)"""
        if all(_is(c, "ids") for d in o[1] for c in (d[1] if _is(d, "and") else [d])):
            return [], o  # (dimension-only: the OR itself is a bitmap pre-filter, TPC-H Q7)
        extra = _or_implied(o)
        if not extra:
            return [], o
        imp = {lf[1]: lf[2] for lf in extra}
        ds_ = []
        for d in o[1]:
            conj = d[1] if _is(d, "and") else [d]
            keep = [c for c in conj if not (_is(c, "ids") and c[1] in imp and np.array_equal(c[2], imp[c[1]]))]
            ds_.append(b_and(keep))
        return extra, b_or(ds_)

    if _is(x, "or"):
        extra, rest = split(x)
        return b_and(extra + [rest]) if extra else x
    if _is(x, "and") and any(_is(c, "or") for c in x[1]):
        out = []
        for c in x[1]:
            if _is(c, "or"):
                extra, rest = split(c)
                out += extra + [rest]
            else:
                out.append(c)
        return b_and(out)
    return x


def b_not(x):
    k = x[0]
    if k == "true":
        return FALSE
    if k == "false":
        return TRUE
    if k == "not":
        return x[1]
    if k == "and":
        return b_or([b_not(c) for c in x[1]])
    if k == "or":
        return b_and([b_not(c) for c in x[1]])
    if k == "ids":
        return ("ids", x[1], ~x[2])
    return ("not", x)


# =================================================================================== extraction
def _fn_key(fn) -> Optional[str]:
    """Cache key of an extraction function: its Druid JSON (JavaScript functions carry their
    source, which the SQL planner generates from the grouping expression)."""
    try:
        import json

        return json.dumps(fn.to_json(), sort_keys=True, default=str)
    except Exception:  # noqa: BLE001
        return None


def extraction_callable(fn) -> Callable[[Any], Any]:
    """Python callable for a Druid extraction function (evaluated over a dictionary)."""
    if fn is None:
        return lambda v: v
    if isinstance(fn, S.RegexExtractionFunctionSpec):
        rx = re.compile(fn.expr)

        def f(v):
            if v is None:
                return None
            m = rx.search(str(v))
            if not m:
                return v
            return m.group(1) if m.groups() else m.group(0)

        return f
    if isinstance(fn, S.PartialExtractionFunctionSpec):
        rx = re.compile(fn.expr)
        return lambda v: v if v is not None and rx.search(str(v)) else None
    if isinstance(fn, S.SearchQueryExtractionFunctionSpec):
        q = str(fn.query).lower()
        return lambda v: v if v is not None and q in str(v).lower() else None
    if isinstance(fn, S.SubstringExtractionFunctionSpec):
        i, n = int(fn.index), fn.length
        return lambda v: None if v is None else (str(v)[i:i + int(n)] if n is not None else str(v)[i:]) or None
    if isinstance(fn, S.UpperExtractionFunctionSpec):
        return lambda v: None if v is None else str(v).upper()
    if isinstance(fn, S.LowerExtractionFunctionSpec):
        return lambda v: None if v is None else str(v).lower()
    if isinstance(fn, S.TimeParsingExtractionFunctionSpec):
        inf, outf = fn.timeFormat, fn.resultFormat

        def f(v):
            ms = joda.parse(inf, v)
            return None if ms is None else joda.format_ms(outf, ms)

        return f
    if isinstance(fn, S.TimeFormatExtractionFunctionSpec):
        fmt = fn.format

        def f(v):
            if v is None:
                return None
            if isinstance(v, (int, np.integer)):
                ms = int(v)
            else:
                try:
                    ms = parse_iso_ms(str(v))
                except ValueError:
                    return None
            return joda.format_ms(fmt, ms)

        return f
    if isinstance(fn, S.JavaScriptExtractionFunctionSpec):
        py = getattr(fn, "_pyfn", None)
        if py is not None:
            return py
        jf = compile_function(fn.function)

        def f(v):
            r = jf(v)
            if isinstance(r, float) and r.is_integer():
                return str(int(r))
            return None if r is None else (r if isinstance(r, str) else str(r))

        return f
    if isinstance(fn, S.InExtractionFnSpec):
        mp = (fn.lookup or {}).get("map", {})
        keep, repl = fn.retainMissingValue, fn.replaceMissingValueWith

        def f(v):
            key = None if v is None else _druid_str(v)
            if key in mp:
                return mp[key]
            return v if keep else repl

        return f
    raise LoweringError(f"unsupported extraction function {type(fn).__name__}")


def _druid_str(v) -> str:
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return str(v)


def tz_offset_ms(tz: Optional[str], at_ms: int = 0) -> int:
    if tz is None or tz.upper() in ("UTC", "Z", "GMT", "ETC/UTC"):
        return 0
    m = re.match(r"^(?:UTC|GMT)?([+-])(\d{1,2}):?(\d{2})?$", tz)
    if m:
        sgn = -1 if m.group(1) == "-" else 1
        return sgn * (int(m.group(2)) * 60 + int(m.group(3) or 0)) * 60_000
    try:
        import datetime as _dt
        from zoneinfo import ZoneInfo

        z = ZoneInfo(tz)
        dt = _dt.datetime.fromtimestamp(at_ms / 1000.0, tz=_dt.timezone.utc).astimezone(z)
        return int(dt.utcoffset().total_seconds() * 1000)
    except Exception:
        return 0


# =================================================================================== program
@dataclass
class KeyComp:
    name: str
    kind: int
    col: str
    card: int
    stride: int = 1
    base: int = 0
    tfield: int = 0
    tz_ms: int = 0
    period_ms: int = 0
    origin_ms: int = 0
    remap: Optional[np.ndarray] = None
    decoder: Optional[Callable[[np.ndarray], np.ndarray]] = None
    collapse: bool = False        # decoded values may coincide: re-aggregate on host
    is_timestamp: bool = False    # granularity bucket (output 'timestamp' ms)
    orig: Optional[np.ndarray] = None  # compacted key: key id -> original dictionary id
    col_idx: int = -1             # descriptor column index (payload section)
    dictionary: Any = None        # plain dictionary-id key: its dictionary (device-side typed decode)
    # K_TIME over a coarse time unit (days): the key of every raw time value of the cluster-wide
    # data span, precomputed (``Lowerer._attach_time_lut``) -- the JIT kernel gathers
    # ``tlut[v - tlut_lo]`` instead of running the calendar arithmetic (civil_from_days: several
    # 64-bit divisions) for all 64 lanes of every word a filter leaves non-empty
    tlut: Optional[np.ndarray] = None
    tlut_lo: int = 0


@dataclass
class AggOut:
    name: str
    kind: str                     # count|sum_i|sum_f|sum_fx|min_i|max_i|min_f|max_f|hll|theta
    slot: int = -1
    slot2: int = -1               # sum_fx: fraction slot (value = slot + slot2 * 2^-32)
    hll_index: int = -1
    scale: int = 0                # decimal digits of an exact integer sum
    out_type: str = "double"      # long|double
    combine: str = "sum"          # host re-aggregation: sum|min|max|hll


@dataclass
class ScanProgram:
    ds: DataSource
    fcols: List[str] = field(default_factory=list)      # filter-phase columns -> desc.cols[0..8)
    pcols: List[str] = field(default_factory=list)      # payload columns      -> desc.cols[8..24)
    section: str = "p"                                  # where col() registers
    fops: List[tuple] = field(default_factory=list)     # (op, col, flags, lo, hi, flo, fhi, bits_tensor)
    filter_len: int = 0
    pre_off: int = 0
    pre_len: int = 0
    final_pre: bool = False
    bm_leaves: List[Tuple[torch.Tensor, int, int]] = field(default_factory=list)  # (first row, stride, count)
    keys: List[KeyComp] = field(default_factory=list)
    aops: List[dict] = field(default_factory=list)
    eops: List[tuple] = field(default_factory=list)
    zones: List[tuple] = field(default_factory=list)    # (col, lo, hi)
    ranges: List[Tuple[int, int]] = field(default_factory=list)
    slots: List[Tuple[int, int]] = field(default_factory=list)  # (slot op, init)
    aggs: List[AggOut] = field(default_factory=list)
    nhll: int = 0
    hll_p: int = HLL_P
    G: int = 1
    est_rows: float = 0.0
    empty: bool = False
    bexpr: Any = TRUE                                    # normalized filter (for the reference executor)
    agg_filters: List[Any] = field(default_factory=list) # per aop bexpr or None
    keepalive: List[torch.Tensor] = field(default_factory=list)
    thetas: List[Tuple[str, str, int]] = field(default_factory=list)  # (name, column, size)
    luts: Dict[str, torch.Tensor] = field(default_factory=dict)       # dim -> f64 value per dictionary id
    lut_ptrs: Dict[float, torch.Tensor] = field(default_factory=dict)  # E_LUT operand -> its table
    # grouping keys functionally determined by a packed key: (key, index of determinant in keys,
    # device int32 table determinant dictionary id -> dependent dictionary id)
    derived: List[Tuple["KeyComp", int, torch.Tensor]] = field(default_factory=list)
    key_order: List[str] = field(default_factory=list)  # output order of all grouping keys
    presence_only: bool = False  # no aggregator reads slot 0's count: group existence only
    presence_bytes: bool = False  # (set by the device executor) existence table is one byte per group
    # min/max of a metric constant per group key: (AggOut, determinant key index, device int64 table
    # determinant dictionary id -> stored metric value); no accumulator, gathered at finalize
    derived_aggs: List[Tuple["AggOut", int, torch.Tensor]] = field(default_factory=list)
    # hyperUnique over rolled-up sketch metrics: (output name, metric, aggregator filter or None);
    # their registers follow the scan's ``nhll`` query-time HLL blocks in Partials.hll
    stored_hll: List[Tuple[str, str, Any]] = field(default_factory=list)

    @property
    def nhll_total(self) -> int:
        return self.nhll + len(self.stored_hll)

    def col(self, name: str) -> int:
        """Absolute descriptor column index of `name` in the current section."""
        if self.section == "f":
            if name not in self.fcols:
                if len(self.fcols) >= D.PAYLOAD_BASE:
                    raise LoweringError("too many filter columns in one query")
                self.fcols.append(name)
            return self.fcols.index(name)
        if name not in self.pcols:
            if len(self.pcols) >= D.MAX_COLS - D.PAYLOAD_BASE:
                raise LoweringError("too many payload columns in one query")
            self.pcols.append(name)
        return D.PAYLOAD_BASE + self.pcols.index(name)

    def colname(self, idx: int) -> str:
        return self.fcols[idx] if idx < D.PAYLOAD_BASE else self.pcols[idx - D.PAYLOAD_BASE]

    @property
    def cols(self) -> List[str]:
        return self.fcols + self.pcols

    def bm_leaf(self, row: torch.Tensor, stride: int, count: int) -> int:
        if len(self.bm_leaves) >= D.MAX_BM:
            raise LoweringError("too many bitmap leaves")
        self.bm_leaves.append((row, stride, count))
        return len(self.bm_leaves) - 1

    @property
    def nslots(self) -> int:
        return len(self.slots)

    @property
    def rows_in_ranges(self) -> int:
        return sum(b - a for a, b in self.ranges)


def column_tensor(ds: DataSource, name: str) -> torch.Tensor:
    if name == TIME:
        return ds.time
    if name in ds.dims:
        return ds.dims[name].ids
    if name in ds.metrics:
        return ds.metrics[name].data
    if "#hll" in name:
        from ..segment.hllcode import lookup

        t = lookup(ds, name)
        if t is not None:
            return t
    raise LoweringError(f"unknown column {name!r} in datasource {ds.name}")


class Lowerer:
    """QuerySpec -> ScanProgram for a datasource shard."""

    def __init__(self, ds: DataSource, bitmap_max_values: int = 4, world=None, deterministic: bool = False):
        self.ds = ds
        self.bitmap_max_values = bitmap_max_values
        self.world = world
        # floating-point sums in exact 64.32 fixed point (two integer slots) instead of f64 atomics:
        # integer addition is associative, so per-wave LDS folds, workgroup flush atomics, segment
        # batches and the cross-GPU merge give bitwise-identical results in any order
        self.deterministic = deterministic
        self._tv_cache: Optional[np.ndarray] = None

    # ------------------------------------------------------------------ filters -> IR
    def filter_ir(self, f) -> tuple:
        """Filter spec -> normalized boolean IR (constant-folded id-set leaves)."""
        return b_and([self._filter_ir(f)])

    def _filter_ir(self, f) -> tuple:
        ds = self.ds
        if f is None or isinstance(f, S.NoopFilterSpec):
            return TRUE
        if isinstance(f, S.LogicalFilterSpec):
            parts = [self._filter_ir(c) for c in f.fields]
            return b_and(parts) if f.type == "and" else b_or(parts)
        if isinstance(f, S.NotFilterSpec):
            return b_not(self._filter_ir(f.field))
        if isinstance(f, S.ExpressionFilterSpec):
            return self._expression_filter(f.expression)
        dim = getattr(f, "dimension", None)
        if dim == TIME or (dim is not None and dim not in ds.dims and dim not in ds.metrics and dim == "timestamp"):
            return self._time_filter(f)
        if dim is not None and dim in ds.metrics and not isinstance(f, S.SpatialFilterSpec):
            return self._metric_filter(f, dim)
        if isinstance(f, S.SpatialFilterSpec):
            return self._spatial(f)
        if dim not in ds.dims:
            raise LoweringError(f"filter on unknown dimension {dim!r}")
        d = ds.dims[dim].dictionary
        if isinstance(f, S.IdRangeFilterSpec):
            mask = np.zeros(len(d), dtype=bool)
            mask[max(0, int(f.lo)): min(len(d), int(f.hi))] = True
            return ("ids", dim, mask)
        if isinstance(f, S.SelectorFilterSpec):
            v = f.value
            mask = np.zeros(len(d), dtype=bool)
            i = d.lookup(None if v in (None, "") and d.has_null else v)
            if i >= 0:
                mask[i] = True
            return ("ids", dim, mask)
        if isinstance(f, S.InFilterSpec):
            mask = np.zeros(len(d), dtype=bool)
            for v in f.values:
                i = d.lookup(v)
                if i >= 0:
                    mask[i] = True
            return ("ids", dim, mask)
        if isinstance(f, S.BoundFilterSpec):
            if f.alphaNumeric and d.vtype == "string":
                lo = None if f.lower is None else float(f.lower)
                hi = None if f.upper is None else float(f.upper)

                def pred(v):
                    try:
                        x = float(v)
                    except (TypeError, ValueError):
                        return False
                    ok = True
                    if lo is not None:
                        ok = ok and (x > lo if f.lowerStrict else x >= lo)
                    if hi is not None:
                        ok = ok and (x < hi if f.upperStrict else x <= hi)
                    return ok

                return ("ids", dim, d.eval_mask(pred))
            a, b = d.id_range(f.lower, f.lowerStrict, f.upper, f.upperStrict)
            mask = np.zeros(len(d), dtype=bool)
            mask[a:b] = True
            return ("ids", dim, mask)
        if isinstance(f, S.RegexFilterSpec):
            rx = re.compile(f.pattern)
            return ("ids", dim, d.eval_mask(lambda v: v is not None and rx.search(str(v)) is not None))
        if isinstance(f, S.ContainsFilterSpec):
            q = f.query or {}
            val = str(q.get("value", ""))
            cs = bool(q.get("caseSensitive", False)) and q.get("type") != "insensitive_contains"
            if cs:
                return ("ids", dim, d.eval_mask(lambda v: v is not None and val in str(v)))
            lv = val.lower()
            return ("ids", dim, d.eval_mask(lambda v: v is not None and lv in str(v).lower()))
        if isinstance(f, S.ExtractionFilterSpec):
            ef = f.extractionFn
            if isinstance(ef, S.InExtractionFnSpec) and _druid_str(f.value) == "true" and \
                    not ef.retainMissingValue and ef.replaceMissingValueWith in (None, "") and \
                    (ef.lookup or {}).get("type", "map") == "map" and getattr(d, "lazy", False):
                # IN list over a large lazy dictionary (o_orderkey IN (subquery)): one lookup per
                # listed value instead of evaluating every dictionary entry
                mask = np.zeros(len(d), dtype=bool)
                for v, out in (ef.lookup.get("map") or {}).items():
                    if _druid_str(out) == "true":
                        i = d.lookup(v)
                        if i >= 0:
                            mask[i] = True
                return ("ids", dim, mask)
            fn = extraction_callable(f.extractionFn)
            target = f.value

            def pred(v):
                r = fn(v)
                return r is not None and _druid_str(r) == _druid_str(target)

            return ("ids", dim, d.eval_mask(pred))
        if isinstance(f, S.JavascriptFilterSpec):
            pl = getattr(f, "_pylike", None)
            if pl is not None and hasattr(d, "like_mask"):
                # structured LIKE over a lazy phrase dictionary (no per-entry strings)
                m = d.like_mask(pl[0])
                if m is not None:
                    if pl[1]:
                        m = ~m
                        if d.has_null:
                            m[0] = False
                    return ("ids", dim, m)
            pv = getattr(f, "_pyvec", None)
            if pv is not None:  # vectorised dictionary-domain predicate (SQL planner)
                return ("ids", dim, np.asarray(pv(d.all_values()), dtype=bool))
            py = getattr(f, "_pyfn", None)
            if py is None:
                jf = compile_function(f.function)
                py = lambda v: bool(jf(v))  # noqa: E731
            return ("ids", dim, d.eval_mask(py))
        raise LoweringError(f"unsupported filter {type(f).__name__}")

    def _expression_filter(self, text: str) -> tuple:
        """``<arith> <cmp> <arith>`` -> ("fexpr", ast of lhs - rhs, lo, hi, flags): a row predicate
        the scan kernel evaluates in its expression VM (F_EXPR).  Two bare string dimensions are
        compared through rank tables over the union of their dictionaries (exact string order /
        equality, ISO dates included); anything else compares numeric values (metrics, numeric
        dimension values through E_LUT)."""
        m = re.match(r"^(.*?)(==|!=|<=|>=|<|>)(.*)$", text.strip(), re.S)
        if m is None:
            raise LoweringError(f"expression filter needs one comparison: {text!r}")
        lhs, op, rhs = m.group(1).strip(), m.group(2), m.group(3).strip()
        try:
            la, ra = parse_expr(lhs), parse_expr(rhs)
        except JSError as e:
            raise LoweringError(f"expression filter not translatable: {e}")
        for a in (la, ra):
            for name in _ast_cols(a):
                if name != TIME and name not in self.ds.dims and name not in self.ds.metrics:
                    raise LoweringError(f"expression filter over unknown column {name!r}")
        if la[0] == "col" and ra[0] == "col" and la[1] in self.ds.dims and ra[1] in self.ds.dims and \
                (self.ds.dims[la[1]].dictionary.vtype == "string" or self.ds.dims[ra[1]].dictionary.vtype == "string"):
            lt, rt = rank_luts(self.ds, la[1], ra[1])
            la, ra = ("lut", la[1], lt), ("lut", ra[1], rt)
        ast = ("sub", la, ra)
        inf = math.inf
        lo, hi, flags = {"<": (-inf, 0.0, 2), "<=": (-inf, 0.0, 0), ">": (0.0, inf, 1), ">=": (0.0, inf, 0),
                         "==": (0.0, 0.0, 0), "!=": (0.0, 0.0, 0)}[op]
        leaf = ("fexpr", ast, lo, hi, flags)
        if op == "!=":
            # NaN (NULL) operands fail both the leaf and its negation, like SQL's 3-valued logic
            return b_and([b_not(leaf), ("fexpr", ast, -inf, inf, 0)])
        return leaf

    def _time_values(self) -> np.ndarray:
        if self._tv_cache is None:
            self._tv_cache = self.ds.distinct_times()
        return self._tv_cache

    def _time_filter(self, f) -> tuple:
        ds = self.ds
        u = ds.time_unit_ms
        if isinstance(f, S.SelectorFilterSpec):
            if f.value is None or f.value == "":
                return FALSE  # __time is never null (the reference's NULL-scan marker)
            ms = _to_ms(f.value)
            return ("time", ms, ms + 1)
        if isinstance(f, S.BoundFilterSpec):
            lo = -(2 ** 62) if f.lower is None else _to_ms(f.lower) + (1 if f.lowerStrict else 0)
            hi = 2 ** 62 if f.upper is None else _to_ms(f.upper) + (0 if f.upperStrict else 1)
            return ("time", lo, hi)
        if isinstance(f, S.IntervalFilterSpec):
            return b_or([("time", iv.lo, iv.hi) for iv in (Interval.parse(s) for s in f.intervals)])
        # generic predicate over the distinct time values -> set of allowed time units
        if isinstance(f, S.JavascriptFilterSpec):
            pv = getattr(f, "_pyvec", None)
            if pv is not None:  # vectorised over the distinct time values (SQL planner)
                tv = self._time_values()
                return ("timeset", tv[np.asarray(pv(tv.astype(np.int64) * u), dtype=bool)])
            py = getattr(f, "_pyfn", None)
            if py is None:
                jf = compile_function(f.function)
                py = lambda ms: bool(jf(joda.format_ms("yyyy-MM-dd'T'HH:mm:ss.SSS'Z'", ms)))  # noqa: E731
        elif isinstance(f, S.ExtractionFilterSpec):
            fn = extraction_callable(f.extractionFn)
            tgt = _druid_str(f.value)
            py = lambda ms: (lambda r: r is not None and _druid_str(r) == tgt)(fn(ms))  # noqa: E731
        else:
            raise LoweringError(f"unsupported time filter {type(f).__name__}")
        tv = self._time_values()
        ok = np.fromiter((bool(py(int(t) * u)) for t in tv), dtype=bool, count=len(tv))
        return ("timeset", tv[ok])

    def _metric_filter(self, f, name) -> tuple:
        m = self.ds.metrics[name]
        scale = 10 ** m.scale if m.kind == "decimal" else 1
        if isinstance(f, S.SelectorFilterSpec):
            v = float(f.value)
            if m.is_integral:
                x = v * scale
                if x != math.floor(x):
                    return FALSE
                return ("int", name, int(x), int(x))
            return ("flt", name, v, v, 0)
        if isinstance(f, S.BoundFilterSpec):
            lo = None if f.lower is None else float(f.lower)
            hi = None if f.upper is None else float(f.upper)
            if m.is_integral:
                ilo = -(2 ** 62) if lo is None else (math.floor(lo * scale) + 1 if f.lowerStrict else math.ceil(lo * scale))
                ihi = 2 ** 62 if hi is None else (math.ceil(hi * scale) - 1 if f.upperStrict else math.floor(hi * scale))
                return ("int", name, int(ilo), int(ihi))
            flags = (1 if f.lowerStrict else 0) | (2 if f.upperStrict else 0)
            return ("flt", name, -math.inf if lo is None else lo, math.inf if hi is None else hi, flags)
        raise LoweringError(f"unsupported metric filter {type(f).__name__}")

    def _spatial(self, f) -> tuple:
        comps = self.ds.spatial.get(f.dimension) if hasattr(self.ds, "spatial") else None
        if not comps:
            raise LoweringError(f"no spatial dimension {f.dimension!r}")
        b = f.bound
        mins, maxs = b.get("minCoords", []), b.get("maxCoords", [])
        parts = [("flt", comps[i], float(mins[i]), float(maxs[i]), 0) for i in range(min(len(comps), len(mins)))]
        return b_and(parts)

    # ------------------------------------------------------------------ intervals
    def query_ranges(self, intervals: Sequence[str], bexpr) -> Tuple[List[Tuple[int, int]], tuple, List[Interval]]:
        """Row ranges from the query intervals AND top-level time conjuncts (pruning)."""
        ivs = [Interval.parse(s) for s in intervals] if intervals else [Interval.eternity()]
        rest = bexpr
        conj = bexpr[1] if _is(bexpr, "and") else [bexpr]
        tleaves = [c for c in conj if _is(c, "time")]
        if tleaves:
            t = Interval(-(2 ** 62), 2 ** 62)
            for lf in tleaves:
                t = t.intersect(Interval(lf[1], lf[2]))
            ivs = [iv.intersect(t) for iv in ivs]
            others = [c for c in conj if not _is(c, "time")]
            rest = b_and(others) if others else TRUE
        ivs = [iv for iv in ivs if not iv.empty]
        ranges = []
        for iv in sorted(ivs, key=lambda i: i.lo):
            a, b = self.ds.rows_for_interval(iv.lo, iv.hi)
            if b > a:
                if ranges and a <= ranges[-1][1]:
                    ranges[-1] = (ranges[-1][0], max(ranges[-1][1], b))
                else:
                    ranges.append((a, b))
        if len(ranges) > D.MAX_RANGES:  # coalesce: keep exactness through a time filter
            lo_all, hi_all = ranges[0][0], ranges[-1][1]
            rest = b_and([rest, b_or([("time", iv.lo, iv.hi) for iv in ivs])])
            ranges = [(lo_all, hi_all)]
        return ranges, rest, ivs

    # ------------------------------------------------------------------ emit filter program
    def emit_filter(self, prog: ScanProgram, x) -> int:
        """Append postfix ops for x; returns max stack depth used."""
        k = x[0]
        if k == "true":
            prog.fops.append((D.F_TRUE, 0, 0, 0, 0, 0.0, 0.0, None))
            return 1
        if k == "false":
            prog.fops.append((D.F_FALSE, 0, 0, 0, 0, 0.0, 0.0, None))
            return 1
        if k in ("and", "or"):
            kids = sorted(x[1], key=_depth, reverse=True)
            d = self.emit_filter(prog, kids[0])
            for c in kids[1:]:
                d = max(d, 1 + self.emit_filter(prog, c))
                prog.fops.append((D.F_AND if k == "and" else D.F_OR, 0, 0, 0, 0, 0.0, 0.0, None))
            return d
        if k == "not":
            d = self.emit_filter(prog, x[1])
            prog.fops.append((D.F_NOT, 0, 0, 0, 0, 0.0, 0.0, None))
            return d
        if k == "ids":
            return self._emit_ids(prog, x[1], x[2])
        if k == "time":
            ci = prog.col(TIME)
            u = self.ds.time_unit_ms
            lo = -(-x[1] // u)
            hi = -(-x[2] // u) - 1
            prog.fops.append((D.F_INT_RANGE, ci, 0, max(lo, -(2 ** 62)), min(hi, 2 ** 62), 0.0, 0.0, None))
            return 1
        if k == "timeset":
            vals = x[1]
            if len(vals) == 0:
                prog.fops.append((D.F_FALSE, 0, 0, 0, 0, 0.0, 0.0, None))
                return 1
            ci = prog.col(TIME)
            # contiguous runs of allowed time values -> OR of ranges (typically 1-2 runs)
            tv = self._time_values()
            allowed = np.isin(tv, vals)
            runs = _runs(allowed)
            for j, (a, b) in enumerate(runs):
                prog.fops.append((D.F_INT_RANGE, ci, 0, int(tv[a]), int(tv[b - 1]), 0.0, 0.0, None))
                if j:
                    prog.fops.append((D.F_OR, 0, 0, 0, 0, 0.0, 0.0, None))
            return 2 if len(runs) > 1 else 1
        if k == "int":
            ci = prog.col(x[1])
            prog.fops.append((D.F_INT_RANGE, ci, 0, int(x[2]), int(x[3]), 0.0, 0.0, None))
            return 1
        if k == "flt":
            ci = prog.col(x[1])
            prog.fops.append((D.F_FLT_RANGE, ci, int(x[4]), 0, 0, float(x[2]), float(x[3]), None))
            return 1
        if k == "fexpr":
            eops = self._emit_expr(prog, x[1], {})
            off = len(prog.eops)
            prog.eops.extend(eops)
            prog.fops.append((D.F_EXPR, 0, int(x[4]), off, len(eops), float(x[2]), float(x[3]), None))
            return 1
        raise LoweringError(f"bad filter IR {k}")

    def bitmap_plan(self, dim: str, mask: np.ndarray):
        """(negate, runs) when the id set is cheap as OR of inverted-bitmap rows, else None."""
        dc = self.ds.dims.get(dim)
        if dc is None or dc.bitmap is None:
            return None
        st = mask_stats(mask)
        if st.k == 0 or st.k == len(mask):
            return None
        lim = self.bitmap_max_values
        for use_neg, nr in ((False, st.runs), (True, st.neg_runs)):
            if nr > lim:
                continue
            rr = _runs(~mask if use_neg else mask)
            if sum(b - a for a, b in rr) <= 64:
                return (use_neg, rr)
        return None

    def bitmap_only(self, x) -> int:
        """number of bitmap leaves x needs if it is evaluable from bitmaps alone, else -1"""
        k = x[0]
        if k in ("true", "false"):
            return 0
        if k in ("and", "or"):
            tot = 0
            for c in x[1]:
                n = self.bitmap_only(c)
                if n < 0:
                    return -1
                tot += n
            return tot
        if k == "not":
            return self.bitmap_only(x[1])
        if k == "ids":
            plan = self.bitmap_plan(x[1], x[2])
            return -1 if plan is None else len(plan[1])
        return -1

    def _emit_ids(self, prog: ScanProgram, dim: str, mask: np.ndarray) -> int:
        dc = self.ds.dims[dim]
        card = len(mask)
        st = mask_stats(mask)
        k = st.k
        if k == 0:
            prog.fops.append((D.F_FALSE, 0, 0, 0, 0, 0.0, 0.0, None))
            return 1
        if k == card:
            prog.fops.append((D.F_TRUE, 0, 0, 0, 0, 0.0, 0.0, None))
            return 1
        plan = self.bitmap_plan(dim, mask)
        if plan is not None and len(prog.bm_leaves) + len(plan[1]) <= D.MAX_BM:
            use_neg, rr = plan
            nw = dc.bitmap.shape[1]
            for j, (a, b) in enumerate(rr):
                leaf = prog.bm_leaf(dc.bitmap[a], nw, b - a)
                prog.fops.append((D.F_BITMAP, 0, 0, leaf, 0, 0.0, 0.0, None))
                if j:
                    prog.fops.append((D.F_OR, 0, 0, 0, 0, 0.0, 0.0, None))
            if use_neg:
                prog.fops.append((D.F_NOT, 0, 0, 0, 0, 0.0, 0.0, None))
            return 2 if len(rr) > 1 else 1
        ci = prog.col(dim)
        if st.runs == 1:
            prog.fops.append((D.F_ID_RANGE, ci, 0, st.lo, st.hi, 0.0, 0.0, None))
            return 1
        if st.neg_runs == 1:
            (a, b), = _runs(~mask)
            prog.fops.append((D.F_ID_RANGE, ci, 0, a, b, 0.0, 0.0, None))
            prog.fops.append((D.F_NOT, 0, 0, 0, 0, 0.0, 0.0, None))
            return 1
        dk = str(self.ds.device)
        t = st.words.get(dk)
        if t is None:  # (read-only on the device: plans of one cached mask share the words)
            t = torch.from_numpy(pack_bitset(mask)).to(self.ds.device)
            if len(mask) >= _MASK_STATS_MIN:
                st.words[dk] = t
        prog.keepalive.append(t)
        prog.fops.append((D.F_IN_SET, ci, 0, 0, 0, 0.0, 0.0, t))
        return 1

    # ------------------------------------------------------------------ zones
    def pick_zones(self, prog: ScanProgram, bexpr) -> None:
        conj = bexpr[1] if _is(bexpr, "and") else [bexpr]
        cands = []
        for c in conj:
            if _is(c, "ids") and self.ds.dims[c[1]].zmin is not None:
                st = mask_stats(c[2])
                if st.k == 0:
                    continue
                lo, hi = st.lo, st.hi
                frac = (hi - lo) / max(1, len(c[2]))
                if frac < 0.9:
                    cands.append((frac, c[1], lo, hi))
        cands.sort()
        for frac, dim, lo, hi in cands[: D.MAX_ZONES]:
            prog.zones.append((dim, lo, hi))

    # ------------------------------------------------------------------ selectivity
    def selectivity(self, x) -> float:
        k = x[0]
        if k == "true":
            return 1.0
        if k == "false":
            return 0.0
        if k == "and":
            p = 1.0
            for c in x[1]:
                p *= self.selectivity(c)
            return p
        if k == "or":
            return min(1.0, sum(self.selectivity(c) for c in x[1]))
        if k == "not":
            return 1.0 - self.selectivity(x[1])
        if k == "ids":
            return mask_stats(x[2]).k / max(1, len(x[2]))
        return 1.0 / 3.0

    # ------------------------------------------------------------------ dimensions
    def key_for_dimension(self, dspec, ivs: List[Interval]) -> KeyComp:
        ds = self.ds
        if isinstance(dspec, str):
            dspec = S.DefaultDimensionSpec(dspec)
        dim = dspec.dimension
        name = dspec.outputName or dim
        fn = getattr(dspec, "extractionFn", None) if isinstance(dspec, S.ExtractionDimensionSpec) else None
        if dim == TIME:
            return self._time_key(name, fn, ivs)
        if dim in ds.metrics and dim not in ds.dims and fn is None:
            return self._metric_key(name, dim)
        if dim not in ds.dims:
            raise LoweringError(f"group by unknown dimension {dim!r}")
        d = ds.dims[dim].dictionary
        if fn is None:
            return KeyComp(name, D.K_ID, dim, len(d), decoder=lambda ids, _d=d: DictColumn(ids, _d), dictionary=d)
        if isinstance(fn, S.TimeFormatExtractionFunctionSpec) and d.vtype != "string":
            pass
        # the derived dictionary + id remap depend only on (dictionary, extraction function): cached
        # on the dictionary, so every statement of one shape -- a dashboard's parameterizations --
        # maps the dictionary domain once (the Joda formatting of 2,400 dates was ~65 ms a query)
        ck = _fn_key(fn)
        cache = d.__dict__.setdefault("_derived_keys", {}) if ck is not None else None
        hit = cache.get(ck) if cache is not None else None
        if hit is None:
            pv = getattr(fn, "_pyvec", None)
            if pv is not None:  # vectorised dictionary-domain extraction (SQL planner)
                derived = np.asarray(pv(d.all_values()), dtype=object)
            else:
                derived = d.map_values(extraction_callable(fn))
            vals = derived.tolist()
            uniq = sorted({v for v in vals if v is not None}, key=lambda v: (str(type(v)), v))
            has_null = any(v is None for v in vals)
            numeric = all(isinstance(v, (int, float)) and not isinstance(v, bool) for v in uniq)
            # non-numeric, non-string derived values (dates, timestamps, booleans) keep their Python objects
            dd = Dictionary(uniq, "double" if numeric and uniq else "string", has_null)
            pos = {v: i + (1 if has_null else 0) for i, v in enumerate(uniq)}
            remap = np.array([0 if v is None else pos[v] for v in vals], dtype=np.int32)
            remap.setflags(write=False)
            hit = (dd, remap)
            if cache is not None:
                cache[ck] = hit
        dd, remap = hit
        return KeyComp(name, D.K_REMAP, dim, len(dd), remap=remap, decoder=lambda ids, _d=dd: DictColumn(ids, _d))

    def _metric_range(self, metric: str) -> Tuple[int, int]:
        """Global (all ranks) min/max of a metric's stored integer values, cached on the metric."""
        # a streamed window (segment/streamed.py) measures (and caches on) its whole host shard
        src = getattr(self.ds, "fd_source", None) or self.ds
        m = src.metrics[metric]
        rng = getattr(m, "_value_range", None)
        if rng is None:
            # global value range (every rank must build the same key space)
            t = column_tensor(src, metric)[:src.num_rows]
            big = 2 ** 62
            lo_t = (t.min() if t.numel() else torch.tensor(big, device=t.device)).to(torch.int64).reshape(1)
            hi_t = (t.max() if t.numel() else torch.tensor(-big, device=t.device)).to(torch.int64).reshape(1)
            if self.world is not None and self.world.distributed:
                lo_t = self.world.all_reduce(lo_t, "min")
                hi_t = self.world.all_reduce(hi_t, "max")
            lo, hi = int(lo_t.item()), int(hi_t.item())
            rng = (lo, hi) if lo <= hi else (0, 0)
            m._value_range = rng  # type: ignore[attr-defined]
        return rng

    def _exact_decimal(self, ast, mapping: Dict[str, str]) -> Optional[int]:
        """Result scale when ``ast`` is +,-,* over decimal/long metrics and decimal constants and the
        scaled value stays exactly representable (row < 2^52, total < 2^62); else None."""
        def rec(n):
            k = n[0]
            if k == "const":
                v = float(n[1])
                if not math.isfinite(v):
                    return None
                txt = repr(v)
                if "e" in txt or "E" in txt:
                    return None
                sc = len(txt.split(".")[1].rstrip("0")) if "." in txt else 0
                return sc, abs(v)
            if k == "col":
                name = mapping.get(n[1], n[1])
                m = self.ds.metrics.get(name)
                if m is None or name in self.ds.dims or not m.is_integral:
                    return None
                lo, hi = self._metric_range(name)
                sc = m.scale if m.kind == "decimal" else 0
                return sc, max(abs(lo), abs(hi)) / 10.0 ** sc
            if k == "neg":
                return rec(n[1])
            if k in ("add", "sub", "mul"):
                a, b = rec(n[1]), rec(n[2])
                if a is None or b is None:
                    return None
                if k == "mul":
                    return a[0] + b[0], a[1] * b[1]
                return max(a[0], b[0]), a[1] + b[1]
            return None

        r = rec(ast)
        if r is None:
            return None
        sc, bound = r
        if sc > 9:
            return None
        row = bound * 10.0 ** sc
        rows = self.ds.num_rows * (self.world.size if self.world is not None else 1)
        if row >= 2.0 ** 52 or row * max(rows, 1) >= 2.0 ** 62:
            return None
        return sc

    def _metric_key(self, name: str, metric: str) -> KeyComp:
        """Group by an integral metric (K_INT over its stored value range, <= 2^20 values)."""
        m = self.ds.metrics[metric]
        if not m.is_integral:
            raise LoweringError(f"cannot group by floating metric {metric!r}")
        lo, hi = self._metric_range(metric)
        card = hi - lo + 1
        if card > (1 << 20):
            raise LoweringError(f"metric {metric!r} spans {card} values: too many to group by")
        scale = m.scale if m.kind == "decimal" else 0

        def decode(ids, _lo=lo, _sc=scale):
            v = np.asarray(ids, dtype=np.int64) + _lo
            return v / (10.0 ** _sc) if _sc else v

        return KeyComp(name, D.K_INT, metric, card, base=lo, decoder=decode)

    def _time_key(self, name, fn, ivs: List[Interval]) -> KeyComp:
        lo, hi = self._data_span(ivs)
        if fn is None:
            tf, exact, fmt, tz = self._unit_field(), True, None, 0
        elif isinstance(fn, S.TimeFormatExtractionFunctionSpec):
            tz = tz_offset_ms(fn.timeZone, lo)
            tf, exact = joda.format_to_field(fn.format)
            fmt = fn.format
        else:
            tf, exact, fmt, tz = self._unit_field(), False, None, 0
        kc = KeyComp(name, D.K_TIME, TIME, 1, tfield=tf, tz_ms=tz)
        if tf in joda.ABSOLUTE:
            b0 = bucket_value(lo + tz, tf)
            b1 = bucket_value(hi - 1 + tz, tf)
            kc.base, kc.card = b0, max(1, b1 - b0 + 1)
        else:
            a, b = joda.field_domain(tf)
            kc.base, kc.card = a, b - a + 1
        self._attach_time_lut(kc)
        base, tfv = kc.base, tf
        if fn is None:
            kc.decoder = lambda ids: np.array([bucket_start_from_value(int(i) + base, tfv) for i in ids], dtype=np.int64)
        elif fmt is not None:
            tzv = tz
            kc.decoder = lambda ids: np.array(
                [joda.format_ms(fmt, joda.representative_ms(tfv, int(i) + base) - (tzv if tfv in joda.ABSOLUTE else 0), tzv if tfv in joda.ABSOLUTE else 0)
                 for i in ids], dtype=object)
            kc.collapse = not exact
        else:
            f = extraction_callable(fn)
            kc.decoder = lambda ids: np.array([f(bucket_start_from_value(int(i) + base, tfv)) for i in ids], dtype=object)
            kc.collapse = True
        return kc

    TIME_LUT_MAX = 1 << 16

    def _attach_time_lut(self, kc: KeyComp) -> None:
        """Key table over the raw time values of the cluster-wide data span (identical on every
        rank), when the storage unit is coarse enough for it to stay small (days: ~2,600 entries
        for TPC-H).  Values are the reference executor's own (ops/reference.py _time_field), so
        the LUT and the arithmetic paths agree bit for bit; out-of-span values clamp like the key."""
        ds = self.ds
        u = int(ds.time_unit_ms)
        if u < 1000:
            return
        lo, hi = self._data_span([])
        v0, v1 = lo // u, (hi - 1) // u
        span = v1 - v0 + 1
        if span <= 0 or span > self.TIME_LUT_MAX:
            return
        from ..ops.reference import _time_field

        vals = torch.arange(v0, v1 + 1, dtype=torch.int64)
        t = (_time_field(vals * u, kc) - kc.base).clamp(0, max(0, kc.card - 1))
        kc.tlut = t.numpy().astype(np.int32)
        kc.tlut_lo = int(v0)

    def _unit_field(self) -> int:
        from ..query.granularity import T_DAY, T_MS, T_SECOND

        u = self.ds.time_unit_ms
        return T_DAY if u == 86_400_000 else (T_SECOND if u == 1000 else T_MS)

    def _data_span(self, ivs: List[Interval]) -> Tuple[int, int]:
        ds = self.ds
        gi = getattr(ds, "global_interval_ms", None)
        # every rank keys time buckets from the CLUSTER-wide span (Session._global_interval), so
        # shards covering different periods still produce identically laid-out partials
        lo, hi = gi if gi is not None else (ds.min_time_ms(), ds.max_time_ms() + ds.time_unit_ms)
        if ivs:
            lo = max(lo, min(iv.lo for iv in ivs))
            hi = min(hi, max(iv.hi for iv in ivs))
        if hi <= lo:
            hi = lo + 1
        return lo, hi

    def granularity_key(self, g: Granularity, ivs: List[Interval]) -> Optional[KeyComp]:
        if g is None or g.is_all:
            return None
        tf, p, o = g.kernel_field()
        lo, hi = self._data_span(ivs)
        b0 = bucket_value(lo + g.tz_ms, tf, p, o)
        b1 = bucket_value(hi - 1 + g.tz_ms, tf, p, o)
        kc = KeyComp("timestamp", D.K_TIME, TIME, max(1, b1 - b0 + 1), base=b0, tfield=tf, tz_ms=g.tz_ms,
                     period_ms=p, origin_ms=o, is_timestamp=True)
        self._attach_time_lut(kc)
        kc.decoder = lambda ids: np.array([bucket_start_from_value(int(i) + b0, tf, p, o) - g.tz_ms for i in ids],
                                          dtype=np.int64)
        return kc

    # ------------------------------------------------------------------ aggregators
    def add_aggregator(self, prog: ScanProgram, a, filt=None) -> None:
        ds = self.ds
        if isinstance(a, S.FilteredAggregationSpec):
            inner = a.aggregator.copy(name=a.name or a.aggregator.name)
            fx = self.filter_ir(a.filter)
            if filt is not None:
                fx = b_and([filt, fx])
            return self.add_aggregator(prog, inner, fx)
        if len(prog.aops) >= D.MAX_AOPS:
            raise LoweringError("too many aggregators")

        def aop(kind, col=-1, expr=None):
            d = {"kind": kind, "col": col, "expr": expr, "filter": filt, "slot": -1, "hll": -1}
            prog.aops.append(d)
            return d

        def slot(op, init, d):
            # identical aggregators (count(*) for both COUNT and AVG, ...) share one accumulator: every
            # slot is one more update per row in the scan kernel's inner loop
            sig = (d["kind"], d["col"], repr(d["expr"]), repr(d["filter"]), op, init)
            for prev in prog.aops[:-1]:
                if prev.get("sig") == sig:
                    prog.aops.pop()
                    return prev["slot"]
            d["sig"] = sig
            if len(prog.slots) >= D.MAX_SLOTS:
                raise LoweringError("too many accumulator slots")
            prog.slots.append((op, init))
            return len(prog.slots) - 1

        def fixed_sum(name, eops, out_type="double"):
            # value v -> floor(v) (integer part) and rint((v - floor(v)) * 2^32) (fraction), each an
            # exact integer sum; finalize returns int + frac * 2^-32.  |v| < 2^63 per row, |sum| <
            # 2^63; per-row resolution 2^-33, the same for every order of accumulation.
            if len(prog.aops) + 1 >= D.MAX_AOPS:
                raise LoweringError("too many aggregators")
            if _eops_depth(eops) + 1 > 4:
                raise LoweringError("aggregator expression too deep for a deterministic sum")
            hi = aop(D.A_SUM_X, -1, list(eops) + [(D.E_FLOOR, 0, 0.0)])
            hi["slot"] = slot(D.S_SUM_I, 0, hi)
            lo = aop(D.A_SUM_X, -1, list(eops) + list(eops) + [(D.E_FLOOR, 0, 0.0), (D.E_SUB, 0, 0.0),
                                                                 (D.E_CONST, 0, FIX_ONE), (D.E_MUL, 0, 0.0)])
            lo["slot"] = slot(D.S_SUM_I, 0, lo)
            prog.aggs.append(AggOut(name, "sum_fx", hi["slot"], slot2=lo["slot"], out_type=out_type))

        if isinstance(a, S.FunctionAggregationSpec):
            t = a.type
            if t == "count":
                d = aop(D.A_COUNT)
                d["slot"] = slot(D.S_SUM_I, 0, d)
                prog.aggs.append(AggOut(a.name, "count", d["slot"], out_type="long"))
                return
            fname = a.fieldName
            if fname == "count" and fname not in ds.metrics:
                # longSum(count) over an index without an explicit count metric == count
                d = aop(D.A_COUNT)
                d["slot"] = slot(D.S_SUM_I, 0, d)
                prog.aggs.append(AggOut(a.name, "count", d["slot"], out_type="long"))
                return
            if fname == TIME and t in ("longMin", "longMax"):
                # longMin/longMax over __time (epoch ms): through the f64 expression path (exact
                # below 2^53 ms)
                mn = t == "longMin"
                d = aop(D.A_MIN_F if mn else D.A_MAX_F, -1, [(D.E_COL, prog.col(TIME), float(ds.time_unit_ms))])
                init = _f2ord(math.inf) if mn else _f2ord(-math.inf)
                d["slot"] = slot(D.S_MIN_I if mn else D.S_MAX_I, init, d)
                prog.aggs.append(AggOut(a.name, "min_f" if mn else "max_f", d["slot"], out_type="long",
                                        combine="min" if mn else "max"))
                return
            if fname not in ds.metrics:
                raise LoweringError(f"aggregation over unknown metric {fname!r}")
            m = ds.metrics[fname]
            ci = prog.col(fname)
            is_long = t.startswith("long")
            op = t[4:] if is_long else t[6:]  # Sum / Min / Max
            integral = m.is_integral
            scale = m.scale if m.kind == "decimal" else 0
            if op == "Sum":
                if integral or is_long:
                    d = aop(D.A_SUM_I, ci)
                    d["slot"] = slot(D.S_SUM_I, 0, d)
                    prog.aggs.append(AggOut(a.name, "sum_i", d["slot"], scale=scale if not is_long else scale,
                                            out_type="long" if is_long and scale == 0 else "double"))
                elif self.deterministic:
                    fixed_sum(a.name, [(D.E_COL, ci, 0.0)])
                else:
                    d = aop(D.A_SUM_F, ci)
                    d["slot"] = slot(D.S_SUM_F, 0, d)
                    prog.aggs.append(AggOut(a.name, "sum_f", d["slot"], out_type="double"))
                return
            mn = op == "Min"
            if integral or is_long:
                d = aop(D.A_MIN_I if mn else D.A_MAX_I, ci)
                d["slot"] = slot(D.S_MIN_I if mn else D.S_MAX_I, D.INT64_MAX if mn else D.INT64_MIN, d)
                prog.aggs.append(AggOut(a.name, "min_i" if mn else "max_i", d["slot"], scale=scale,
                                        out_type="long" if is_long and scale == 0 else "double",
                                        combine="min" if mn else "max"))
            else:
                d = aop(D.A_MIN_F if mn else D.A_MAX_F, ci)
                init = _f2ord(math.inf) if mn else _f2ord(-math.inf)
                d["slot"] = slot(D.S_MIN_I if mn else D.S_MAX_I, init, d)
                prog.aggs.append(AggOut(a.name, "min_f" if mn else "max_f", d["slot"], out_type="double",
                                        combine="min" if mn else "max"))
            return
        if isinstance(a, S.HyperUniqueAggregationSpec) and a.fieldName in ds.metrics and \
                ds.metrics[a.fieldName].sketch is not None:
            # rolled-up hyperUnique metric: the rows' stored sparse sketches are unioned after the
            # scan (sketch.hip hll_merge_stored) into the same register layout as query-time HLL
            sk = ds.metrics[a.fieldName].sketch
            if sk.kind != "hll" or sk.p != prog.hll_p:
                raise LoweringError(f"hyperUnique over a {sk.kind} sketch metric {a.fieldName!r}")
            prog.stored_hll.append((a.name, a.fieldName, filt))
            prog.aggs.append(AggOut(a.name, "hll", hll_index=-len(prog.stored_hll), out_type="double", combine="hll"))
            # the JIT scan unions each selected row's stored pairs in place (A_HLL_STORED); without
            # the JIT the executor does it after the scan (engine/executor.py _merge_stored_hll)
            d = aop(D.A_HLL_STORED)
            d["stored"] = len(prog.stored_hll) - 1
            return
        if isinstance(a, (S.CardinalityAggregationSpec, S.HyperUniqueAggregationSpec)):
            fields = a.fieldNames if isinstance(a, S.CardinalityAggregationSpec) else [a.fieldName]
            if len(fields) != 1:
                raise LoweringError("cardinality over several fields is not supported")
            col = fields[0]
            if col not in ds.dims and col not in ds.metrics:
                raise LoweringError(f"cardinality over unknown column {col!r}")
            if col in ds.metrics and ds.metrics[col].sketch is not None:
                raise LoweringError(f"cardinality by row over the sketch metric {col!r}")
            from ..segment.hllcode import code_column

            code = code_column(ds, col, prog.hll_p, _salt(col))
            # a resident (bucket, rho) code plane when the dimension has one (segment/hllcode.py):
            # half the bytes of an int32 id and no per-row hashing; registers are identical
            d = aop(D.A_HLL_CODE, prog.col(code)) if code is not None else aop(D.A_HLL, prog.col(col))
            d["hll"] = prog.nhll
            d["salt"] = _salt(col)
            prog.aggs.append(AggOut(a.name, "hll", hll_index=prog.nhll, out_type="double", combine="hll"))
            prog.nhll += 1
            return
        if isinstance(a, S.JavascriptAggregationSpec):
            try:
                op, params, expr = jsagg_to_expr(a.fnAggregate)
            except JSError as e:
                raise LoweringError(f"javascript aggregator not translatable: {e}")
            ast = parse_expr(expr)
            mapping = dict(zip(params, a.fieldNames))
            eops = self._emit_expr(prog, ast, mapping)
            if op == "sum":
                ex = self._exact_decimal(ast, mapping)
                if ex is not None:
                    # exact decimal sum: per-row value * 10^scale rounded to int64 (exact: the bound
                    # keeps every row < 2^52 and the total < 2^62), summed like a long metric --
                    # deterministic under any atomic order and equal across queries (Q15's
                    # total_revenue = max(total_revenue))
                    sc = ex
                    d = aop(D.A_SUM_X, -1, eops + [(D.E_CONST, 0, float(10 ** sc)), (D.E_MUL, 0, 0.0)])
                    d["slot"] = slot(D.S_SUM_I, 0, d)
                    prog.aggs.append(AggOut(a.name, "sum_i", d["slot"], scale=sc, out_type="double"))
                    return
            if op == "sum" and self.deterministic:
                fixed_sum(a.name, eops)
                return
            kind = {"sum": D.A_SUM_F, "max": D.A_MAX_F, "min": D.A_MIN_F}[op]
            d = aop(kind, -1, eops)
            if op == "sum":
                d["slot"] = slot(D.S_SUM_F, 0, d)
                prog.aggs.append(AggOut(a.name, "sum_f", d["slot"]))
            else:
                mn = op == "min"
                d["slot"] = slot(D.S_MIN_I if mn else D.S_MAX_I, _f2ord(math.inf) if mn else _f2ord(-math.inf), d)
                prog.aggs.append(AggOut(a.name, "min_f" if mn else "max_f", d["slot"], combine=op))
            return
        if isinstance(a, S.ThetaSketchAggregationSpec):
            if a.fieldName not in ds.dims and a.fieldName not in ds.metrics:
                raise LoweringError(f"thetaSketch over unknown column {a.fieldName!r}")
            m = ds.metrics.get(a.fieldName)
            if m is not None and m.sketch is not None and m.sketch.kind != "theta":
                raise LoweringError(f"thetaSketch over the {m.sketch.kind} sketch metric {a.fieldName!r}")
            prog.thetas.append((a.name, a.fieldName, int(a.size)))
            prog.aggs.append(AggOut(a.name, "theta", combine="theta"))
            return
        raise LoweringError(f"unsupported aggregator {type(a).__name__}")

    def _emit_expr(self, prog: ScanProgram, ast, mapping: Dict[str, str]) -> List[tuple]:
        out: List[tuple] = []

        def rec(n, depth):
            k = n[0]
            if k == "const":
                out.append((D.E_CONST, 0, float(n[1])))
                return 1
            if k == "lut":  # explicit per-dictionary table (rank_luts)
                t = n[2]
                prog.keepalive.append(t)
                c = _ptr_as_double(t.data_ptr())
                prog.lut_ptrs[c] = t
                out.append((D.E_LUT, prog.col(n[1]), c))
                return 1
            if k == "col":
                name = mapping.get(n[1], n[1])
                vl = virtual_lut(self.ds, name)
                if vl is not None:
                    # an expression over one dimension evaluated per dictionary entry by the SQL
                    # layer (druid_rewrite._dim_expr_agg): one f64 table lookup by the row's id
                    col, lut = vl
                    prog.keepalive.append(lut)
                    c = _ptr_as_double(lut.data_ptr())
                    prog.lut_ptrs[c] = lut
                    out.append((D.E_LUT, prog.col(col), c))
                    return 1
                if name == TIME:
                    # __time in epoch ms (stored in time units)
                    out.append((D.E_COL, prog.col(TIME), float(self.ds.time_unit_ms)))
                    return 1
                if name in self.ds.dims:
                    # a dimension in a row expression: the value is its dictionary entry read as a
                    # number (javascript coercion: numeric strings -> numbers, ISO dates -> epoch
                    # ms, anything else NaN), one f64 table lookup per row (E_LUT)
                    lut = dim_numeric_lut(self.ds, name)
                    prog.luts[name] = lut
                    prog.keepalive.append(lut)
                    c = _ptr_as_double(lut.data_ptr())
                    prog.lut_ptrs[c] = lut
                    out.append((D.E_LUT, prog.col(name), c))
                    return 1
                if name not in self.ds.metrics:
                    raise LoweringError(f"unknown column {name!r} in expression")
                m = self.ds.metrics.get(name)
                sc = (10.0 ** -m.scale) if (m is not None and m.kind == "decimal" and m.scale) else 0.0
                out.append((D.E_COL, prog.col(name), sc))
                return 1
            unary = {"neg": D.E_NEG, "abs": D.E_ABS, "floor": D.E_FLOOR, "ceil": D.E_CEIL, "sqrt": D.E_SQRT,
                     "log": D.E_LOG, "exp": D.E_EXP}
            if k in unary:
                d = rec(n[1], depth)
                out.append((unary[k], 0, 0.0))
                return d
            op = {"add": D.E_ADD, "sub": D.E_SUB, "mul": D.E_MUL, "div": D.E_DIV, "min": D.E_MIN, "max": D.E_MAX,
                  "mod": D.E_MOD, "pmod": D.E_PMOD, "pow": D.E_POW}[k]
            d1 = rec(n[1], depth)
            d2 = rec(n[2], depth + 1)
            out.append((op, 0, 0.0))
            return max(d1, d2 + 1)

        if rec(ast, 0) > 4:
            raise LoweringError("aggregator expression too deep for the device VM")
        return out

    def fold_presence_slot(self, prog: ScanProgram) -> None:
        """The hidden presence count (slot 0) only has to be > 0 for groups that exist.  An
        unfiltered long sum over a metric whose values are all >= 1 (l_quantity) has exactly that
        property, so it becomes slot 0 and the scan does one atomic less per row (TPC-H Q18 over
        150M order groups: 3 -> 2 HBM atomics per line)."""
        if not FOLD_PRESENCE or len(prog.aops) < 2 or prog.aops[0]["slot"] != 0:
            return
        if any(d["slot"] == 0 for d in prog.aops[1:]) or any(a.slot == 0 for a in prog.aggs):
            return  # a user count(*) already shares the presence slot
        for d in prog.aops[1:]:
            if d["kind"] != D.A_SUM_I or d["filter"] is not None or d["expr"] is not None or d["col"] < 0:
                continue
            name = prog.colname(d["col"])
            m = self.ds.metrics.get(name)
            if m is None or name in self.ds.dims or not m.is_integral or self._metric_range(name)[0] < 1:
                continue
            s_old = d["slot"]
            if sum(1 for x in prog.aops if x["slot"] == s_old) != 1:
                continue
            prog.aops.pop(0)
            prog.slots.pop(s_old)
            for x in prog.aops:
                if x is d:
                    x["slot"] = 0
                elif x["slot"] > s_old:
                    x["slot"] -= 1
            for a in prog.aggs:
                if a.slot == s_old:
                    a.slot = 0
                elif a.slot > s_old:
                    a.slot -= 1
            return

    # ------------------------------------------------------------------ functional dependencies
    def eliminate_dependent_keys(self, prog: ScanProgram) -> None:
        """Drop grouping keys that another grouping key functionally determines in the data
        (``s_name, s_address, s_phone`` given ``l_suppkey``; ``o_orderdate, o_custkey`` given
        ``o_orderkey``).  They do not split groups, so the packed key covers the determinants only
        -- wide TPC-H group-bys (Q2, Q10, Q18) stay far inside 64 bits and in the dense/LDS
        paths -- and the dependent values are decoded from the determinant's id through the FD
        table (``prog.derived``).  The reference only declares FDs for its cost model
        (``functionalDependencies`` DDL option, ``sd/FunctionalDependencies.scala``); here they
        are verified on the index itself (and across ranks), so no declaration can make results
        wrong."""
        if not FD_KEYS:
            return
        cand = [i for i, kc in enumerate(prog.keys) if kc.kind == D.K_ID and kc.card > 1]
        if len(cand) < 2:
            return
        alive = set(cand)
        derived = []
        while True:
            best, best_deps = None, []
            for i in sorted(alive):
                deps = [j for j in sorted(alive) if j != i and fd_table(self.ds, prog.keys[i].col, prog.keys[j].col,
                                                                         self.world) is not None]
                if len(deps) > len(best_deps):
                    best, best_deps = i, deps
            if not best_deps:
                break
            for j in best_deps:
                alive.discard(j)
                derived.append((j, best))
            alive.discard(best)
        if not derived:
            return
        drop = {j for j, _ in derived}
        keep = [i for i in range(len(prog.keys)) if i not in drop]
        pos = {old: new for new, old in enumerate(keep)}
        for j, i in derived:
            kc = prog.keys[j]
            lut = fd_table(self.ds, prog.keys[i].col, kc.col, self.world)
            prog.derived.append((kc, pos[i], lut))
        prog.keys = [prog.keys[i] for i in keep]

    def eliminate_dependent_aggs(self, prog: ScanProgram) -> None:
        """MIN/MAX of a metric that is constant per value of a grouping key (TPC-H Q18
        ``max(o_totalprice)`` per order, Q10 ``max(c_acctbal)`` per customer) needs no per-row
        accumulator: the value is gathered per result group from an FD table (verified on the
        index, all ranks).  Q18 over 150M order groups: one HBM atomic less per line."""
        if not FD_KEYS or any(kc.collapse for kc in prog.keys):
            return
        dets = [i for i, kc in enumerate(prog.keys) if kc.kind == D.K_ID and kc.card > 1]
        if not dets:
            return
        for a in list(prog.aggs):
            s = a.slot
            if a.kind not in ("min_i", "max_i") or s <= 0:
                continue
            users = [d for d in prog.aops if d["slot"] == s]
            if len(users) != 1 or any(x is not a and x.slot == s for x in prog.aggs):
                continue
            d = users[0]
            if d["filter"] is not None or d["expr"] is not None or d["col"] < 0:
                continue
            name = prog.colname(d["col"])
            if name not in self.ds.metrics or name in self.ds.dims:
                continue
            hit = None
            for i in dets:
                lut = fd_metric_table(self.ds, prog.keys[i].col, name, self.world)
                if lut is not None:
                    hit = (i, lut)
                    break
            if hit is None:
                continue
            prog.aops.remove(d)
            prog.slots.pop(s)
            for x in prog.aops:
                if x["slot"] > s:
                    x["slot"] -= 1
            for x in prog.aggs:
                if x.slot > s:
                    x.slot -= 1
            a.slot = -1
            prog.derived_aggs.append((a, hit[0], hit[1]))

    # ------------------------------------------------------------------ whole query
    def lower_aggregate(self, intervals, filter_spec, dimensions, granularity, aggregations,
                        extra_keys: Sequence[KeyComp] = ()) -> ScanProgram:
        try:
            return self._lower_aggregate(intervals, filter_spec, dimensions, granularity, aggregations, extra_keys)
        except LoweringError:
            if not IMPLY_OR:
                raise
            # (the implied conjuncts made the program too large: lower the filter as written)
            return self._lower_aggregate(intervals, filter_spec, dimensions, granularity, aggregations, extra_keys,
                                         imply=False)

    def _lower_aggregate(self, intervals, filter_spec, dimensions, granularity, aggregations,
                         extra_keys: Sequence[KeyComp] = (), imply: bool = True) -> ScanProgram:
        prog = ScanProgram(self.ds)
        bexpr = self.filter_ir(filter_spec)
        bexpr = imply_or_conjuncts(bexpr) if imply else bexpr
        ranges, bexpr, ivs = self.query_ranges(intervals, bexpr)
        prog.ranges = ranges
        prog.bexpr = bexpr
        if _is(bexpr, "false") or not ranges:
            prog.empty = True
        # hidden presence count (slot 0)
        prog.slots.append((D.S_SUM_I, 0))
        prog.aops.append({"kind": D.A_COUNT, "col": -1, "expr": None, "filter": None, "slot": 0, "hll": -1,
                          "sig": (D.A_COUNT, -1, "None", "None", D.S_SUM_I, 0)})
        gk = self.granularity_key(granularity, ivs)
        if gk is not None:
            prog.keys.append(gk)
        for dspec in dimensions:
            prog.keys.append(self.key_for_dimension(dspec, ivs))
        prog.keys.extend(extra_keys)
        if len(prog.keys) > D.MAX_KOPS:
            raise LoweringError("too many grouping keys")
        for a in aggregations:
            self.add_aggregator(prog, a)
        for a in prog.aggs:  # stored-sketch registers come after the scan's HLL blocks
            if a.kind == "hll" and a.hll_index < 0:
                a.hll_index = prog.nhll + (-a.hll_index - 1)
        prog.presence_only = not aggregations and not extra_keys
        self.fold_presence_slot(prog)
        prog.key_order = [kc.name for kc in prog.keys]
        self.eliminate_dependent_keys(prog)
        self.eliminate_dependent_aggs(prog)
        # filter-implied key domains: a dimension the filter pins to a few values only needs
        # that many key slots (Q7: s_nation x c_nation shrinks 25x25 -> 2x2), which keeps the
        # accumulators in LDS instead of contended HBM atomics
        for i, kc in enumerate(prog.keys):
            if kc.kind == D.K_ID:
                imp = implied_ids(bexpr, kc.col)
                if imp is not None and int(imp.sum()) < kc.card:
                    prog.keys[i] = compact_key(kc, imp)
        # mixed radix strides (last key fastest)
        G = 1
        for kc in reversed(prog.keys):
            kc.stride = G
            G *= max(1, kc.card)
        if G >= 2 ** 62:
            raise LoweringError("group key space exceeds 64 bits")
        prog.G = G
        prog.est_rows = prog.rows_in_ranges * self.selectivity(bexpr)
        w = self.world
        if w is not None and w.distributed and getattr(self.ds, "fd_source", None) is None:
            # the group-by table (and so the partials' dense/sparse layout) is planned from the row
            # estimate: every rank must decide alike, also when shards differ in size
            prog.est_rows = w.max_float(float(prog.est_rows))
        if not prog.empty:
            for kc in prog.keys:
                kc.col_idx = prog.col(kc.col)  # payload section
            self.emit_main_filter(prog, bexpr)
            prog.section = "p"
            for d in prog.aops:
                if d["filter"] is not None:
                    off = len(prog.fops)
                    dep = self.emit_filter(prog, d["filter"])
                    if dep > D.STACK_DEPTH:
                        raise LoweringError("aggregator filter too deep")
                    d["filt_off"], d["filt_len"] = off, len(prog.fops) - off
            for d in prog.aops:
                if d["expr"] is not None:
                    d["expr_off"] = len(prog.eops)
                    prog.eops.extend(d["expr"])
                    d["expr_len"] = len(d["expr"])
            if len(prog.fops) > D.MAX_FOPS or len(prog.eops) > D.MAX_EOPS:
                raise LoweringError("query program too large for the device descriptor")
            self.pick_zones(prog, bexpr)
        return prog

    def emit_main_filter(self, prog: ScanProgram, bexpr) -> None:
        """Split the filter's top-level conjuncts: bitmap-only ones become the chunk-level
        pre-filter (one vector load per leaf per 4096 rows, lane = 64-row word); the rest is the
        per-word program over filter-phase columns staged into LDS."""
        conj = bexpr[1] if _is(bexpr, "and") else ([] if _is(bexpr, "true") else [bexpr])
        pre, rest, nleaves = [], [], 0
        for c in conj:
            n = self.bitmap_only(c)
            if n >= 0 and nleaves + n <= D.MAX_BM:
                pre.append(c)
                nleaves += n
            else:
                rest.append(c)
        # the pre-filter is emitted first so its bitmap leaves are reserved (the per-row section may
        # then fall back to column tests where leaves run out; the chunk-level pre-filter cannot),
        # and placed after the per-row section
        head = prog.fops
        prog.fops = []
        if pre:
            depth = self.emit_filter(prog, b_and(pre))
            if depth > D.STACK_DEPTH:
                raise LoweringError("filter too deep for the device stack")
            if any(int(f[0]) not in _PRE_OPS for f in prog.fops):
                raise LoweringError("chunk pre-filter is not bitmap-only")
        pre_ops = prog.fops
        prog.fops = head
        prog.section = "f"
        if rest:
            depth = self.emit_filter(prog, b_and(rest))
            if depth > D.STACK_DEPTH:
                raise LoweringError("filter too deep for the device stack")
        prog.filter_len = len(prog.fops)
        prog.final_pre = not rest
        prog.pre_off = len(prog.fops)
        prog.fops.extend(pre_ops)
        prog.pre_len = len(prog.fops) - prog.pre_off
        prog.section = "p"

    def lower_mask(self, intervals, filter_spec) -> ScanProgram:
        try:
            return self._lower_mask(intervals, filter_spec)
        except LoweringError:
            if not IMPLY_OR:
                raise
            return self._lower_mask(intervals, filter_spec, imply=False)

    def _lower_mask(self, intervals, filter_spec, imply: bool = True) -> ScanProgram:
        prog = ScanProgram(self.ds)
        bexpr = self.filter_ir(filter_spec)
        bexpr = imply_or_conjuncts(bexpr) if imply else bexpr
        ranges, bexpr, ivs = self.query_ranges(intervals, bexpr)
        prog.ranges, prog.bexpr = ranges, bexpr
        if _is(bexpr, "false") or not ranges:
            prog.empty = True
            return prog
        self.emit_main_filter(prog, bexpr)
        self.pick_zones(prog, bexpr)
        return prog


FIX_ONE = float(1 << 32)  # fixed-point unit of deterministic float sums (AggOut.kind sum_fx)


def fixed_value(hi, lo):
    """Value of a deterministic float sum from its integer-part and fraction slots (numpy or
    torch int64 arrays) as float64."""
    return hi.astype(np.float64) + lo.astype(np.float64) / FIX_ONE if isinstance(hi, np.ndarray) else \
        hi.to(torch.float64) + lo.to(torch.float64) / FIX_ONE


def _eops_depth(eops) -> int:
    """Peak stack depth of a postfix expression program (the device VM keeps 4 registers)."""
    d = peak = 0
    for op, _, _ in eops:
        if op in (D.E_COL, D.E_CONST, D.E_LUT):
            d += 1
        elif op not in D.E_UNARY:
            d -= 1
        peak = max(peak, d)
    return peak


def _ptr_as_double(ptr: int) -> float:
    import struct

    return struct.unpack("<d", struct.pack("<Q", int(ptr)))[0]


def _numeric_value(v) -> float:
    if v is None:
        return math.nan
    if isinstance(v, (bool, np.bool_)):
        return float(v)
    if isinstance(v, (int, float, np.integer, np.floating)):
        return float(v)
    s = str(v).strip()
    try:
        return float(s)
    except ValueError:
        pass
    if len(s) >= 10 and s[4:5] == "-" and s[7:8] == "-":
        try:
            return float(parse_iso_ms(s))
        except Exception:  # noqa: BLE001
            return math.nan
    return math.nan


def _ast_cols(a) -> List[str]:
    if a[0] == "col":
        return [a[1]]
    if a[0] in ("const", "lut"):
        return []
    return [c for x in a[1:] for c in _ast_cols(x)]


_FD_CHUNK = 1 << 26


_FD_MISSING = -(2 ** 63)


def _fd_lut(ids_a: torch.Tensor, card_a: int, vals_b: torch.Tensor, n: int, world=None) -> Optional[torch.Tensor]:
    """int64 table a-id -> b-value when every row's b is a function of its a (all ranks), with
    _FD_MISSING for a-ids no rank holds; None when the dependency does not hold."""
    dev = ids_a.device
    lut = torch.full((card_a,), _FD_MISSING, dtype=torch.int64, device=dev)
    for s0 in range(0, n, _FD_CHUNK):
        lut.scatter_(0, ids_a[s0:min(n, s0 + _FD_CHUNK)].to(torch.int64), vals_b[s0:min(n, s0 + _FD_CHUNK)].to(torch.int64))
    ok = torch.ones((), dtype=torch.int64, device=dev)
    for s0 in range(0, n, _FD_CHUNK):
        ia = ids_a[s0:min(n, s0 + _FD_CHUNK)].to(torch.int64)
        ok &= (lut[ia] == vals_b[s0:min(n, s0 + _FD_CHUNK)].to(torch.int64)).all().to(torch.int64)
    if world is not None and world.distributed:
        hi = world.all_reduce(lut.clone(), "max")
        big = torch.iinfo(torch.int64).max
        lo = world.all_reduce(torch.where(lut == _FD_MISSING, torch.full_like(lut, big), lut), "min")
        ok &= ((lo == big) | (lo == hi)).all().to(torch.int64)
        ok = world.all_reduce(ok, "min")
        lut = hi
    return lut if bool(ok.item()) else None


def fd_metric_table(ds: DataSource, a: str, metric: str, world=None) -> Optional[torch.Tensor]:
    """Device table a-id -> stored metric value when the metric is constant per value of
    dimension ``a`` (o_totalprice per order, c_acctbal per customer); cached per datasource."""
    cache = ds.__dict__.setdefault("_fd_cache", {})
    key = (a, "metric:" + metric)
    ds = getattr(ds, "fd_source", None) or ds  # streamed window: decide over the whole shard
    if key not in cache:
        from ..utils.streams import publish

        cache[key] = publish(_fd_lut(ds.dims[a].ids, len(ds.dims[a].dictionary), column_tensor(ds, metric),
                                     ds.num_rows, world), ds.dims[a].ids.device)
    return cache[key]


def virtual_lut(ds, name: str):
    """(column, device f64 table) of a per-dictionary-entry expression table registered by the SQL
    rewrite under ``name`` (``__vx_*``), or None."""
    src = getattr(ds, "fd_source", None) or ds
    reg = src.__dict__.get("_virtual_luts") if hasattr(src, "__dict__") else None
    if not reg or name not in reg:
        return None
    cache = src.__dict__.setdefault("_virtual_luts_dev", {})
    t = cache.get(name)
    col, arr = reg[name]
    if t is None:
        dev = src.time.device if col == TIME else src.dims[col].ids.device
        t = cache[name] = torch.from_numpy(arr).to(dev)
    return col, t


def fd_table(ds: DataSource, a: str, b: str, world=None) -> Optional[torch.Tensor]:
    """If dimension ``a`` functionally determines dimension ``b`` over every row of the index
    (all shards), the device table a-id -> b-id (int32, -1 for ids absent everywhere); else None.
    Two scatter/gather passes over the id columns on the device, cached per datasource."""
    cache = ds.__dict__.setdefault("_fd_cache", {})
    key = (a, b)
    if key in cache:
        return cache[key]
    ds = getattr(ds, "fd_source", None) or ds  # streamed window: decide over the whole shard
    da, db = ds.dims[a], ds.dims[b]
    ca = len(da.dictionary)
    dev = da.ids.device
    lut = torch.full((ca,), -1, dtype=torch.int64, device=dev)
    n = ds.num_rows
    for s0 in range(0, n, _FD_CHUNK):  # (id columns are padded past num_rows)
        ia = da.ids[s0:min(n, s0 + _FD_CHUNK)].to(torch.int64)
        ib = db.ids[s0:min(n, s0 + _FD_CHUNK)].to(torch.int64)
        lut.scatter_(0, ia, ib)
    ok = torch.ones((), dtype=torch.int64, device=dev)
    for s0 in range(0, n, _FD_CHUNK):
        ia = da.ids[s0:min(n, s0 + _FD_CHUNK)].to(torch.int64)
        ib = db.ids[s0:min(n, s0 + _FD_CHUNK)].to(torch.int64)
        ok &= (lut[ia] == ib).all().to(torch.int64)
    if world is not None and world.distributed:
        # global FD: every rank's table agrees wherever two ranks both saw an a-id
        hi = world.all_reduce(lut.clone(), "max")
        big = torch.iinfo(torch.int64).max
        lo = world.all_reduce(torch.where(lut < 0, torch.full_like(lut, big), lut), "min")
        ok &= ((lo == big) | (lo == hi)).all().to(torch.int64)
        ok = world.all_reduce(ok, "min")
        lut = hi
    # kept on the device (int32): finalize gathers the dependent ids of the result groups there --
    # a host gather into a 150M-entry table costs a cache miss per group
    from ..utils.streams import publish

    out = lut.to(torch.int32) if bool(ok.item()) else None
    cache[key] = publish(out, dev)
    if TRACE_FD:
        print(f"[fd] {a} -> {b}: {'yes' if out is not None else 'no'}", flush=True)
    return out


def rank_luts(ds: DataSource, a: str, b: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """f64 rank of every dictionary value of dims a and b in the sorted union of both
    dictionaries (NULL -> NaN): comparing ranks == comparing the values as strings."""
    key = ("_ranklut", a, b)
    cache = ds.__dict__.setdefault("_lut_cache", {})
    if key in cache:
        return cache[key]
    va = ds.dims[a].dictionary.all_values()
    vb = ds.dims[b].dictionary.all_values()

    def strs(vs):
        return [None if v is None else str(v) for v in vs]

    sa, sb = strs(va), strs(vb)
    union = sorted({v for v in sa + sb if v is not None})
    pos = {v: float(i) for i, v in enumerate(union)}
    dev = ds.dims[a].ids.device
    ta = torch.tensor([pos[v] if v is not None else math.nan for v in sa], dtype=torch.float64, device=dev)
    tb = torch.tensor([pos[v] if v is not None else math.nan for v in sb], dtype=torch.float64, device=dev)
    from ..utils.streams import publish

    cache[key] = publish((ta, tb), dev)
    return ta, tb


def dim_numeric_lut(ds: DataSource, dim: str) -> torch.Tensor:
    """f64 value of every dictionary entry of `dim` (cached on the column)."""
    dc = ds.dims[dim]
    lut = getattr(dc, "_numlut", None)
    if lut is not None:
        return lut
    dic = dc.dictionary
    if dic.vtype != "string" and (dic.lazy or not dic.has_null):
        vals = np.asarray(dic.values, dtype=np.float64) if not dic.lazy else \
            dic.decode(np.arange(len(dic))).astype(np.float64)
    else:
        vals = np.asarray(dic.map_values(_numeric_value), dtype=np.float64)
    lut = torch.from_numpy(np.ascontiguousarray(vals)).to(dc.ids.device)
    dc._numlut = lut  # type: ignore[attr-defined]
    return lut


def implied_ids(x, dim: str) -> Optional[np.ndarray]:
    """Ids of `dim` that can satisfy filter x (None = unrestricted)."""
    k = x[0]
    if k == "ids":
        return x[2] if x[1] == dim else None
    if k == "and":
        out = None
        for c in x[1]:
            m = implied_ids(c, dim)
            if m is not None:
                out = m.copy() if out is None else (out & m)
        return out
    if k == "or":
        out = None
        for c in x[1]:
            m = implied_ids(c, dim)
            if m is None:
                return None
            out = m.copy() if out is None else (out | m)
        return out
    if k == "false":
        return None
    return None


def compact_key(kc: KeyComp, mask: np.ndarray) -> KeyComp:
    ids = np.flatnonzero(mask)
    if len(ids) == 0:
        ids = np.array([0])
    a, n = int(ids[0]), len(ids)
    if kc.kind == D.K_ID and kc.base == 0 and int(ids[-1]) - a + 1 == n and n > 1:
        # a contiguous id run (a value range, a key-range pass): a key window [a, a+n) -- the
        # kernel subtracts the base, no remap table to upload or gather through
        dec = kc.decoder
        ids_t = ids.astype(np.int64)
        out = KeyComp(kc.name, D.K_ID, kc.col, n, base=a, orig=ids_t,
                      decoder=(lambda c: dec(np.asarray(c, dtype=np.int64) + a)) if dec else (lambda c: np.asarray(c) + a))
        out.dictionary = getattr(kc, "dictionary", None)
        return out
    remap = np.zeros(len(mask), dtype=np.int32)
    remap[ids] = np.arange(len(ids), dtype=np.int32)
    dec = kc.decoder
    ids_t = ids.astype(np.int64)
    return KeyComp(kc.name, D.K_REMAP, kc.col, len(ids), remap=remap, orig=ids_t,
                   decoder=(lambda c: dec(ids_t[np.asarray(c, dtype=np.int64)])) if dec else (lambda c: ids_t[c]))


def pack_bitset(mask: np.ndarray) -> np.ndarray:
    """bool[n] -> int64 words, bit (i & 63) of word (i >> 6) == mask[i] (the kernel's F_IN_SET layout)"""
    n64 = (len(mask) + 63) // 64
    b = np.packbits(np.asarray(mask, dtype=bool), bitorder="little")
    buf = np.zeros(n64 * 8, dtype=np.uint8)
    buf[:len(b)] = b
    return buf.view("<i8").astype(np.int64, copy=False)


def _depth(x) -> int:
    if x[0] in ("and", "or"):
        ds = sorted((_depth(c) for c in x[1]), reverse=True)
        return max(ds[0], 1 + (ds[1] if len(ds) > 1 else 0))
    if x[0] == "not":
        return _depth(x[1])
    return 1


def _runs(mask: np.ndarray, limit: Optional[int] = None) -> Optional[List[Tuple[int, int]]]:
    """[(start, end)] of the True runs of ``mask``; None when there are more than ``limit`` (a
    LIKE over a 20M-value dictionary has ~1M runs: counting them is cheap, listing them is not)."""
    if limit is not None and mask_stats(mask).runs > limit:
        return None
    m = np.concatenate([[False], mask.astype(bool), [False]])
    d = np.diff(m.astype(np.int8))
    starts = np.flatnonzero(d == 1)
    ends = np.flatnonzero(d == -1)
    return list(zip(starts.tolist(), ends.tolist()))


class MaskStats:
    """Counts of a dictionary-id mask the lowering asks for more than once: set size, True / False
    run counts, first / last True id, and its packed F_IN_SET words per device."""
    __slots__ = ("k", "runs", "neg_runs", "lo", "hi", "words", "mask")

    def __init__(self, mask: np.ndarray):
        m = mask.astype(bool, copy=False)
        n = len(m)
        self.mask = mask  # (pins the id this entry is cached under)
        self.k = int(np.count_nonzero(m))
        if n == 0 or self.k == 0:
            self.runs, self.neg_runs, self.lo, self.hi = 0, min(n, 1), 0, 0
        else:
            self.runs = int(np.count_nonzero(np.greater(m[1:], m[:-1]))) + int(m[0])
            self.neg_runs = self.runs - 1 + int(not m[0]) + int(not m[-1])
            self.lo = int(np.argmax(m))
            self.hi = n - int(np.argmax(m[::-1]))
        self.words: Dict[str, torch.Tensor] = {}


_MASK_STATS: "Dict[int, MaskStats]" = {}
_MASK_STATS_MIN = 1 << 16   # smaller masks are recomputed (cheap, and usually fresh arrays)
_MASK_STATS_MAX = 16   # (each entry pins its mask: up to a few MB of host memory)


def mask_stats(mask: np.ndarray) -> MaskStats:
    """``MaskStats`` of ``mask``, cached by identity for large masks: a dictionary's LIKE / regex
    masks are cached per pattern (segment/dictionary.py ``like_mask``), so every parameterization of
    a template that filters ``p_name LIKE '%green%'`` hands the lowering the same 20M-entry array."""
    if len(mask) < _MASK_STATS_MIN:
        return MaskStats(mask)
    st = _MASK_STATS.get(id(mask))
    if st is None or st.mask is not mask:
        st = MaskStats(mask)
        if len(_MASK_STATS) >= _MASK_STATS_MAX:
            _MASK_STATS.pop(next(iter(_MASK_STATS)))
        _MASK_STATS[id(mask)] = st
    return st


def _f2ord(f: float) -> int:
    b = int(np.array([f], dtype=np.float64).view(np.int64)[0])
    return b if b >= 0 else b ^ 0x7FFFFFFFFFFFFFFF


def ord2f(v: np.ndarray) -> np.ndarray:
    v = np.asarray(v, dtype=np.int64)
    b = np.where(v >= 0, v, v ^ np.int64(0x7FFFFFFFFFFFFFFF))
    return b.view(np.float64)


def _salt(col: str) -> int:
    import zlib

    return zlib.crc32(col.encode()) & 0x7FFFFFFF


def _to_ms(v) -> int:
    if isinstance(v, (int, np.integer)):
        return int(v)
    if isinstance(v, float):
        return int(v)
    s = str(v)
    if re.fullmatch(r"-?\d+", s):
        return int(s)
    return parse_iso_ms(s)


def col_meta(t: torch.Tensor, plane: int) -> Tuple[int, int]:
    """(meta, planes) for the kernel's LDS staging: lg | signed << 4 | float << 5 | plane << 8"""
    lg = {1: 0, 2: 1, 4: 2, 8: 3}[t.element_size()]
    sgn = 1 if t.dtype in (torch.int16, torch.int32, torch.int64) else 0
    flt = 1 if t.dtype.is_floating_point else 0
    return lg | (sgn << 4) | (flt << 5) | (plane << 8), (2 if lg == 3 else 1)


def lds_layout(prog: ScanProgram, acc_hll_bytes: int, unroll: int, waves: int) -> Tuple[int, int, int, int]:
    """(cache_off, wave_bytes, nplanes, total_lds) of the kernel's dynamic LDS."""
    nplanes = 0
    for name in prog.cols:
        nplanes += 2 if column_tensor(prog.ds, name).element_size() == 8 else 1
    cache_off = (acc_hll_bytes + 15) // 16 * 16
    wave_bytes = nplanes * unroll * 256 + len(prog.bm_leaves) * 512
    wave_bytes = (wave_bytes + 15) // 16 * 16
    return cache_off, wave_bytes, nplanes, cache_off + waves * wave_bytes


def pack(prog: ScanProgram, mode: int, dedup: int, hll_lds: int, lds_bytes: int, out_acc: int, out_keys: int,
         hash_cap: int, overflow: int, out_mask: int, out_count: int, hll_ptrs: Sequence[int],
         hll_lds_offs: Sequence[int], unroll: int = 2, cache_off: int = 0, wave_bytes: int = 0) -> np.ndarray:
    """Serialize a program into ScanDesc bytes (device pointers are plain integers)."""
    ds = prog.ds
    d = D.new_desc()
    r = d[0]
    r["ncols"] = len(prog.cols)
    plane = 0
    packed = getattr(prog, "packed", None) or {}
    for base, names in ((0, prog.fcols), (D.PAYLOAD_BASE, prog.pcols)):
        for j, name in enumerate(names):
            t = column_tensor(ds, name)
            meta, npl = col_meta(t, plane)
            plane += npl
            c = r["cols"][base + j]
            # the JIT kernel of this program reads the bit-packed copy (segment/packed.py)
            ptr = packed[name].data.data_ptr() if name in packed else t.data_ptr()
            c["ptr"], c["dtype"], c["meta"] = ptr, dtype_code(t), meta
    r["nfc"], r["npc"], r["nplanes"] = len(prog.fcols), len(prog.pcols), plane
    r["lds_cache_off"], r["lds_wave_bytes"], r["unroll"] = cache_off, wave_bytes, unroll
    if ds.device.type == "cuda":
        from ..ops import native

        r["narrow4"] = native.narrow4()
    r["pre_off"], r["pre_len"], r["final_pre"] = prog.pre_off, prog.pre_len, 1 if prog.final_pre else 0
    r["nbm"] = len(prog.bm_leaves)
    for j, (row, stride, count) in enumerate(prog.bm_leaves):
        r["bm_bits"][j], r["bm_stride"][j], r["bm_count"][j] = row.data_ptr(), stride, count
    r["nfops"] = len(prog.fops)
    r["filter_len"] = prog.filter_len
    for i, (op, col, flags, lo, hi, flo, fhi, bits) in enumerate(prog.fops):
        f = r["fops"][i]
        f["op"], f["col"], f["flags"], f["lo"], f["hi"], f["flo"], f["fhi"] = op, col, flags, lo, hi, flo, fhi
        f["bits"] = bits.data_ptr() if bits is not None else 0
    r["nkops"] = len(prog.keys)
    for i, kc in enumerate(prog.keys):
        k = r["kops"][i]
        k["kind"], k["col"], k["tfield"] = kc.kind, kc.col_idx, kc.tfield
        k["stride"], k["base"], k["card"] = kc.stride, kc.base, kc.card
        k["unit_ms"] = ds.time_unit_ms
        k["tz_ms"], k["period_ms"], k["origin_ms"] = kc.tz_ms, kc.period_ms or 1, kc.origin_ms
        table = kc.remap if kc.remap is not None else (kc.tlut if kc.kind == D.K_TIME else None)
        if table is not None:
            t = getattr(kc, "_remap_dev", None)
            if t is None or t.device != ds.device:
                # (cached remap tables are read-only arrays: torch gets its own copy)
                t = torch.from_numpy(table if table.flags.writeable else table.copy()).to(ds.device)
                kc._remap_dev = t  # type: ignore[attr-defined]
            prog.keepalive.append(t)
            k["remap"] = t.data_ptr()
    r["naggs"] = len(prog.aops)
    for i, a in enumerate(prog.aops):
        o = r["aops"][i]
        o["kind"], o["col"], o["slot"] = a["kind"], a["col"], max(a["slot"], 0)
        o["expr_off"], o["expr_len"] = a.get("expr_off", 0), a.get("expr_len", 0)
        o["filt_off"], o["filt_len"] = a.get("filt_off", 0), a.get("filt_len", 0)
        if a["kind"] in D.HLL_KINDS:
            o["hll_regs"] = hll_ptrs[a["hll"]]
            o["hll_lds_off"] = hll_lds_offs[a["hll"]] if hll_lds_offs else 0
            o["salt"] = a.get("salt", 0)
        elif a["kind"] == D.A_HLL_STORED and len(hll_ptrs) > prog.nhll + a["stored"]:
            # (registers exist only when the JIT fuses the union: PreparedScan allocates them)
            sk = ds.metrics[prog.stored_hll[a["stored"]][1]].sketch
            o["hll_regs"] = hll_ptrs[prog.nhll + a["stored"]]
            o["sk_off"], o["sk_val"] = sk.offsets.data_ptr(), sk.values.data_ptr()
    r["neops"] = len(prog.eops)
    for i, (op, col, c) in enumerate(prog.eops):
        e = r["eops"][i]
        e["op"], e["col"], e["c"] = op, col, c
    r["nzones"] = len(prog.zones)
    for i, (dim, lo, hi) in enumerate(prog.zones):
        z = r["zones"][i]
        dc = ds.dims[dim]
        z["col"], z["lo"], z["hi"] = 0, lo, hi
        z["zmin"], z["zmax"] = dc.zmin.data_ptr(), dc.zmax.data_ptr()
    total = 0
    r["nranges"] = len(prog.ranges)
    for i, (a, b) in enumerate(prog.ranges):
        g = r["ranges"][i]
        c0 = a // CHUNK_ROWS
        c1 = (b + CHUNK_ROWS - 1) // CHUNK_ROWS
        g["lo"], g["hi"], g["chunk_begin"], g["nchunks"] = a, b, c0, c1 - c0
        total += c1 - c0
    r["total_chunks"] = total
    r["num_rows"] = ds.num_rows
    r["nslots"] = len(prog.slots)
    for i, (op, init) in enumerate(prog.slots):
        r["slot_op"][i] = op
        r["slot_init"][i] = init
    r["mode"], r["dedup"], r["hll_lds"], r["hll_p"], r["nhll"] = mode, dedup, hll_lds, prog.hll_p, prog.nhll
    r["lds_bytes"] = lds_bytes
    r["G"] = prog.G
    r["out_acc"], r["out_keys"], r["hash_cap"], r["overflow"] = out_acc, out_keys, hash_cap, overflow
    r["out_mask"], r["out_count"] = out_mask, out_count
    return d
