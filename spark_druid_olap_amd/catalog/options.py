"""Druid relation options (the DDL ``OPTIONS(...)``) and the session configuration registry.

Option names, defaults and the per-session overrides keep the reference's surface so existing DDL
runs unchanged: ``sd/DefaultSource.scala:197-308`` (options), ``sd/metadata/DruidRelationInfo.scala:84-140``
(``DruidRelationOptions`` + ``spark.sparklinedata.druid.option.<name>`` overrides),
``asd/DruidPlanner.scala:60-169`` (SQLConf keys).  Options that only made sense for a remote Druid
cluster (ZooKeeper, Smile, HTTP pools) are accepted and recorded; they have no effect in-process.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional

REQUIRED = ("sourceDataframe", "druidDatasource", "timeDimensionColumn")

NON_AGG_HANDLING = ("push_none", "push_filters", "push_project_and_filters")


def _bool(v) -> bool:
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() in ("true", "1", "yes", "y")


@dataclass
class DruidRelationOptions:
    maxCardinality: int = 1_000_000               # maxResultCardinality (dead in reference too)
    cardinalityPerDruidQuery: int = 100_000       # maxCardinalityPerQuery (dead)
    pushHLLTODruid: bool = True
    streamDruidQueryResults: bool = True          # (dead)
    loadMetadataFromAllSegments: bool = True
    zkSessionTimeoutMs: int = 30000
    zkEnableCompression: bool = True
    zkDruidPath: str = "/druid"
    queryHistoricalServers: bool = False
    zkQualifyDiscoveryNames: bool = False
    numSegmentsPerHistoricalQuery: int = 2 ** 31 - 1
    useSmile: bool = True
    nonAggQueryHandling: str = "push_none"
    queryGranularity: str = "none"                # (dead)
    allowTopN: bool = False
    topNMaxThreshold: int = 100000
    numProcessingThreadsPerHistorical: Optional[int] = None

    @staticmethod
    def from_options(opts: Dict[str, str]) -> "DruidRelationOptions":
        g = opts.get
        o = DruidRelationOptions()
        o.maxCardinality = int(g("maxResultCardinality", o.maxCardinality))
        o.cardinalityPerDruidQuery = int(g("maxCardinalityPerQuery", o.cardinalityPerDruidQuery))
        o.pushHLLTODruid = _bool(g("pushHLLTODruid", True))
        o.streamDruidQueryResults = _bool(g("streamDruidQueryResults", True))
        o.loadMetadataFromAllSegments = _bool(g("loadMetadataFromAllSegments", True))
        o.zkSessionTimeoutMs = int(g("zkSessionTimeoutMilliSecs", o.zkSessionTimeoutMs))
        o.zkEnableCompression = _bool(g("zkEnableCompression", True))
        o.zkDruidPath = g("zkDruidPath", o.zkDruidPath)
        o.queryHistoricalServers = _bool(g("queryHistoricalServers", False))
        o.zkQualifyDiscoveryNames = _bool(g("zkQualifyDiscoveryNames", False))
        o.numSegmentsPerHistoricalQuery = int(g("numSegmentsPerHistoricalQuery", o.numSegmentsPerHistoricalQuery))
        o.useSmile = _bool(g("useSmile", True))
        nah = g("nonAggregateQueryHandling", "push_none").lower()
        if nah not in NON_AGG_HANDLING:
            raise ValueError(f"nonAggregateQueryHandling must be one of {NON_AGG_HANDLING}")
        o.nonAggQueryHandling = nah
        o.queryGranularity = g("queryGranularity", "none")
        o.allowTopN = _bool(g("allowTopNRewrite", False))
        o.topNMaxThreshold = int(g("topNMaxThreshold", o.topNMaxThreshold))
        nt = g("numProcessingThreadsPerHistorical")
        o.numProcessingThreadsPerHistorical = int(nt) if nt is not None else None
        return o

    # session overrides (DruidRelationInfo.scala:103-138)
    def allow_topn(self, conf: "Conf") -> bool:
        v = conf.get("spark.sparklinedata.druid.option.allowTopN")
        if v is None:
            v = conf.get("spark.sparklinedata.druid.allowTopN")
            if v is not None and not _bool(v):
                return self.allowTopN
        return _bool(v) if v is not None else self.allowTopN

    def topn_max_threshold(self, conf: "Conf") -> int:
        v = conf.get("spark.sparklinedata.druid.option.topNMaxThreshold")
        return int(v) if v is not None else self.topNMaxThreshold

    def query_historical(self, conf: "Conf") -> bool:
        v = conf.get("spark.sparklinedata.druid.option.queryHistoricalServers")
        return _bool(v) if v is not None else self.queryHistoricalServers

    def num_segments_per_query(self, conf: "Conf") -> int:
        v = conf.get("spark.sparklinedata.druid.option.numSegmentsPerHistoricalQuery")
        return int(v) if v is not None else self.numSegmentsPerHistoricalQuery

    def to_dict(self) -> Dict[str, Any]:
        return {f.name: getattr(self, f.name) for f in fields(self)}


# ------------------------------------------------------------------------------------------------
# session conf
@dataclass
class ConfEntry:
    key: str
    default: Any
    doc: str
    kind: type = str


CONF_ENTRIES: List[ConfEntry] = [
    ConfEntry("spark.sparklinedata.druid.cache.tables.tocheck", "", "tables whose cached copies may be star-joined"),
    ConfEntry("spark.sparklinedata.druid.debug.transformations", False, "log every planner transformation", bool),
    ConfEntry("spark.sparklinedata.tz.id", "UTC", "time zone for date/time evaluation"),
    ConfEntry("spark.sparklinedata.druid.selectquery.pagesize", 10000, "rows per Select page", int),
    ConfEntry("spark.sparklinedata.druid.stream.results", True,
              "Thrift server: stream Select-backed and large groupBy results page by page instead of materialising them", bool),
    ConfEntry("spark.sparklinedata.druid.max.connections", 100, "(remote Druid only)", int),
    ConfEntry("spark.sparklinedata.druid.max.connections.per.route", 20, "(remote Druid only)", int),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.enabled", True, "use the cost model", bool),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.histMergeCostFactor", 0.07, "", float),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.histSegsPerQueryLimit", 5, "", int),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.queryintervalScalingForDistinctValues", 3.0, "", float),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.historicalProcessingCost", 0.1, "", float),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.historicalTimeSeriesProcessingCost", 0.07, "", float),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.sparkSchedulingCost", 1.0, "", float),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.sparkAggregatingCost", 0.15, "", float),
    ConfEntry("spark.sparklinedata.druid.querycostmodel.druidOutputTransportCost", 0.4, "", float),
    ConfEntry("spark.sparklinedata.druid.option.useSmile", True, "(remote Druid only)", bool),
    ConfEntry("spark.sparklinedata.druid.allowTopN", False, "allow TopN rewrites", bool),
    ConfEntry("spark.sparklinedata.druid.topNMaxThreshold", 100000, "max TopN threshold", int),
    ConfEntry("spark.sparklinedata.druid.option.use.v2.groupByEngine", False, "groupByStrategy v2 hint", bool),
    ConfEntry("spark.sparklinedata.enable.druid.query.history", False, "record executed Druid queries", bool),
    ConfEntry("spark.sparklinedata.druid.window.rankone.pushdown", True,
              "pre-filter rank()/dense_rank() = 1 windows over a pushed groupBy on the device", bool),
    ConfEntry("spark.sparklinedata.modules", "", "extra planner modules (python import paths)"),
    # MI355X engine knobs (new)
    ConfEntry("spark.sparklinedata.druid.approxCountDistinct", False,
              "push COUNT(DISTINCT x) as a cardinality (HLL) aggregator instead of the exact 2-level rewrite", bool),
    ConfEntry("spark.sparklinedata.druid.planCache.enabled", True, "cache optimized plans by SQL text", bool),
    ConfEntry("spark.sparklinedata.druid.query.timeout.ms", 0, "per-query deadline (0 = none)", int),
    ConfEntry("spark.sparklinedata.druid.fuse.groupingsets", True,
              "answer the per-set Druid queries of CUBE / ROLLUP / GROUPING SETS from one scan", bool),
    ConfEntry("spark.sparklinedata.druid.deterministic", False,
              "float sums in exact fixed point: bitwise reproducible results under any reduction order", bool),
    ConfEntry("sparkline.queryhistory.maxsize", 500, "query history capacity", int),
]
_BY_KEY = {e.key: e for e in CONF_ENTRIES}


class Conf:
    """Layered config: defaults <- SDO_CONF_* environment <- session SET."""

    def __init__(self, init: Optional[Dict[str, Any]] = None):
        self._vals: Dict[str, str] = {}
        self._key: Optional[str] = None  # canonical form of the SET values (plan-cache key part)
        for k, v in os.environ.items():
            if k.startswith("SDO_CONF_"):
                self._vals[k[len("SDO_CONF_"):].replace("__", ".")] = v
        if init:
            for k, v in init.items():
                self.set(k, v)

    def copy(self) -> "Conf":
        c = Conf.__new__(Conf)
        c._vals = dict(self._vals)
        c._key = self._key
        return c

    def set(self, key: str, value: Any) -> None:
        self._vals[key] = value if isinstance(value, str) else json.dumps(value) if not isinstance(
            value, (int, float, bool)) else str(value).lower() if isinstance(value, bool) else str(value)
        self._key = None

    def unset(self, key: str) -> None:
        self._vals.pop(key, None)
        self._key = None

    def cache_key(self) -> str:
        """The SET values in canonical form, recomputed only after a SET / UNSET (every statement's
        plan-cache lookup uses it)."""
        k = self._key
        if k is None:
            k = self._key = json.dumps(sorted(self._vals.items()))
        return k

    def get(self, key: str, default: Any = None) -> Optional[str]:
        if key in self._vals:
            return self._vals[key]
        if default is not None:
            return default
        return None

    def typed(self, key: str) -> Any:
        e = _BY_KEY.get(key)
        raw = self._vals.get(key)
        if e is None:
            return raw
        if raw is None:
            return e.default
        if e.kind is bool:
            return _bool(raw)
        return e.kind(raw)

    def items(self) -> Dict[str, str]:
        out = {e.key: str(e.default).lower() if isinstance(e.default, bool) else str(e.default)
               for e in CONF_ENTRIES}
        out.update(self._vals)
        return out
