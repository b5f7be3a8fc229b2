"""Metadata views ``d$druidrelations``, ``d$druidservers``, ``d$druidsegments``,
``d$druidserverassignments``, ``d$druidqueries``.

Parity: ``sd/metadata/DruidMetadataViews.scala:25-225`` (view names and columns) and
``asql/hive/sparklinedata/SPLSessionState.scala:39-75`` (the catalog serves them before the regular
lookup).  "Servers" are the GPUs of the process group: each rank is one historical holding its
shard's segments; assignments are segment -> GPU.
"""
from __future__ import annotations

import json
from typing import Callable, Dict, List

import pandas as pd

VIEW_NAMES = ("d$druidrelations", "d$druidservers", "d$druidsegments", "d$druidserverassignments",
              "d$druidqueries")


def _relations(session) -> pd.DataFrame:
    rows = []
    for t in session.catalog.druid_tables():
        info = t.info
        ds = info.datasource
        rows.append({
            "sparkRelation": t.qualified_name, "druidDataSource": info.ds_name,
            "timeDimensionCol": info.time_dim_col, "sourceDataFrame": info.source_name,
            "columnMapping": json.dumps({c.column: c.druid_column for c in info.column_map.values()}),
            "functionalDeps": json.dumps([f.__dict__ for f in info.fds]),
            "starSchema": json.dumps(info.star.info.to_json()),
            "options": json.dumps(info.options.to_dict(), default=str),
            "numRows": int(getattr(ds, "global_num_rows", ds.num_rows)),
        })
    return pd.DataFrame(rows, columns=["sparkRelation", "druidDataSource", "timeDimensionCol", "sourceDataFrame",
                                       "columnMapping", "functionalDeps", "starSchema", "options", "numRows"])


def _servers(session) -> pd.DataFrame:
    w = session.engine.world
    rows = []
    info = {}
    try:
        from ..ops import native

        info = native.device_info() if session.engine.use_native else {}
    except Exception:
        info = {}
    for r in range(w.size):
        rows.append({"druidHost": f"gpu:{r}", "host": f"rank{r}", "maxSize": int(info.get("total_mem", 0)),
                     "serverType": "historical", "tier": "_default_tier", "priority": 0,
                     "numSegments": sum(len(ds.segments) for ds in session.catalog.cluster.datasources.values()),
                     "currSize": int(sum(ds.size_bytes() for ds in session.catalog.cluster.datasources.values()))})
    return pd.DataFrame(rows)


def _segments(session) -> pd.DataFrame:
    rows = []
    for name, ds in session.catalog.cluster.datasources.items():
        for s in ds.segments:
            rows.append({"druidHost": f"gpu:{session.engine.world.rank}", "druidDataSource": name,
                         "interval": s.identifier.split("_")[0], "version": s.version, "binaryVersion": "sdo-1",
                         "size": int((s.row_hi - s.row_lo) * max(1, ds.size_bytes() // max(ds.num_rows, 1))),
                         "identifier": s.identifier, "shardSpec": json.dumps({"partitionNum": s.partition}),
                         "numRows": int(s.row_hi - s.row_lo)})
    return pd.DataFrame(rows, columns=["druidHost", "druidDataSource", "interval", "version", "binaryVersion", "size",
                                       "identifier", "shardSpec", "numRows"])


def _assignments(session) -> pd.DataFrame:
    seg = _segments(session)
    if seg.empty:
        return pd.DataFrame(columns=["druidHost", "druidDataSource", "segIdentifier"])
    return pd.DataFrame({"druidHost": seg["druidHost"], "druidDataSource": seg["druidDataSource"],
                         "segIdentifier": seg["identifier"]})


def _queries(session) -> pd.DataFrame:
    rows = session.history.rows()
    cols = ["queryId", "stageId", "partitionId", "taskAttemptId", "druidQueryServer", "druidSegIntervals",
            "startTime", "druidExecTime", "queryExecTime", "numRows", "druidQuery", "sqlStmt"]
    return pd.DataFrame(rows, columns=cols)


VIEWS: Dict[str, Callable] = {
    "d$druidrelations": _relations,
    "d$druidservers": _servers,
    "d$druidsegments": _segments,
    "d$druidserverassignments": _assignments,
    "d$druidqueries": _queries,
}


def schema_of(df: pd.DataFrame) -> List[tuple]:
    out = []
    for c in df.columns:
        k = df[c].dtype.kind
        out.append((c, "bigint" if k in "iu" else "double" if k == "f" else "string"))
    return out
