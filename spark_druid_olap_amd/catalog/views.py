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


SEGMENT_COLS = ["druidHost", "druidDataSource", "interval", "version", "binaryVersion", "size",
                "identifier", "shardSpec", "numRows"]


def _local_inventory(session) -> dict:
    """This rank's server record + segment list (the coordinator's ``servers?full=true`` entry for
    one historical, ``sd/client/DruidClient.scala:488-492``)."""
    w = session.engine.world
    host = f"gpu:{w.rank}"
    info = {}
    try:
        from ..ops import native

        info = native.device_info() if session.engine.use_native else {}
    except Exception:
        info = {}
    dss = session.catalog.cluster.datasources
    segs = []
    for name, ds in dss.items():
        row_bytes = max(1, ds.size_bytes() // max(ds.num_rows, 1))
        for s in ds.segments:
            segs.append({"druidHost": host, "druidDataSource": name,
                         "interval": s.identifier.split("_")[0], "version": s.version, "binaryVersion": "sdo-1",
                         "size": int((s.row_hi - s.row_lo) * row_bytes),
                         "identifier": s.identifier, "shardSpec": json.dumps({"partitionNum": s.partition}),
                         "numRows": int(s.row_hi - s.row_lo)})
    server = {"druidHost": host, "host": f"rank{w.rank}", "maxSize": int(info.get("totalGlobalMem", 0)),
              "serverType": "historical", "tier": "_default_tier", "priority": 0,
              "numSegments": len(segs), "currSize": int(sum(ds.size_bytes() for ds in dss.values()))}
    return {"server": server, "segments": segs}


def cluster_inventory(session) -> List[dict]:
    """Every rank's inventory, in rank order.  Collective when the world is distributed: view
    queries run SPMD like every other statement (server/spmd.py), so all ranks reach it together."""
    return session.engine.world.all_gather_object(_local_inventory(session))


def _servers(session) -> pd.DataFrame:
    return pd.DataFrame([inv["server"] for inv in cluster_inventory(session)])


def _segments(session) -> pd.DataFrame:
    rows = [s for inv in cluster_inventory(session) for s in inv["segments"]]
    return pd.DataFrame(rows, columns=SEGMENT_COLS)


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
