""""Druid Query Details" page: the reference's Spark UI tab over the query history
(``asql/hive/thriftserver/sparklinedata/ui/DruidQueriesTab.scala:25-43``,
``.../ui/DruidQueriesPage.scala:27-78``), served as plain HTML by the Druid HTTP endpoint at
``/sparklinedata/druid/queries`` (JSON at ``/sparklinedata/druid/queries.json``) and attached by the
Thrift server when ``spark.sparklinedata.enable.druid.query.history`` is on, like the reference's
``HiveThriftServer2`` (73-77)."""
from __future__ import annotations

import html
from typing import Iterable

COLUMNS = ["queryId", "stageId", "partitionId", "taskAttemptId", "druidQueryServer", "druidSegIntervals",
           "startTime", "druidExecTime", "queryExecTime", "numRows", "druidQuery", "sqlStmt"]


class HTMLPage(str):
    """Marker type: the HTTP layer sends it as text/html."""


def queries_page(views: Iterable, title: str = "Druid Query Details") -> HTMLPage:
    rows = []
    for v in reversed(list(views)):  # newest first, like the Spark UI table
        d = v.__dict__ if hasattr(v, "__dict__") else dict(v)
        cells = []
        for c in COLUMNS:
            x = d.get(c)
            s = "" if x is None else str(x)
            if c in ("druidQuery", "sqlStmt") and len(s) > 120:
                s = f"<details><summary>{html.escape(s[:120])}&hellip;</summary><pre>{html.escape(s)}</pre></details>"
            else:
                s = html.escape(s)
            cells.append(f"<td>{s}</td>")
        rows.append("<tr>" + "".join(cells) + "</tr>")
    head = "".join(f"<th>{c}</th>" for c in COLUMNS)
    return HTMLPage(
        "<!DOCTYPE html><html><head><meta charset='utf-8'><title>" + html.escape(title) + "</title>"
        "<style>body{font-family:sans-serif}table{border-collapse:collapse}td,th{border:1px solid #ccc;"
        "padding:3px 6px;font-size:12px;vertical-align:top}th{background:#eee}</style></head><body>"
        f"<h3>{html.escape(title)}</h3><p>{len(rows)} queries</p>"
        f"<table><thead><tr>{head}</tr></thead><tbody>{''.join(rows)}</tbody></table></body></html>")
