"""Druid-compatible HTTP API served by the GPU engine.

The reference is a *client* of Druid's broker / historical / coordinator / overlord HTTP APIs
(``sd/client/DruidClient.scala:130-500``, ``sd/client/DruidOverlordClient.scala:51-129``).  This
module serves those same endpoints from the in-process MI355X engine, so any Druid client (including
the reference itself) can use the GPUs as its "Druid cluster":

  POST   /druid/v2/                      native JSON query -> Druid-format result array
  DELETE /druid/v2/{queryId}             cancel
  GET    /druid/v2/datasources[/{ds}]    datasource list / dimensions+metrics
  GET    /druid/coordinator/v1/datasources[/{ds}[/segments]]
  GET    /druid/coordinator/v1/servers?full       one "historical" per GPU rank
  GET    /druid/coordinator/v1/leader
  POST   /druid/indexer/v1/task          index task (JSON spec) -> {"task": id}
  GET    /druid/indexer/v1/task/{id}/status
  GET    /status

``timeBoundary`` and ``segmentMetadata`` queries are answered from the catalog (K19 in SURVEY §2.3).
Request bodies may be JSON or Smile (``client/smile.py``, the reference's ``useSmile`` wire format);
a Smile request (or ``Accept: application/x-jackson-smile``) gets a Smile response.
"""
from __future__ import annotations

import json
import logging
import threading
import time
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional
from urllib.parse import parse_qs, urlparse

import numpy as np

from ..client import smile
from ..query import spec as S
from ..query.intervals import fmt_iso
from .ui import HTMLPage, queries_page

log = logging.getLogger("sdo.druid_http")


def _py(v):
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, float) and v != v:
        return None
    return v


def format_result(spec, res) -> List[Dict[str, Any]]:
    """Engine QueryResult -> Druid's JSON result layout for the query type."""
    from ..engine.columns import materialize

    qt = spec.queryType
    cols = {c: materialize(res.data[c]) for c in res.columns}
    n = res.num_rows
    start = spec.intervals[0].split("/")[0] if getattr(spec, "intervals", None) else fmt_iso(0)
    try:
        from ..query.intervals import Interval

        ts0 = fmt_iso(Interval.parse(spec.intervals[0]).lo)
    except Exception:  # noqa: BLE001
        ts0 = start
    names = [c for c in res.columns if c != "timestamp"]

    def ts_of(i):
        if "timestamp" in cols:
            t = cols["timestamp"][i]
            return fmt_iso(int(t)) if isinstance(t, (int, np.integer)) else str(t)
        return ts0

    if qt == "groupBy":
        return [{"version": "v1", "timestamp": ts_of(i), "event": {c: _py(cols[c][i]) for c in names}}
                for i in range(n)]
    if qt == "timeseries":
        return [{"timestamp": ts_of(i), "result": {c: _py(cols[c][i]) for c in names}} for i in range(n)]
    if qt == "topN":
        return [{"timestamp": ts0, "result": [{c: _py(cols[c][i]) for c in names} for i in range(n)]}]
    if qt == "search":
        return [{"timestamp": ts0, "result": [{"dimension": _py(cols["dimension"][i]), "value": _py(cols["value"][i]),
                                               "count": _py(cols["count"][i]) if "count" in cols else None}
                                              for i in range(n)]}]
    if qt == "select":
        events = []
        for i in range(n):
            ev = {c: _py(cols[c][i]) for c in res.columns}
            if "timestamp" in ev and isinstance(ev["timestamp"], int):
                ev["timestamp"] = fmt_iso(ev["timestamp"])
            events.append({"segmentId": f"{spec.dataSource}_{ts0}", "offset": i, "event": ev})
        return [{"timestamp": ts0, "result": {"pagingIdentifiers": res.paging or {}, "events": events}}]
    return [{c: _py(cols[c][i]) for c in res.columns} for i in range(n)]


def time_boundary(ds) -> List[Dict[str, Any]]:
    from ..sql.druid_rewrite import data_interval

    lo = ds.min_time_ms()
    hi = ds.max_time_ms()
    return [{"timestamp": fmt_iso(lo), "result": {"minTime": fmt_iso(lo), "maxTime": fmt_iso(hi)}}]


def segment_metadata(ds) -> List[Dict[str, Any]]:
    from ..sql.druid_rewrite import data_interval

    lo, hi = data_interval(ds)
    cols = {"__time": {"type": "LONG", "size": int(ds.num_rows * 8), "cardinality": None, "errorMessage": None}}
    for n, d in ds.dims.items():
        cols[n] = {"type": "STRING", "size": int(d.ids.numel() * d.ids.element_size()),
                   "cardinality": int(len(d.dictionary)), "errorMessage": None}
    for n, m in ds.metrics.items():
        t = {"long": "LONG", "decimal": "FLOAT", "double": "FLOAT", "hll": "hyperUnique"}.get(m.kind, "FLOAT")
        cols[n] = {"type": t, "size": int(m.data.numel() * m.data.element_size()), "cardinality": None,
                   "errorMessage": None}
    return [{"id": f"merged_{ds.name}", "intervals": [f"{fmt_iso(lo)}/{fmt_iso(hi)}"], "columns": cols,
             "size": int(ds.size_bytes()), "numRows": int(getattr(ds, "global_num_rows", ds.num_rows))}]


class JSONStream(list):
    """Marker type: a large result array sent with chunked transfer encoding, rows serialized a
    block at a time (the client can start parsing before the last row is encoded)."""


STREAM_ROWS = 4096  # results with more rows than this are streamed


class PlainText(str):
    """Marker type: sent as text/plain (Prometheus exposition format)."""


class DruidHTTPServer:
    def __init__(self, session, host: str = "127.0.0.1", port: int = 8082):
        self.session = session
        self.host = host
        self.port = port
        self.lock = threading.Lock()
        self.running: Dict[str, Any] = {}  # queryId -> CancelToken of the running query
        self.cancelled: set = set()
        self._srv: Optional[ThreadingHTTPServer] = None
        from ..segment.ingest import Overlord

        self.overlord = Overlord(session, device=str(session.engine.world.device()))

    # -------------------------------------------------------------------------------- queries
    def query(self, body: Dict[str, Any]) -> List[Dict[str, Any]]:
        qt = body.get("queryType")
        cluster = self.session.catalog.cluster
        ds_name = body.get("dataSource")
        if isinstance(ds_name, dict):
            ds_name = ds_name.get("name")
        ds = cluster.get(ds_name)
        if qt == "timeBoundary":
            return time_boundary(ds)
        if qt == "segmentMetadata":
            return segment_metadata(ds)
        spec = S.query_from_json(body)
        ctx = body.get("context") or {}
        qid = ctx.get("queryId") or uuid.uuid4().hex
        from ..utils.cancel import CancelToken, scope

        # Druid's context timeout (ms); DELETE /druid/v2/{queryId} cancels the token of a running
        # query, which the engine honours at its next stage boundary (before each scan / batch)
        token = CancelToken(float(ctx["timeout"]) if ctx.get("timeout") else None)
        with self.lock:
            self.running[qid] = token
            if qid in self.cancelled:
                self.cancelled.discard(qid)
                token.cancel(f"query {qid} cancelled")
        t0 = time.perf_counter()
        ok = False
        try:
            with scope(token):
                token.check()
                res = self.session.engine.coalescer().run(None, lambda: self.session.engine.execute(spec, ds)) \
                    if not self.session.engine.world.distributed else self.session.engine.execute(spec, ds)
            if self.session.conf.typed("spark.sparklinedata.enable.druid.query.history"):
                self.session.history.record(spec, res.stats.get("exec_ms", 0.0), res.stats.get("exec_ms", 0.0),
                                            res.num_rows, "http", None)
            out = format_result(spec, res)
            ok = True
            if isinstance(out, list) and len(out) > STREAM_ROWS:
                return JSONStream(out)
            return out
        finally:
            self.running.pop(qid, None)
            from ..utils.metrics import metrics_of

            metrics_of(self.session).record("druid_http", (time.perf_counter() - t0) * 1e3, ok)

    # -------------------------------------------------------------------------------- routes
    def handle(self, method: str, path: str, query: Dict[str, List[str]], body: Optional[bytes]):
        cluster = self.session.catalog.cluster
        parts = [p for p in path.split("/") if p]
        if method == "GET" and parts == ["sparklinedata", "druid", "queries"]:
            return 200, queries_page(self.session.history.entries())
        if method == "GET" and parts == ["sparklinedata", "druid", "queries.json"]:
            return 200, self.session.history.rows()
        if method == "GET" and parts == ["sparklinedata", "metrics"]:
            from ..utils.metrics import metrics_of

            return 200, metrics_of(self.session).snapshot()
        if method == "GET" and parts == ["metrics"]:  # Prometheus text exposition
            from ..utils.metrics import metrics_of

            return 200, PlainText(metrics_of(self.session).prometheus())
        if method == "GET" and parts == ["status"]:
            return 200, {"version": "spark-druid-olap-amd", "modules": [], "gpus": self.session.engine.world.size}
        if parts[:2] == ["druid", "v2"]:
            if method == "POST" and len(parts) == 2:
                return 200, self.query(json.loads(body or b"{}"))
            if method == "DELETE" and len(parts) == 3:
                with self.lock:
                    tok = self.running.get(parts[2])
                    if tok is not None:
                        tok.cancel(f"query {parts[2]} cancelled")
                    else:  # not started yet: cancel it on arrival
                        self.cancelled.add(parts[2])
                return 202, {}
            if method == "GET" and len(parts) >= 3 and parts[2] == "datasources":
                if len(parts) == 3:
                    return 200, sorted(cluster.datasources)
                ds = cluster.get(parts[3])
                return 200, {"dimensions": sorted(ds.dims), "metrics": sorted(ds.metrics)}
        if parts[:3] == ["druid", "coordinator", "v1"]:
            rest = parts[3:]
            if rest == ["leader"]:
                return 200, f"{self.host}:{self.port}"
            if rest == ["datasources"]:
                if "full" in query:
                    return 200, [self._ds_full(n) for n in sorted(cluster.datasources)]
                return 200, sorted(cluster.datasources)
            if len(rest) >= 2 and rest[0] == "datasources":
                ds = cluster.get(rest[1])
                if len(rest) == 3 and rest[2] == "segments":
                    segs = [s.identifier for s in ds.segments]
                    if "full" in query:
                        return 200, [self._seg(ds, s) for s in ds.segments]
                    return 200, segs
                return 200, self._ds_full(rest[1])
            if rest == ["servers"]:
                return 200, self._servers(full="full" in query)
        if parts[:3] == ["druid", "indexer", "v1"]:
            rest = parts[3:]
            if method == "POST" and rest == ["task"]:
                spec = json.loads(body or b"{}")
                with self.lock:
                    tid = self.overlord.submit_task(spec)
                return 200, {"task": tid}
            if method == "GET" and len(rest) == 3 and rest[0] == "task" and rest[2] == "status":
                st = self.overlord.task_status(rest[1])
                return 200, {"task": rest[1], "status": {"id": rest[1], **st}}
        return 404, {"error": f"no route for {method} {path}"}

    def _seg(self, ds, s):
        return {"dataSource": ds.name, "interval": f"{fmt_iso(s.interval_lo_ms)}/{fmt_iso(s.interval_hi_ms)}",
                "version": s.version, "shardSpec": {"type": "linear", "partitionNum": s.partition},
                "size": int((s.row_hi - s.row_lo) * max(1, ds.size_bytes() // max(ds.num_rows, 1))),
                "identifier": s.identifier, "numRows": int(s.row_hi - s.row_lo)}

    def _ds_full(self, name):
        ds = self.session.catalog.cluster.get(name)
        return {"name": name, "properties": {"created": time.strftime("%Y-%m-%dT%H:%M:%SZ")},
                "segments": [self._seg(ds, s) for s in ds.segments]}

    def _servers(self, full: bool):
        w = self.session.engine.world
        cl = self.session.catalog.cluster
        out = []
        for r in range(w.size):
            srv = {"host": f"gpu{r}:{self.port}", "tier": "_default_tier", "type": "historical", "priority": 0,
                   "currSize": int(sum(ds.size_bytes() for ds in cl.datasources.values())), "maxSize": 288 << 30}
            if full:
                srv["segments"] = {s.identifier: self._seg(ds, s) for ds in cl.datasources.values() for s in ds.segments}
            out.append(srv)
        return out

    # -------------------------------------------------------------------------------- server
    def start(self) -> "DruidHTTPServer":
        app = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):  # quiet
                log.debug(*a)

            def _do(self, method):
                u = urlparse(self.path)
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else None
                ctype = self.headers.get("Content-Type", "application/json")
                self._smile = "smile" in ctype or "smile" in (self.headers.get("Accept") or "")
                if body and "smile" in ctype:
                    try:
                        body = json.dumps(smile.loads(body), default=_py).encode()
                    except smile.SmileError as e:
                        return self._send(400, {"error": "bad Smile body", "errorMessage": str(e)})
                try:
                    code, obj = app.handle(method, u.path, parse_qs(u.query, keep_blank_values=True), body)
                except KeyError as e:
                    code, obj = 404, {"error": str(e)}
                except Exception as e:  # noqa: BLE001
                    log.exception("request failed")
                    code, obj = 500, {"error": type(e).__name__, "errorMessage": str(e)}
                self._send(code, obj)

            def _send(self, code, obj):
                if isinstance(obj, JSONStream) and not getattr(self, "_smile", False):
                    self.send_response(code)
                    self.send_header("Content-Type", "application/json")
                    self.send_header("Transfer-Encoding", "chunked")
                    self.end_headers()

                    def chunk(b: bytes):
                        self.wfile.write(b"%x\r\n" % len(b) + b + b"\r\n")

                    try:
                        chunk(b"[")
                        for i in range(0, len(obj), 1024):
                            part = ",".join(json.dumps(r, default=_py) for r in obj[i:i + 1024])
                            chunk(((b"," if i else b"") + part.encode()))
                        chunk(b"]")
                        self.wfile.write(b"0\r\n\r\n")
                    except (BrokenPipeError, ConnectionResetError):
                        self.close_connection = True  # the client stopped reading (closed its iterator)
                    return
                if isinstance(obj, HTMLPage):
                    data, ct = obj.encode("utf-8"), "text/html; charset=utf-8"
                elif isinstance(obj, PlainText):
                    data, ct = obj.encode("utf-8"), "text/plain; version=0.0.4"
                elif getattr(self, "_smile", False):
                    data, ct = smile.dumps(json.loads(json.dumps(obj, default=_py))), smile.MIME
                else:
                    data, ct = json.dumps(obj, default=_py).encode(), "application/json"
                self.send_response(code)
                self.send_header("Content-Type", ct)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                self._do("GET")

            def do_POST(self):
                self._do("POST")

            def do_DELETE(self):
                self._do("DELETE")

        self._srv = ThreadingHTTPServer((self.host, self.port), H)
        self._srv.daemon_threads = True
        self.port = self._srv.server_address[1]
        threading.Thread(target=self._srv.serve_forever, daemon=True, name="druid-http").start()
        disc = getattr(self.session, "discovery", None)
        self._announced = []
        if disc is not None:
            # one endpoint plays every Druid service role (CuratorConnection.getBroker/getCoordinator)
            for svc in ("broker", "coordinator", "overlord"):
                self._announced.append(disc.announce_service(svc, self.host, self.port))
        return self

    def stop(self):
        disc = getattr(self.session, "discovery", None)
        for p in getattr(self, "_announced", []):
            disc.unannounce(p)
        self._announced = []
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
            self._srv = None
