"""HiveServer2-compatible Thrift endpoint over a ``Session`` (the reference's
``HiveThriftServer2``, ``asql/hive/thriftserver/sparklinedata/HiveThriftServer2.scala:48-148``).

JDBC / ODBC / beeline clients connect with ``jdbc:hive2://host:10000/default`` (SASL PLAIN, the
HiveServer2 default) or ``;auth=noSasl`` (raw binary protocol); the server detects which from the
first byte.  Statements run through the SQL front-end, so Druid rewrites, the ``d$*`` views,
``EXPLAIN DRUID REWRITE`` and ``ON DRUIDDATASOURCE ... EXECUTE QUERY`` all work remotely.  Results
go back as column-based ``TRowSet`` pages (protocol V8).

Every client session gets its own ``Session`` view (``Session.new_session``: own ``SET`` conf,
current database and temporary views; shared tables, datasources and cached plans).  On one GPU,
statements from different sessions execute concurrently on K HIP-stream slots with per-slot device
buffers, and identical queued statements run once (``engine/scheduler.py``).  With several ranks
(one per GPU) rank 0 serves the clients and broadcasts every statement to the other ranks, which
execute it over their shards (``server/spmd.py``).  Query history records the SQL text of every
Druid query (the ``HS2Listener``).
"""
from __future__ import annotations

import logging
import os
import socket
import socketserver
import struct
import threading
import time
import uuid
from typing import Any, Dict, List, Optional

import numpy as np
import pandas as pd

from . import thrift as T

log = logging.getLogger("sdo.thriftserver")

SASL_START, SASL_OK, SASL_BAD, SASL_ERROR, SASL_COMPLETE = 1, 2, 3, 4, 5


class Operation:
    def __init__(self, session_id: bytes, kind: int = 0):
        self.id = uuid.uuid4().bytes
        self.secret = uuid.uuid4().bytes
        self.session_id = session_id
        self.kind = kind
        self.state = T.OP_INITIALIZED
        self.error: Optional[str] = None
        self.names: List[str] = []
        self.types: List[str] = []
        self.cols: List[list] = []
        self.nrows = 0
        self.cursor = 0
        self.base = 0
        self.stream = None
        self.factory = None
        self.close_hook = None  # releases an open multi-rank cursor (server/spmd.py streams)
        self.started = int(time.time() * 1000)
        self.completed = 0
        self.thread: Optional[threading.Thread] = None
        self.cancelled = threading.Event()
        from ..utils.cancel import CancelToken

        self.token = CancelToken()

    def handle(self) -> Dict[str, Any]:
        return {"operationId": {"guid": self.id, "secret": self.secret}, "operationType": self.kind,
                "hasResultSet": True}

    def set_frame(self, names, types, df: pd.DataFrame):
        self.names, self.types = list(names), list(types)
        self.cols = [df.iloc[:, i].tolist() for i in range(df.shape[1])]
        self.nrows = len(df)
        self.base = 0
        self.stream = None

    def set_stream(self, names, types, pages_factory):
        """Rows produced page by page (a pushed Select's cursor, session.DataFrame.iter_batches):
        FetchResults pulls pages on demand and only the unread rows stay buffered."""
        self.names, self.types = list(names), list(types)
        self.cols = [[] for _ in self.names]
        self.nrows = 0
        self.base = 0  # absolute offset of the first buffered row
        self.factory = pages_factory
        self.stream = pages_factory()

    def fill(self, upto: int) -> None:
        """Buffer rows until ``upto`` (absolute) rows are available or the stream ends."""
        while self.stream is not None and self.nrows < upto:
            page = next(self.stream, None)
            if page is None:
                self.stream = None
                break
            for i in range(len(self.names)):
                self.cols[i].extend(page.iloc[:, i].tolist())
            self.nrows += len(page)

    def trim(self) -> None:
        """Drop rows before the cursor (streamed results keep one page of lookahead)."""
        k = self.cursor - self.base
        if self.factory is not None and k > 0:
            self.cols = [c[k:] for c in self.cols]
            self.base = self.cursor

    def rewind(self) -> None:
        if getattr(self, "factory", None) is not None and self.base > 0:
            self.cols = [[] for _ in self.names]
            self.nrows = self.base = 0
            self.stream = self.factory()
        self.cursor = 0


class HiveThriftServer:
    def __init__(self, session, host: str = "127.0.0.1", port: int = 10000, auth: str = "auto", world=None):
        self.session = session
        self.host = host
        self.port = port
        self.auth = auth
        self.sessions: Dict[bytes, Dict[str, Any]] = {}
        self.ops: Dict[bytes, Operation] = {}
        self.world = world if world is not None else session.engine.world
        self.spmd = None
        if self.world.distributed:
            from .spmd import SpmdDispatcher

            self.spmd = SpmdDispatcher(session, self.world)
        self._srv: Optional[socketserver.ThreadingTCPServer] = None
        self._thread: Optional[threading.Thread] = None

    # ------------------------------------------------------------------------------ lifecycle
    def start(self) -> "HiveThriftServer":
        from ..utils.memory import reserve_runtime_memory, serving_gc

        serving_gc()
        reserve_runtime_memory()  # device memory the HIP runtime allocates outside torch (scratch, RCCL)
        server = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                server._serve_connection(self.request)

        class Srv(socketserver.ThreadingTCPServer):
            allow_reuse_address = True
            daemon_threads = True

        self._srv = Srv((self.host, self.port), Handler)
        self.port = self._srv.server_address[1]
        self._thread = threading.Thread(target=self._srv.serve_forever, daemon=True, name="hs2-accept")
        self._thread.start()
        log.info("HiveServer2 endpoint on %s:%d", self.host, self.port)
        return self

    def stop(self):
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
            self._srv = None
        if self.spmd is not None:
            self.spmd.shutdown()

    def serve_forever(self):
        self.start()
        try:
            while True:
                time.sleep(3600)
        except KeyboardInterrupt:
            self.stop()

    # ------------------------------------------------------------------------------ transport
    def _serve_connection(self, sock: socket.socket):
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        f = sock.makefile("rb")
        try:
            first = f.peek(1)[:1] if hasattr(f, "peek") else b""
            if not first:
                return
            if first[0] == SASL_START and self.auth in ("auto", "sasl"):
                self._sasl_handshake(f, sock)
                framed = True
            else:
                framed = False
            while True:
                if framed:
                    hdr = _read_exact(f, 4)
                    if hdr is None:
                        return
                    (n,) = struct.unpack("!i", hdr)
                    msg = _read_exact(f, n)
                    if msg is None:
                        return
                else:
                    msg = _read_unframed_message(f)
                    if msg is None:
                        return
                out = self._dispatch(msg)
                if framed:
                    sock.sendall(struct.pack("!i", len(out)) + out)
                else:
                    sock.sendall(out)
        except (ConnectionError, T.ProtocolError, OSError) as e:
            log.debug("connection closed: %s", e)
        finally:
            try:
                f.close()
                sock.close()
            except OSError:
                pass

    def _sasl_handshake(self, f, sock):
        # START: status(1) len(4) mechanism ; then OK frames with PLAIN payload "\0user\0password"
        st = f.read(1)
        (n,) = struct.unpack("!i", f.read(4))
        mech = f.read(n).decode()
        if mech.upper() not in ("PLAIN", "ANONYMOUS"):
            sock.sendall(bytes([SASL_BAD]) + struct.pack("!i", 0))
            raise ConnectionError(f"unsupported SASL mechanism {mech}")
        st = f.read(1)
        (n,) = struct.unpack("!i", f.read(4))
        _payload = f.read(n)
        sock.sendall(bytes([SASL_COMPLETE]) + struct.pack("!i", 0))

    # ------------------------------------------------------------------------------ RPC
    def _dispatch(self, msg: bytes) -> bytes:
        name, mtype, seqid, req = T.decode_call(msg)
        fn = getattr(self, "rpc_" + name, None)
        if fn is None:
            return T.encode_exception(name, seqid, f"method {name} not implemented", 1)
        try:
            resp = fn(req)
        except Exception as e:  # noqa: BLE001
            log.exception("rpc %s failed", name)
            resp = {"status": _err(str(e))}
        return T.encode_reply(name, seqid, resp)

    def rpc_OpenSession(self, req):
        sid = uuid.uuid4().bytes
        conf, db = {}, None
        for k, v in (req.get("configuration") or {}).items():
            if k.startswith("set:hiveconf:") or k.startswith("set:hivevar:"):
                conf[k.split(":", 2)[2]] = v
            elif k == "use:database" and v.lower() in self.session.catalog.dbs:
                db = v
        if self.spmd is not None:
            self.spmd.open_session(sid, conf, db)
            sess = self.spmd.session(sid)
        else:
            sess = self.session.new_session()
            for k, v in conf.items():
                sess.conf.set(k, v)
            if db:
                sess.catalog.use(db)
        self.sessions[sid] = {"user": req.get("username"), "conf": dict(req.get("configuration") or {}),
                              "opened": time.time(), "session": sess}
        proto = min(int(req.get("client_protocol", T.PROTOCOL_V8)), T.PROTOCOL_V8)
        return {"status": _ok(), "serverProtocolVersion": proto,
                "sessionHandle": {"sessionId": {"guid": sid, "secret": uuid.uuid4().bytes}}, "configuration": {}}

    def rpc_CloseSession(self, req):
        sid = _sid(req)
        if self.sessions.pop(sid, None) is not None and self.spmd is not None:
            self.spmd.close_session(sid)
        for oid in [k for k, o in self.ops.items() if o.session_id == sid]:
            self.ops.pop(oid, None)
        return {"status": _ok()}

    def rpc_GetInfo(self, req):
        t = req.get("infoType", 0)
        vals = {0: "MAX_DRIVER_CONNECTIONS", 18: "spark-druid-olap-amd", 20: "SparklineData SQL", 13: "2.0"}
        if t in (18, 20, 13):
            return {"status": _ok(), "infoValue": {"stringValue": vals[t]}}
        return {"status": _ok(), "infoValue": {"integerFlag": 0}}

    def rpc_ExecuteStatement(self, req):
        sid = _sid(req)
        if sid not in self.sessions:
            return {"status": {"statusCode": T.INVALID_HANDLE, "errorMessage": "invalid session"}}
        op = Operation(sid, 0)
        self.ops[op.id] = op
        stmt = req.get("statement", "")
        overlay = req.get("confOverlay") or {}
        if req.get("queryTimeout"):
            op.token.deadline = time.monotonic() + float(req["queryTimeout"])
        if req.get("runAsync"):
            op.state = T.OP_RUNNING
            op.thread = threading.Thread(target=self._run, args=(op, stmt, overlay), daemon=True)
            op.thread.start()
        else:
            self._run(op, stmt, overlay)
            if op.state == T.OP_ERROR:
                return {"status": _err(op.error), "operationHandle": op.handle()}
        return {"status": _ok(), "operationHandle": op.handle()}

    def _run(self, op: Operation, stmt: str, overlay: Dict[str, str]):
        from ..utils.metrics import metrics_of

        t0 = time.perf_counter()
        try:
            self._run_stmt(op, stmt, overlay)
        finally:
            metrics_of(self.session).record("thrift", (time.perf_counter() - t0) * 1e3, op.state != T.OP_ERROR)

    def _run_stmt(self, op: Operation, stmt: str, overlay: Dict[str, str]):
        op.state = T.OP_RUNNING
        try:
            if op.cancelled.is_set():
                op.state = T.OP_CANCELED
                return
            stmt = stmt.strip().rstrip(";")
            if self.spmd is not None:
                tmo = None
                if op.token.deadline is not None:
                    tmo = max(0.001, op.token.deadline - time.monotonic())
                sp = self.spmd
                df, pdf = sp.execute(op.session_id, stmt, overlay, tmo, stream=True)
                if isinstance(pdf, tuple) and pdf and pdf[0] == "stream":
                    # Select-backed result over every rank: pages pulled on demand through the
                    # broadcast stream (each rank advances its cursor on the same message)
                    first = [pdf[1]]

                    def pages(first=first, sid=op.session_id, stmt=stmt, overlay=dict(overlay), tmo=tmo):
                        sid_ = first.pop() if first else sp.execute(sid, stmt, overlay, tmo, stream=True)[1][1]
                        op.close_hook = lambda: sp.close_stream(sid_)
                        while True:
                            page = sp.stream_next(sid_)
                            if page is None:
                                op.close_hook = None
                                return
                            yield page

                    op.set_stream(df.columns, [t for _, t in df.schema], pages)
                    op.fill(1)  # the first page now: errors surface in ExecuteStatement
                    op.state = T.OP_FINISHED if not op.cancelled.is_set() else T.OP_CANCELED
                    op.completed = int(time.time() * 1000)
                    return
            else:
                sess = self.sessions[op.session_id]["session"]
                for k, v in overlay.items():
                    sess.conf.set(k, v)
                df = sess.sql(stmt)
                if df.plan is not None and sess.conf.typed("spark.sparklinedata.druid.stream.results") and \
                        (df._stream_source()[1] is not None or df.agg_streamable()):
                    # Select-backed or large groupBy result: stream pages to the client instead of
                    # materialising it
                    op.set_stream(df.columns, [t for _, t in df.schema],
                                  lambda df=df: df.iter_batches(token=op.token))
                    op.fill(1)  # run the scan now: errors surface in ExecuteStatement
                    op.state = T.OP_FINISHED if not op.cancelled.is_set() else T.OP_CANCELED
                    op.completed = int(time.time() * 1000)
                    return
                if df.plan is None:  # a command: already executed by sql()
                    pdf = df.to_pandas()
                else:
                    # a stream slot per execution; identical queued statements (same cached plan,
                    # i.e. same text + conf + database) execute once
                    df.prepare()  # lowering / compiling before a stream slot is leased
                    co = sess.engine.coalescer()
                    key = id(df) if sess.conf.typed("spark.sparklinedata.druid.planCache.enabled") and \
                        os.environ.get("SDO_COALESCE", "1") != "0" else None
                    pdf = co.run(key, lambda: df.to_pandas(token=op.token))
            # row-set encoding (host only) runs after the slot is released
            op.set_frame(df.columns, [t for _, t in df.schema], pdf)
            op.state = T.OP_FINISHED if not op.cancelled.is_set() else T.OP_CANCELED
        except Exception as e:  # noqa: BLE001
            op.error = f"{type(e).__name__}: {e}"
            op.state = T.OP_ERROR
        op.completed = int(time.time() * 1000)

    def rpc_GetOperationStatus(self, req):
        op = self.ops.get(_oid(req))
        if op is None:
            return {"status": {"statusCode": T.INVALID_HANDLE, "errorMessage": "invalid operation handle"}}
        r = {"status": _ok(), "operationState": op.state, "operationStarted": op.started,
             "operationCompleted": op.completed, "hasResultSet": True}
        if op.state == T.OP_ERROR:
            r.update(errorMessage=op.error, sqlState="42000", errorCode=0)
        return r

    def rpc_CancelOperation(self, req):
        op = self.ops.get(_oid(req))
        if op is not None:
            op.cancelled.set()
            op.token.cancel("cancelled by client")
            if op.state in (T.OP_INITIALIZED, T.OP_RUNNING):
                op.state = T.OP_CANCELED
        return {"status": _ok()}

    def rpc_CloseOperation(self, req):
        op = self.ops.pop(_oid(req), None)
        hook = getattr(op, "close_hook", None) if op is not None else None
        if hook is not None:  # an unfinished cursor over every rank: release it everywhere
            try:
                hook()
            except Exception:  # noqa: BLE001
                log.debug("closing the statement's cursor failed", exc_info=True)
        return {"status": _ok()}

    def rpc_GetResultSetMetadata(self, req):
        op = self.ops.get(_oid(req))
        if op is None:
            return {"status": {"statusCode": T.INVALID_HANDLE, "errorMessage": "invalid operation handle"}}
        cols = []
        for i, (n, t) in enumerate(zip(op.names, op.types)):
            tid = T.TYPE_IDS.get(t.split("(")[0], T.TYPE_IDS["string"])
            cols.append({"columnName": n, "typeDesc": {"types": [{"primitiveEntry": {"type": tid}}]},
                         "position": i + 1})
        return {"status": _ok(), "schema": {"columns": cols}}

    def rpc_FetchResults(self, req):
        op = self.ops.get(_oid(req))
        if op is None:
            return {"status": {"statusCode": T.INVALID_HANDLE, "errorMessage": "invalid operation handle"}}
        if req.get("fetchType", 0) == 1:  # operation log
            return {"status": _ok(), "hasMoreRows": False,
                    "results": {"startRowOffset": 0, "rows": [], "columns": [{"stringVal": {"values": [], "nulls": b""}}]}}
        if op.thread is not None:
            op.thread.join()
        if op.state == T.OP_ERROR:
            return {"status": _err(op.error)}
        if req.get("orientation", 0) == 4:  # FETCH_FIRST
            op.rewind()
        n = int(req.get("maxRows", 1000) or 1000)
        try:
            op.fill(op.cursor + n + 1)  # one row of lookahead decides hasMoreRows
        except Exception as e:  # noqa: BLE001  (a streamed page failed)
            return {"status": _err(f"{type(e).__name__}: {e}")}
        a, b = op.cursor, min(op.nrows, op.cursor + n)
        cols = [_tcolumn(op.types[i], op.cols[i][a - op.base:b - op.base]) for i in range(len(op.names))]
        op.cursor = b
        op.trim()
        return {"status": _ok(), "hasMoreRows": b < op.nrows or op.stream is not None,
                "results": {"startRowOffset": a, "rows": [], "columns": cols}}

    # metadata calls -> result sets
    def _meta_op(self, req, kind, names, types, rows):
        sid = _sid(req)
        op = Operation(sid, kind)
        op.set_frame(names, types, pd.DataFrame(rows, columns=names) if rows else pd.DataFrame({n: [] for n in names}))
        op.state = T.OP_FINISHED
        self.ops[op.id] = op
        return {"status": _ok(), "operationHandle": op.handle()}

    def rpc_GetCatalogs(self, req):
        return self._meta_op(req, 2, ["TABLE_CAT"], ["string"], [])

    def rpc_GetSchemas(self, req):
        pat = _like(req.get("schemaName"))
        rows = [(db, "") for db in sorted(self.session.catalog.dbs) if pat(db)]
        return self._meta_op(req, 3, ["TABLE_SCHEM", "TABLE_CATALOG"], ["string", "string"], rows)

    def rpc_GetTables(self, req):
        sp, tp = _like(req.get("schemaName")), _like(req.get("tableName"))
        rows = []
        for db, tabs in sorted(self.session.catalog.dbs.items()):
            if not sp(db):
                continue
            for t in tabs.values():
                if tp(t.name):
                    rows.append(("", db, t.name, "VIEW" if t.kind == "view" else "TABLE", ""))
        return self._meta_op(req, 4, ["TABLE_CAT", "TABLE_SCHEM", "TABLE_NAME", "TABLE_TYPE", "REMARKS"],
                             ["string"] * 5, rows)

    def rpc_GetTableTypes(self, req):
        return self._meta_op(req, 5, ["TABLE_TYPE"], ["string"], [("TABLE",), ("VIEW",)])

    def rpc_GetTypeInfo(self, req):
        rows = [(t.upper(), tid) for t, tid in T.TYPE_IDS.items()]
        return self._meta_op(req, 1, ["TYPE_NAME", "DATA_TYPE"], ["string", "int"], rows)

    def rpc_GetColumns(self, req):
        sp, tp, cp = _like(req.get("schemaName")), _like(req.get("tableName")), _like(req.get("columnName"))
        rows = []
        for db, tabs in sorted(self.session.catalog.dbs.items()):
            if not sp(db):
                continue
            for t in tabs.values():
                if not tp(t.name):
                    continue
                for i, (c, ty) in enumerate(t.schema):
                    if cp(c):
                        rows.append(("", db, t.name, c, T.TYPE_IDS.get(ty.split("(")[0], 7), ty.upper(), i + 1))
        return self._meta_op(req, 6, ["TABLE_CAT", "TABLE_SCHEM", "TABLE_NAME", "COLUMN_NAME", "DATA_TYPE",
                                      "TYPE_NAME", "ORDINAL_POSITION"],
                             ["string", "string", "string", "string", "int", "string", "int"], rows)

    def rpc_GetFunctions(self, req):
        from ..sql.functions import function_names

        fp = _like(req.get("functionName"))
        rows = [("", "", f, "", 1, f) for f in function_names() if fp(f)]
        return self._meta_op(req, 7, ["FUNCTION_CAT", "FUNCTION_SCHEM", "FUNCTION_NAME", "REMARKS", "FUNCTION_TYPE",
                                      "SPECIFIC_NAME"], ["string", "string", "string", "string", "int", "string"],
                             rows)


# ------------------------------------------------------------------------------------------------
def _ok():
    return {"statusCode": T.SUCCESS}


def _err(msg):
    return {"statusCode": T.ERROR, "errorMessage": msg or "error", "sqlState": "42000", "errorCode": 0}


def _sid(req) -> bytes:
    return req["sessionHandle"]["sessionId"]["guid"]


def _oid(req) -> bytes:
    return req["operationHandle"]["operationId"]["guid"]


def _like(p: Optional[str]):
    import re

    if not p or p in ("%", "*"):
        return lambda s: True
    rx = re.compile("^" + re.escape(p).replace("%", ".*").replace("_", ".").replace("\\*", ".*") + "$", re.I)
    return lambda s: rx.match(s) is not None


def _nulls(vals) -> bytes:
    n = len(vals)
    bits = bytearray((n + 7) // 8)
    for i, v in enumerate(vals):
        if v is None or v is pd.NA or v is pd.NaT or (isinstance(v, float) and v != v):
            bits[i // 8] |= 1 << (i % 8)
    return bytes(bits)


def _is_null(v) -> bool:
    return v is None or v is pd.NA or v is pd.NaT or (isinstance(v, float) and v != v)


def _tcolumn(t: str, vals: list) -> Dict[str, Any]:
    base_ = t.split("(")[0]
    nulls = _nulls(vals)
    if base_ == "boolean":
        return {"boolVal": {"values": [bool(v) if not _is_null(v) else False for v in vals], "nulls": nulls}}
    if base_ in ("tinyint",):
        return {"byteVal": {"values": [int(v) if not _is_null(v) else 0 for v in vals], "nulls": nulls}}
    if base_ in ("smallint",):
        return {"i16Val": {"values": [int(v) if not _is_null(v) else 0 for v in vals], "nulls": nulls}}
    if base_ in ("int",):
        return {"i32Val": {"values": [int(v) if not _is_null(v) else 0 for v in vals], "nulls": nulls}}
    if base_ in ("bigint",):
        return {"i64Val": {"values": [int(v) if not _is_null(v) else 0 for v in vals], "nulls": nulls}}
    if base_ in ("double", "float", "decimal"):
        return {"doubleVal": {"values": [float(v) if not _is_null(v) else 0.0 for v in vals], "nulls": nulls}}
    out = []
    for v in vals:
        if _is_null(v):
            out.append("")
        elif isinstance(v, pd.Timestamp):
            out.append(v.strftime("%Y-%m-%d") if base_ == "date" else str(v))
        else:
            out.append(str(v))
    return {"stringVal": {"values": out, "nulls": nulls}}


def _read_exact(f, n: int) -> Optional[bytes]:
    b = f.read(n)
    if not b or len(b) < n:
        return None
    return b


def _read_unframed_message(f) -> Optional[bytes]:
    """Read one complete unframed binary-protocol CALL (message header + args struct)."""
    buf = bytearray()
    rd = _Tee(f, buf)
    try:
        v = rd.i32()
    except EOFError:
        return None
    if v < 0:
        rd.string()
        rd.i32()
    else:
        rd.take(v)
        rd.take(1)
        rd.i32()
    rd.skip(T.STRUCT)
    return bytes(buf)


class _Tee:
    """Streams bytes from a socket file while skipping over a thrift value (to find its end)."""

    def __init__(self, f, buf):
        self.f, self.buf = f, buf

    def take(self, n):
        b = self.f.read(n)
        if len(b) < n:
            raise EOFError
        self.buf += b
        return b

    def i8(self):
        return struct.unpack("!b", self.take(1))[0]

    def i16(self):
        return struct.unpack("!h", self.take(2))[0]

    def i32(self):
        return struct.unpack("!i", self.take(4))[0]

    def string(self):
        n = self.i32()
        return self.take(n)

    def skip(self, t):
        if t == T.BOOL or t == T.BYTE:
            self.take(1)
        elif t == T.I16:
            self.take(2)
        elif t == T.I32:
            self.take(4)
        elif t in (T.I64, T.DOUBLE):
            self.take(8)
        elif t == T.STRING:
            self.string()
        elif t == T.STRUCT:
            while True:
                ft = self.i8()
                if ft == T.STOP:
                    return
                self.i16()
                self.skip(ft)
        elif t in (T.LIST, T.SET):
            et = self.i8()
            n = self.i32()
            for _ in range(n):
                self.skip(et)
        elif t == T.MAP:
            kt, vt = self.i8(), self.i8()
            n = self.i32()
            for _ in range(n):
                self.skip(kt)
                self.skip(vt)
        else:
            raise T.ProtocolError(f"bad type {t}")


def _load_datasources(sess, world, ingest_specs, store, dev) -> None:
    """Deployment: datasources from index tasks (``--ingest``) and/or a persisted segment store
    (``--segments``: ``<store>/<datasource>/rank<r>/manifest.json`` per shard, written by
    ``DataSource.save``).  A shard saved for a different world size is refused: its rows belong to
    another partitioning."""
    from ..segment.datasource import DataSource
    from ..segment.ingest import ingest

    log = logging.getLogger("sdo.thrift")
    for item in ingest_specs:
        spec, _, data_dir = item.partition("@")
        ds = ingest(spec, dev, rank=world.rank, world=world.size, data_dir=data_dir or None)
        sess.register_datasource(ds)
        log.info("ingested %s: %d rows on rank %d (%d total)", ds.name, ds.num_rows, world.rank, ds.global_num_rows)
        if store:
            ds.save(os.path.join(store, ds.name, f"rank{world.rank}"))
    if store and not ingest_specs and os.path.isdir(store):
        for name in sorted(os.listdir(store)):
            shard = os.path.join(store, name, f"rank{world.rank}")
            if not os.path.exists(os.path.join(shard, "manifest.json")):
                continue
            ds = DataSource.load(shard, dev)
            if ds.num_partitions != world.size:
                raise RuntimeError(f"segment store {shard} was written by {ds.num_partitions} ranks, "
                                   f"this server has {world.size}")
            sess.register_datasource(ds)
            log.info("loaded %s: %d rows on rank %d", ds.name, ds.num_rows, world.rank)


def main(argv=None):
    """``python -m spark_druid_olap_amd.server.hive_server --port 10000 [--tpch-sf 1] [--gpus N]``
    (the ``start-sparklinedatathriftserver.sh`` entry, scripts/start-sparklinedatathriftserver.sh).

    ``--gpus N`` (without torchrun): starts N rank processes, one per GPU; every rank holds
    ``--tpch-sf`` of synthetic TPC-H as its shard, rank 0 serves the clients and the others execute
    the broadcast statement stream (server/spmd.py)."""
    import argparse

    from ..utils.memory import serving_allocator_conf

    serving_allocator_conf()  # (before this process's first device allocation)
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=int(os.environ.get("SDO_THRIFT_PORT", "10000")))
    ap.add_argument("--tpch-sf", type=float, default=0.0, help="preload a synthetic TPC-H datasource (per rank)")
    ap.add_argument("--init-sql", default=None, help="file of ';'-separated statements to run at startup")
    ap.add_argument("--ui-port", type=int, default=int(os.environ.get("SDO_UI_PORT", "4040")),
                    help="Druid HTTP API + 'Druid Query Details' page (0 = any free port, -1 = off)")
    ap.add_argument("--conf", action="append", default=[], help="key=value session conf (repeatable)")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU) to start when not under torchrun")
    ap.add_argument("--port-file", default=None, help="write the bound Thrift port here (rank 0)")
    ap.add_argument("--ingest", action="append", default=[], metavar="SPEC[@DATA_DIR]",
                    help="run a Druid index task (JSON spec file) at startup; every rank keeps its hash "
                         "partition (repeatable)")
    ap.add_argument("--segments", default=None,
                    help="segment store root: load every datasource saved under DIR/<datasource>/rank<r> "
                         "(resume after restart); with --ingest, the ingested shards are saved there")
    ap.add_argument("--warmup", default=None,
                    help="file of ';'-separated statements the server runs (on its execution slots) before "
                         "taking clients; the slots' device memory is then sized for the largest "
                         "(server/gateway.py warm_up)")
    ap.add_argument("--gpu-wait", default="spin", choices=["blocking", "spin"],
                    help="HIP's wait mode for server threads (utils/hipsync.py): spin (HIP's default; the "
                         "engine's own waits sleep after 2 ms anyway) or blocking (every wait sleeps on the "
                         "completion interrupt: least CPU, less throughput near capacity)")
    ap.add_argument("--elastic", action="store_true",
                    help="survive a lost GPU process: heartbeats, communicator rebuild over the survivors and "
                         "re-homing of its shards from --segments (parallel/recovery.py)")
    a = ap.parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import sys

        from ..utils.launch import spawn_ranks

        sys.exit(spawn_ranks(a.gpus, [sys.executable, "-m", "spark_druid_olap_amd.server.hive_server"] +
                             list(argv if argv is not None else sys.argv[1:]), quiet_peers=False))
    logging.basicConfig(level=logging.INFO)
    if a.gpu_wait != "spin":
        # first thing, before torch or the world touch the device (the flag only takes then)
        from ..utils.hipsync import set_wait_mode

        set_wait_mode(a.gpu_wait, int(os.environ.get("LOCAL_RANK", "0")))
    import torch

    from ..parallel.world import init_world
    from ..session import Session

    world = init_world()
    dev = world.device()
    sess = Session(conf=dict(kv.split("=", 1) for kv in a.conf), world=world)
    if a.tpch_sf > 0:
        from ..models import tpch

        ds = tpch.to_datasource(tpch.generate_flat(a.tpch_sf, dev, rank=world.rank, world=world.size),
                                profile="bench")
        sess.register_datasource(ds)
        sess.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
        sess.sql(tpch.druid_ddl(with_column_mapping=False))
    _load_datasources(sess, world, a.ingest, a.segments, dev)
    if a.elastic and world.distributed:
        from ..parallel import recovery

        recovery.enable(world, segment_store=a.segments)
    if a.init_sql:
        with open(a.init_sql) as f:
            for st in f.read().split(";"):
                if st.strip():
                    sess.sql(st)
    if a.warmup and not world.distributed:
        from .gateway import warm_up

        with open(a.warmup) as f:
            stmts = [st for st in f.read().split(";") if st.strip()]
        logging.getLogger("sdo.thrift").info("warm-up: %s", warm_up(sess, stmts))
    if world.rank != 0:
        from ..parallel.world import shutdown
        from .spmd import serve_peer

        serve_peer(sess, world)
        shutdown()
        return
    if a.ui_port >= 0 and not world.distributed:
        # the reference attaches its "Druid Query Details" UI tab next to the Thrift server
        # (HiveThriftServer2.scala:73-77); here the same process also serves the Druid HTTP API
        from .druid_http import DruidHTTPServer

        ui = DruidHTTPServer(sess, a.host, a.ui_port).start()
        logging.getLogger("sdo.thrift").info("query history page: http://%s:%d/sparklinedata/druid/queries",
                                             a.host, ui.port)
    from .gateway import make_server

    srv = make_server(sess, a.host, a.port, world=world).start()  # native gateway unless SDO_NATIVE_GATEWAY=0
    if a.port_file:
        with open(a.port_file + ".tmp", "w") as f:
            f.write(str(srv.port))
        os.replace(a.port_file + ".tmp", a.port_file)
    import signal

    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    try:
        while not stop.wait(1.0):
            pass
    except KeyboardInterrupt:
        pass
    srv.stop()
    if world.distributed:
        from ..parallel.world import shutdown

        shutdown()


if __name__ == "__main__":
    main()
