"""Minimal HiveServer2 client (DB-API-like) speaking the same Thrift subset.

Used by the tests, the ``sdo-beeline`` CLI (``tools/beeline.py``) and the concurrency soak
(BASELINE config 5: many concurrent clients).  SASL PLAIN framing (HiveServer2 default) or raw
``noSasl`` transport."""
from __future__ import annotations

import socket
import struct
import threading
from typing import Any, Dict, List, Optional, Tuple

from . import thrift as T
from .hive_server import SASL_COMPLETE, SASL_OK, SASL_START, _read_unframed_message


class HiveError(RuntimeError):
    pass


class Connection:
    def __init__(self, host: str = "127.0.0.1", port: int = 10000, user: str = "anonymous",
                 password: str = "anonymous", sasl: bool = True, database: Optional[str] = None,
                 configuration: Optional[Dict[str, str]] = None, timeout: float = 600.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.f = self.sock.makefile("rb")
        self.sasl = sasl
        self.seq = 0
        self._lock = threading.Lock()
        if sasl:
            mech = b"PLAIN"
            self.sock.sendall(bytes([SASL_START]) + struct.pack("!i", len(mech)) + mech)
            payload = b"\0" + user.encode() + b"\0" + password.encode()
            self.sock.sendall(bytes([SASL_OK]) + struct.pack("!i", len(payload)) + payload)
            st = self.f.read(1)
            (n,) = struct.unpack("!i", self.f.read(4))
            self.f.read(n)
            if not st or st[0] != SASL_COMPLETE:
                raise HiveError("SASL negotiation failed")
        conf = dict(configuration or {})
        if database:
            conf["use:database"] = database
        r = self.call("OpenSession", {"client_protocol": T.PROTOCOL_V8, "username": user, "configuration": conf})
        _check(r)
        self.session = r["sessionHandle"]

    def call(self, method: str, req: Dict[str, Any]) -> Dict[str, Any]:
        with self._lock:
            self.seq += 1
            msg = T.encode_call(method, self.seq, req)
            if self.sasl:
                self.sock.sendall(struct.pack("!i", len(msg)) + msg)
                (n,) = struct.unpack("!i", self.f.read(4))
                data = self.f.read(n)
            else:
                self.sock.sendall(msg)
                data = _read_unframed_message(self.f)
            return T.decode_reply(data, method)

    def cursor(self) -> "Cursor":
        return Cursor(self)

    def close(self):
        try:
            self.call("CloseSession", {"sessionHandle": self.session})
        finally:
            self.f.close()
            self.sock.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _check(r):
    st = r.get("status", {})
    if st.get("statusCode", 0) not in (T.SUCCESS, T.SUCCESS_WITH_INFO):
        raise HiveError(st.get("errorMessage", "error"))


_ID_TO_TYPE = {v: k for k, v in T.TYPE_IDS.items()}


class Cursor:
    def __init__(self, conn: Connection):
        self.conn = conn
        self.op = None
        self.description: Optional[List[Tuple[str, str]]] = None
        self.arraysize = 10000

    def execute(self, sql: str, run_async: bool = False) -> "Cursor":
        r = self.conn.call("ExecuteStatement", {"sessionHandle": self.conn.session, "statement": sql,
                                                "runAsync": run_async})
        _check(r)
        self.op = r["operationHandle"]
        if run_async:
            while True:
                s = self.conn.call("GetOperationStatus", {"operationHandle": self.op})
                if s.get("operationState") in (T.OP_FINISHED, T.OP_ERROR, T.OP_CANCELED, T.OP_CLOSED):
                    if s.get("operationState") == T.OP_ERROR:
                        raise HiveError(s.get("errorMessage"))
                    break
        m = self.conn.call("GetResultSetMetadata", {"operationHandle": self.op})
        _check(m)
        cols = (m.get("schema") or {}).get("columns", [])
        self.description = [(c["columnName"], _ID_TO_TYPE.get(c["typeDesc"]["types"][0]["primitiveEntry"]["type"],
                                                              "string")) for c in cols]
        return self

    def fetchmany(self, n: Optional[int] = None) -> List[tuple]:
        r = self.conn.call("FetchResults", {"operationHandle": self.op, "orientation": 0,
                                            "maxRows": n or self.arraysize})
        _check(r)
        rs = r.get("results") or {}
        cols = rs.get("columns") or []
        out_cols = []
        for c in cols:
            (kind, v), = c.items()
            vals = v.get("values", [])
            nulls = v.get("nulls", b"") or b""
            out_cols.append([None if (i // 8 < len(nulls) and nulls[i // 8] >> (i % 8) & 1) else x
                             for i, x in enumerate(vals)])
        self._more = bool(r.get("hasMoreRows"))
        return list(zip(*out_cols)) if out_cols else []

    def fetchall(self) -> List[tuple]:
        out = []
        while True:
            page = self.fetchmany()
            out += page
            if not self._more:
                break
        return out

    def close(self):
        if self.op is not None:
            self.conn.call("CloseOperation", {"operationHandle": self.op})
            self.op = None


def connect(*a, **k) -> Connection:
    return Connection(*a, **k)
