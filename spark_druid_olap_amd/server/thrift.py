"""Thrift binary protocol (strict) + the HiveServer2 ``TCLIService`` schema subset.

No thrift library exists in the image, so the wire format is implemented here: messages
(``0x80010000 | type``, name, seqid), structs of typed fields, lists/maps, and the TCLIService
structs a JDBC/ODBC/beeline client needs (OpenSession, ExecuteStatement, GetOperationStatus,
GetResultSetMetadata, FetchResults with column-based row sets (protocol >= V6), CloseOperation,
CloseSession, GetInfo, GetTables, GetSchemas, GetCatalogs, GetColumns, GetTableTypes, GetTypeInfo,
GetFunctions, CancelOperation).  Field ids follow Hive's ``TCLIService.thrift``.
"""
from __future__ import annotations

import struct
from typing import Any, Dict, Tuple

STOP, BOOL, BYTE, DOUBLE, I16, I32, I64, STRING, STRUCT, MAP, SET, LIST = 0, 2, 3, 4, 6, 8, 10, 11, 12, 13, 14, 15
BINARY = "binary"   # STRING on the wire, bytes in Python

CALL, REPLY, EXCEPTION, ONEWAY = 1, 2, 3, 4
VERSION_1 = 0x80010000


def L(e):
    return ("list", e)


def M(k, v):
    return ("map", k, v)


def St(n):
    return ("struct", n)


SCHEMAS: Dict[str, Dict[int, Tuple[str, Any]]] = {
    "TStatus": {1: ("statusCode", I32), 2: ("infoMessages", L(STRING)), 3: ("sqlState", STRING),
                4: ("errorCode", I32), 5: ("errorMessage", STRING)},
    "THandleIdentifier": {1: ("guid", BINARY), 2: ("secret", BINARY)},
    "TSessionHandle": {1: ("sessionId", St("THandleIdentifier"))},
    "TOperationHandle": {1: ("operationId", St("THandleIdentifier")), 2: ("operationType", I32),
                         3: ("hasResultSet", BOOL), 4: ("modifiedRowCount", DOUBLE)},
    "TOpenSessionReq": {1: ("client_protocol", I32), 2: ("username", STRING), 3: ("password", STRING),
                        4: ("configuration", M(STRING, STRING))},
    "TOpenSessionResp": {1: ("status", St("TStatus")), 2: ("serverProtocolVersion", I32),
                         3: ("sessionHandle", St("TSessionHandle")), 4: ("configuration", M(STRING, STRING))},
    "TCloseSessionReq": {1: ("sessionHandle", St("TSessionHandle"))},
    "TCloseSessionResp": {1: ("status", St("TStatus"))},
    "TExecuteStatementReq": {1: ("sessionHandle", St("TSessionHandle")), 2: ("statement", STRING),
                             3: ("confOverlay", M(STRING, STRING)), 4: ("runAsync", BOOL), 5: ("queryTimeout", I64)},
    "TExecuteStatementResp": {1: ("status", St("TStatus")), 2: ("operationHandle", St("TOperationHandle"))},
    "TGetOperationStatusReq": {1: ("operationHandle", St("TOperationHandle")), 2: ("getProgressUpdate", BOOL)},
    "TGetOperationStatusResp": {1: ("status", St("TStatus")), 2: ("operationState", I32), 3: ("sqlState", STRING),
                                4: ("errorCode", I32), 5: ("errorMessage", STRING), 6: ("taskStatus", STRING),
                                7: ("operationStarted", I64), 8: ("operationCompleted", I64),
                                9: ("hasResultSet", BOOL)},
    "TCancelOperationReq": {1: ("operationHandle", St("TOperationHandle"))},
    "TCancelOperationResp": {1: ("status", St("TStatus"))},
    "TCloseOperationReq": {1: ("operationHandle", St("TOperationHandle"))},
    "TCloseOperationResp": {1: ("status", St("TStatus"))},
    "TGetResultSetMetadataReq": {1: ("operationHandle", St("TOperationHandle"))},
    "TGetResultSetMetadataResp": {1: ("status", St("TStatus")), 2: ("schema", St("TTableSchema"))},
    "TTableSchema": {1: ("columns", L(St("TColumnDesc")))},
    "TColumnDesc": {1: ("columnName", STRING), 2: ("typeDesc", St("TTypeDesc")), 3: ("position", I32),
                    4: ("comment", STRING)},
    "TTypeDesc": {1: ("types", L(St("TTypeEntry")))},
    "TTypeEntry": {1: ("primitiveEntry", St("TPrimitiveTypeEntry"))},
    "TPrimitiveTypeEntry": {1: ("type", I32), 2: ("typeQualifiers", St("TTypeQualifiers"))},
    "TTypeQualifiers": {1: ("qualifiers", M(STRING, St("TTypeQualifierValue")))},
    "TTypeQualifierValue": {1: ("i32Value", I32), 2: ("stringValue", STRING)},
    "TFetchResultsReq": {1: ("operationHandle", St("TOperationHandle")), 2: ("orientation", I32),
                         3: ("maxRows", I64), 4: ("fetchType", I16)},
    "TFetchResultsResp": {1: ("status", St("TStatus")), 2: ("hasMoreRows", BOOL), 3: ("results", St("TRowSet"))},
    "TRowSet": {1: ("startRowOffset", I64), 2: ("rows", L(St("TRow"))), 3: ("columns", L(St("TColumn"))),
                4: ("binaryColumns", BINARY), 5: ("columnCount", I32)},
    "TRow": {1: ("colVals", L(St("TColumnValue")))},
    "TColumnValue": {1: ("boolVal", St("TBoolValue")), 2: ("byteVal", St("TByteValue")),
                     3: ("i16Val", St("TI16Value")), 4: ("i32Val", St("TI32Value")), 5: ("i64Val", St("TI64Value")),
                     6: ("doubleVal", St("TDoubleValue")), 7: ("stringVal", St("TStringValue"))},
    "TBoolValue": {1: ("value", BOOL)}, "TByteValue": {1: ("value", BYTE)}, "TI16Value": {1: ("value", I16)},
    "TI32Value": {1: ("value", I32)}, "TI64Value": {1: ("value", I64)}, "TDoubleValue": {1: ("value", DOUBLE)},
    "TStringValue": {1: ("value", STRING)},
    "TColumn": {1: ("boolVal", St("TBoolColumn")), 2: ("byteVal", St("TByteColumn")),
                3: ("i16Val", St("TI16Column")), 4: ("i32Val", St("TI32Column")), 5: ("i64Val", St("TI64Column")),
                6: ("doubleVal", St("TDoubleColumn")), 7: ("stringVal", St("TStringColumn")),
                8: ("binaryVal", St("TBinaryColumn"))},
    "TBoolColumn": {1: ("values", L(BOOL)), 2: ("nulls", BINARY)},
    "TByteColumn": {1: ("values", L(BYTE)), 2: ("nulls", BINARY)},
    "TI16Column": {1: ("values", L(I16)), 2: ("nulls", BINARY)},
    "TI32Column": {1: ("values", L(I32)), 2: ("nulls", BINARY)},
    "TI64Column": {1: ("values", L(I64)), 2: ("nulls", BINARY)},
    "TDoubleColumn": {1: ("values", L(DOUBLE)), 2: ("nulls", BINARY)},
    "TStringColumn": {1: ("values", L(STRING)), 2: ("nulls", BINARY)},
    "TBinaryColumn": {1: ("values", L(BINARY)), 2: ("nulls", BINARY)},
    "TGetInfoReq": {1: ("sessionHandle", St("TSessionHandle")), 2: ("infoType", I32)},
    "TGetInfoResp": {1: ("status", St("TStatus")), 2: ("infoValue", St("TGetInfoValue"))},
    "TGetInfoValue": {1: ("stringValue", STRING), 2: ("smallIntValue", I16), 3: ("integerBitmask", I32),
                      4: ("integerFlag", I32), 5: ("binaryValue", I32), 6: ("lenValue", I64)},
    "TGetTablesReq": {1: ("sessionHandle", St("TSessionHandle")), 2: ("catalogName", STRING),
                      3: ("schemaName", STRING), 4: ("tableName", STRING), 5: ("tableTypes", L(STRING))},
    "TGetSchemasReq": {1: ("sessionHandle", St("TSessionHandle")), 2: ("catalogName", STRING),
                       3: ("schemaName", STRING)},
    "TGetCatalogsReq": {1: ("sessionHandle", St("TSessionHandle"))},
    "TGetTableTypesReq": {1: ("sessionHandle", St("TSessionHandle"))},
    "TGetTypeInfoReq": {1: ("sessionHandle", St("TSessionHandle"))},
    "TGetColumnsReq": {1: ("sessionHandle", St("TSessionHandle")), 2: ("catalogName", STRING),
                       3: ("schemaName", STRING), 4: ("tableName", STRING), 5: ("columnName", STRING)},
    "TGetFunctionsReq": {1: ("sessionHandle", St("TSessionHandle")), 2: ("catalogName", STRING),
                         3: ("schemaName", STRING), 4: ("functionName", STRING)},
    "TGetMetadataResp": {1: ("status", St("TStatus")), 2: ("operationHandle", St("TOperationHandle"))},
}

# method -> (request struct, response struct)
METHODS = {
    "OpenSession": ("TOpenSessionReq", "TOpenSessionResp"),
    "CloseSession": ("TCloseSessionReq", "TCloseSessionResp"),
    "GetInfo": ("TGetInfoReq", "TGetInfoResp"),
    "ExecuteStatement": ("TExecuteStatementReq", "TExecuteStatementResp"),
    "GetOperationStatus": ("TGetOperationStatusReq", "TGetOperationStatusResp"),
    "CancelOperation": ("TCancelOperationReq", "TCancelOperationResp"),
    "CloseOperation": ("TCloseOperationReq", "TCloseOperationResp"),
    "GetResultSetMetadata": ("TGetResultSetMetadataReq", "TGetResultSetMetadataResp"),
    "FetchResults": ("TFetchResultsReq", "TFetchResultsResp"),
    "GetTables": ("TGetTablesReq", "TGetMetadataResp"),
    "GetSchemas": ("TGetSchemasReq", "TGetMetadataResp"),
    "GetCatalogs": ("TGetCatalogsReq", "TGetMetadataResp"),
    "GetTableTypes": ("TGetTableTypesReq", "TGetMetadataResp"),
    "GetTypeInfo": ("TGetTypeInfoReq", "TGetMetadataResp"),
    "GetColumns": ("TGetColumnsReq", "TGetMetadataResp"),
    "GetFunctions": ("TGetFunctionsReq", "TGetMetadataResp"),
}

# enums
SUCCESS, SUCCESS_WITH_INFO, STILL_EXECUTING, ERROR, INVALID_HANDLE = 0, 1, 2, 3, 4
OP_INITIALIZED, OP_RUNNING, OP_FINISHED, OP_CANCELED, OP_CLOSED, OP_ERROR = 0, 1, 2, 3, 4, 5
PROTOCOL_V8 = 7
TYPE_IDS = {"boolean": 0, "tinyint": 1, "smallint": 2, "int": 3, "bigint": 4, "float": 5, "double": 6,
            "string": 7, "timestamp": 8, "binary": 9, "decimal": 15, "null": 16, "date": 17}


class ProtocolError(IOError):
    pass


# ------------------------------------------------------------------------------------------------
class Writer:
    def __init__(self):
        self.buf = bytearray()

    def i8(self, v):
        self.buf += struct.pack("!b", v)

    def i16(self, v):
        self.buf += struct.pack("!h", v)

    def i32(self, v):
        self.buf += struct.pack("!i", v)

    def i64(self, v):
        self.buf += struct.pack("!q", v)

    def dbl(self, v):
        self.buf += struct.pack("!d", v)

    def string(self, v):
        b = v if isinstance(v, (bytes, bytearray)) else str(v).encode("utf-8")
        self.i32(len(b))
        self.buf += b

    def message_begin(self, name: str, mtype: int, seqid: int):
        self.buf += struct.pack("!I", VERSION_1 | mtype)
        self.string(name)
        self.i32(seqid)

    def value(self, spec, v):
        t = _wire(spec)
        if t == BOOL:
            self.i8(1 if v else 0)
        elif t == BYTE:
            self.i8(v)
        elif t == I16:
            self.i16(v)
        elif t == I32:
            self.i32(v)
        elif t == I64:
            self.i64(v)
        elif t == DOUBLE:
            self.dbl(v)
        elif t == STRING:
            self.string(v)
        elif t == STRUCT:
            self.struct(spec[1], v)
        elif t == LIST:
            et = spec[1]
            self.i8(_wire(et))
            self.i32(len(v))
            for x in v:
                self.value(et, x)
        elif t == MAP:
            self.i8(_wire(spec[1]))
            self.i8(_wire(spec[2]))
            self.i32(len(v))
            for k, x in v.items():
                self.value(spec[1], k)
                self.value(spec[2], x)
        else:
            raise ProtocolError(f"cannot write type {spec}")

    def struct(self, name: str, d: Dict[str, Any]):
        sch = SCHEMAS[name]
        for fid, (fname, spec) in sorted(sch.items()):
            v = d.get(fname)
            if v is None:
                continue
            self.i8(_wire(spec))
            self.i16(fid)
            self.value(spec, v)
        self.i8(STOP)

    def raw_result(self, resp_struct: str, d: Dict[str, Any]):
        """``<Method>_result { 0: <Resp> success }``"""
        self.i8(STRUCT)
        self.i16(0)
        self.struct(resp_struct, d)
        self.i8(STOP)

    def raw_args(self, req_struct: str, d: Dict[str, Any]):
        """``<Method>_args { 1: <Req> req }``"""
        self.i8(STRUCT)
        self.i16(1)
        self.struct(req_struct, d)
        self.i8(STOP)


def _wire(spec) -> int:
    if spec == BINARY:
        return STRING
    if isinstance(spec, tuple):
        return {"struct": STRUCT, "list": LIST, "map": MAP}[spec[0]]
    return spec


class Reader:
    def __init__(self, data: bytes):
        self.d = memoryview(data)
        self.p = 0

    def _take(self, n):
        if self.p + n > len(self.d):
            raise ProtocolError("truncated message")
        b = self.d[self.p:self.p + n]
        self.p += n
        return b

    def i8(self):
        return struct.unpack("!b", self._take(1))[0]

    def i16(self):
        return struct.unpack("!h", self._take(2))[0]

    def i32(self):
        return struct.unpack("!i", self._take(4))[0]

    def i64(self):
        return struct.unpack("!q", self._take(8))[0]

    def dbl(self):
        return struct.unpack("!d", self._take(8))[0]

    def binary(self):
        n = self.i32()
        return bytes(self._take(n))

    def message_begin(self):
        v = self.i32()
        if v < 0:
            v &= 0xFFFFFFFF
            if v & 0xFFFF0000 != VERSION_1:
                raise ProtocolError("bad protocol version")
            mtype = v & 0xFF
            name = self.binary().decode()
            seqid = self.i32()
            return name, mtype, seqid
        # old non-strict: v is name length
        name = bytes(self._take(v)).decode()
        mtype = self.i8()
        seqid = self.i32()
        return name, mtype, seqid

    def value(self, t, spec=None):
        if t == BOOL:
            return self.i8() != 0
        if t == BYTE:
            return self.i8()
        if t == I16:
            return self.i16()
        if t == I32:
            return self.i32()
        if t == I64:
            return self.i64()
        if t == DOUBLE:
            return self.dbl()
        if t == STRING:
            b = self.binary()
            if spec == BINARY:
                return b
            try:
                return b.decode("utf-8")
            except UnicodeDecodeError:
                return b
        if t == STRUCT:
            if isinstance(spec, tuple) and spec[0] == "struct":
                return self.struct(spec[1])
            return self.struct(None)
        if t in (LIST, SET):
            et = self.i8()
            n = self.i32()
            es = spec[1] if isinstance(spec, tuple) and spec[0] == "list" else None
            return [self.value(et, es) for _ in range(n)]
        if t == MAP:
            kt = self.i8()
            vt = self.i8()
            n = self.i32()
            ks = spec[1] if isinstance(spec, tuple) and spec[0] == "map" else None
            vs = spec[2] if isinstance(spec, tuple) and spec[0] == "map" else None
            return {self.value(kt, ks): self.value(vt, vs) for _ in range(n)}
        raise ProtocolError(f"unknown wire type {t}")

    def struct(self, name):
        sch = SCHEMAS.get(name, {}) if name else {}
        out: Dict[str, Any] = {}
        while True:
            t = self.i8()
            if t == STOP:
                return out
            fid = self.i16()
            f = sch.get(fid)
            v = self.value(t, f[1] if f else None)
            out[f[0] if f else f"_{fid}"] = v


def encode_call(method: str, seqid: int, req: Dict[str, Any]) -> bytes:
    w = Writer()
    w.message_begin(method, CALL, seqid)
    w.raw_args(METHODS[method][0], req)
    return bytes(w.buf)


def encode_reply(method: str, seqid: int, resp: Dict[str, Any]) -> bytes:
    w = Writer()
    w.message_begin(method, REPLY, seqid)
    w.raw_result(METHODS[method][1], resp)
    return bytes(w.buf)


def encode_exception(method: str, seqid: int, msg: str, code: int = 6) -> bytes:
    """TApplicationException { 1: message, 2: type }"""
    w = Writer()
    w.message_begin(method, EXCEPTION, seqid)
    w.i8(STRING)
    w.i16(1)
    w.string(msg)
    w.i8(I32)
    w.i16(2)
    w.i32(code)
    w.i8(STOP)
    return bytes(w.buf)


def decode_call(data: bytes):
    r = Reader(data)
    name, mtype, seqid = r.message_begin()
    req_name = METHODS.get(name, (None, None))[0]
    args = r.struct(None) if req_name is None else _args(r, req_name)
    return name, mtype, seqid, args


def _args(r: Reader, req_name: str):
    out = None
    while True:
        t = r.i8()
        if t == STOP:
            return out or {}
        fid = r.i16()
        if fid == 1 and t == STRUCT:
            out = r.struct(req_name)
        else:
            r.value(t)


def decode_reply(data: bytes, method: str):
    r = Reader(data)
    name, mtype, seqid = r.message_begin()
    if mtype == EXCEPTION:
        e = r.struct(None)
        raise ProtocolError(f"server exception: {e.get('_1')}")
    resp_name = METHODS[method][1]
    out = None
    while True:
        t = r.i8()
        if t == STOP:
            return out
        fid = r.i16()
        if fid == 0 and t == STRUCT:
            out = r.struct(resp_name)
        else:
            r.value(t)
