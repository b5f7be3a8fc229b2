"""Smile (binary JSON) codec -- the reference's ``useSmile`` wire format.

The reference posts query specs and reads results as Smile when ``useSmile`` is on
(``sd/client/DruidClient.scala:183-189, 244-251, 304-314``; json4s glue
``src/main/scala/org/json4s/jackson/sparklinedata/SmileJsonMethods.scala:24-39``) and forces ints
to be written as Smile ints because Druid type-checks its context fields
(``SmileJson4sScalaModule.scala:42-83``).  This is a from-scratch encoder/decoder of the Smile
format as Jackson writes it by default:

* header ``:)\\n`` + version/flags byte (bit0 shared property names, bit1 shared string values,
  bit2 raw binary); we write shared names on, shared values off (Jackson's defaults) and read all
  three;
* key tokens: short shared-name refs (0x40-0x7F), long shared-name refs (0x30-0x33), short
  ASCII / Unicode names (0x80-0xBF / 0xC0-0xF7), long names (0x34 ... 0xFC), ``""`` (0x20);
* value tokens: small ints (0xC0-0xDF, zigzag), int32 / int64 / BigInteger (0x24-0x26, zigzag
  VInts), float32 / float64 (0x28 / 0x29, 7-bit packed), tiny / small ASCII and Unicode strings,
  long strings (0xE0 / 0xE4 ... 0xFC), shared-value refs, 7-bit binary (0xE8), raw binary (0xFD),
  arrays / objects (0xF8-0xFB), end-of-content 0xFF.

Python ints are written as Smile ints (so ``context.timeout`` stays an int, the reason the
reference needed a custom json4s module); bools, None, floats, str, bytes, lists/tuples, dicts
map to their Smile tokens.
"""
from __future__ import annotations

import struct
from typing import Any, List, Optional, Tuple

HEADER = b":)\n"
MIME = "application/x-jackson-smile"
F_SHARED_NAMES = 0x01
F_SHARED_VALUES = 0x02
F_RAW_BINARY = 0x04
MAX_SHARED = 1024
MAX_SHARED_VALUE_BYTES = 64


class SmileError(ValueError):
    pass


def is_smile(data: bytes) -> bool:
    return data[:3] == HEADER


# ----------------------------------------------------------------------------------- primitives
def _zz(v: int) -> int:
    return (v << 1) ^ (v >> 63) if -(1 << 63) <= v < (1 << 63) else (v << 1) ^ (-1 if v < 0 else 0)


def _unzz(u: int) -> int:
    return (u >> 1) ^ -(u & 1)


def _vint(v: int) -> bytes:
    """Smile VInt: big-endian 7-bit groups (MSB clear), last byte MSB set with 6 data bits."""
    if v < 0:
        raise SmileError("negative VInt")
    last = 0x80 | (v & 0x3F)
    v >>= 6
    out = []
    while v:
        out.append(v & 0x7F)
        v >>= 7
    return bytes(reversed(out)) + bytes([last])


def _pack7(data: bytes) -> bytes:
    """7-bit binary encoding: every 7 raw bytes -> 8 bytes of 7 bits; a trailing group of n bytes
    -> n + 1 bytes (last byte right-aligned)."""
    out = bytearray()
    i, n = 0, len(data)
    while i + 7 <= n:
        acc = int.from_bytes(data[i:i + 7], "big")
        out.extend(((acc >> (7 * (7 - k))) & 0x7F) for k in range(8))
        i += 7
    r = n - i
    if r:
        acc = int.from_bytes(data[i:], "big")
        bits = 8 * r
        groups = r + 1
        pad = 7 * groups - bits
        acc <<= pad
        vals = [((acc >> (7 * (groups - 1 - k))) & 0x7F) for k in range(groups)]
        vals[-1] >>= pad
        out.extend(vals)
    return bytes(out)


def _unpack7(buf: bytes, pos: int, nraw: int) -> Tuple[bytes, int]:
    out = bytearray()
    full, r = divmod(nraw, 7)
    for _ in range(full):
        acc = 0
        for k in range(8):
            acc = (acc << 7) | (buf[pos + k] & 0x7F)
        out.extend(acc.to_bytes(7, "big"))
        pos += 8
    if r:
        groups = r + 1
        pad = 7 * groups - 8 * r
        acc = 0
        for k in range(groups):
            b = buf[pos + k] & 0x7F
            if k == groups - 1:
                acc = (acc << (7 - pad)) | b
            else:
                acc = (acc << 7) | b
        out.extend(acc.to_bytes(r, "big"))
        pos += groups
    return bytes(out), pos


# ----------------------------------------------------------------------------------- encoder
class _Encoder:
    def __init__(self, shared_names: bool, shared_values: bool):
        self.out = bytearray()
        self.shared_names = shared_names
        self.shared_values = shared_values
        self.names: dict = {}
        self.values: dict = {}

    def name(self, k: str) -> None:
        o = self.out
        if k == "":
            o.append(0x20)
            return
        if self.shared_names:
            ix = self.names.get(k)
            if ix is not None:
                if ix < 64:
                    o.append(0x40 | ix)
                else:
                    o.extend((0x30 | (ix >> 8), ix & 0xFF))
                return
        b = k.encode("utf-8")
        n = len(b)
        if n <= 64 and len(k) == n:
            o.append(0x80 | (n - 1))
            o.extend(b)
        elif 2 <= n <= 57 and len(k) != n:
            o.append(0xC0 | (n - 2))
            o.extend(b)
        else:
            o.append(0x34)
            o.extend(b)
            o.append(0xFC)
        if self.shared_names:
            if len(self.names) >= MAX_SHARED:
                self.names.clear()
            self.names[k] = len(self.names)

    def string(self, s: str) -> None:
        o = self.out
        if s == "":
            o.append(0x20)
            return
        b = s.encode("utf-8")
        n = len(b)
        if self.shared_values and n <= MAX_SHARED_VALUE_BYTES:
            ix = self.values.get(s)
            if ix is not None:
                if ix < 31:
                    o.append(ix + 1)
                else:
                    o.extend((0xEC | (ix >> 8), ix & 0xFF))
                return
        ascii_ = len(s) == n
        if ascii_ and n <= 32:
            o.append(0x40 | (n - 1))
            o.extend(b)
        elif ascii_ and n <= 64:
            o.append(0x60 | (n - 33))
            o.extend(b)
        elif not ascii_ and 2 <= n <= 33:
            o.append(0x80 | (n - 2))
            o.extend(b)
        elif not ascii_ and 34 <= n <= 65:
            o.append(0xA0 | (n - 34))
            o.extend(b)
        else:
            o.append(0xE0 if ascii_ else 0xE4)
            o.extend(b)
            o.append(0xFC)
        if self.shared_values and n <= MAX_SHARED_VALUE_BYTES:
            if len(self.values) >= MAX_SHARED:
                self.values.clear()
            self.values[s] = len(self.values)

    def value(self, v: Any) -> None:
        o = self.out
        if v is None:
            o.append(0x21)
        elif v is True:
            o.append(0x23)
        elif v is False:
            o.append(0x22)
        elif isinstance(v, int):
            if -16 <= v <= 15:
                o.append(0xC0 | _zz(v))
            elif -(1 << 31) <= v < (1 << 31):
                o.append(0x24)
                o.extend(_vint(_zz(v)))
            elif -(1 << 63) <= v < (1 << 63):
                o.append(0x25)
                o.extend(_vint(_zz(v)))
            else:
                raw = v.to_bytes((v.bit_length() + 8) // 8, "big", signed=True)
                o.append(0x26)
                o.extend(_vint(len(raw)))
                o.extend(_pack7(raw))
        elif isinstance(v, float):
            bits = struct.unpack(">Q", struct.pack(">d", v))[0]
            o.append(0x29)
            o.append((bits >> 63) & 0x01)
            o.extend(((bits >> (7 * (8 - k))) & 0x7F) for k in range(9))
        elif isinstance(v, str):
            self.string(v)
        elif isinstance(v, (bytes, bytearray, memoryview)):
            raw = bytes(v)
            o.append(0xE8)
            o.extend(_vint(len(raw)))
            o.extend(_pack7(raw))
        elif isinstance(v, dict):
            o.append(0xFA)
            for k, x in v.items():
                self.name(str(k))
                self.value(x)
            o.append(0xFB)
        elif isinstance(v, (list, tuple)):
            o.append(0xF8)
            for x in v:
                self.value(x)
            o.append(0xF9)
        else:
            try:  # numpy scalars
                import numpy as np

                if isinstance(v, np.generic):
                    return self.value(v.item())
            except ImportError:  # pragma: no cover
                pass
            raise SmileError(f"cannot encode {type(v).__name__}")


def dumps(obj: Any, shared_names: bool = True, shared_values: bool = False, end_marker: bool = False) -> bytes:
    enc = _Encoder(shared_names, shared_values)
    flags = (F_SHARED_NAMES if shared_names else 0) | (F_SHARED_VALUES if shared_values else 0)
    enc.out.extend(HEADER)
    enc.out.append(flags)
    enc.value(obj)
    if end_marker:
        enc.out.append(0xFF)
    return bytes(enc.out)


# ----------------------------------------------------------------------------------- decoder
class _Decoder:
    def __init__(self, buf: bytes, shared_names: bool, shared_values: bool):
        self.b = buf
        self.p = 0
        self.shared_names = shared_names
        self.shared_values = shared_values
        self.names: List[str] = []
        self.values: List[str] = []

    def _byte(self) -> int:
        if self.p >= len(self.b):
            raise SmileError("unexpected end of Smile content")
        c = self.b[self.p]
        self.p += 1
        return c

    def _take(self, n: int) -> bytes:
        if self.p + n > len(self.b):
            raise SmileError("unexpected end of Smile content")
        s = self.b[self.p:self.p + n]
        self.p += n
        return s

    def _until_fc(self) -> bytes:
        j = self.b.find(b"\xfc", self.p)
        if j < 0:
            raise SmileError("unterminated long string")
        s = self.b[self.p:j]
        self.p = j + 1
        return s

    def _vint(self) -> int:
        v = 0
        while True:
            c = self._byte()
            if c & 0x80:
                return (v << 6) | (c & 0x3F)
            v = (v << 7) | c

    def _seen_name(self, s: str) -> str:
        if self.shared_names:
            if len(self.names) >= MAX_SHARED:
                self.names.clear()
            self.names.append(s)
        return s

    def _seen_value(self, s: str, nbytes: int) -> str:
        if self.shared_values and nbytes <= MAX_SHARED_VALUE_BYTES:
            if len(self.values) >= MAX_SHARED:
                self.values.clear()
            self.values.append(s)
        return s

    def name(self, c: int) -> str:
        if c == 0x20:
            return ""
        if 0x40 <= c <= 0x7F:
            return self.names[c & 0x3F]
        if 0x30 <= c <= 0x33:
            return self.names[((c & 0x03) << 8) | self._byte()]
        if 0x80 <= c <= 0xBF:
            return self._seen_name(self._take((c & 0x3F) + 1).decode("ascii"))
        if 0xC0 <= c <= 0xF7:
            return self._seen_name(self._take((c & 0x3F) + 2).decode("utf-8"))
        if c == 0x34:
            return self._seen_name(self._until_fc().decode("utf-8"))
        raise SmileError(f"invalid key token 0x{c:02x}")

    def value(self) -> Any:
        c = self._byte()
        if c < 0x20:
            if c == 0:
                raise SmileError("invalid value token 0x00")
            return self.values[c - 1]
        if c == 0x20:
            return ""
        if c == 0x21:
            return None
        if c == 0x22:
            return False
        if c == 0x23:
            return True
        if c in (0x24, 0x25):
            return _unzz(self._vint())
        if c == 0x26:
            n = self._vint()
            raw, self.p = _unpack7(self.b, self.p, n)
            return int.from_bytes(raw, "big", signed=True)
        if c == 0x28:
            bits = 0
            for _ in range(5):
                bits = (bits << 7) | (self._byte() & 0x7F)
            return struct.unpack(">f", struct.pack(">I", bits & 0xFFFFFFFF))[0]
        if c == 0x29:
            bits = 0
            for _ in range(10):
                bits = (bits << 7) | (self._byte() & 0x7F)
            return struct.unpack(">d", struct.pack(">Q", bits & 0xFFFFFFFFFFFFFFFF))[0]
        if c == 0x2A:  # BigDecimal: scale (zigzag VInt) + 7-bit unscaled magnitude
            scale = _unzz(self._vint())
            n = self._vint()
            raw, self.p = _unpack7(self.b, self.p, n)
            from decimal import Decimal

            return float(Decimal(int.from_bytes(raw, "big", signed=True)).scaleb(-scale))
        if 0x40 <= c <= 0x5F:
            n = (c & 0x1F) + 1
            return self._seen_value(self._take(n).decode("ascii"), n)
        if 0x60 <= c <= 0x7F:
            n = (c & 0x1F) + 33
            return self._seen_value(self._take(n).decode("ascii"), n)
        if 0x80 <= c <= 0x9F:
            n = (c & 0x1F) + 2
            return self._seen_value(self._take(n).decode("utf-8"), n)
        if 0xA0 <= c <= 0xBF:
            n = (c & 0x1F) + 34
            return self._seen_value(self._take(n).decode("utf-8"), n)
        if 0xC0 <= c <= 0xDF:
            return _unzz(c & 0x1F)
        if c in (0xE0, 0xE4):
            return self._until_fc().decode("utf-8")
        if c == 0xE8:
            n = self._vint()
            raw, self.p = _unpack7(self.b, self.p, n)
            return raw
        if 0xEC <= c <= 0xEF:
            return self.values[((c & 0x03) << 8) | self._byte()]
        if c == 0xFD:
            return self._take(self._vint())
        if c == 0xF8:
            out = []
            while True:
                if self.b[self.p] == 0xF9:
                    self.p += 1
                    return out
                out.append(self.value())
        if c == 0xFA:
            obj = {}
            while True:
                k = self._byte()
                if k == 0xFB:
                    return obj
                key = self.name(k)
                obj[key] = self.value()
        raise SmileError(f"invalid value token 0x{c:02x}")


def loads(data: bytes) -> Any:
    """Decode one Smile document (header required, as Jackson writes it by default)."""
    data = bytes(data)
    if not is_smile(data) or len(data) < 4:
        raise SmileError("missing Smile header ':)\\n'")
    flags = data[3]
    if flags >> 4:
        raise SmileError(f"unsupported Smile version {flags >> 4}")
    dec = _Decoder(data, bool(flags & F_SHARED_NAMES), bool(flags & F_SHARED_VALUES))
    dec.p = 4
    v = dec.value()
    return v


def decode_body(data: bytes, content_type: Optional[str] = None) -> Any:
    """JSON or Smile request/response body -> Python object."""
    import json

    if (content_type and "smile" in content_type) or is_smile(data):
        return loads(data)
    return json.loads(data.decode("utf-8") if isinstance(data, (bytes, bytearray)) else data)
