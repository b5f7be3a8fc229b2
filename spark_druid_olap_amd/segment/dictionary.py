"""Sorted, typed dimension dictionaries.

Druid stores every dimension as dictionary-encoded strings per segment.  Here dictionaries are
*global per datasource* (ids agree across segments and across GPUs, so partial aggregates merge
by position) and *sorted in the natural order of the value type*, so:

* bound / range predicates become id ranges (``searchsorted``),
* arbitrary single-dimension predicates (the reference's JavaScript filters,
  ``asd/ProjectFilterTransfom.scala:406-413``) are evaluated ONCE per dictionary entry
  ("dictionary-domain evaluation") instead of once per row,
* time-format / expression extractions on a dimension become id -> id remap tables.

``FormattedDictionary`` / ``RangeDictionary`` are lazy dictionaries for synthetic
high-cardinality columns (values are generated from the id and are monotone in it), so a
150M-entry o_orderkey dictionary costs no memory.
"""
from __future__ import annotations

from typing import Any, Callable, Iterable, Optional, Sequence, Tuple

import numpy as np

STRING = "string"
LONG = "long"
DOUBLE = "double"


class Dictionary:
    """Materialized sorted dictionary."""

    lazy = False

    def __init__(self, values: Sequence[Any], vtype: str = STRING, has_null: bool = False):
        if vtype == STRING:
            arr = np.asarray(values, dtype=object)
        elif vtype == LONG:
            arr = np.asarray(values, dtype=np.int64)
        else:
            arr = np.asarray(values, dtype=np.float64)
        self.values = arr
        self.vtype = vtype
        self.has_null = has_null  # id 0 is NULL when set (sorts first)
        self._index = None

    # ---------------------------------------------------------------- basics
    def __len__(self) -> int:
        return int(len(self.values)) + (1 if self.has_null else 0)

    @property
    def cardinality(self) -> int:
        return len(self)

    def _off(self) -> int:
        return 1 if self.has_null else 0

    def value(self, i: int):
        if self.has_null:
            if i == 0:
                return None
            i -= 1
        v = self.values[i]
        return v.item() if hasattr(v, "item") else v

    def decode(self, ids: np.ndarray) -> np.ndarray:
        ids = np.asarray(ids, dtype=np.int64)
        if self.has_null:
            out = np.empty(len(ids), dtype=object)
            nz = ids > 0
            out[~nz] = None
            vals = self.values[ids[nz] - 1]
            out[nz] = vals
            return out
        vals = self.values[ids]
        return vals

    def coerce(self, v):
        if v is None:
            return None
        if self.vtype == STRING:
            return str(v)
        if self.vtype == LONG:
            try:
                f = float(v)
            except (TypeError, ValueError):
                return None
            return int(f) if f == int(f) else f
        try:
            return float(v)
        except (TypeError, ValueError):
            return None

    def lookup(self, v) -> int:
        """id of value v, or -1."""
        if v is None:
            return 0 if self.has_null else -1
        v = self.coerce(v)
        if v is None:
            return -1
        if self._index is None and self.vtype == STRING and len(self.values) <= 1 << 22:
            self._index = {s: i for i, s in enumerate(self.values)}
        if self._index is not None:
            i = self._index.get(v, -1)
            return i + self._off() if i >= 0 else -1
        i = int(np.searchsorted(self.values, v))
        if i < len(self.values) and self.values[i] == v:
            return i + self._off()
        return -1

    def id_range(self, lo=None, lo_strict=False, hi=None, hi_strict=False) -> Tuple[int, int]:
        """Half-open id range [a, b) of non-null values within the bounds (natural order)."""
        a, b = 0, len(self.values)
        if lo is not None:
            lo = self.coerce(lo)
            if lo is None:
                return (self._off(), self._off())
            a = int(np.searchsorted(self.values, lo, side="right" if lo_strict else "left"))
        if hi is not None:
            hi = self.coerce(hi)
            if hi is None:
                return (self._off(), self._off())
            b = int(np.searchsorted(self.values, hi, side="left" if hi_strict else "right"))
        if b < a:
            b = a
        return (a + self._off(), b + self._off())

    def eval_mask(self, fn: Callable[[Any], bool]) -> np.ndarray:
        """Dictionary-domain evaluation of a predicate: one call per entry (not per row)."""
        out = np.zeros(len(self), dtype=bool)
        off = self._off()
        if self.has_null:
            try:
                out[0] = bool(fn(None))
            except Exception:
                out[0] = False
        vals = self.values
        for i in range(len(vals)):
            v = vals[i]
            try:
                out[i + off] = bool(fn(v.item() if hasattr(v, "item") else v))
            except Exception:
                out[i + off] = False
        return out

    def map_values(self, fn: Callable[[Any], Any]) -> np.ndarray:
        """Apply fn to every entry (ids order), returns object array."""
        out = np.empty(len(self), dtype=object)
        off = self._off()
        if self.has_null:
            out[0] = fn(None)
        for i, v in enumerate(self.values):
            out[i + off] = fn(v.item() if hasattr(v, "item") else v)
        return out

    def all_values(self) -> np.ndarray:
        if self.has_null:
            out = np.empty(len(self), dtype=object)
            out[0] = None
            out[1:] = self.values
            return out
        return self.values

    def to_json(self) -> dict:
        vals = self.values.tolist()
        return {"kind": "materialized", "vtype": self.vtype, "has_null": self.has_null, "values": vals}

    @staticmethod
    def from_json(d: dict) -> "Dictionary":
        k = d.get("kind", "materialized")
        if k == "formatted":
            return FormattedDictionary(d["prefix"], d["width"], d["n"], d.get("start", 0), d.get("suffix", ""))
        if k == "range":
            return RangeDictionary(d["start"], d["n"])
        return Dictionary(d["values"], d["vtype"], d.get("has_null", False))

    @staticmethod
    def build(values: Iterable[Any], vtype: str = STRING) -> Tuple["Dictionary", np.ndarray]:
        """Sort-unique encode a column: returns (dictionary, int64 ids)."""
        arr = np.asarray(list(values) if not isinstance(values, np.ndarray) else values, dtype=object)
        nulls = np.array([v is None or (isinstance(v, float) and np.isnan(v)) for v in arr], dtype=bool)
        has_null = bool(nulls.any())
        nn = arr[~nulls]
        if vtype == STRING:
            nn = nn.astype(str).astype(object)
            uniq = np.array(sorted(set(nn.tolist())), dtype=object)
        elif vtype == LONG:
            nn = nn.astype(np.int64)
            uniq = np.unique(nn)
        else:
            nn = nn.astype(np.float64)
            uniq = np.unique(nn)
        d = Dictionary(uniq, vtype, has_null)
        ids = np.zeros(len(arr), dtype=np.int64)
        if len(nn):
            pos = np.searchsorted(uniq, nn) if vtype != STRING else np.searchsorted(uniq.astype(str), nn.astype(str))
            ids[~nulls] = pos + (1 if has_null else 0)
        return d, ids


class RangeDictionary(Dictionary):
    """Lazy dictionary of consecutive integers start .. start+n-1 (id = value - start)."""

    lazy = True

    def __init__(self, start: int, n: int):
        self.start = int(start)
        self.n = int(n)
        self.vtype = LONG
        self.has_null = False
        self._index = None

    def __len__(self):
        return self.n

    @property
    def values(self):  # materialize on demand (small n only)
        if self.n > 1 << 24:
            raise MemoryError("refusing to materialize a huge lazy dictionary")
        return np.arange(self.start, self.start + self.n, dtype=np.int64)

    def value(self, i):
        return self.start + int(i)

    def decode(self, ids):
        return np.asarray(ids, dtype=np.int64) + self.start

    def lookup(self, v):
        v = self.coerce(v)
        if v is None or not float(v).is_integer():
            return -1
        i = int(v) - self.start
        return i if 0 <= i < self.n else -1

    def id_range(self, lo=None, lo_strict=False, hi=None, hi_strict=False):
        import math

        a, b = 0, self.n
        if lo is not None:
            lv = float(self.coerce(lo))
            a = (math.floor(lv) + 1 if lo_strict else math.ceil(lv)) - self.start
        if hi is not None:
            hv = float(self.coerce(hi))
            b = (math.ceil(hv) if hi_strict else math.floor(hv) + 1) - self.start
        a = max(0, min(self.n, a))
        b = max(a, min(self.n, b))
        return (a, b)

    def eval_mask(self, fn):
        if self.n > 1 << 22:
            raise MemoryError("dictionary-domain evaluation over a huge lazy dictionary")
        return np.fromiter((bool(fn(self.start + i)) for i in range(self.n)), dtype=bool, count=self.n)

    def map_values(self, fn):
        if self.n > 1 << 22:
            raise MemoryError("dictionary-domain evaluation over a huge lazy dictionary")
        out = np.empty(self.n, dtype=object)
        for i in range(self.n):
            out[i] = fn(self.start + i)
        return out

    def all_values(self):
        return self.values

    def to_json(self):
        return {"kind": "range", "start": self.start, "n": self.n}


class FormattedDictionary(Dictionary):
    """Lazy string dictionary: value(id) = prefix + zero-padded (start+id) + suffix(id).

    Zero padding keeps lexicographic order == id order, so range filters stay id ranges."""

    lazy = True

    def __init__(self, prefix: str, width: int, n: int, start: int = 0, suffix: str = ""):
        self.prefix = prefix
        self.width = int(width)
        self.n = int(n)
        self.start = int(start)
        self.suffix = suffix
        self.vtype = STRING
        self.has_null = False
        self._index = None

    def __len__(self):
        return self.n

    def value(self, i):
        return f"{self.prefix}{self.start + int(i):0{self.width}d}{self.suffix}"

    @property
    def values(self):
        if self.n > 1 << 22:
            raise MemoryError("refusing to materialize a huge lazy dictionary")
        return np.array([self.value(i) for i in range(self.n)], dtype=object)

    def decode(self, ids):
        ids = np.asarray(ids, dtype=np.int64)
        return np.array([self.value(i) for i in ids], dtype=object)

    def lookup(self, v):
        if v is None:
            return -1
        s = str(v)
        if not (s.startswith(self.prefix) and s.endswith(self.suffix)):
            return -1
        core = s[len(self.prefix): len(s) - len(self.suffix) if self.suffix else len(s)]
        if len(core) != self.width or not core.isdigit():
            return -1
        i = int(core) - self.start
        return i if 0 <= i < self.n else -1

    def _pos(self, s: str, side: str) -> int:
        lo, hi = 0, self.n
        while lo < hi:
            mid = (lo + hi) // 2
            v = self.value(mid)
            if v < s or (side == "right" and v == s):
                lo = mid + 1
            else:
                hi = mid
        return lo

    def id_range(self, lo=None, lo_strict=False, hi=None, hi_strict=False):
        a, b = 0, self.n
        if lo is not None:
            a = self._pos(str(lo), "right" if lo_strict else "left")
        if hi is not None:
            b = self._pos(str(hi), "left" if hi_strict else "right")
        return (a, max(a, b))

    def eval_mask(self, fn):
        if self.n > 1 << 22:
            raise MemoryError("dictionary-domain evaluation over a huge lazy dictionary")
        return np.fromiter((bool(fn(self.value(i))) for i in range(self.n)), dtype=bool, count=self.n)

    def map_values(self, fn):
        if self.n > 1 << 22:
            raise MemoryError("dictionary-domain evaluation over a huge lazy dictionary")
        out = np.empty(self.n, dtype=object)
        for i in range(self.n):
            out[i] = fn(self.value(i))
        return out

    def all_values(self):
        return self.values

    def to_json(self):
        return {"kind": "formatted", "prefix": self.prefix, "width": self.width, "n": self.n,
                "start": self.start, "suffix": self.suffix}


def id_dtype_for(card: int) -> str:
    """Narrowest storage type for dictionary ids (bandwidth is the scan's roofline)."""
    if card <= 256:
        return "uint8"
    if card <= 32767:
        return "int16"
    return "int32"
