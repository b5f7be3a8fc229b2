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

import math
from typing import Any, Callable, Dict, Iterable, Optional, Sequence, Tuple

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
        if k == "words":
            return WordsDictionary(d["vocab"], d["k"], d["n"])
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
        ids = np.asarray(ids, dtype=np.int64) + self.start
        fmt = self.prefix.replace("%", "%%") + f"%0{self.width}d" + self.suffix.replace("%", "%%")
        return np.array([fmt % i for i in ids.tolist()], dtype=object)

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


class WordsDictionary(Dictionary):
    """Lazy dictionary of k-word phrases over a vocabulary (TPC-H ``p_name`` colour names, comment
    text).  Entry i is the i-th of n phrases spread evenly over the V^k word combinations: the
    combination index ``i * step`` written in base V picks the words (most significant first).
    With the vocabulary sorted and all words free of characters below ' ', phrase order == tuple
    order == id order, so the dictionary stays sorted like every Druid dictionary.

    LIKE patterns whose literal pieces contain no space are evaluated structurally
    (``like_mask``): a per-word automaton table over (pieces matched so far, word) -- V x (m+2)
    entries -- is applied column by column to the k word codes of all n entries, instead of
    materializing n strings (20M part names at SF100, 150M order comments)."""

    lazy = True
    _CHUNK = 1 << 22

    def __init__(self, vocab: Sequence[str], k: int, n: int):
        self.vocab = sorted(set(vocab))
        assert all(min(w) > " " for w in self.vocab), "vocabulary words must not contain spaces"
        self.k = int(k)
        self.n = int(n)
        V = len(self.vocab)
        total = V ** self.k
        if total < self.n:
            raise ValueError(f"{V}^{k} phrases cannot hold {n} distinct entries")
        step = max(1, total // max(self.n, 1))
        while step > 1 and math.gcd(step, V) != 1:  # keep the last word cycling through the vocabulary
            step -= 1
        self.step = step
        self.vtype = STRING
        self.has_null = False
        self._index = None
        self._like_cache: Dict[Tuple[str, bool], np.ndarray] = {}

    def __len__(self):
        return self.n

    # -- codes -------------------------------------------------------------------------------
    def codes(self, ids) -> np.ndarray:
        """[len(ids), k] word indices of the given entries."""
        x = np.asarray(ids, dtype=np.int64) * self.step
        V = len(self.vocab)
        out = np.empty((x.shape[0], self.k), dtype=np.int16)
        for j in range(self.k - 1, -1, -1):
            out[:, j] = x % V
            x = x // V
        return out

    def value(self, i):
        return " ".join(self.vocab[c] for c in self.codes([int(i)])[0])

    @property
    def values(self):
        if self.n > 1 << 22:
            raise MemoryError("refusing to materialize a huge lazy dictionary")
        return self.decode(np.arange(self.n))

    def decode(self, ids):
        voc = np.asarray(self.vocab, dtype=object)
        c = self.codes(ids)
        if c.shape[0] == 0:
            return np.empty(0, dtype=object)
        out = voc[c[:, 0]]
        for j in range(1, self.k):
            out = out + " " + voc[c[:, j]]
        return out.astype(object)

    def lookup(self, v):
        if v is None:
            return -1
        ws = str(v).split(" ")
        if len(ws) != self.k:
            return -1
        pos = {w: i for i, w in enumerate(self.vocab)}
        x = 0
        for w in ws:
            if w not in pos:
                return -1
            x = x * len(self.vocab) + pos[w]
        if x % self.step:
            return -1
        i = x // self.step
        return i if i < self.n else -1

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
        vals = self.values
        return np.fromiter((bool(fn(v)) for v in vals), dtype=bool, count=self.n)

    def map_values(self, fn):
        vals = self.values
        out = np.empty(self.n, dtype=object)
        for i, v in enumerate(vals):
            out[i] = fn(v)
        return out

    def all_values(self):
        return self.values

    def to_json(self):
        return {"kind": "words", "vocab": list(self.vocab), "k": self.k, "n": self.n}

    # -- structured LIKE ---------------------------------------------------------------------
    def like_mask(self, pattern: str, escape: str = "\\") -> Optional[np.ndarray]:
        """bool[n]: entries matching the SQL LIKE ``pattern``; None when the pattern is outside the
        structured subset ('_' wildcards, a space inside a literal piece, no '%' at all)."""
        key = (pattern, escape)
        hit = self._like_cache.get(key)
        if hit is not None:
            return hit
        pieces, cur, i = [], [], 0
        while i < len(pattern):
            ch = pattern[i]
            if escape and ch == escape and i + 1 < len(pattern):
                cur.append(pattern[i + 1])
                i += 2
                continue
            if ch == "%":
                pieces.append("".join(cur))
                cur = []
            elif ch == "_":
                return None
            else:
                cur.append(ch)
            i += 1
        pieces.append("".join(cur))
        if len(pieces) < 2:
            return None  # no '%': an equality, handled by lookup()
        a_start, a_end = pieces[0] != "", pieces[-1] != ""
        segs = [p for p in pieces if p != ""]
        if any(" " in s for s in segs):
            return None
        m = len(segs)
        if m == 0:
            out = np.ones(self.n, dtype=bool)
            self._like_cache[key] = out
            return out
        DEAD = m + 1

        def advance(s, w, first, last):
            if s == DEAD:
                return DEAD
            pos = 0
            if first and a_start:
                if not w.startswith(segs[0]):
                    return DEAD
                pos, s = len(segs[0]), 1
            if last and a_end:
                while s < m - 1:
                    p = w.find(segs[s], pos)
                    if p < 0:
                        return DEAD
                    pos, s = p + len(segs[s]), s + 1
                if s == m - 1:
                    ok = w.endswith(segs[-1]) and len(w) - len(segs[-1]) >= pos
                    return m if ok else DEAD
                return DEAD
            limit = m - 1 if a_end else m
            while s < limit:
                p = w.find(segs[s], pos)
                if p < 0:
                    break
                pos, s = p + len(segs[s]), s + 1
            return s

        V = len(self.vocab)
        tables = {}
        for first in (False, True):
            for last in (False, True):
                t = np.empty((m + 2, V), dtype=np.int8)
                for s in range(m + 2):
                    for wi, w in enumerate(self.vocab):
                        t[s, wi] = advance(s, w, first, last)
                tables[(first, last)] = t
        out = np.empty(self.n, dtype=bool)
        for a in range(0, self.n, self._CHUNK):
            c = self.codes(np.arange(a, min(self.n, a + self._CHUNK)))
            st = np.zeros(c.shape[0], dtype=np.int8)
            for j in range(self.k):
                st = tables[(j == 0, j == self.k - 1)][st, c[:, j]]
            out[a:a + c.shape[0]] = st == m
        if len(self._like_cache) > 32:
            self._like_cache.clear()
        self._like_cache[key] = out
        return out
