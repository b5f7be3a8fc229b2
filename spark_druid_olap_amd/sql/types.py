"""SQL types and their columnar (pandas) representation.

Column values on the host are pandas Series with nullable dtypes so that SQL three-valued logic and
null propagation come from pandas:

  int/bigint/smallint/tinyint -> Int64      double/float/decimal -> Float64
  string -> string (pd.StringDtype)          boolean -> boolean (Kleene logic)
  date/timestamp -> datetime64[ns] (NaT)     (sparkline ``dateTime`` values are timestamps)

Scalars (literals, constant-folded values) are plain Python values with ``None`` as NULL.
"""
from __future__ import annotations

import datetime as _dt
import math
import re
from typing import Any, Optional

import numpy as np
import pandas as pd

INTEGRAL = ("tinyint", "smallint", "int", "bigint")
FRACTIONAL = ("float", "double")
NUMERIC_ORDER = ["tinyint", "smallint", "int", "bigint", "decimal", "float", "double"]


class AnalysisError(ValueError):
    pass


def base(t: str) -> str:
    return "decimal" if t.startswith("decimal") else t


def is_numeric(t: str) -> bool:
    return base(t) in NUMERIC_ORDER or t == "null"


def is_integral(t: str) -> bool:
    return t in INTEGRAL


def is_datetime(t: str) -> bool:
    return t in ("date", "timestamp")


def wider(a: str, b: str) -> str:
    """Common type for arithmetic / comparison / union (Spark's TypeCoercion, simplified)."""
    if a == b:
        return a
    if a == "null":
        return b
    if b == "null":
        return a
    ba, bb = base(a), base(b)
    if ba in NUMERIC_ORDER and bb in NUMERIC_ORDER:
        w = max(ba, bb, key=NUMERIC_ORDER.index)
        if w == "decimal":
            return "double" if (ba in FRACTIONAL or bb in FRACTIONAL) else (a if ba == "decimal" else b)
        return w
    if {ba, bb} == {"date", "timestamp"}:
        return "timestamp"
    if "string" in (ba, bb):
        other = bb if ba == "string" else ba
        if other in NUMERIC_ORDER:
            return "double"
        if other in ("date", "timestamp"):
            return other
        return "string"
    if ba == "boolean" or bb == "boolean":
        return "boolean" if ba == bb else "string"
    return "string"


def pandas_dtype(t: str):
    bt = base(t)
    if bt in INTEGRAL:
        return "Int64"
    if bt in FRACTIONAL or bt == "decimal":
        return "Float64"
    if bt == "boolean":
        return "boolean"
    if bt in ("date", "timestamp"):
        return "datetime64[ns]"
    if bt == "null":
        return "object"
    return "string"


EPOCH = pd.Timestamp("1970-01-01")


# ------------------------------------------------------------------------------------------------
# scalar helpers
_TZ_SUFFIX = re.compile(r"(Z|[+-]\d{2}:?\d{2})$")


def _parse_date(s: str):
    """ISO-ish date/timestamp string -> naive UTC pd.Timestamp (offsets are applied, like Spark with
    the session time zone set to UTC); unparseable -> None."""
    s = s.strip()
    try:
        if len(s) == 10 and s[4] == "-":
            return pd.Timestamp(s)
        if _TZ_SUFFIX.search(s):
            t = pd.Timestamp(s)
            return t.tz_convert("UTC").tz_localize(None) if t.tzinfo is not None else t
        parts = s.split()
        if len(parts) == 3 and re.match(r"^[A-Z]{2,5}$", parts[2]):
            s = parts[0] + " " + parts[1]  # trailing zone abbreviation (e.g. PST): ignored
        return pd.Timestamp(s.replace("T", " ")[:26])
    except (ValueError, TypeError):
        return None


def scalar_cast(v: Any, frm: str, to: str) -> Any:
    if v is None:
        return None
    bt = base(to)
    try:
        if bt in INTEGRAL:
            if isinstance(v, str):
                v = v.strip()
                if not v or not _is_number(v):
                    return None
                return int(float(v)) if any(c in v for c in ".eE") else int(v)
            if isinstance(v, (pd.Timestamp, _dt.datetime)):
                return int(pd.Timestamp(v).value // 10 ** 9)
            if isinstance(v, float):
                if math.isnan(v) or math.isinf(v):
                    return None
                return int(v)
            return int(v)
        if bt in FRACTIONAL or bt == "decimal":
            if isinstance(v, str):
                v = v.strip()
                return float(v) if _is_number(v) else None
            if isinstance(v, (pd.Timestamp, _dt.datetime)):
                return pd.Timestamp(v).value / 1e9
            f = float(v)
            if bt == "decimal":
                sc = _dec_scale(to)
                f = round(f, sc)
            return f
        if bt == "string":
            return format_value(v, frm)
        if bt == "boolean":
            if isinstance(v, str):
                s = v.strip().lower()
                return True if s in ("true", "t", "1", "yes", "y") else False if s in ("false", "f", "0", "no", "n") else None
            return bool(v)
        if bt == "date":
            ts = _parse_date(v) if isinstance(v, str) else pd.Timestamp(v)
            return None if ts is None or ts is pd.NaT else ts.normalize()
        if bt == "timestamp":
            if isinstance(v, str):
                return _parse_date(v)
            if isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool):
                return pd.Timestamp(int(v * 10 ** 9))
            return pd.Timestamp(v)
    except (ValueError, TypeError, OverflowError):
        return None
    return v


def _is_number(s: str) -> bool:
    try:
        float(s)
        return True
    except ValueError:
        return False


def _dec_scale(t: str) -> int:
    if "(" in t:
        parts = t[t.index("(") + 1:-1].split(",")
        return int(parts[1]) if len(parts) > 1 else 0
    return 0


def format_value(v: Any, t: str) -> Optional[str]:
    """Spark's cast-to-string of a value of type t."""
    if v is None or (isinstance(v, float) and math.isnan(v)) or v is pd.NaT:
        return None
    bt = base(t)
    if bt == "date":
        return pd.Timestamp(v).strftime("%Y-%m-%d")
    if bt == "timestamp":
        ts = pd.Timestamp(v)
        s = ts.strftime("%Y-%m-%d %H:%M:%S")
        if ts.microsecond:
            s += ("." + f"{ts.microsecond:06d}").rstrip("0")
        return s
    if bt == "boolean":
        return "true" if v else "false"
    if isinstance(v, (bytes, bytearray)):
        return bytes(v).decode("utf-8", errors="replace")
    if isinstance(v, float):
        if v == int(v) and abs(v) < 1e7:
            return f"{v:.1f}"
        return repr(v)
    return str(v)


# ------------------------------------------------------------------------------------------------
# vector helpers
def is_vec(x) -> bool:
    return isinstance(x, pd.Series)


def broadcast(x, n: int, t: str) -> pd.Series:
    if is_vec(x):
        return x
    return pd.Series([x] * n, dtype=pandas_dtype(t)) if x is not None else pd.Series([None] * n, dtype=pandas_dtype(t))


def fast_series(arr) -> pd.Series:
    """``pd.Series(arr)`` for a numpy array or pandas ExtensionArray without pandas' input
    sanitising (about half the construction cost; result columns of small queries are built many
    times per second).  Falls back to the public constructor if the internal API moves."""
    try:
        n = len(arr)
        idx = _RANGES.get(n)
        if idx is None:
            idx = pd.RangeIndex(n)
            if n <= 4096:  # immutable, shared by every small result column of that length
                if len(_RANGES) > 256:
                    _RANGES.clear()
                _RANGES[n] = idx
        mgr = _SBM.from_array(arr, idx)
        out = pd.Series._from_mgr(mgr, mgr.axes)
        out._name = None
        return out
    except Exception:  # pragma: no cover - pandas internals changed
        return pd.Series(arr)


_RANGES: dict = {}

try:
    from pandas.core.internals import SingleBlockManager as _SBM
except ImportError:  # pragma: no cover
    _SBM = None


def to_series(values, t: str) -> pd.Series:
    """Build a typed Series from raw values (numpy / list / Series)."""
    pdt = pandas_dtype(t)
    if isinstance(values, pd.Series):
        s = values.reset_index(drop=True)
    else:
        s = pd.Series(values)
    if pdt == "datetime64[ns]":
        if s.dtype.kind == "M":
            out = s.astype("datetime64[ns]")
        elif s.dtype == object or str(s.dtype) == "string":
            out = pd.to_datetime(s.astype("string").str.replace("Z", "", regex=False), errors="coerce",
                                 format="mixed" if _pd2() else None)
        else:
            out = pd.to_datetime(s, errors="coerce")
        return out.dt.normalize() if base(t) == "date" else out
    if pdt == "string":
        if s.dtype == object or str(s.dtype) == "string":
            return s.astype("string")
        if s.dtype.kind == "f":
            return pd.Series([format_value(None if (v is None or v != v) else float(v), "double") for v in s],
                             dtype="string")
        if s.dtype.kind == "M":
            return pd.Series([format_value(v, "timestamp" if base(t) != "date" else "date") if v is not pd.NaT else None
                              for v in s], dtype="string")
        if s.dtype.kind == "b" or str(s.dtype) == "boolean":
            return s.map(lambda v: None if v is None or v is pd.NA else ("true" if v else "false")).astype("string")
        return s.astype("string")
    if pdt == "Int64":
        if s.dtype == object:
            try:
                return pd.Series(pd.array(s.to_numpy(), dtype="Int64"))
            except (TypeError, ValueError):
                return _str_to_int(s)
        if str(s.dtype) == "string":
            return _str_to_int(s)
        if s.dtype.kind == "f" or str(s.dtype) == "Float64":
            return _float_to_int(s.astype("Float64").to_numpy(dtype="float64", na_value=np.nan))
        if s.dtype.kind == "M":
            return (s.astype("int64") // 10 ** 9).astype("Int64")
        return s.astype("Int64")
    if pdt == "Float64":
        if s.dtype == object:
            try:
                return pd.Series(pd.array(s.to_numpy(), dtype="Float64"))
            except (TypeError, ValueError):
                pass
        if s.dtype == object or str(s.dtype) == "string":
            return pd.to_numeric(s.astype("string"), errors="coerce").astype("Float64")
        if s.dtype.kind == "M":
            return (s.astype("int64") / 1e9).astype("Float64")
        out = s.astype("Float64")
        if base(t) == "decimal":
            out = out.round(_dec_scale(t))
        return out
    if pdt == "boolean":
        if s.dtype == object or str(s.dtype) == "string":
            m = {"true": True, "t": True, "1": True, "false": False, "f": False, "0": False}
            return s.map(lambda v: m.get(str(v).strip().lower()) if v is not None and v is not pd.NA else None
                         ).astype("boolean")
        return s.astype("boolean")
    return s


def _pd2() -> bool:
    return int(pd.__version__.split(".")[0]) >= 2


def _str_to_int(s: pd.Series) -> pd.Series:
    f = pd.to_numeric(s.astype("string").str.strip(), errors="coerce")
    return _float_to_int(pd.Series(f).astype("Float64").to_numpy(dtype="float64", na_value=np.nan))


def _float_to_int(f: pd.Series) -> pd.Series:
    arr = np.asarray(f, dtype=np.float64)
    ok = np.isfinite(arr)
    out = np.zeros(len(arr), dtype=np.int64)
    out[ok] = np.trunc(arr[ok]).astype(np.int64)
    return pd.Series(pd.arrays.IntegerArray(out, ~ok))


def cast_vec(x, frm: str, to: str, n: int):
    if not is_vec(x):
        return scalar_cast(x, frm, to)
    if base(frm) == base(to) and base(to) != "decimal":
        return x
    bt = base(to)
    if bt == "date" and base(frm) == "timestamp":
        return x.dt.normalize()
    if bt == "string" and base(frm) in ("date", "timestamp"):
        fmt = "%Y-%m-%d" if base(frm) == "date" else "%Y-%m-%d %H:%M:%S"
        return x.dt.strftime(fmt).astype("string")
    if bt in INTEGRAL and base(frm) == "boolean":
        return x.astype("Int64")
    if bt == "string" and base(frm) == "binary":
        return pd.Series([None if v is None or v is pd.NA else format_value(v, "binary") for v in x],
                         dtype="string")
    return to_series(x, to)


def to_python(v: Any):
    if v is None or v is pd.NA or v is pd.NaT:
        return None
    if isinstance(v, float) and math.isnan(v):
        return None
    if isinstance(v, np.generic):
        return v.item()
    return v


def series_to_list(s: pd.Series, t: str) -> list:
    bt = base(t)
    if bt == "date":
        return [None if v is pd.NaT or v is None else pd.Timestamp(v).date() for v in s]
    if bt == "timestamp":
        return [None if v is pd.NaT or v is None else pd.Timestamp(v).to_pydatetime() for v in s]
    return [to_python(v) for v in s.tolist()]
