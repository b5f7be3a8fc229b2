"""Druid query / segment granularities (reference ``sd/DruidQueryGranularity.scala:29-126``).

Each granularity knows how to bucket epoch-ms on the host (for result formatting and segment
boundaries) and how to lower itself into a kernel time-key component (``TField`` in
ops/csrc/scan_desc.h), where the bucket is computed in registers with civil-from-days math.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Optional, Union

from .intervals import civil_from_days, days_from_civil, parse_iso_ms

# TField codes (scan_desc.h)
T_MS, T_SECOND, T_MINUTE, T_HOUR, T_DAY, T_WEEK, T_MONTH, T_QUARTER, T_YEAR = range(9)
T_MOY, T_DOM, T_DOW, T_HOD, T_MOH, T_DOY, T_SOM, T_QOY, T_PERIOD = range(9, 18)

SIMPLE = {
    "none": (T_MS, 1), "second": (T_SECOND, 1000), "minute": (T_MINUTE, 60_000),
    "fifteen_minute": (T_PERIOD, 900_000), "thirty_minute": (T_PERIOD, 1_800_000),
    "hour": (T_HOUR, 3_600_000), "day": (T_DAY, 86_400_000), "week": (T_WEEK, 7 * 86_400_000),
    "month": (T_MONTH, None), "quarter": (T_QUARTER, None), "year": (T_YEAR, None),
}


def bucket_value(ms: int, tfield: int, period_ms: int = 0, origin_ms: int = 0) -> int:
    """Python mirror of the kernel's time_field() (absolute buckets and field extracts)."""
    if tfield == T_MS:
        return ms
    if tfield == T_SECOND:
        return ms // 1000
    if tfield == T_MINUTE:
        return ms // 60_000
    if tfield == T_HOUR:
        return ms // 3_600_000
    if tfield == T_DAY:
        return ms // 86_400_000
    if tfield == T_WEEK:
        return (ms // 86_400_000 + 3) // 7
    if tfield == T_PERIOD:
        return (ms - origin_ms) // period_ms
    if tfield == T_HOD:
        return (ms // 3_600_000) % 24
    if tfield == T_MOH:
        return (ms // 60_000) % 60
    if tfield == T_SOM:
        return (ms // 1000) % 60
    days = ms // 86_400_000
    if tfield == T_DOW:
        return (days + 3) % 7 + 1
    y, m, d = civil_from_days(days)
    if tfield == T_MONTH:
        return y * 12 + (m - 1)
    if tfield == T_QUARTER:
        return y * 4 + (m - 1) // 3
    if tfield == T_YEAR:
        return y
    if tfield == T_MOY:
        return m
    if tfield == T_DOM:
        return d
    if tfield == T_QOY:
        return (m - 1) // 3 + 1
    if tfield == T_DOY:
        return days - days_from_civil(y, 1, 1) + 1
    raise ValueError(tfield)


def bucket_start_from_value(v: int, tfield: int, period_ms: int = 0, origin_ms: int = 0) -> int:
    """Start (ms) of an absolute bucket value."""
    if tfield == T_MS:
        return v
    if tfield == T_SECOND:
        return v * 1000
    if tfield == T_MINUTE:
        return v * 60_000
    if tfield == T_HOUR:
        return v * 3_600_000
    if tfield == T_DAY:
        return v * 86_400_000
    if tfield == T_WEEK:
        return (v * 7 - 3) * 86_400_000
    if tfield == T_PERIOD:
        return origin_ms + v * period_ms
    if tfield == T_MONTH:
        return days_from_civil(v // 12, v % 12 + 1, 1) * 86_400_000
    if tfield == T_QUARTER:
        return days_from_civil(v // 4, (v % 4) * 3 + 1, 1) * 86_400_000
    if tfield == T_YEAR:
        return days_from_civil(v, 1, 1) * 86_400_000
    raise ValueError(f"not an absolute bucket: {tfield}")


_PERIOD = re.compile(r"^P(?:(\d+)Y)?(?:(\d+)M)?(?:(\d+)W)?(?:(\d+)D)?(?:T(?:(\d+)H)?(?:(\d+)M)?(?:(\d+)S)?)?$")


@dataclass(frozen=True)
class Granularity:
    """name in SIMPLE, or 'duration'/'period' with period_ms (fixed-length only)."""
    name: str = "all"
    period_ms: int = 0
    origin_ms: int = 0
    tz_ms: int = 0
    calendar: Optional[str] = None  # for period P1M / P3M / P1Y: month/quarter/year

    @property
    def is_all(self) -> bool:
        return self.name == "all"

    def kernel_field(self):
        """(tfield, period_ms, origin_ms)"""
        if self.name in ("duration", "period"):
            if self.calendar:
                return (SIMPLE[self.calendar][0], 0, 0)
            return (T_PERIOD, self.period_ms, self.origin_ms)
        tf, p = SIMPLE[self.name]
        if tf == T_PERIOD:
            return (T_PERIOD, p, 0)
        return (tf, 0, 0)

    def bucket_start(self, ms: int) -> int:
        tf, p, o = self.kernel_field()
        return bucket_start_from_value(bucket_value(ms + self.tz_ms, tf, p, o), tf, p, o) - self.tz_ms

    def to_json(self):
        if self.name in SIMPLE or self.name == "all":
            return self.name
        if self.name == "duration":
            return {"type": "duration", "duration": self.period_ms, "origin": self.origin_ms}
        d = {"type": "period", "period": self._period_str()}
        return d

    def _period_str(self) -> str:
        if self.calendar == "month":
            return "P1M"
        if self.calendar == "quarter":
            return "P3M"
        if self.calendar == "year":
            return "P1Y"
        ms = self.period_ms
        if ms % 86_400_000 == 0:
            return f"P{ms // 86_400_000}D"
        return f"PT{ms // 1000}S"

    @staticmethod
    def parse(g: Union[str, dict, None]) -> "Granularity":
        if g is None:
            return Granularity("all")
        if isinstance(g, str):
            n = g.lower()
            if n == "all" or n in SIMPLE:
                return Granularity(n)
            raise ValueError(f"unknown granularity {g!r}")
        t = g.get("type")
        if t == "duration":
            origin = g.get("origin", 0)
            if isinstance(origin, str):
                origin = parse_iso_ms(origin)
            return Granularity("duration", int(g["duration"]), int(origin or 0))
        if t == "period":
            p = g["period"]
            m = _PERIOD.match(p)
            if not m:
                raise ValueError(f"bad period {p!r}")
            yy, mm, ww, dd, hh, mi, ss = (int(x) if x else 0 for x in m.groups())
            origin = g.get("origin", 0)
            if isinstance(origin, str):
                origin = parse_iso_ms(origin)
            if yy == 1 and not any((mm, ww, dd, hh, mi, ss)):
                return Granularity("period", 0, 0, calendar="year")
            if mm in (1, 3) and not any((yy, ww, dd, hh, mi, ss)):
                return Granularity("period", 0, 0, calendar="month" if mm == 1 else "quarter")
            if yy or mm:
                raise ValueError(f"unsupported calendar period {p!r}")
            ms = ((((ww * 7 + dd) * 24 + hh) * 60 + mi) * 60 + ss) * 1000
            return Granularity("period", ms, int(origin or 0))
        raise ValueError(f"unknown granularity spec {g!r}")


def bucket_start_ms(ms: int, name: str) -> int:
    return Granularity.parse(name).bucket_start(ms)


def next_bucket_ms(start_ms: int, name: str) -> int:
    g = Granularity.parse(name)
    tf, p, o = g.kernel_field()
    v = bucket_value(start_ms, tf, p, o)
    return bucket_start_from_value(v + 1, tf, p, o)
