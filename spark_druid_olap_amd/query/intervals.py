"""ISO-8601 intervals and the folding of time predicates into query intervals.

Behavioural parity with ``sd/QueryIntervals.scala:24-132``: time conditions on the time
dimension are intersected into ONE interval (the empty interval when they do not overlap);
an interval list is what the scan uses for row-range pruning (binary search on ``__time``).
All times are epoch milliseconds (UTC); offsets in ISO strings are honoured.
"""
from __future__ import annotations

import datetime as _dt
import re
from dataclasses import dataclass
from typing import List, Optional, Tuple

EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)
MIN_MS = -(2 ** 62)
MAX_MS = 2 ** 62

_ISO = re.compile(
    r"^(?P<y>[+-]?\d{4,})(?:-(?P<mo>\d{2})(?:-(?P<d>\d{2}))?)?"
    r"(?:[T ](?P<h>\d{2})(?::(?P<mi>\d{2})(?::(?P<s>\d{2})(?:[.,](?P<f>\d{1,9}))?)?)?)?"
    r"\s*(?P<tz>Z|[+-]\d{2}(?::?\d{2})?)?$"
)


def parse_iso_ms(s: str, default_tz_ms: int = 0) -> int:
    s = s.strip()
    m = _ISO.match(s)
    if not m:
        raise ValueError(f"bad ISO timestamp: {s!r}")
    y = int(m.group("y"))
    mo = int(m.group("mo") or 1)
    d = int(m.group("d") or 1)
    h = int(m.group("h") or 0)
    mi = int(m.group("mi") or 0)
    sec = int(m.group("s") or 0)
    frac = m.group("f") or "0"
    ms = int((frac + "000")[:3])
    tz = m.group("tz")
    if tz is None:
        off = default_tz_ms
    elif tz == "Z":
        off = 0
    else:
        sign = -1 if tz[0] == "-" else 1
        t = tz[1:].replace(":", "")
        off = sign * (int(t[:2]) * 3600 + (int(t[2:4]) if len(t) > 2 else 0) * 60) * 1000
    days = days_from_civil(y, mo, d)
    return ((days * 24 + h) * 60 + mi) * 60_000 + sec * 1000 + ms - off


def days_from_civil(y: int, m: int, d: int) -> int:
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    doy = (153 * (m + (-3 if m > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def civil_from_days(z: int) -> Tuple[int, int, int]:
    z += 719468
    era = (z if z >= 0 else z - 146096) // 146097
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = mp + 3 if mp < 10 else mp - 9
    return (y + (m <= 2), m, d)


def fmt_iso(ms: int) -> str:
    days, rem = divmod(ms, 86_400_000)
    y, m, d = civil_from_days(days)
    h, rem = divmod(rem, 3_600_000)
    mi, rem = divmod(rem, 60_000)
    s, msr = divmod(rem, 1000)
    return f"{y:04d}-{m:02d}-{d:02d}T{h:02d}:{mi:02d}:{s:02d}.{msr:03d}Z"


def date_to_ms(s: str) -> int:
    return parse_iso_ms(s)


@dataclass(frozen=True)
class Interval:
    lo: int  # inclusive ms
    hi: int  # exclusive ms

    @property
    def empty(self) -> bool:
        return self.hi <= self.lo

    def intersect(self, o: "Interval") -> "Interval":
        return Interval(max(self.lo, o.lo), min(self.hi, o.hi))

    def overlaps(self, o: "Interval") -> bool:
        return max(self.lo, o.lo) < min(self.hi, o.hi)

    def to_iso(self) -> str:
        return f"{fmt_iso(self.lo)}/{fmt_iso(self.hi)}"

    @staticmethod
    def parse(s: str) -> "Interval":
        a, b = s.split("/")
        return Interval(parse_iso_ms(a), parse_iso_ms(b))

    @staticmethod
    def eternity() -> "Interval":
        return Interval(MIN_MS, MAX_MS)


class QueryIntervals:
    """Accumulates time conditions into a single interval (reference QueryIntervals.add)."""

    def __init__(self, index_interval: Interval):
        self.index_interval = index_interval
        self.current: Optional[Interval] = None

    def _add(self, i: Interval) -> "QueryIntervals":
        self.current = i if self.current is None else self.current.intersect(i)
        return self

    def gt(self, ms: int):
        return self._add(Interval(ms + 1, self.index_interval.hi))

    def gte(self, ms: int):
        return self._add(Interval(ms, self.index_interval.hi))

    def lt(self, ms: int):
        return self._add(Interval(self.index_interval.lo, ms))

    def lte(self, ms: int):
        return self._add(Interval(self.index_interval.lo, ms + 1))

    def eq(self, ms: int):
        return self._add(Interval(ms, ms + 1))

    def intervals(self) -> List[Interval]:
        i = self.current if self.current is not None else self.index_interval
        return [i if not i.empty else Interval(i.lo, i.lo)]
