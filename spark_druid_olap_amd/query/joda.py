"""Joda-time format patterns (the reference's time extraction / parsing vocabulary,
``sd/DateTimeExtractor.scala:159-176, 358-372`` and Druid ``timeFormat`` / ``time`` extraction
functions) -- formatting epoch-ms, parsing strings, and mapping a pattern to the kernel's
time-bucket field.
"""
from __future__ import annotations

import re
from functools import lru_cache
from typing import List, Optional, Tuple

from .granularity import (T_DAY, T_DOM, T_DOW, T_DOY, T_HOD, T_HOUR, T_MINUTE, T_MOH, T_MONTH, T_MOY, T_MS,
                          T_QOY, T_SECOND, T_SOM, T_WEEK, T_YEAR, bucket_start_from_value)
from .intervals import civil_from_days, days_from_civil

MONTHS = ["January", "February", "March", "April", "May", "June", "July", "August", "September", "October",
          "November", "December"]
DAYS = ["Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday", "Sunday"]


@lru_cache(maxsize=256)
def tokenize(fmt: str) -> Tuple[Tuple[str, str], ...]:
    """[(kind, text)] kind in {'lit', 'field'}; field text is a run of one pattern letter."""
    out: List[Tuple[str, str]] = []
    i = 0
    while i < len(fmt):
        c = fmt[i]
        if c == "'":
            j = fmt.find("'", i + 1)
            if j == -1:
                j = len(fmt)
            lit = fmt[i + 1:j]
            out.append(("lit", "'" if lit == "" else lit))
            i = j + 1
        elif c.isalpha():
            j = i
            while j < len(fmt) and fmt[j] == c:
                j += 1
            out.append(("field", fmt[i:j]))
            i = j
        else:
            out.append(("lit", c))
            i += 1
    return tuple(out)


def _fields(ms: int):
    days, rem = divmod(ms, 86_400_000)
    y, m, d = civil_from_days(days)
    h, rem = divmod(rem, 3_600_000)
    mi, rem = divmod(rem, 60_000)
    s, msr = divmod(rem, 1000)
    dow = (days + 3) % 7 + 1
    doy = days - days_from_civil(y, 1, 1) + 1
    return y, m, d, h, mi, s, msr, dow, doy, days


def iso_week(days: int) -> Tuple[int, int]:
    y, m, d = civil_from_days(days)
    dow = (days + 3) % 7 + 1
    thursday = days - dow + 4
    ty, _, _ = civil_from_days(thursday)
    jan1 = days_from_civil(ty, 1, 1)
    return ty, (thursday - jan1) // 7 + 1


def format_ms(fmt: str, ms: int, tz_ms: int = 0) -> str:
    ms += tz_ms
    y, m, d, h, mi, s, msr, dow, doy, days = _fields(ms)
    out = []
    for kind, t in tokenize(fmt):
        if kind == "lit":
            out.append(t)
            continue
        c, n = t[0], len(t)
        if c in "yY":
            out.append(f"{y % 100:02d}" if n == 2 else f"{y:0{max(n, 4)}d}")
        elif c == "x":
            out.append(f"{iso_week(days)[0]:04d}")
        elif c == "M":
            out.append(MONTHS[m - 1] if n >= 4 else MONTHS[m - 1][:3] if n == 3 else f"{m:0{n}d}")
        elif c == "d":
            out.append(f"{d:0{n}d}")
        elif c == "D":
            out.append(f"{doy:0{n}d}")
        elif c == "E":
            out.append(DAYS[dow - 1] if n >= 4 else DAYS[dow - 1][:3])
        elif c == "e":
            out.append(f"{dow:0{n}d}")
        elif c == "w":
            out.append(f"{iso_week(days)[1]:0{n}d}")
        elif c == "H":
            out.append(f"{h:0{n}d}")
        elif c == "k":
            out.append(f"{h if h else 24:0{n}d}")
        elif c in "hK":
            hh = h % 12
            if c == "h" and hh == 0:
                hh = 12
            out.append(f"{hh:0{n}d}")
        elif c == "a":
            out.append("AM" if h < 12 else "PM")
        elif c == "m":
            out.append(f"{mi:0{n}d}")
        elif c == "s":
            out.append(f"{s:0{n}d}")
        elif c == "S":
            out.append(f"{msr:03d}"[:n] if n <= 3 else f"{msr:03d}" + "0" * (n - 3))
        elif c == "Z":
            out.append("Z" if tz_ms == 0 else ("+" if tz_ms >= 0 else "-") + f"{abs(tz_ms) // 3_600_000:02d}"
                       + (":" if n >= 2 else "") + f"{abs(tz_ms) // 60_000 % 60:02d}")
        elif c == "G":
            out.append("AD")
        else:
            out.append(t)
    return "".join(out)


@lru_cache(maxsize=256)
def _parse_regex(fmt: str):
    parts, names = [], []
    for kind, t in tokenize(fmt):
        if kind == "lit":
            parts.append(re.escape(t))
            continue
        c, n = t[0], len(t)
        if c in "yYx":
            parts.append(r"([+-]?\d{1,9})")
        elif c == "M" and n >= 3:
            parts.append(r"([A-Za-z]+)")
        elif c == "E":
            parts.append(r"([A-Za-z]+)")
        elif c == "a":
            parts.append(r"([AaPp][Mm])")
        elif c == "S":
            parts.append(r"(\d{1,9})")
        elif c == "Z":
            parts.append(r"(Z|[+-]\d{2}:?\d{2})")
        else:
            parts.append(r"(\d{1,%d})" % max(n, 2) if n <= 2 else r"(\d{%d})" % n)
        names.append(t)
    return re.compile("^" + "".join(parts) + "$"), names


def parse(fmt: str, s: str, tz_ms: int = 0) -> Optional[int]:
    """Parse s with a Joda pattern into epoch ms (None when it does not match)."""
    if s is None:
        return None
    rx, names = _parse_regex(fmt)
    m = rx.match(str(s).strip())
    if not m:
        return None
    y, mo, d, h, mi, sec, msr, pm, off = 1970, 1, 1, 0, 0, 0, 0, None, None
    for t, v in zip(names, m.groups()):
        c = t[0]
        if c in "yYx":
            y = int(v)
            if len(t) == 2 and abs(y) < 100:
                y += 2000 if y < 50 else 1900
        elif c == "M":
            mo = int(v) if v.isdigit() else [x[:3].lower() for x in MONTHS].index(v[:3].lower()) + 1
        elif c == "d":
            d = int(v)
        elif c in "Hk":
            h = int(v) % 24
        elif c in "hK":
            h = int(v) % 12
        elif c == "a":
            pm = v.lower() == "pm"
        elif c == "m":
            mi = int(v)
        elif c == "s":
            sec = int(v)
        elif c == "S":
            msr = int((v + "000")[:3])
        elif c == "Z":
            if v == "Z":
                off = 0
            else:
                sign = -1 if v[0] == "-" else 1
                vv = v[1:].replace(":", "")
                off = sign * (int(vv[:2]) * 60 + int(vv[2:4])) * 60_000
    if pm is not None and pm:
        h += 12
    ms = ((days_from_civil(y, mo, d) * 24 + h) * 60 + mi) * 60_000 + sec * 1000 + msr
    return ms - (off if off is not None else tz_ms)


_EXACT = {
    "yyyy": T_YEAR, "YYYY": T_YEAR, "yyyy-MM": T_MONTH, "yyyy-MM-dd": T_DAY, "YYYY-MM-dd": T_DAY,
    "MM": T_MOY, "M": T_MOY, "MMM": T_MOY, "MMMM": T_MOY, "dd": T_DOM, "d": T_DOM, "EEEE": T_DOW, "EEE": T_DOW,
    "E": T_DOW, "e": T_DOW, "HH": T_HOD, "H": T_HOD, "mm": T_MOH, "ss": T_SOM, "D": T_DOY, "DDD": T_DOY,
    "yyyy-MM-dd HH": T_HOUR, "yyyy-MM-dd'T'HH": T_HOUR, "yyyy-MM-dd HH:mm": T_MINUTE,
    "yyyy-MM-dd HH:mm:ss": T_SECOND, "yyyy-MM-dd'T'HH:mm:ss": T_SECOND,
}

ABSOLUTE = {T_MS, T_SECOND, T_MINUTE, T_HOUR, T_DAY, T_WEEK, T_MONTH, T_YEAR}


def format_to_field(fmt: str) -> Tuple[int, bool]:
    """(tfield, exact): exact means format(bucket) is injective over the bucket field."""
    if fmt in _EXACT:
        return _EXACT[fmt], True
    letters = {t[0] for k, t in tokenize(fmt) if k == "field"}
    for c, tf in (("S", T_MS), ("s", T_SECOND), ("m", T_MINUTE), ("H", T_HOUR), ("h", T_HOUR), ("k", T_HOUR),
                  ("K", T_HOUR), ("a", T_HOUR), ("d", T_DAY), ("D", T_DAY), ("E", T_DAY), ("e", T_DAY),
                  ("w", T_WEEK), ("M", T_MONTH), ("y", T_YEAR), ("Y", T_YEAR), ("x", T_YEAR)):
        if c in letters:
            return tf, False
    return T_DAY, False


def representative_ms(tfield: int, v: int) -> int:
    """An instant whose field value is v (for formatting field-extract buckets)."""
    if tfield in ABSOLUTE:
        return bucket_start_from_value(v, tfield)
    if tfield == T_MOY:
        return days_from_civil(2001, v, 1) * 86_400_000
    if tfield == T_QOY:
        return days_from_civil(2001, (v - 1) * 3 + 1, 1) * 86_400_000
    if tfield == T_DOM:
        return days_from_civil(2001, 1, v) * 86_400_000
    if tfield == T_DOW:
        return (days_from_civil(2001, 1, 1) + (v - 1)) * 86_400_000  # 2001-01-01 was a Monday
    if tfield == T_DOY:
        return (days_from_civil(2001, 1, 1) + v - 1) * 86_400_000
    if tfield == T_HOD:
        return v * 3_600_000
    if tfield == T_MOH:
        return v * 60_000
    if tfield == T_SOM:
        return v * 1000
    raise ValueError(tfield)


def field_domain(tfield: int) -> Tuple[int, int]:
    """(min, max) of a field-extract."""
    return {T_MOY: (1, 12), T_QOY: (1, 4), T_DOM: (1, 31), T_DOW: (1, 7), T_DOY: (1, 366), T_HOD: (0, 23),
            T_MOH: (0, 59), T_SOM: (0, 59)}[tfield]
