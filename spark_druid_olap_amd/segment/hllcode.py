"""HLL code columns: the per-row (bucket, rho) of a dimension's HyperLogLog update, precomputed.

A query-time ``cardinality`` / ``hyperUnique`` aggregator over a dimension (the reference's
TpchBenchMark Q1 / Basic Aggregation count distinct ``o_orderkey``,
``/root/reference/src/main/scala/org/sparklinedata/druid/tools/TpchBenchMark.scala:137-160``;
Druid's CardinalityAggregator hashes each row's value) costs the scan kernel a 4-byte id read, a
32-bit mix and a register update per row.  The (bucket, rho) pair depends only on the row's id, the
column's salt and the precision p, so it is computed once per (column, p) and kept resident next to
the column as a u16 ``bucket << 5 | rho`` plane: the scan reads half the bytes of an int32 id and
does no hashing (TPC-H Q1's HLL-only part 1.23 -> see profiles/r3).  Like the bit-packed copies
(``segment/packed.py``) it is an encoding of an input column, built on first use and cached on the
datasource -- never a cached result: every query still updates its registers from the rows it
selects.

Exactness: for ids in [0, 2^32) (every dictionary id) ``hll_bucket_rho`` takes the 32-bit mix whose
rho is at most 33 - p; with p <= 11 the code fits 16 bits.  The plane is bit-identical to what the
kernels compute per row (``ops/reference.py:hll_update_values``), so registers -- and the estimates
and cross-GPU merges built from them -- do not change."""
from __future__ import annotations

from typing import Optional

import torch

ENABLED = True
MAX_P = 11            # bucket (p bits) + rho (5 bits) in 16
MIN_ID_BYTES = 2      # byte-wide dimensions read no fewer bytes through a u16 plane
CHUNK = 1 << 24       # rows per build step (bounded int64 temporaries)
# total bytes of code planes per datasource (HBM is 288 GB; SF100's o_orderkey plane is 1.2 GB)
MAX_BYTES = 16 << 30


def code_name(col: str, p: int, salt: int) -> str:
    return f"{col}#hll{p}.{salt:x}"


def codes(vals: torch.Tensor, salt: int, p: int) -> torch.Tensor:
    """int32 codes ``bucket << 5 | rho`` of non-negative ids < 2^32 (bit-exact twin of the kernels'
    hash, ``ops/reference.py:hll_update_values``)."""
    from ..ops.reference import hll_update_values

    b, r = hll_update_values(vals, salt, p)
    return ((b << 5) | r).to(torch.int32)


def code_column(ds, col: str, p: int, salt: int) -> Optional[str]:
    """Name of the resident code plane of dimension ``col`` (built now if needed), or None when the
    column does not qualify: not a dimension, ids narrower than ``MIN_ID_BYTES``, p too large, a
    streamed window (its columns are staged per window), or the plane budget exhausted."""
    if not ENABLED or p > MAX_P or col not in getattr(ds, "dims", {}) or not getattr(ds, "hll_codes_ok", True):
        return None
    ids = ds.dims[col].ids
    if ids.dtype.is_floating_point or ids.element_size() < MIN_ID_BYTES:
        return None
    name = code_name(col, p, salt)
    cache = ds.__dict__.setdefault("_hll_codes", {})
    if name in cache:
        return name
    n = ids.numel()
    if sum(t.numel() * 2 for t in cache.values()) + n * 2 > MAX_BYTES:
        return None
    out = torch.zeros(n, dtype=torch.int16, device=ids.device)
    rows = int(getattr(ds, "num_rows", n))
    for lo in range(0, rows, CHUNK):
        hi = min(rows, lo + CHUNK)
        v = ids[lo:hi].to(torch.int64)
        if v.numel() and int(v.min()) < 0:  # (ids are never negative; a 64-bit-mix value has no u16 code)
            return None
        out[lo:hi] = codes(v, salt, p).to(torch.int16)  # low 16 bits (two's complement wrap)
    from ..utils.streams import publish

    # (complete before any slot's stream can find it: utils/streams.py)
    cache[name] = publish(out.view(torch.uint16) if hasattr(torch, "uint16") else out, ids.device)
    return name


def lookup(ds, name: str) -> Optional[torch.Tensor]:
    c = ds.__dict__.get("_hll_codes")
    return None if c is None else c.get(name)
