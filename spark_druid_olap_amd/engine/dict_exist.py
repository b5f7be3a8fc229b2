"""Group existence over the dictionary domain instead of the rows.

An existence-only group-by (no aggregator reads the groups' counts: the inner level of TPC-H Q13's
``count(distinct o_orderkey)``, Search queries, DISTINCT) keyed on ONE dimension ``K``, over the
whole shard (no time restriction), whose filter only reads ``K`` itself or dimensions that ``K``
functionally determines, has the answer

    { k : k occurs in the shard  and  filter(FD(k)) }

-- a predicate over ``C_K`` dictionary entries instead of ``N`` rows.  This is the dictionary-domain
evaluation of SURVEY K3 ("O(C_d) instead of O(N)") carried one step further, and the GPU analogue
of what Druid answers from its per-value bitmap indexes (a value's bitmap is non-empty iff it
occurs).  Q13 at SF100: 600M rows -> 150M order ids; the per-row random byte stores into a 150 MB
presence table disappear.

The per-dimension occurrence bitmap and the FD tables (``lower.fd_table``) are computed once per
shard on the device and cached, like the dictionaries themselves.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ..ops import desc as D
from .partials import Partials

_CHUNK = 1 << 27


_OCC_LOCK = __import__("threading").Lock()


def occurrence(ds, col: str) -> torch.Tensor:
    """bool [C_col]: dictionary id occurs in this shard (cached on the datasource).

    Queries of the stream scheduler run on different HIP streams of one process: the bitmap is
    published to the cache only after the producing stream finished its scatter, so a query on
    another stream never reads a half-built table (it would drop keys from an existence group-by)."""
    cache = ds.__dict__.setdefault("_occurrence_cache", {})
    t = cache.get(col)
    if t is not None:
        return t
    with _OCC_LOCK:
        t = cache.get(col)
        if t is None:
            d = ds.dims[col]
            t = torch.zeros(len(d.dictionary), dtype=torch.bool, device=d.ids.device)
            n = ds.num_rows
            for s0 in range(0, n, _CHUNK):  # (id columns are padded past num_rows)
                t[d.ids[s0:min(n, s0 + _CHUNK)].to(torch.int64)] = True
            if t.is_cuda:
                torch.cuda.current_stream(t.device).synchronize()
            cache[col] = t
    return t


def _leaf_cols(x, out: set) -> bool:
    """Collect the dimensions the filter reads; False if it has anything but id-set leaves."""
    k = x[0]
    if k in ("true", "false"):
        return True
    if k in ("and", "or"):
        return all(_leaf_cols(c, out) for c in x[1])
    if k == "not":
        return _leaf_cols(x[1], out)
    if k == "ids":
        out.add(x[1])
        return True
    return False  # time / numeric / expression leaves read rows


_TRACE = False  # (tools: print the dictionary-domain decisions)


def plan(prog) -> Optional[Tuple[str, Tuple[str, ...]]]:
    """(key dimension, dimensions the filter reads) when the program qualifies, else None.
    Structural checks only (no device work)."""
    r, why = _plan(prog)
    if _TRACE:
        print(f"[dict_exist] plan keys={[k.name for k in prog.keys]} G={prog.G} -> {r or why}", flush=True)
    return r


def _plan(prog):
    ds = prog.ds
    if prog.empty or not prog.presence_only or prog.nhll or prog.stored_hll or prog.thetas:
        return None, "not existence-only"
    if len(prog.keys) != 1 or prog.nslots != 1 or getattr(ds, "fd_source", None) is not None:
        return None, "not one key"
    kc = prog.keys[0]
    if kc.kind not in (D.K_ID, D.K_REMAP) or kc.col not in ds.dims:
        return None, "key not a dimension id"
    covered = sum(hi - lo for lo, hi in prog.ranges)
    if covered < ds.num_rows:
        return None, f"time restriction ({covered} of {ds.num_rows} rows)"  # rows decide
    cols: set = set()  # (zone maps are chunk-pruning hints implied by these leaves)
    if not _leaf_cols(prog.bexpr, cols) or any(c not in ds.dims for c in cols):
        return None, "filter reads more than id sets"
    if len(ds.dims[kc.col].dictionary) > ds.num_rows:
        return None, "dictionary larger than the shard"  # the scan is cheaper
    return (kc.col, tuple(sorted(cols - {kc.col}))), ""


_MASKS: "dict" = {}  # id(host id-set array) -> (array, device copy)
_MASKS_LOCK = __import__("threading").Lock()


def _device_mask(arr, dev) -> torch.Tensor:
    """The device copy of a filter leaf's id set, made once per lowered program: TPC-H Q13's
    o_comment set has one entry per distinct comment (~150M at SF100) and its pageable upload was
    9 of the query's 17 ms.  Keyed by the array object (kept alive in the entry, so the id is not
    reused while cached); bounded to the most recent leaves."""
    k = (id(arr), str(dev))
    with _MASKS_LOCK:
        hit = _MASKS.get(k)
    if hit is not None and hit[0] is arr:
        m = hit[1]
        if m.is_cuda:  # (statements on other slot streams read it: an eviction must wait for them)
            m.record_stream(torch.cuda.current_stream(m.device))
        return m
    m = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.bool_)).to(dev)
    with _MASKS_LOCK:
        _MASKS[k] = (arr, m)
        while len(_MASKS) > 64:
            _MASKS.pop(next(iter(_MASKS)))
    return m


def _eval(x, key_col: str, masks: dict, n: int, dev) -> torch.Tensor:
    k = x[0]
    if k == "true":
        return torch.ones(n, dtype=torch.bool, device=dev)
    if k == "false":
        return torch.zeros(n, dtype=torch.bool, device=dev)
    if k == "and":
        out = torch.ones(n, dtype=torch.bool, device=dev)
        for c in x[1]:
            out &= _eval(c, key_col, masks, n, dev)
        return out
    if k == "or":
        out = torch.zeros(n, dtype=torch.bool, device=dev)
        for c in x[1]:
            out |= _eval(c, key_col, masks, n, dev)
        return out
    if k == "not":
        return ~_eval(x[1], key_col, masks, n, dev)
    m = _device_mask(x[2], dev)
    if x[1] == key_col:
        return m[:n] if m.numel() >= n else torch.nn.functional.pad(m, (0, n - m.numel()))
    fd = masks[x[1]]  # key id -> dependent id (int32; -1: absent everywhere, so never occurring)
    return torch.index_select(m, 0, fd.clamp(min=0))


def run(prog, key_col: str, dep_cols, world=None) -> Optional[Partials]:
    """The existence partials (sparse: group keys + a count slot of ones, like the presence-byte
    scan), or None when a filter dimension is not functionally determined by the key."""
    from .lower import fd_table

    ds = prog.ds
    fds = {}
    for c in dep_cols:
        t = fd_table(ds, key_col, c, world)
        if t is None:
            if _TRACE:
                print(f"[dict_exist] {key_col} does not determine {c}: scanning rows", flush=True)
            return None
        fds[c] = t
    occ = occurrence(ds, key_col)
    n = occ.numel()
    # the filter over the key's domain depends only on the program's (constant) predicate and the
    # shard's FD tables: composed once per lowered program, like the predicate's own evaluation
    # over each dictionary at lowering -- TPC-H Q13's o_comment set gathered through the
    # o_orderkey -> o_comment table is 150M random reads (2.8 ms) per run otherwise
    cache = prog.__dict__.setdefault("_dict_exist_filter", {})
    f = cache.get((key_col, n))
    if f is None:
        from ..utils.streams import publish

        # (the prepared program is shared by concurrent statements on other slots' streams)
        f = cache[(key_col, n)] = publish(_eval(prog.bexpr, key_col, fds, n, occ.device), occ.device)
    sel = occ & f
    if sel.is_cuda:
        from ..ops import native

        ids = native.nonzero_rows(sel.view(torch.uint8))  # ballot + compaction kernels
    else:
        ids = torch.nonzero(sel).flatten()
    kc = prog.keys[0]
    if kc.kind == D.K_REMAP:
        rm = torch.from_numpy(np.asarray(kc.remap, dtype=np.int64)).to(ids.device)
        keys = rm[ids]
        keys = torch.sort(keys[keys >= 0]).values
    elif kc.base == 0 and kc.card >= n:
        keys = ids  # (every dictionary id is a key: nothing to shift or drop)
    else:
        keys = ids - kc.base
        keys = keys[(keys >= 0) & (keys < kc.card)]
    return Partials("sparse", torch.ones((keys.numel(), 1), dtype=torch.int64, device=keys.device), keys, [])
