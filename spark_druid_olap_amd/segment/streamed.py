"""Shards larger than HBM: host-resident segments streamed through the GPU window by window
("segments are double-buffered H2D on a copy stream, the scan overlaps, and partial
aggregates stay resident").

The reference bounds memory with time-partitioned segments and per-batch historical queries
(``asd/DruidQueryCostModel.scala:505-547``, ``sd/DruidRDD.scala:244-269``).  Here a shard whose
columns do not fit (or should not stay) in HBM lives in pinned host memory (``HostShard``); a
query is lowered once against the whole shard to learn which columns, bitmaps and zone maps it
reads, then executed over chunk-aligned row windows:

* window j+1's columns are copied host->device on a dedicated copy stream while window j scans on
  the compute stream (two staging slots, event-ordered -- classic double buffering);
* every window is a regular device ``DataSource`` view (``_WindowDataSource``) of its rows, so the
  lowering, JIT kernels and modes of the resident engine apply unchanged; window-independent
  lowering state (functional-dependency tables, metric value ranges, the time span that fixes
  time-bucket key bases) is decided once over the whole shard (``fd_source``), so every window's
  partial aggregates share one key/slot layout;
* partials accumulate on the device (``combine_local``) and only the combined result is merged
  across ranks and finalized -- exactly the resident path's tail.

Only the columns a query reads cross the host link (TPC-H Q1 reads ~16 of ~170 bytes per row).
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Set, Tuple

import numpy as np
import torch

from .datasource import CHUNK_ROWS, DataSource, DimColumn, MetricColumn, SketchColumn, padded_len


class _WindowDataSource(DataSource):
    """Rows [lo, hi) of a host shard on the device.  Reports the WHOLE shard's time span so
    time-bucket key bases (lower.granularity_key) agree across windows."""

    hll_codes_ok = False  # columns are staged per window: no resident derived planes (segment/hllcode.py)

    def min_time_ms(self) -> int:
        return self.fd_source.min_time_ms()

    def max_time_ms(self) -> int:
        return self.fd_source.max_time_ms()


class HostShard:
    """A datasource shard in (pinned) host memory, served to queries in row windows of
    ``window_rows`` (rounded to whole 4096-row chunks)."""

    def __init__(self, ds: DataSource, device, window_rows: int = 1 << 26, pin: bool = True):
        if ds.device.type != "cpu":
            raise ValueError("HostShard wraps a host-resident (CPU) datasource")
        self.ds = ds
        ds.hll_codes_ok = False  # programs lowered over the shard read only columns a window stages
        self.device = torch.device(device)
        self.window_rows = max(CHUNK_ROWS, window_rows // CHUNK_ROWS * CHUNK_ROWS)
        if pin and torch.cuda.is_available():
            for d in ds.dims.values():
                d.ids = d.ids.pin_memory()
                if d.bitmap is not None:
                    d.bitmap = d.bitmap.pin_memory()
            for m in ds.metrics.values():
                m.data = m.data.pin_memory()
            ds.time = ds.time.pin_memory()
        # zone maps are tiny ([chunks] int32): resident on the device for every window
        self._zones = {k: (d.zmin.to(self.device), d.zmax.to(self.device)) for k, d in ds.dims.items()
                       if d.zmin is not None}
        self.windows: List[Tuple[int, int]] = [(lo, min(ds.num_rows, lo + self.window_rows))
                                               for lo in range(0, ds.num_rows, self.window_rows)]
        self.copy_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self.bytes_copied = 0

    @property
    def name(self) -> str:
        return self.ds.name

    def __getattr__(self, item):
        # catalog / planner / views read the shard's metadata (dictionaries, segments, metrics)
        if item.startswith("__") or item == "ds":
            raise AttributeError(item)
        return getattr(self.ds, item)

    # ------------------------------------------------------------------ windows
    def window(self, j: int, dims: Set[str], metrics: Set[str], bitmaps: Dict[str, Set[int]]) -> _WindowDataSource:
        """Device view of window ``j`` holding only the listed columns (the rest are empty
        placeholders: any access would fail loudly).  Copies are issued on the copy stream; the
        caller orders the compute stream after ``ready``."""
        ds = self.ds
        lo, hi = self.windows[j]
        n = hi - lo
        P = padded_len(n)
        dev = self.device
        c0 = lo // CHUNK_ROWS
        nch = P // CHUNK_ROWS
        w0 = lo // 64
        nw = P // 64
        ctx = torch.cuda.stream(self.copy_stream) if self.copy_stream is not None else _null()
        with ctx:
            def rows(t: torch.Tensor) -> torch.Tensor:
                out = torch.zeros(P, dtype=t.dtype, device=dev)
                m = min(P, t.numel() - lo)
                out[:m].copy_(t[lo: lo + m], non_blocking=True)
                self.bytes_copied += m * t.element_size()
                return out

            time_t = rows(ds.time)
            dcols: Dict[str, DimColumn] = {}
            for k, d in ds.dims.items():
                ids = rows(d.ids) if k in dims else torch.empty(0, dtype=d.ids.dtype, device=dev)
                bm = None
                if d.bitmap is not None and k in bitmaps:
                    # only the value planes the query's bitmap leaves read, each a contiguous copy
                    # (a whole [card, words] window of a 150-value dimension is ~19 B/row)
                    bm = torch.zeros((d.bitmap.shape[0], nw), dtype=torch.int64, device=dev)
                    m = min(nw, d.bitmap.shape[1] - w0)
                    for v in sorted(bitmaps[k]):
                        bm[v, :m].copy_(d.bitmap[v, w0: w0 + m], non_blocking=True)
                    self.bytes_copied += len(bitmaps[k]) * m * 8
                    bm.staged_values = frozenset(bitmaps[k])
                zmin = zmax = None
                if k in self._zones:
                    zm, zx = self._zones[k]
                    zmin = torch.zeros(nch, dtype=zm.dtype, device=dev)
                    zmax = torch.zeros(nch, dtype=zx.dtype, device=dev)
                    m = min(nch, zm.numel() - c0)
                    zmin[:m] = zm[c0: c0 + m]
                    zmax[:m] = zx[c0: c0 + m]
                dcols[k] = DimColumn(k, d.dictionary, ids, bm, zmin, zmax, d.spatial)
            mcols: Dict[str, MetricColumn] = {}
            for k, m_ in ds.metrics.items():
                data = rows(m_.data) if k in metrics else torch.empty(0, dtype=m_.data.dtype, device=dev)
                sk = None
                if m_.sketch is not None and k in metrics:
                    a, b = int(m_.sketch.offsets[lo]), int(m_.sketch.offsets[hi])
                    sk = SketchColumn(k, m_.sketch.kind, (m_.sketch.offsets[lo: hi + 1] - a).to(dev, non_blocking=True),
                                      m_.sketch.values[a:b].to(dev, non_blocking=True), m_.sketch.p, m_.sketch.salt,
                                      m_.sketch.size)
                mcols[k] = MetricColumn(k, m_.kind, data, m_.scale, sk)
            ready = None
            if self.copy_stream is not None:
                ready = torch.cuda.Event()
                ready.record(self.copy_stream)
        w = _WindowDataSource(ds.name, n, time_t, ds.time_unit_ms, dcols, mcols, ds.segment_granularity,
                              ds.query_granularity, ds.partition, ds.num_partitions,
                              time_host=ds.time_host[lo:hi])
        w.fd_source = ds
        w.__dict__["_fd_cache"] = ds.__dict__.setdefault("_fd_cache", {})
        w.shard_key = ds.shard_key
        w.spatial = getattr(ds, "spatial", {})
        w.rollup = getattr(ds, "rollup", False)
        w.global_num_rows = ds.global_num_rows
        w.global_interval_ms = getattr(ds, "global_interval_ms", None)
        w.window = (lo, hi)
        w.ready = ready
        return w


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _columns_of(prog) -> Tuple[Set[str], Set[str], Set[str]]:
    """(dimensions, metrics, bitmap dimensions) a lowered program reads."""
    ds = prog.ds
    cols = set(prog.cols) | {kc.col for kc in prog.keys}
    dims = {c for c in cols if c in ds.dims}
    mets = {c for c in cols if c in ds.metrics}
    mets |= {m for _, m, _ in getattr(prog, "stored_hll", [])}
    dims |= {dim for dim, _, _ in prog.zones}
    # the reference executor (and filter fallbacks) evaluate the normalized filter over ids
    named = set()

    def walk(x):
        if isinstance(x, str):
            named.add(x)
        elif isinstance(x, (tuple, list)):
            for y in x:
                walk(y)

    walk(prog.bexpr)
    for d in prog.aops:
        walk(d.get("filter"))
    dims |= {c for c in named if c in ds.dims}
    mets |= {c for c in named if c in ds.metrics}
    bitmaps: Dict[str, Set[int]] = {}
    for row, _, count in prog.bm_leaves:  # a leaf addresses `count` value planes of one bitmap index
        p = row.data_ptr()
        for k, d in ds.dims.items():
            b = d.bitmap
            if b is not None and b.data_ptr() <= p < b.data_ptr() + b.numel() * 8:
                v0 = (p - b.data_ptr()) // (b.shape[1] * 8)
                bitmaps.setdefault(k, set()).update(range(v0, v0 + count))
    return dims, mets, bitmaps


class StreamedQuery:
    """Run a QuerySpec over a ``HostShard`` window by window (see the module doc)."""

    def __init__(self, engine, qs, shard: HostShard):
        from ..engine.executor import PreparedQuery
        from ..engine.lower import LoweringError

        qt = qs.queryType
        if qt not in ("groupBy", "timeseries", "topN"):
            raise LoweringError(f"streamed execution runs aggregate queries, not {qt}")
        self.engine, self.qs, self.shard = engine, qs, shard
        # lower once over the whole host shard (CPU): which columns every window must carry
        host_pq = PreparedQuery(_HostEngine(engine), qs, shard.ds)
        self._cols = _columns_of(host_pq._full_prog)
        if host_pq._full_prog.thetas:
            raise LoweringError("thetaSketch aggregations are not streamed")
        self.stats: Dict[str, float] = {}

    def run(self):
        import torch

        from ..engine.executor import PreparedQuery, combine_local
        from ..parallel.merge import merge_partials
        from ..engine.partials import finalize

        t0 = time.perf_counter()
        sh = self.shard
        dims, mets, bms = self._cols
        parts, progs = [], []
        first_pq = None
        nxt = sh.window(0, dims, mets, bms) if sh.windows else None
        for j in range(len(sh.windows)):
            cur = nxt
            if j + 1 < len(sh.windows):  # prefetch the next window while this one scans
                nxt = sh.window(j + 1, dims, mets, bms)
            if cur.ready is not None:
                torch.cuda.current_stream(sh.device).wait_event(cur.ready)
            pq = PreparedQuery(_LocalEngine(self.engine), self.qs, cur)
            prog = pq._full_prog
            _check_resident(prog, cur)
            _, p_, prep = pq.scans[0]
            part = pq._scan(p_, prep)
            if pq.window is not None:
                part = pq.window.to_global(part)
            parts.append(_own(part))
            progs.append(prog)
            if first_pq is None:
                first_pq = pq
            if sh.copy_stream is not None:
                # the staging buffers of `cur` may be reused once this window's scan is done
                sh.copy_stream.wait_stream(torch.cuda.current_stream(sh.device))
        if first_pq is None:
            raise ValueError("empty shard")
        prog = progs[0]
        if any(p.G != prog.G or p.slots != prog.slots for p in progs[1:]):
            raise RuntimeError("streamed windows lowered to different layouts")
        part = combine_local(prog, parts) if len(parts) > 1 else parts[0]
        t1 = time.perf_counter()
        world = self.engine.world
        disjoint = bool(sh.ds.shard_key) and any(k.col == sh.ds.shard_key for k in prog.keys)
        part = merge_partials(world, prog, part, disjoint_keys=disjoint)
        first_pq.world = world
        part, hv = first_pq._device_having(prog, part)
        part = first_pq._device_prune(prog, part, hv)
        cols = finalize(prog, part, getattr(self, "out_types", None))
        res = first_pq._post(prog, cols)
        res.stats.update(windows=len(sh.windows), scan_ms=(t1 - t0) * 1e3,
                         exec_ms=(time.perf_counter() - t0) * 1e3, h2d_bytes=sh.bytes_copied)
        return res


def _check_resident(prog, w) -> None:
    """Every column the window's kernel will dereference must have been staged (a placeholder
    read would be an out-of-bounds device access): fail on the host instead."""
    from ..engine.lower import column_tensor

    for c in prog.cols:
        if column_tensor(w, c).numel() < w.padded_rows:
            raise RuntimeError(f"streamed window lowered to read column {c!r} that was not staged")
    for row, _, count in prog.bm_leaves:
        if row.numel() == 0 or row.device != w.device:
            raise RuntimeError("streamed window lowered to read a bitmap that was not staged")
        for d in w.dims.values():
            b = d.bitmap
            if b is not None and b.data_ptr() <= row.data_ptr() < b.data_ptr() + b.numel() * 8:
                v0 = (row.data_ptr() - b.data_ptr()) // (b.shape[1] * 8)
                staged = getattr(b, "staged_values", frozenset())
                if any(v not in staged for v in range(v0, v0 + count)):
                    raise RuntimeError(f"streamed window reads bitmap planes of {d.name!r} that were not staged")


def _own(part):
    """Partials that survive the next window's scan (the prepared buffers are per window, but a
    dense result aliases its accumulator table)."""
    from ..engine.partials import Partials

    return Partials(part.kind, part.acc.clone(), None if part.keys is None else part.keys.clone(),
                    [h.clone() for h in part.hll])


class _HostEngine:
    """Engine facade for the one-off host lowering: the torch path, no collectives."""

    def __init__(self, engine):
        from ..parallel.world import World

        self.world = World()
        self.use_native = False
        self.deterministic = engine.deterministic


class _LocalEngine:
    """Engine facade for a window: the real engine's kernels, but a single-rank world -- windows
    combine locally and merge across ranks once, after the last window."""

    def __init__(self, engine):
        from ..parallel.world import World

        self.world = World()
        self.use_native = engine.use_native
        self.deterministic = engine.deterministic
