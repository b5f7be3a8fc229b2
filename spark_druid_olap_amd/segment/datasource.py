"""Device-resident, time-sorted, dictionary-encoded datasource shards.

This is the MI355X replacement for a Druid datasource served by historicals
(reference metadata model: ``sd/metadata/DruidDataSource.scala:24-153``; segment inventory
``sd/metadata/DruidMetadataCache.scala:64-148``).  Design points:

* One rank (GPU) holds one shard: a hash partition of EVERY time segment, concatenated in time
  order.  A time-range query therefore loads every GPU equally (time-sharding would leave most
  GPUs idle for a one-year predicate), and row ranges come from a binary search on ``__time``.
* Columns are padded to a multiple of ``CHUNK_ROWS`` (+1 chunk) so the scan kernel may issue its
  unrolled loads past the last row without bounds checks.
* Dimension ids use the narrowest integer type (u8 / i16 / i32) -- the scan is HBM-bound, so
  bytes per row is the speed-of-light.  Decimal metrics are stored as scaled int32/int64 and
  aggregated exactly in int64 (Druid stored them as float, see BASELINE.md accuracy row).
* Low-cardinality dimensions get an inverted bitmap index ``[card, nwords]`` of u64 words: one
  word per 64-row wavefront step, so bitmap filters cost one scalar load per 64 rows.
* Every dimension gets a zone map (min/max id per 4096-row chunk); dimensions correlated with
  time (o_orderdate vs l_shipdate) prune most chunks of a date-range query.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .dictionary import Dictionary, id_dtype_for

CHUNK_ROWS = 4096
MS_PER_DAY = 86_400_000

TORCH_DT = {"uint8": torch.uint8, "int16": torch.int16, "int32": torch.int32, "int64": torch.int64,
            "float32": torch.float32, "float64": torch.float64}
# kernel dtype codes (scan_desc.h DType)
DT_CODE = {torch.uint8: 0, torch.int16: 1, torch.int32: 2, torch.int64: 3, torch.float32: 4, torch.float64: 5}
if hasattr(torch, "uint16"):
    DT_CODE[torch.uint16] = 6  # HLL code planes (segment/hllcode.py)


def dtype_code(t: torch.Tensor) -> int:
    return DT_CODE[t.dtype]


def padded_len(n: int) -> int:
    return (max(n, 1) + CHUNK_ROWS - 1) // CHUNK_ROWS * CHUNK_ROWS + CHUNK_ROWS


def _pad(t: torch.Tensor, n: int, fill=0) -> torch.Tensor:
    P = padded_len(n)
    out = torch.full((P,), fill, dtype=t.dtype, device=t.device)
    out[:n] = t[:n]
    return out


@dataclass
class DimColumn:
    name: str
    dictionary: Dictionary
    ids: torch.Tensor                       # padded, narrow int
    bitmap: Optional[torch.Tensor] = None   # [card, nwords] int64 (u64 bit patterns)
    zmin: Optional[torch.Tensor] = None     # [nchunks] int32
    zmax: Optional[torch.Tensor] = None
    spatial: bool = False

    @property
    def cardinality(self) -> int:
        return len(self.dictionary)


@dataclass
class SketchColumn:
    """A sketch metric kept per rolled-up row (segment/ingest.py), CSR over the shard's rows:
    row r owns ``values[offsets[r]:offsets[r+1]]``.  hll: packed (bucket << 8 | rho) int32 pairs,
    distinct buckets with their max rho; theta: the row's k smallest distinct 62-bit hashes."""
    name: str
    kind: str                 # hll | theta
    offsets: torch.Tensor     # [num_rows + 1] int64
    values: torch.Tensor
    p: int = 11
    salt: int = 0
    size: int = 16384

    def nbytes(self) -> int:
        return self.offsets.numel() * 8 + self.values.numel() * self.values.element_size()


@dataclass
class MetricColumn:
    name: str
    kind: str                 # long | double | decimal | hll | theta
    data: torch.Tensor        # padded (a one-byte placeholder when ``sketch`` holds the values)
    scale: int = 0            # decimal digits for kind == decimal
    sketch: Optional[SketchColumn] = None  # rolled-up sketch metric (hyperUnique / thetaSketch)

    @property
    def is_integral(self) -> bool:
        return self.kind in ("long", "decimal", "hll") and self.sketch is None


@dataclass
class SegmentInfo:
    """One (interval, partition) Druid segment == a row range of this shard."""
    interval_lo_ms: int
    interval_hi_ms: int
    row_lo: int
    row_hi: int
    partition: int
    version: str = "v1"

    @property
    def identifier(self) -> str:
        from ..query.intervals import fmt_iso

        return f"{fmt_iso(self.interval_lo_ms)}/{fmt_iso(self.interval_hi_ms)}_{self.version}_{self.partition}"


class DataSource:
    """A datasource shard resident on one device."""

    def __init__(self, name: str, num_rows: int, time: torch.Tensor, time_unit_ms: int,
                 dims: Dict[str, DimColumn], metrics: Dict[str, MetricColumn],
                 segment_granularity: str = "month", query_granularity: str = "none",
                 partition: int = 0, num_partitions: int = 1, time_host: Optional[np.ndarray] = None):
        self.name = name
        self.num_rows = int(num_rows)
        self.time = time
        self.time_unit_ms = int(time_unit_ms)
        self.dims = dims
        self.metrics = metrics
        self.segment_granularity = segment_granularity
        self.query_granularity = query_granularity
        self.partition = partition
        self.num_partitions = num_partitions
        self.time_host = time_host if time_host is not None else time[: self.num_rows].cpu().numpy()
        self.segments: List[SegmentInfo] = self._compute_segments()
        self.global_num_rows = self.num_rows  # set by the parallel layer after sharding
        self.shard_key: Optional[str] = None  # dimension rows are hash/range partitioned on

    # ----------------------------------------------------------------- properties
    @property
    def device(self) -> torch.device:
        return self.time.device

    @property
    def padded_rows(self) -> int:
        return int(self.time.numel())

    @property
    def num_chunks(self) -> int:
        return self.padded_rows // CHUNK_ROWS

    @property
    def nwords(self) -> int:
        return self.padded_rows // 64

    def column_names(self) -> List[str]:
        return ["__time"] + list(self.dims) + list(self.metrics)

    def min_time_ms(self) -> int:
        return int(self.time_host[0]) * self.time_unit_ms if self.num_rows else 0

    def max_time_ms(self) -> int:
        return int(self.time_host[-1]) * self.time_unit_ms if self.num_rows else 0

    def size_bytes(self) -> int:
        n = self.time.numel() * self.time.element_size()
        for d in self.dims.values():
            n += d.ids.numel() * d.ids.element_size()
            if d.bitmap is not None:
                n += d.bitmap.numel() * 8
        for m in self.metrics.values():
            n += m.data.numel() * m.data.element_size()
            if m.sketch is not None:
                n += m.sketch.nbytes()
        return n

    # ----------------------------------------------------------------- time
    def distinct_times(self) -> np.ndarray:
        """The distinct __time values (in time units), ascending -- cached.  The column is sorted,
        so this hops from value to value with binary searches (~2,500 days at SF100: a few
        milliseconds, where np.unique over 600M rows took seconds per lowered query)."""
        tv = self.__dict__.get("_distinct_times")
        if tv is None:
            t = self.time_host
            if len(t) > 1 and not bool((t[1:] >= t[:-1]).all()):  # (once per datasource)
                tv = self._distinct_times = np.unique(t)
                return tv
            out = []
            i, n = 0, len(t)
            while i < n:
                v = t[i]
                out.append(v)
                i = int(np.searchsorted(t, v, side="right"))
            tv = self._distinct_times = np.asarray(out, dtype=t.dtype)
        return tv

    def rows_for_interval(self, lo_ms: int, hi_ms: int):
        """Half-open row range whose __time is in [lo_ms, hi_ms)."""
        u = self.time_unit_ms
        lo_u = -(-lo_ms // u)  # ceil
        hi_u = -(-hi_ms // u)
        a = int(np.searchsorted(self.time_host, lo_u, side="left"))
        b = int(np.searchsorted(self.time_host, hi_u, side="left"))
        return a, max(a, b)

    def _compute_segments(self) -> List[SegmentInfo]:
        if self.num_rows == 0:
            return []
        from ..query.granularity import bucket_start_ms, next_bucket_ms

        segs = []
        t = self.time_host
        u = self.time_unit_ms
        start = bucket_start_ms(int(t[0]) * u, self.segment_granularity)
        last = int(t[-1]) * u
        while start <= last:
            nxt = next_bucket_ms(start, self.segment_granularity)
            a, b = self.rows_for_interval(start, nxt)
            if b > a:
                segs.append(SegmentInfo(start, nxt, a, b, self.partition))
            start = nxt
        return segs

    # ----------------------------------------------------------------- indexes
    def build_indexes(self, bitmap_max_card: int = 256, bitmap_budget_bytes: Optional[int] = None,
                      zone_maps: bool = True) -> None:
        """Build zone maps for every dimension and inverted bitmaps for low-card dimensions."""
        nch = self.num_chunks
        for d in self.dims.values():
            if zone_maps:
                v = d.ids.view(nch, CHUNK_ROWS)
                # padded tail rows must not widen the last real chunk's zone
                zmin = v.to(torch.int32).amin(dim=1)
                zmax = v.to(torch.int32).amax(dim=1)
                if self.num_rows % CHUNK_ROWS:
                    last = self.num_rows // CHUNK_ROWS
                    tail = d.ids[last * CHUNK_ROWS: self.num_rows].to(torch.int32)
                    zmin[last] = tail.min()
                    zmax[last] = tail.max()
                d.zmin, d.zmax = zmin.contiguous(), zmax.contiguous()
        if bitmap_max_card <= 0:
            return
        budget = bitmap_budget_bytes if bitmap_budget_bytes is not None else 1 << 62
        used = 0
        for d in sorted(self.dims.values(), key=lambda x: x.cardinality):
            card = d.cardinality
            if card > bitmap_max_card or d.spatial:
                continue
            need = card * self.nwords * 8
            if used + need > budget:
                continue
            d.bitmap = build_bitmap(d.ids, self.num_rows, card)
            used += need

    # ----------------------------------------------------------------- persistence
    def save(self, path: str) -> None:
        """Segment store: one .npy per column + a JSON manifest (checkpoint / resume)."""
        os.makedirs(path, exist_ok=True)
        n = self.num_rows
        np.save(os.path.join(path, "__time.npy"), self.time[:n].cpu().numpy())
        man = {"name": self.name, "num_rows": n, "time_unit_ms": self.time_unit_ms,
               "segment_granularity": self.segment_granularity, "query_granularity": self.query_granularity,
               "partition": self.partition, "num_partitions": self.num_partitions,
               "shard_key": self.shard_key, "global_num_rows": int(self.global_num_rows), "dims": {}, "metrics": {}}
        for name, d in self.dims.items():
            np.save(os.path.join(path, f"dim.{name}.npy"), d.ids[:n].cpu().numpy())
            man["dims"][name] = {"dictionary": d.dictionary.to_json(), "spatial": d.spatial}
        for name, m in self.metrics.items():
            np.save(os.path.join(path, f"met.{name}.npy"), m.data[:n].cpu().numpy())
            man["metrics"][name] = {"kind": m.kind, "scale": m.scale}
            if m.sketch is not None:
                sk = m.sketch
                np.save(os.path.join(path, f"sk.{name}.offsets.npy"), sk.offsets.cpu().numpy())
                np.save(os.path.join(path, f"sk.{name}.values.npy"), sk.values.cpu().numpy())
                man["metrics"][name]["sketch"] = {"kind": sk.kind, "p": sk.p, "salt": sk.salt, "size": sk.size}
        man["spatial"] = getattr(self, "spatial", {})
        man["rollup"] = bool(getattr(self, "rollup", False))
        with open(os.path.join(path, "manifest.json"), "w") as f:
            json.dump(man, f)

    def to(self, device) -> "DataSource":
        """A copy of this shard on ``device`` (host <-> HBM), indexes and sketches included."""
        dev = torch.device(device)
        mv = lambda t: None if t is None else t.to(dev)  # noqa: E731
        dims = {k: DimColumn(k, d.dictionary, mv(d.ids), mv(d.bitmap), mv(d.zmin), mv(d.zmax), d.spatial)
                for k, d in self.dims.items()}
        mets = {}
        for k, m in self.metrics.items():
            sk = m.sketch
            if sk is not None:
                sk = SketchColumn(k, sk.kind, mv(sk.offsets), mv(sk.values), sk.p, sk.salt, sk.size)
            mets[k] = MetricColumn(k, m.kind, mv(m.data), m.scale, sk)
        ds = DataSource(self.name, self.num_rows, mv(self.time), self.time_unit_ms, dims, mets,
                        self.segment_granularity, self.query_granularity, self.partition, self.num_partitions,
                        time_host=self.time_host)
        for a in ("global_num_rows", "shard_key", "spatial", "rollup", "global_interval_ms"):
            if hasattr(self, a):
                setattr(ds, a, getattr(self, a))
        return ds

    @staticmethod
    def concat(shards: Sequence["DataSource"]) -> "DataSource":
        return concat_shards(shards)

    @staticmethod
    def load(path: str, device="cpu", bitmap_max_card: int = 256) -> "DataSource":
        with open(os.path.join(path, "manifest.json")) as f:
            man = json.load(f)
        n = man["num_rows"]
        dev = torch.device(device)
        t = torch.from_numpy(np.load(os.path.join(path, "__time.npy"), allow_pickle=False))
        dims = {}
        for name, meta in man["dims"].items():
            ids = torch.from_numpy(np.load(os.path.join(path, f"dim.{name}.npy"), allow_pickle=False))
            dims[name] = DimColumn(name, Dictionary.from_json(meta["dictionary"]), _pad(ids.to(dev), n),
                                   spatial=meta.get("spatial", False))
        metrics = {}
        for name, meta in man["metrics"].items():
            data = torch.from_numpy(np.load(os.path.join(path, f"met.{name}.npy"), allow_pickle=False))
            metrics[name] = MetricColumn(name, meta["kind"], _pad(data.to(dev), n), meta.get("scale", 0))
            if "sketch" in meta:
                sm = meta["sketch"]
                off = torch.from_numpy(np.load(os.path.join(path, f"sk.{name}.offsets.npy"), allow_pickle=False))
                val = torch.from_numpy(np.load(os.path.join(path, f"sk.{name}.values.npy"), allow_pickle=False))
                metrics[name].sketch = SketchColumn(name, sm["kind"], off.to(dev), val.to(dev), sm["p"], sm["salt"],
                                                    sm["size"])
        th = t.numpy().astype(np.int64)
        ds = DataSource(man["name"], n, _pad(t.to(dev), n, fill=int(t[-1]) if n else 0), man["time_unit_ms"],
                        dims, metrics, man["segment_granularity"], man["query_granularity"],
                        man.get("partition", 0), man.get("num_partitions", 1), time_host=th)
        ds.shard_key = man.get("shard_key")
        ds.global_num_rows = man.get("global_num_rows", n)
        ds.spatial = man.get("spatial", {})
        ds.rollup = man.get("rollup", False)
        ds.build_indexes(bitmap_max_card=bitmap_max_card)
        return ds


def concat_shards(shards: Sequence["DataSource"]) -> "DataSource":
    """One shard holding the rows of several shards of the same datasource (same global
    dictionaries), time-ordered: how a surviving GPU adopts a lost GPU's segments
    (parallel/recovery.py).  Sketch columns (CSR) are re-offset row by row."""
    a = shards[0]
    for b in shards[1:]:
        if set(b.dims) != set(a.dims) or set(b.metrics) != set(a.metrics):
            raise ValueError("shards of different schemas")
        for k, d in a.dims.items():
            if len(d.dictionary) != len(b.dims[k].dictionary):
                raise ValueError(f"dimension {k!r}: shards were encoded with different dictionaries")
    dev = a.device
    units = {s.time_unit_ms for s in shards}
    unit = min(units)
    th = np.concatenate([s.time_host.astype(np.int64) * (s.time_unit_ms // unit) for s in shards])
    perm_h = np.argsort(th, kind="stable")
    perm = torch.from_numpy(perm_h).to(dev)
    n = len(th)

    def cat(get):
        return torch.cat([get(s)[: s.num_rows] for s in shards])

    time_units = torch.from_numpy(th[perm_h]).to(dev)
    dim_ids = {k: cat(lambda s, k=k: s.dims[k].ids)[perm] for k in a.dims}
    dicts = {k: d.dictionary for k, d in a.dims.items()}
    mdata = {k: cat(lambda s, k=k: s.metrics[k].data)[perm] for k in a.metrics}
    ds = make_datasource(a.name, n, time_units, unit, dim_ids, dicts, mdata, {k: m.kind for k, m in a.metrics.items()},
                         {k: m.scale for k, m in a.metrics.items()}, a.segment_granularity, a.query_granularity,
                         a.partition, a.num_partitions, [k for k, d in a.dims.items() if d.spatial])
    for k, m in a.metrics.items():
        if m.sketch is None:
            continue
        offs, vals, base = [], [], 0
        for s in shards:
            sk = s.metrics[k].sketch
            offs.append(sk.offsets[:-1] + base)
            vals.append(sk.values)
            base += int(sk.values.numel())
        start = torch.cat(offs)
        allv = torch.cat(vals)
        cnt = torch.cat([s.metrics[k].sketch.offsets.diff() for s in shards])
        start, cnt = start[perm], cnt[perm]
        new_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        new_off[1:] = torch.cumsum(cnt, 0)
        idx = torch.repeat_interleave(start - new_off[:-1], cnt) + torch.arange(int(cnt.sum()), device=dev)
        ds.metrics[k].sketch = SketchColumn(k, m.sketch.kind, new_off, allv[idx].contiguous(), m.sketch.p,
                                            m.sketch.salt, m.sketch.size)
    ds.shard_key = a.shard_key
    ds.spatial = getattr(a, "spatial", {})
    ds.rollup = getattr(a, "rollup", False)
    ds.global_num_rows = a.global_num_rows
    ds.build_indexes(bitmap_max_card=max((d.cardinality for d in a.dims.values() if d.bitmap is not None),
                                         default=0))
    return ds


def build_bitmap(ids: torch.Tensor, num_rows: int, card: int) -> torch.Tensor:
    """Inverted bitmap index [card, nwords] (u64 words as int64)."""
    P = ids.numel()
    nwords = P // 64
    out = torch.zeros((card, nwords), dtype=torch.int64, device=ids.device)
    if ids.is_cuda:
        from ..ops import native

        native.bitmap_build(ids, num_rows, out, card)
        return out
    v = ids[:num_rows].to(torch.int64)
    words = torch.arange(num_rows, dtype=torch.int64) // 64
    bits = torch.ones(num_rows, dtype=torch.int64) << (torch.arange(num_rows, dtype=torch.int64) % 64)
    flat = out.view(-1)
    # each (value, word) cell gets the OR of its row bits; bits are disjoint so sum == OR
    flat.index_add_(0, v * nwords + words, bits)
    return out


def make_datasource(name: str, num_rows: int, time_units: torch.Tensor, time_unit_ms: int,
                    dim_ids: Dict[str, torch.Tensor], dictionaries: Dict[str, Dictionary],
                    metric_data: Dict[str, torch.Tensor], metric_kinds: Dict[str, str],
                    metric_scales: Optional[Dict[str, int]] = None, segment_granularity: str = "month",
                    query_granularity: str = "none", partition: int = 0, num_partitions: int = 1,
                    spatial_dims: Sequence[str] = ()) -> DataSource:
    """Assemble a datasource from time-sorted unpadded columns (narrowing id types)."""
    dev = time_units.device
    dims = {}
    for k, ids in dim_ids.items():
        card = len(dictionaries[k])
        dt = TORCH_DT[id_dtype_for(card)]
        dims[k] = DimColumn(k, dictionaries[k], _pad(ids.to(dt), num_rows), spatial=k in spatial_dims)
    mets = {}
    for k, data in metric_data.items():
        mets[k] = MetricColumn(k, metric_kinds[k], _pad(data, num_rows), (metric_scales or {}).get(k, 0))
    th = time_units[:num_rows].cpu().numpy().astype(np.int64)
    last = int(th[-1]) if num_rows else 0
    tpad = _pad(time_units.to(torch.int32), num_rows, fill=last)
    return DataSource(name, num_rows, tpad, time_unit_ms, dims, mets, segment_granularity, query_granularity,
                      partition, num_partitions, time_host=th)
