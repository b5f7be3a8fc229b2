"""Bit-packed copies of integer columns for the scan kernels.

A Druid segment stores dictionary-encoded dimensions with the narrowest byte width the
dictionary allows and compresses metric columns (``CompressedVSizeIndexedSupplier`` /
compressed longs in Druid 0.9).  The MI355X scan is HBM-bound on wide scans -- TPC-H Q1 reads
16 bytes per row at ~5.7 TB/s -- so the kernels read columns packed to the exact bit width of
their value range instead of their byte width:

* frame of reference: ``value = base + field``, ``field`` in ``[0, 2^W)``, ``W`` = bits of
  ``max - min`` (the shard's own range, so every rank packs its shard independently);
* 64-row words, the natural unit of the kernels (one row per lane of a wave): a word is ``W``
  64-bit integers (``8 W`` bytes) and row ``l`` of the word sits at bits ``[l W, l W + W)``;
* a lane reads the 8 bytes at the dword holding its first bit -- ``((l W) >> 5) * 4`` -- and
  shifts by ``(l W) & 31``: at most 31 + 32 bits, always inside that one 8-byte load, and the
  wave's 64 loads cover the word's ``8 W`` bytes contiguously (fully coalesced).

TPC-H Q1 / Basic Aggregation: returnflag 8 -> 2 bits, linestatus 8 -> 1, extendedprice 32 -> 24,
supplycost 32 -> 17, availqty 16 -> 14, orderkey 32 -> 28 (SF100): 16 -> 10.75 bytes per row.

The decoded column stays resident next to the packed copy (HBM is 288 GB): the torch paths,
bitmap indexes, zone maps and the host read it; only the fused scan kernels (ops/jit.py) read the
packed bits.  ``unpack`` is the exact inverse used by the tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch

ENABLED = os.environ.get("SDO_PACKED", "0") not in ("0", "")
_CHUNK_ROWS = 1 << 26   # packing works through the column in pieces (bounded temporaries)


@dataclass
class PackedColumn:
    data: torch.Tensor     # int64 [nwords * W + 1] (one spare word: the last lane's 8-byte read)
    width: int             # W, bits per row
    base: int              # frame of reference: value = base + field
    nrows: int

    @property
    def word_bytes(self) -> int:
        return 8 * self.width

    @property
    def nbytes(self) -> int:
        return int(self.data.numel()) * 8


def _range(t: torch.Tensor, n: int):
    if n == 0:
        return 0, 0
    lo, hi = torch.aminmax(t[:n])
    return int(lo), int(hi)


def width_for(lo: int, hi: int) -> int:
    return max(1, int(hi - lo).bit_length())


def worth_packing(t: torch.Tensor, width: int) -> bool:
    """Pack when it saves bytes: the packed width is below the stored width."""
    return width < 8 * t.element_size()


def pack(t: torch.Tensor, n: Optional[int] = None, lo: Optional[int] = None, hi: Optional[int] = None) -> PackedColumn:
    """Bit-pack the first ``n`` values of integer tensor ``t`` (any device)."""
    n = int(t.numel() if n is None else n)
    if lo is None or hi is None:
        lo, hi = _range(t, n)
    W = width_for(lo, hi)
    if W > 32:
        raise ValueError("value range wider than 32 bits")
    nwords = (n + 63) // 64
    out = torch.zeros(nwords * W + 1, dtype=torch.int64, device=t.device)
    for r0 in range(0, n, _CHUNK_ROWS):
        r1 = min(n, r0 + _CHUNK_ROWS)
        u = t[r0:r1].to(torch.int64) - lo                      # [0, 2^W)
        r = torch.arange(r0, r1, dtype=torch.int64, device=t.device)
        bit = (r >> 6) * (64 * W) + (r & 63) * W              # absolute bit offset of each row
        idx = bit >> 6
        sh = bit & 63
        # bits of different rows are disjoint, so adding the shifted fields is OR-ing them; the
        # 64-bit wrap of ``u << sh`` drops exactly the bits that spill into the next integer
        out.index_add_(0, idx, torch.bitwise_left_shift(u, sh))
        spill = sh + W > 64
        if bool(spill.any()):
            s_idx = idx[spill] + 1
            s_val = torch.bitwise_right_shift(u[spill], 64 - sh[spill])
            out.index_add_(0, s_idx, s_val)
        del u, r, bit, idx, sh, spill
    return PackedColumn(out, W, int(lo), n)


def unpack(pc: PackedColumn) -> torch.Tensor:
    """Decode every row (int64) -- the kernels' ``ld_pk`` / shift / mask, on the host or device."""
    n, W = pc.nrows, pc.width
    r = torch.arange(n, dtype=torch.int64, device=pc.data.device)
    lane_bit = (r & 63) * W
    dword = (r >> 6) * (2 * W) + (lane_bit >> 5)              # 32-bit unit holding the first bit
    sh = lane_bit & 31
    d32 = pc.data.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    lo32 = d32[dword]
    hi32 = d32[dword + 1]
    word = lo32 | (hi32 << 32)
    field = torch.bitwise_right_shift(word, sh) & ((1 << W) - 1)
    # (>> of a negative int64 is arithmetic; the mask keeps only the field's W bits)
    return field + pc.base


def packed_column(ds, name: str) -> Optional[PackedColumn]:
    """The packed copy of column ``name`` of a device-resident shard, built once and cached on the
    datasource; None when the column is not an integer column worth packing."""
    if not ENABLED:
        return None
    cache = ds.__dict__.setdefault("_packed", {})
    if name in cache:
        return cache[name]
    from ..engine.lower import column_tensor

    t = column_tensor(ds, name)
    pc = None
    if not t.is_floating_point() and t.dtype in (torch.uint8, torch.int16, torch.int32, torch.int64) and \
            t.device.type == "cuda":  # (not the u16 HLL code planes, segment/hllcode.py)
        n = int(ds.num_rows)
        lo, hi = _range(t, n)
        W = width_for(lo, hi)
        if W <= 32 and worth_packing(t, W) and n > 0:
            pc = pack(t, n, lo, hi)
    cache[name] = pc
    return pc
