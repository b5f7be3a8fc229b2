"""Bit-packed copies of integer columns for the scan kernels.

A Druid segment stores dictionary-encoded dimensions with the narrowest byte width the
dictionary allows and compresses metric columns (``CompressedVSizeIndexedSupplier`` /
compressed longs in Druid 0.9).  The MI355X scan kernels read columns packed to the exact bit
width of their value range instead of their byte width, in a layout built for the vector memory
path of CDNA4:

* frame of reference: ``value = base + field``, ``field`` in ``[0, 2^W)``, ``W`` = bits of
  ``max - min`` (the shard's own range, so every rank packs its shard independently);
* the kernels' unit is a 64-row word (row ``64 w + l`` belongs to lane ``l``) inside a 4096-row
  chunk; a chunk is two groups of 32 words, and in each group lane ``l`` owns a ``W``-dword
  stream holding its 32 rows' fields back to back (word ``j`` of the group at stream bits
  ``[j W, j W + W)``);
* stream dword ``k`` of lane ``l`` sits at dword ``k * 64 + l`` of the group: ONE 256-byte,
  fully coalesced dword load per stream dword serves the whole wave, and a run of ``U`` words is
  ``U W / 32`` such loads (+1) whose field offsets are compile-time constants in the unrolled
  kernel (ops/jit.py).  The previous row-major word layout needed two dword loads per field per
  word, and the scan was bound by vector-memory address processing, not HBM: a Q1-shaped read
  of five packed columns and one u16 plane ran 1.49 ms (3.7 TB/s) in that layout and 0.91 ms
  (6.1 TB/s, the HBM ceiling) in this one (tools/stream_probe.py, profiles/r4).

A chunk is ``512 W`` bytes, as before.  u8 / u16 columns are packed even at their full width --
the gain there is the access pattern (one dword load per 32 / W words instead of a byte or short
load per word).

The decoded column stays resident next to the packed copy (HBM is 288 GB): the torch paths,
bitmap indexes, zone maps and the host read it; only the fused scan kernels (ops/jit.py) read the
packed bits.  ``unpack`` is the exact inverse used by the tests.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

ENABLED = True  # (tools / tests: False keeps every scan on the byte-wide columns)
CHUNK_ROWS = 4096        # ops/desc.py CHUNK_ROWS
GROUP_WORDS = 32         # words per lane stream
_PIECE_ROWS = 1 << 26    # packing works through the column in pieces (bounded temporaries)


@dataclass
class PackedColumn:
    data: torch.Tensor     # int32 [nchunks * 128 W + 128] (spare dwords: a lane's next stream dword)
    width: int             # W, bits per row
    base: int              # frame of reference: value = base + field
    nrows: int

    @property
    def chunk_bytes(self) -> int:
        return 512 * self.width

    @property
    def nbytes(self) -> int:
        return int(self.data.numel()) * 4


def _range(t: torch.Tensor, n: int):
    if n == 0:
        return 0, 0
    if t.dtype == torch.uint16:  # (no reductions on the bare unsigned dtype)
        lo = hi = None
        for r0 in range(0, n, _PIECE_ROWS):
            a, b = torch.aminmax(t[r0:min(n, r0 + _PIECE_ROWS)].to(torch.int32))
            lo = int(a) if lo is None else min(lo, int(a))
            hi = int(b) if hi is None else max(hi, int(b))
        return lo, hi
    lo, hi = torch.aminmax(t[:n])
    return int(lo), int(hi)


def width_for(lo: int, hi: int) -> int:
    return max(1, int(hi - lo).bit_length())


def worth_packing(t: torch.Tensor, width: int) -> bool:
    """Pack when it saves bytes, and always for 1- and 2-byte columns (the layout's dword loads
    replace a byte / short load per word)."""
    return width < 8 * t.element_size() or (t.element_size() <= 2 and width <= 16)


def _place(r: torch.Tensor, W: int):
    """(dword of the row's first bit, shift) for rows ``r`` (int64)."""
    c, w, lane = r >> 12, (r >> 6) & 63, r & 63
    g, j = w >> 5, w & 31
    bit = j * W
    return c * (128 * W) + g * (64 * W) + (bit >> 5) * 64 + lane, bit & 31


def pack(t: torch.Tensor, n: Optional[int] = None, lo: Optional[int] = None, hi: Optional[int] = None) -> PackedColumn:
    """Bit-pack the first ``n`` values of integer tensor ``t`` (any device)."""
    n = int(t.numel() if n is None else n)
    if lo is None or hi is None:
        lo, hi = _range(t, n)
    W = width_for(lo, hi)
    if W > 32:
        raise ValueError("value range wider than 32 bits")
    nchunks = (n + CHUNK_ROWS - 1) // CHUNK_ROWS
    out = torch.zeros(nchunks * 128 * W + 128, dtype=torch.int32, device=t.device)
    m32 = (1 << 32) - 1

    def to_i32(x):  # u32 bit patterns -> int32 (adding disjoint bit patterns == OR-ing them)
        return torch.where(x >= (1 << 31), x - (1 << 32), x).to(torch.int32)

    for r0 in range(0, n, _PIECE_ROWS):
        r1 = min(n, r0 + _PIECE_ROWS)
        u = t[r0:r1].to(torch.int64) - lo                      # [0, 2^W)
        r = torch.arange(r0, r1, dtype=torch.int64, device=t.device)
        dw, sh = _place(r, W)
        out.index_add_(0, dw, to_i32(torch.bitwise_left_shift(u, sh) & m32))
        spill = sh + W > 32
        if bool(spill.any()):
            out.index_add_(0, dw[spill] + 64, to_i32(torch.bitwise_right_shift(u[spill], 32 - sh[spill])))
        del u, r, dw, sh, spill
    return PackedColumn(out, W, int(lo), n)


def unpack(pc: PackedColumn) -> torch.Tensor:
    """Decode every row (int64) -- the kernels' two-dword window / shift / mask."""
    n, W = pc.nrows, pc.width
    r = torch.arange(n, dtype=torch.int64, device=pc.data.device)
    dw, sh = _place(r, W)
    d32 = pc.data.to(torch.int64) & 0xFFFFFFFF
    word = d32[dw] | (d32[dw + 64] << 32)
    field = torch.bitwise_right_shift(word, sh) & ((1 << W) - 1)
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
    if not t.is_floating_point() and t.dtype in (torch.uint8, torch.int16, torch.uint16, torch.int32, torch.int64) \
            and t.device.type == "cuda":
        n = int(ds.num_rows)
        lo, hi = _range(t, n)
        W = width_for(lo, hi)
        if W <= 32 and worth_packing(t, W) and n > 0:
            pc = pack(t, n, lo, hi)
    from ..utils.streams import publish

    cache[name] = publish(pc, t.device)  # (every slot's stream reads it: complete before it is visible)
    return pc
