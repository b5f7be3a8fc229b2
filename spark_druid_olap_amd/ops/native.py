"""Loader for the in-tree HIP extension (``_sdo_native``).

Policy: on a machine with a GPU the native extension is REQUIRED -- a missing or stale build
raises instead of silently falling back to torch (fallbacks would hide "native code not
loaded").  On a CPU-only machine (CI, this container) the engine uses the torch reference
executor in ``ops/reference.py`` and this module is only imported for layout checks.
"""
from __future__ import annotations

import importlib
import os
import threading

from typing import Optional, Sequence

import torch

_lock = threading.Lock()
_mod = None


class NativeUnavailable(RuntimeError):
    pass


def loaded():
    """The extension module if some caller already loaded it, else None (never builds or imports)."""
    return _mod


def load(build_if_missing: bool = True):
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        from . import build as _build

        alt = os.environ.get("SDO_NATIVE_SO")
        if alt:
            # an instrumented build of the same module (tools/asan_host.py: host-side ASan)
            import sys
            from importlib import util as _ilu

            name = "spark_druid_olap_amd.ops._sdo_native"
            spec = _ilu.spec_from_file_location(name, alt)
            _mod = _ilu.module_from_spec(spec)
            spec.loader.exec_module(_mod)
            sys.modules[name] = _mod
            return _mod
        if not _build.target_path().exists():
            if not build_if_missing:
                raise NativeUnavailable(f"native extension missing: {_build.target_path()}")
            _build.build()
        elif build_if_missing and os.environ.get("SDO_REBUILD", "1") != "0" and not _build.is_fresh():
            try:
                _build.build()
            except Exception as e:  # pragma: no cover - no compiler on the box
                raise NativeUnavailable(f"native extension is stale and rebuild failed: {e}") from e
        _mod = importlib.import_module("spark_druid_olap_amd.ops._sdo_native")
        return _mod


_narrow4 = None


def narrow4() -> int:
    """1 if 1/2-byte LDS-DMA elements land at lane*4 on this GPU (probed once per process)."""
    global _narrow4
    if _narrow4 is None:
        r = load().glds_probe()
        if r not in (1, 4):
            raise NativeUnavailable(f"unexpected LDS-DMA layout (probe={r})")
        _narrow4 = 1 if r == 4 else 0
    return _narrow4


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(dev=None) -> int:
    """The calling thread's current HIP stream handle for ``dev``.  The raw accessor skips
    ``torch.cuda.current_stream``'s Stream object and device-index parsing (~7 us per call on the
    benchmark host, three calls per small query)."""
    if _RAW_STREAM is not None:
        idx = dev.index if isinstance(dev, torch.device) and dev.index is not None else \
            (dev if isinstance(dev, int) else torch.cuda.current_device())
        return _RAW_STREAM(idx)
    return torch.cuda.current_stream(dev).cuda_stream


def scan(desc: torch.Tensor, grid: int, block: int, lds: int, unroll: int) -> None:
    m = load()
    m.scan(desc.data_ptr(), int(grid), int(block), int(lds), int(unroll), _stream(desc.device))


def bitmap_build(ids: torch.Tensor, num_rows: int, out: torch.Tensor, card: int) -> None:
    from ..segment.datasource import dtype_code

    m = load()
    nwords = out.shape[1]
    m.bitmap_build(ids.data_ptr(), dtype_code(ids), int(num_rows), int(nwords), out.data_ptr(), int(card),
                   _stream(ids.device))


def hll_estimate(regs: torch.Tensor, G: int, p: int, est: torch.Tensor) -> None:
    m = load()
    assert regs.dtype == torch.uint8 and regs.is_contiguous() and regs.numel() >= G * (1 << p)
    assert est.dtype == torch.float64 and est.numel() >= G
    m.hll_estimate(regs.data_ptr(), int(G), int(p), est.data_ptr(), _stream(regs.device))


def reset_bufs(acc: Optional[torch.Tensor], init: torch.Tensor, zeros: Sequence[torch.Tensor],
               overflow: Optional[torch.Tensor]) -> None:
    """One launch: ``acc[r, s] = init[s]`` for every row, every tensor in ``zeros`` (<= 4, sizes a
    multiple of 8 bytes) set to 0, ``overflow[0] = 0``."""
    m = load()
    dev = init.device
    zp, zw = [], []
    for z in zeros:
        nb = z.numel() * z.element_size()
        assert z.is_contiguous() and nb % 8 == 0
        zp.append(z.data_ptr())
        zw.append(nb // 8)
    if acc is not None:
        assert acc.dtype == torch.int64 and acc.is_contiguous() and acc.dim() == 2 and acc.shape[1] == init.numel()
    m.reset_bufs(acc.data_ptr() if acc is not None else 0, init.data_ptr(), int(acc.shape[0]) if acc is not None else 0,
                 int(init.numel()), zp, zw, overflow.data_ptr() if overflow is not None else 0, _stream(dev))


def device_info(dev: int = 0) -> dict:
    return load().device_info(dev)


def theta_select(g: torch.Tensor, h: torch.Tensor, G: int, target: torch.Tensor, bits: int):
    """Candidates of a per-group KMV selection (sketch.hip theta_*): (g, h) pairs whose hash lies
    below their group's bound -- the first top-``bits`` bin at which the group's running pair count
    reaches ``target[g]`` -- plus the bounds.  Pairs are int64 on the device; ``g`` in [0, G)."""
    m = load()
    assert g.dtype == torch.int64 and h.dtype == torch.int64 and g.is_cuda and g.numel() == h.numel()
    assert target.dtype == torch.int64 and target.numel() == G
    dev = g.device
    n = g.numel()
    hist = torch.empty(G << bits, dtype=torch.int32, device=dev)
    bound = torch.empty(G, dtype=torch.int64, device=dev)
    count = torch.zeros(1, dtype=torch.int64, device=dev)
    cap = int(min(n, int(target.sum()) * 2 + (1 << 16)))
    st = _stream(dev)
    while True:
        og = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        oh = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        m.theta_select(g.data_ptr(), h.data_ptr(), n, G, bits, hist.data_ptr(), target.data_ptr(), bound.data_ptr(),
                       og.data_ptr(), oh.data_ptr(), count.data_ptr(), cap, st)
        c = int(count.item())
        if c <= cap:
            return og[:c], oh[:c], bound
        cap = c  # a duplicate-heavy bin held more candidates than the first guess: select again


def compact_rows(mask: torch.Tensor) -> torch.Tensor:
    """Row ids (int64, ascending) of the set bits of a [nwords] int64 mask (post_scan.hip
    compact_*: popcount per 65536-row block, one-workgroup offset scan, scatter).  Temporaries are
    O(nwords / 1024); the output is exactly the selected rows."""
    m = load()
    assert mask.dtype == torch.int64 and mask.is_contiguous() and mask.is_cuda
    nw = mask.numel()
    dev = mask.device
    nb = (nw + 1023) // 1024
    if nb == 0:
        return torch.zeros(0, dtype=torch.int64, device=dev)
    counts = torch.empty(nb, dtype=torch.int32, device=dev)
    offs = torch.empty(nb, dtype=torch.int64, device=dev)
    total = torch.empty(1, dtype=torch.int64, device=dev)
    st = _stream(dev)
    m.compact_count(mask.data_ptr(), nw, counts.data_ptr(), offs.data_ptr(), total.data_ptr(), st)
    n = int(total.item())
    rows = torch.empty(n, dtype=torch.int64, device=dev)
    if n:
        m.compact_write(mask.data_ptr(), nw, offs.data_ptr(), rows.data_ptr(), st)
    return rows


def topk_keep(acc: torch.Tensor, slot: int, is_f64: bool, desc: bool, k: int) -> torch.Tensor:
    """Indices (ascending) of the rows of ``acc`` [R, nslots] int64 whose slot value ties or beats
    the bucket of the k-th best (post_scan.hip topk_*: 4-level 12-bit radix select, no host
    round trip until the final compaction): a superset of the top k, exact after an order+limit."""
    m = load()
    assert acc.dtype == torch.int64 and acc.is_contiguous() and acc.dim() == 2 and acc.is_cuda
    R, ns = acc.shape
    dev = acc.device
    state = torch.tensor([0, int(k), 0], dtype=torch.int64, device=dev)
    hist = torch.zeros(4096, dtype=torch.int32, device=dev)
    keep = torch.empty((R + 63) // 64, dtype=torch.int64, device=dev)
    grid = int(max(1, min(2048, (R + 4095) // 4096)))
    m.topk_keep(acc.data_ptr(), R, ns, int(slot), int(bool(is_f64)), int(bool(desc)), state.data_ptr(),
                hist.data_ptr(), keep.data_ptr(), grid, _stream(dev))
    return compact_rows(keep)


def nonzero_rows(col: torch.Tensor) -> torch.Tensor:
    """Indices (int64, ascending) of the non-zero elements of a 1-D (possibly strided) int64 or
    uint8 device tensor: ballot mask (post_scan.hip nonzero_mask) + compact_rows.  Replaces
    ``torch.nonzero`` for group-existence compaction of dense accumulator tables."""
    m = load()
    assert col.dim() == 1 and col.is_cuda and col.dtype in (torch.int64, torch.uint8)
    n = col.numel()
    if n == 0:
        return torch.zeros(0, dtype=torch.int64, device=col.device)
    words = torch.empty((n + 63) // 64, dtype=torch.int64, device=col.device)
    m.nonzero_mask(col.data_ptr(), col.element_size(), n, col.stride(0), words.data_ptr(), _stream(col.device))
    return compact_rows(words)


def touch_compact(touch: torch.Tensor, acc: torch.Tensor, init_row: torch.Tensor):
    """(group ids, accumulator rows) of the groups a first-touch byte table marks, with those rows
    re-initialised to ``init_row`` and their bytes cleared (post_scan.hip touch_*: fused mask +
    count pass, offset scan, one gather / re-init / clear pass).  ``touch`` holds a multiple of 64
    bytes covering every row of ``acc`` [rows, nslots] int64."""
    m = load()
    rows, ns = acc.shape
    nw = (rows + 63) // 64
    assert touch.dtype == torch.uint8 and touch.is_contiguous() and touch.numel() >= nw * 64
    assert acc.dtype == torch.int64 and acc.is_contiguous() and init_row.numel() == ns
    dev = acc.device
    nb = (nw + 1023) // 1024
    words = torch.empty(max(nw, 1), dtype=torch.int64, device=dev)
    counts = torch.empty(max(nb, 1), dtype=torch.int32, device=dev)
    offs = torch.empty(max(nb, 1), dtype=torch.int64, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    st = _stream(dev)
    m.touch_count(touch.data_ptr(), nw, words.data_ptr(), counts.data_ptr(), offs.data_ptr(), total.data_ptr(), st)
    n = int(total.item())
    idx = torch.empty(n, dtype=torch.int64, device=dev)
    out = torch.empty((n, ns), dtype=torch.int64, device=dev)
    if n:
        m.touch_gather(words.data_ptr(), nw, offs.data_ptr(), acc.data_ptr(), ns, init_row.data_ptr(),
                       touch.data_ptr(), idx.data_ptr(), out.data_ptr(), st)
    return idx, out


def histogram(keys: torch.Tensor, nbins: int) -> torch.Tensor:
    """int64 counts per bin of int64 ids in [0, nbins) (post_scan.hip histogram_kernel: 32-bit
    device atomics, no min/max pre-pass); replaces ``torch.bincount`` for nested count levels."""
    m = load()
    assert keys.dim() == 1 and keys.is_cuda and keys.dtype == torch.int64 and keys.is_contiguous()
    assert keys.numel() < (1 << 32)
    if nbins > PART_HIST_MIN_BINS and keys.numel() >= PART_HIST_MIN_KEYS and nbins < (1 << 32):
        return part_histogram(keys, nbins)
    counts = torch.zeros(nbins, dtype=torch.int32, device=keys.device)
    m.histogram(keys.data_ptr(), keys.numel(), nbins, counts.data_ptr(), _stream(keys.device))
    return counts.to(torch.int64)


# Bins beyond the LDS histogram: one random 32-bit device atomic per key runs at the ~20 G/s
# random-update rate (TPC-H Q13: 149M orders into 15M customer bins, 7.5 ms); the radix-partitioned
# path (partition.hip) moves the keys twice at streaming bandwidth and counts in LDS.
PART_HIST_MIN_BINS = 1 << 16
PART_HIST_MIN_KEYS = 1 << 20


def part_histogram(keys: torch.Tensor, nbins: int) -> torch.Tensor:
    """int64 counts per bin via part_keys -> [part_split] -> part_agg (implicit count records)."""
    m = load()
    dev = keys.device
    st = _stream(dev)
    n = keys.numel()
    shift = 12                                   # 4096 int64 counters = 32 KB of LDS per sub-bucket
    gbits = max(1, (nbins - 1).bit_length())
    rem = max(0, gbits - shift)
    if rem <= 10:
        b1, b2 = rem, 0
    else:
        b1 = min(10, (rem + 1) // 2)
        b2 = rem - b1
    P1, P2 = 1 << b1, 1 << b2
    grid = int(max(1, min(2048, (n + 4095) // 4096)))
    u32 = torch.int32
    recs1 = torch.empty(n, dtype=u32, device=dev)
    c1 = torch.empty(P1 * grid, dtype=u32, device=dev)
    t1 = torch.empty(P1, dtype=u32, device=dev)
    base1 = torch.empty(P1 + 1, dtype=u32, device=dev)
    s1 = shift + b2
    m.part_keys(keys.data_ptr(), n, s1, P1, c1.data_ptr(), 0, recs1.data_ptr(), 0, grid, st)
    m.part_scan(c1.data_ptr(), P1, grid, t1.data_ptr(), base1.data_ptr(), st)
    m.part_keys(keys.data_ptr(), n, s1, P1, c1.data_ptr(), base1.data_ptr(), recs1.data_ptr(), 1, grid, st)
    recs, base, nsub = recs1, base1, P1
    if b2:
        K = max(1, min(64, 4096 // P1))
        recs2 = torch.empty_like(recs1)
        c2 = torch.empty(P1 * P2 * K, dtype=u32, device=dev)
        t2 = torch.empty(P1 * P2, dtype=u32, device=dev)
        base2 = torch.empty(P1 * P2 + 1, dtype=u32, device=dev)
        b1p = base1.data_ptr()
        args = (recs1.data_ptr(), 1, b1p, b1p + 4, P1, 1, K, shift, P2, c2.data_ptr())
        m.part_split(*args, 0, 0, 0, st)
        m.part_scan(c2.data_ptr(), P1 * P2, K, t2.data_ptr(), base2.data_ptr(), st)
        m.part_split(*args, base2.data_ptr(), recs2.data_ptr(), 1, st)
        recs, base, nsub = recs2, base2, P1 * P2
    out = torch.empty(nbins, dtype=torch.int64, device=dev)
    m.part_agg(recs.data_ptr(), 1, base.data_ptr(), nsub, nbins, shift, [0], [0], [0], [0], out.data_ptr(),
               [], 1, 0, 0, 0, st)
    return out


def hll_pairs(vals: torch.Tensor, p: int, salt: int) -> torch.Tensor:
    """Packed (bucket << 8 | rho) int32 HLL pair of every 64-bit value (sketch.hip hll_pairs)."""
    m = load()
    v = vals.to(torch.int64).contiguous()
    assert v.is_cuda
    out = torch.empty(v.numel(), dtype=torch.int32, device=v.device)
    m.hll_pairs(v.data_ptr(), v.numel(), int(p), int(salt), out.data_ptr(), _stream(v.device))
    return out


def hll_merge_stored(regs: torch.Tensor, rows: torch.Tensor, gid: torch.Tensor, offsets: torch.Tensor,
                     pairs: torch.Tensor, p: int) -> None:
    """Union the stored sparse HLL sketches of ``rows`` into ``regs[gid[i]]`` (sketch.hip
    hll_merge_stored); ``regs`` is [G, 2^p] uint8 (byte registers), gid < 0 skips a row."""
    m = load()
    G = regs.shape[0]
    assert regs.dtype == torch.uint8 and regs.is_contiguous() and regs.shape[1] == (1 << p) and regs.is_cuda
    assert rows.dtype == torch.int64 and gid.dtype == torch.int64 and rows.numel() == gid.numel()
    assert offsets.dtype == torch.int64 and pairs.dtype == torch.int32
    if rows.numel():
        assert int(rows.max()) < offsets.numel() - 1 and int(rows.min()) >= 0
    m.hll_merge_stored(rows.contiguous().data_ptr(), gid.contiguous().data_ptr(), rows.numel(),
                       offsets.data_ptr(), pairs.data_ptr(), int(p), int(G), regs.data_ptr(), _stream(regs.device))


def run_scan(acc, init, rows, nslots, zptr, zwords, overflow, jit, desc, grid, block, lds, unroll, stream) -> None:
    """Fused buffer reset + scan kernel of a prepared scan (arguments cached by the caller)."""
    load().run_scan(acc, init, rows, nslots, zptr, zwords, overflow, jit, desc, grid, block, lds, unroll, stream)


def fetch_small(acc: torch.Tensor, hll: Sequence[torch.Tensor], G: int, p: int, est_dev: torch.Tensor,
                host: torch.Tensor) -> None:
    """HLL estimates of each register block + the accumulator table and the estimates into the
    pinned ``host`` buffer, then a stream sync -- one native call (bindings.cpp fetch_small)."""
    assert acc.is_contiguous() and host.is_pinned()
    nb = acc.numel() * acc.element_size()
    assert host.numel() * host.element_size() >= nb + len(hll) * G * 8
    assert est_dev.numel() * est_dev.element_size() >= len(hll) * G * 8
    for h in hll:
        assert h.dtype == torch.uint8 and h.is_contiguous() and h.numel() >= G * (1 << p)
    load().fetch_small(acc.data_ptr(), nb, [h.data_ptr() for h in hll], int(G), int(p), est_dev.data_ptr(),
                       host.data_ptr(), _stream(acc.device))



def fetch_small_reset(acc: torch.Tensor, hll: Sequence[torch.Tensor], G: int, p: int, est_dev: torch.Tensor,
                      host: torch.Tensor, reset_args: tuple) -> None:
    """``fetch_small`` + the scan's buffer reset for its next run enqueued behind the copies; waits
    for the copies only.  ``reset_args``: a prepared scan's cached (init, rows, nslots, zero
    pointers, zero words, overflow) -- the reset half of its fused launch arguments (the
    accumulator table reset is ``acc`` itself)."""
    nb = acc.numel() * acc.element_size()
    load().fetch_small_reset(acc.data_ptr(), nb, [h.data_ptr() for h in hll], int(G), int(p), est_dev.data_ptr(),
                             host.data_ptr(), *reset_args, _stream(acc.device))


def read_words(ts, dev) -> list:
    """Values of int64 device words (tensors' first elements) after this thread's stream work, with
    one copy and one wait (bindings.cpp read_words)."""
    for t in ts:
        assert t.is_cuda and t.element_size() in (4, 8) and t.numel() >= 1
    return list(load().read_words([t.data_ptr() for t in ts], [t.element_size() for t in ts], _stream(dev)))


def stream_sync(dev) -> None:
    load().stream_sync(_stream(dev))
