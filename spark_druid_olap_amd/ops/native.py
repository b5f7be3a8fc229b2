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

import torch

_lock = threading.Lock()
_mod = None


class NativeUnavailable(RuntimeError):
    pass


def load(build_if_missing: bool = True):
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        from . import build as _build

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


def _stream(dev=None) -> int:
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
    assert regs.dtype == torch.int32 and regs.is_contiguous() and regs.numel() >= G * (1 << p)
    assert est.dtype == torch.float64 and est.numel() >= G
    m.hll_estimate(regs.data_ptr(), int(G), int(p), est.data_ptr(), _stream(regs.device))


def device_info(dev: int = 0) -> dict:
    return load().device_info(dev)
