"""Bit-packed column copies for the scan kernels (segment/packed.py): exact round trip at every
width 1..32, frame-of-reference bases (negative values), partial last words; and the word layout
the kernels' ld_pk / pk_field read (lane l of a word: the 8 bytes at dword (l W) >> 5, shift
(l W) & 31) decodes every row."""
import numpy as np
import pytest
import torch

from spark_druid_olap_amd.segment.packed import pack, unpack, width_for, worth_packing


@pytest.mark.parametrize("W", [1, 2, 3, 7, 12, 14, 17, 24, 28, 31, 32])
def test_roundtrip_every_width(W):
    g = torch.Generator().manual_seed(W)
    for n in (2, 63, 64, 65, 1000, 4097):
        lo = -7 if W < 32 else 0
        v = torch.randint(0, 2 ** W, (n,), generator=g, dtype=torch.int64) + lo
        v[0], v[-1] = lo, lo + 2 ** W - 1
        pc = pack(v)
        assert pc.width == W and pc.base == lo
        assert pc.data.numel() == ((n + 63) // 64) * W + 1
        assert torch.equal(unpack(pc), v)


def test_kernel_lane_window_decodes_every_row():
    """Emulate the JIT's per-lane read on the packed bytes (numpy, little endian)."""
    g = torch.Generator().manual_seed(3)
    for W in (1, 5, 17, 24, 31):
        n = 64 * 5 + 9
        v = torch.randint(0, 2 ** W, (n,), generator=g, dtype=torch.int64)
        pc = pack(v)
        raw = pc.data.numpy().view(np.uint8)
        for r in range(n):
            word, lane = divmod(r, 64)
            off = word * 8 * W + ((lane * W) >> 5) * 4
            x = int.from_bytes(raw[off: off + 8].tobytes(), "little")
            field = (x >> ((lane * W) & 31)) & ((1 << W) - 1)
            assert field + pc.base == int(v[r]), (W, r)


def test_narrow_types_and_worth():
    ids = torch.tensor([0, 1, 2, 2, 1, 0] * 50, dtype=torch.uint8)
    pc = pack(ids)
    assert pc.width == 2 and torch.equal(unpack(pc), ids.to(torch.int64))
    assert worth_packing(ids, 2) and not worth_packing(ids, 8)
    assert width_for(5, 5) == 1 and width_for(0, 255) == 8 and width_for(-3, 4) == 3
