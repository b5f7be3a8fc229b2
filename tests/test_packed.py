"""Bit-packed column copies for the scan kernels (segment/packed.py): exact round trip at every
width 1..32, frame-of-reference bases (negative values), partial last chunks; and the
lane-interleaved layout the kernels read decodes every row -- the per-word window of ld_il (stream
dwords k and k + 1 of lane l, 256 B apart) and the static U-word runs of ops/jit.py stage_words
(the run's stream dwords loaded once, compile-time field offsets)."""
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
        assert pc.data.numel() == ((n + 4095) // 4096) * 128 * W + 128
        assert torch.equal(unpack(pc), v)


def _dw(raw, i):
    return int.from_bytes(raw[4 * i: 4 * i + 4].tobytes(), "little")


def test_kernel_lane_window_decodes_every_row():
    """Emulate the JIT's per-lane reads on the packed bytes (numpy, little endian)."""
    g = torch.Generator().manual_seed(3)
    for W in (1, 5, 16, 17, 24, 31, 32):
        n = 4096 + 64 * 5 + 9
        v = torch.randint(0, 2 ** W, (n,), generator=g, dtype=torch.int64)
        pc = pack(v)
        raw = pc.data.numpy().view(np.uint8)
        for r in range(n):
            chunk, word, lane = r >> 12, (r >> 6) & 63, r & 63
            gq, j = word >> 5, word & 31
            soff = chunk * 512 * W + gq * 256 * W + (((j * W) >> 5) << 8)  # ld_il: soffset + lane * 4
            x = _dw(raw, (soff >> 2) + lane) | (_dw(raw, (soff >> 2) + 64 + lane) << 32)
            field = (x >> ((j * W) & 31)) & ((1 << W) - 1)
            assert field + pc.base == int(v[r]), (W, r)


@pytest.mark.parametrize("U", [4, 8, 16])
def test_static_runs_decode_every_row(U):
    """ops/jit.py static runs: words g*32 + j0 + u of a chunk from the run's stream dwords
    k0..k1 (one load each) at compile-time bit offsets (j0 + u) W - 32 k0."""
    g = torch.Generator().manual_seed(U)
    for W in (1, 2, 14, 16, 17, 24, 32):
        n = 2 * 4096
        v = torch.randint(0, 2 ** W, (n,), generator=g, dtype=torch.int64)
        pc = pack(v)
        raw = pc.data.numpy().view(np.uint8)
        for chunk in range(2):
            for gq in range(2):
                for j0 in range(0, 32, U):
                    k0, k1 = (j0 * W) >> 5, ((j0 + U) * W - 1) >> 5
                    for lane in (0, 1, 31, 62, 63):
                        xd = [_dw(raw, ((chunk * 512 * W + gq * 256 * W + (k0 + k) * 256) >> 2) + lane)
                              for k in range(k1 - k0 + 1)] + [0]
                        for u in range(U):
                            b = (j0 + u) * W - 32 * k0
                            x = xd[b >> 5] | (xd[(b >> 5) + 1] << 32)
                            r = chunk * 4096 + (gq * 32 + j0 + u) * 64 + lane
                            assert ((x >> (b & 31)) & ((1 << W) - 1)) + pc.base == int(v[r]), (W, U, r)


def test_narrow_types_and_worth():
    ids = torch.tensor([0, 1, 2, 2, 1, 0] * 50, dtype=torch.uint8)
    pc = pack(ids)
    assert pc.width == 2 and torch.equal(unpack(pc), ids.to(torch.int64))
    assert worth_packing(ids, 2) and worth_packing(ids, 8)  # (u8 / u16: the layout's dword loads)
    assert worth_packing(torch.zeros(1, dtype=torch.int32), 31) and not worth_packing(torch.zeros(1, dtype=torch.int32), 32)
    assert width_for(5, 5) == 1 and width_for(0, 255) == 8 and width_for(-3, 4) == 3
