"""A partitioned group-by run uses the layout its buffers were built for (engine/device_exec.py
PreparedScan._run_part_on), never the scan's current one.

Concurrent statements share prepared plans, so two execution slots can run one PreparedScan at
once; a hash-partitioned scan re-lays itself out after a run (sub-bucket overflow: 4x the buckets;
far fewer groups than estimated: fewer buckets), and a literal-specialized kernel swapped in may
carry another resident grid.  A run that picked up the new bucket count with buffers sized for the
old one wrote past them -- the serving fault under 64 BI clients.  Checked here with the native
launches recorded instead of run (no GPU)."""
from types import SimpleNamespace

import torch

from spark_druid_olap_amd.engine import device_exec as DE
from spark_druid_olap_amd.ops import desc as D


class _FakeNative:
    def __init__(self):
        self.calls = []

    def module_launch(self, handle, desc, grid, block, lds, stream):
        self.calls.append(("launch", handle, grid))

    def part_scan(self, counts, rows, cols, totals, base, stream):
        self.calls.append(("scan", rows, cols))

    def part_split(self, recs, rw, seg_lo, seg_hi, groups, spg, k, shift, p, counts, base, out, phase, stream):
        self.calls.append(("split", groups, spg, k, shift, p, phase))

    def part_agg_hll(self, recs, rw, base, nsub, G, shift, *rest):
        self.calls.append(("agg", nsub, shift))


def _layout(p1: int, shift: int) -> dict:
    return {"levels": 1, "shift": shift, "shift1": shift, "p1": p1, "p2": 1, "k": 1, "nsub": p1,
            "fields": [(0, 1)], "rw": 2, "nhll": 0}


def test_partitioned_run_uses_its_buffers_layout_and_grid(monkeypatch):
    nat = _FakeNative()
    monkeypatch.setattr(DE.native, "load", lambda: nat)
    monkeypatch.setattr(DE.native, "_stream", lambda dev: 0)
    old, new = _layout(64, 5), _layout(256, 3)
    sc = DE.PreparedScan.__new__(DE.PreparedScan)
    sc.prog = SimpleNamespace(G=2048, slots=[(D.S_SUM_I, 0)], hll_p=11)
    sc.dev = torch.device("cpu")
    sc.jit = SimpleNamespace(handle=7, lay=SimpleNamespace(total=4096))
    sc.part_having = sc.part_topk = None
    # another slot re-laid the scan out (and swapped in a kernel with another grid) after these
    # buffers were built
    sc.part, sc.grid = new, 999
    u32 = torch.int32
    grid = 12
    pb = {"L": old, "grid": grid, "k1": grid, "npos": grid * 8, "nch": 40, "cap_words": 64, "desc_recs": 0,
          "seg_lo": torch.zeros(grid * 8, dtype=u32), "pend": torch.zeros(grid * 8, dtype=u32),
          "counts1": torch.zeros(old["p1"] * grid, dtype=u32), "totals1": torch.zeros(old["p1"], dtype=u32),
          "base1": torch.zeros(old["p1"] + 1, dtype=u32)}
    b = SimpleNamespace(part=pb, desc=torch.zeros(D.SCANDESC.itemsize, dtype=torch.uint8),
                        acc=torch.zeros((2048, 1), dtype=torch.int64), hll=[])
    slab = SimpleNamespace(recs1=torch.zeros(64, dtype=u32), recs2=torch.zeros(64, dtype=u32))
    assert sc._run_part_on(b, slab) is None
    assert ("launch", 7, grid) in nat.calls
    assert ("scan", old["p1"], grid) in nat.calls
    splits = [c for c in nat.calls if c[0] == "split"]
    assert splits and all(c[3] == grid and c[4] == old["shift1"] and c[5] == old["p1"] for c in splits)
    assert ("agg", old["nsub"], old["shift"]) in nat.calls


def test_layout_packs_a_small_field_of_wide_records_only(ds_small, monkeypatch):
    """part_layout's record packing (engine/device_exec.py _pack_field): a non-negative integer sum
    whose values fit the key word's bits above shift1 rides in the key word after level 1 -- for
    3+ word records only; wide value ranges, negative values and 2-word records stay unpacked."""
    from spark_druid_olap_amd.engine.lower import Lowerer
    from spark_druid_olap_amd.query import spec as S

    def layout(aggs):
        prog = Lowerer(ds_small).lower_aggregate(["1992-01-01/1999-01-01"], None,
                                                 [S.DefaultDimensionSpec("o_orderkey")], None, aggs)
        return DE.part_layout(prog)

    q = S.FunctionAggregationSpec("longSum", "q", "l_quantity")
    tp = S.FunctionAggregationSpec("longSum", "tp", "o_totalprice")
    L = layout([tp, q])  # key + two i32 sums: 3 words
    assert L["rw"] == 3 and L.get("pack") is not None
    j, word = L["pack"]
    assert L["rw1"] == 2 and L["agg_fields"][j][1] == 3 | (L["shift1"] << 8)
    assert [f for i, f in enumerate(L["agg_fields"]) if i != j] == [f for i, f in enumerate(L["fields"]) if i != j]
    assert "pack" not in layout([q])  # 2-word records: unpacked
    monkeypatch.setattr(DE, "_value_range", lambda ds, name: (-5, 10))
    assert "pack" not in layout([tp, q])  # negative values never pack
    monkeypatch.setattr(DE, "_value_range", lambda ds, name: (0, 1 << 31))
    assert "pack" not in layout([tp, q])  # too wide for the free bits
    monkeypatch.setattr(DE, "PACK_RECORDS", False)
    monkeypatch.setattr(DE, "_value_range", lambda ds, name: (0, 10))
    assert "pack" not in layout([tp, q])
