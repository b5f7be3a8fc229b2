"""Slot-buffer hand-over between prepared scans of equal geometry (engine/device_exec.py _steal):
many parameterizations of one dashboard statement share one set of device buffers per execution
slot instead of one each; a scan the current statement has run (pinned) is never robbed."""
import threading
import weakref

import pytest
import torch

from spark_druid_olap_amd.engine import device_exec as DE
from spark_druid_olap_amd.engine.scheduler import pinned, use_slot


class _Fake:
    def __init__(self, geom):
        self._slot_lock = threading.Lock()
        b = DE._Bufs()
        b.geom = geom
        b.acc = torch.zeros(4)
        self._slots = {1: b}


def test_steal_respects_geometry_pins_and_slots():
    g1, g2 = ("cpu", 1, 100, 2, 0, 2048, False, True, False), ("cpu", 1, 200, 2, 0, 2048, False, True, False)
    a, b, c = _Fake(g1), _Fake(g1), _Fake(g2)
    for p in (a, b, c):
        DE._geom_register(p, 1, p._slots[1].geom)
    me = _Fake(g1)
    with use_slot(1):
        pinned().add(id(a))  # a ran in this statement: its buffers may hold live partials
        got = DE._steal(me, 1, g1)
        assert got is not None and got.geom == g1
        assert 1 not in b._slots and 1 in a._slots and 1 in c._slots  # b robbed, a pinned, c other shape
        assert DE._steal(me, 1, g1) is None  # nothing left but the pinned one
        assert DE._steal(me, 2, g1) is None  # other slots hold their own buffers
    assert not pinned()  # the slot's statement ended: pins released
    assert DE._steal(me, 1, g1) is not None  # now a may be handed over
    assert 1 not in a._slots


def test_no_handover_on_unleased_slot_zero():
    """Slot 0 is every unscheduled thread's: another thread may be running a scan there right now
    (advisor r4), so its buffers are never handed over and runs there pin nothing."""
    g = ("cpu", 1, 100, 2, 0, 2048, False, True, False)
    a = _Fake(g)
    a._slots = {0: a._slots[1]}
    DE._geom_register(a, 0, g)
    me = _Fake(g)
    assert DE._steal(me, 0, g) is None
    assert 0 in a._slots


@pytest.mark.gpu
def test_parameterizations_share_one_table_per_slot():
    """Two parameterizations of one large group-by (dense HBM table with a first-touch byte table)
    run alternately: the second takes over the first's table (same device pointer), the first
    takes it back, and both keep answering exactly as freshly prepared scans."""
    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.query import spec as S

    ds = tpch.to_datasource(tpch.generate_flat(0.2, "cuda"), profile="bench")

    def q(seg):
        return S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("o_orderkey")],
                                  aggregations=[S.FunctionAggregationSpec("doubleSum", "p", "l_extendedprice")],
                                  filter=S.SelectorFilterSpec("c_mktsegment", seg), intervals=["1992-01-01/1999-01-01"])

    eng = Engine()
    pa, pb = eng.prepare(q("BUILDING"), ds), eng.prepare(q("MACHINERY"), ds)
    ref_a, ref_b = Engine().execute(q("BUILDING"), ds), Engine().execute(q("MACHINERY"), ds)

    def rows(r):
        return sorted(zip(r.data["o_orderkey"].tolist(), [round(x, 6) for x in r.data["p"].tolist()]))

    ptrs = set()
    for i in range(3):
        with use_slot(1):
            ra = pa.run()
        with use_slot(1):
            rb = pb.run()
        assert rows(ra) == rows(ref_a) and rows(rb) == rows(ref_b), i
        for p in (pa, pb):
            sc = p.scans[0][2]
            if 1 in sc._slots:
                ptrs.add(sc._slots[1].acc.data_ptr())
    assert len(ptrs) == 1, "the parameterizations did not share the slot's table"
