"""Per-slot device arenas (engine/device_exec.py SlotArena): every leased execution slot carves the
large tensors of its current statement's scans from one bump-allocated arena that restarts with the
slot's next statement, so K slots hold K x the largest statement's need instead of one cached table
set per (prepared plan, slot) (the round-4 BI plan ran out of HBM at 6 slots that way)."""
import threading

import pytest
import torch

from spark_druid_olap_amd.engine import device_exec as DE
from spark_druid_olap_amd.engine.scheduler import slot_epoch, use_slot


class _Owner:
    def __init__(self):
        self._slot_lock = threading.Lock()
        self._slots = {}


def test_carve_restarts_per_statement_and_tracks_intact_regions():
    ar = DE.SlotArena("cpu", 91)
    a, b, c = _Owner(), _Owner(), _Owner()
    with use_slot(91):
        ga, oa, ia, _ = ar.carve(1000, a)
        gb, ob, ib, _ = ar.carve(5000, b)
    assert (oa, ob) == (0, 1024) and not ia and not ib  # 256-byte aligned bump, first carve: not intact
    with use_slot(91):  # the same statement again: the same offsets, contents as left
        assert ar.carve(1000, a)[:3] == (ga, 0, True)
        assert ar.carve(5000, b)[:3] == (gb, 1024, True)
    with use_slot(91):  # another statement carves over a's region
        assert ar.carve(3000, c)[1:3] == (0, False)
    with use_slot(91):
        assert ar.carve(1000, a)[1:3] == (0, False)   # a's bytes were overwritten by c
        assert ar.carve(5000, b)[2] is False          # c's 3072 bytes overlapped b's region too
    assert ar.cap == DE.ARENA_MIN  # one storage for all of it


def test_growth_keeps_earlier_views_and_sizes_for_the_whole_statement(monkeypatch):
    monkeypatch.setattr(DE, "ARENA_MIN", 4096)
    ar = DE.SlotArena("cpu", 92)
    a, b = _Owner(), _Owner()
    with use_slot(92):
        g0, off, _, buf = ar.carve(3000, a)
        va = DE.SlotArena.view(buf, off, 375, torch.int64)
        va.fill_(7)
        a._slots[92] = "bufs"
        g1, off_b, _, _ = ar.carve(6000, b)  # does not fit: a new storage, a's view stays valid
        assert g1 == g0 + 1 and off_b == 0
        assert int(va.sum()) == 7 * 375
        assert 92 not in a._slots  # a re-carves at its next run
    assert ar.cap >= 3072 + 6144  # the next statement fits whole
    with use_slot(92):
        assert ar.carve(3000, a)[:2] == (g1, 0)
        assert ar.carve(6000, b)[:2] == (g1, 3072)
    assert ar.gen == g1


def test_release_drops_other_arenas_only():
    a1, a2 = DE.slot_arena("cpu", 93), DE.slot_arena("cpu", 94)
    o1, o2 = _Owner(), _Owner()
    with use_slot(93):
        a1.carve(100, o1)
        o1._slots[93] = "x"
    with use_slot(94):
        a2.carve(100, o2)
        o2._slots[94] = "y"
    DE.release_device_memory(keep_arena=a2) if torch.cuda.is_available() else _release_no_cuda(a2)
    assert a1.buf is None and 93 not in o1._slots
    assert a2.buf is not None and o2._slots[94] == "y"


def _release_no_cuda(keep):
    for ar in list(DE._ARENAS.values()):
        if ar is not keep:
            ar.release()


def test_slot_epochs_count_statements():
    e = slot_epoch(95)
    with use_slot(95):
        assert slot_epoch(95) == e + 1
    with use_slot(95):
        pass
    assert slot_epoch(95) == e + 2


@pytest.mark.gpu
def test_parameterizations_share_the_slot_arena():
    """Two parameterizations of one large group-by (dense HBM table with a first-touch byte table)
    run alternately on slot 1: both carve the same arena region (same device pointer, no second
    table), each re-initialises it when the other wrote over it, and both answer exactly as
    freshly prepared scans on slot 0; a select (mask scan) carves from the arena too."""
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
        for p, ref in ((pa, ref_a), (pa, ref_a), (pb, ref_b)):  # (a twice: its intact re-run skips the reset)
            with use_slot(1):
                r = p.run()
                ptrs.add(p.scans[0][2]._slots[1].acc.data_ptr())
            assert rows(r) == rows(ref), i
    assert len(ptrs) == 1, "the parameterizations did not share the slot's arena region"
    ar = DE.slot_arena(ds.device, 1)
    # (sized for its own need -- or straight to a larger peer slot's size, set by earlier tests)
    peers = max((a.cap for k, a in DE._ARENAS.items() if k[0] == str(ds.device) and a is not ar), default=0)
    assert ar.cap < 4 * ar.need + DE.ARENA_MIN or ar.cap <= peers


def test_partition_scratch_pool_budget_reuse_and_wait(monkeypatch):
    """The device-wide partition scratch (engine/device_exec.py PartScratchPool): slabs are reused
    smallest-fit, a new slab over the byte budget waits for a release from another thread, and a
    thread that already holds one (hashed re-partition) never waits."""
    import time

    monkeypatch.setattr(DE, "PART_SCRATCH_BUDGET", 20000)  # bytes: a 1000-word and a 1250-word slab
    pool = DE.PartScratchPool()
    a = pool.acquire("cpu", 1000)
    assert a.recs1.numel() == 1000 and pool.bytes() == 8000
    nested = pool.acquire("cpu", 1500)  # same thread holds one: over budget without waiting
    assert pool.bytes() == 8000 + 12000
    pool.release(nested)
    got = {}

    def other():
        t0 = time.perf_counter()
        got["slab"] = pool.acquire("cpu", 2000)  # does not fit next to a: waits for a release
        got["waited"] = time.perf_counter() - t0
        pool.release(got["slab"])

    th = threading.Thread(target=other)
    th.start()
    time.sleep(0.3)
    assert "slab" not in got
    pool.release(a)
    th.join(5)
    assert got["slab"].words == 2000 and got["waited"] >= 0.25
    again = pool.acquire("cpu", 900)  # smallest free slab that fits is reused
    assert again.words == 2000 and pool.bytes() == 16000
    pool.release(again)
    pool.clear()
    assert pool.bytes() == 0


def test_out_of_memory_release_skips_arenas_held_by_other_slots(monkeypatch):
    """An out-of-memory release while carving (this arena's lock held) must not wait for another
    slot's arena lock: that slot may be carving too and releasing in turn -- each would hold its own
    lock and wait on the other's (lock-order deadlock).  Busy arenas are skipped."""
    monkeypatch.setattr(DE, "_ARENAS", {})
    a, b = DE.slot_arena("cpu", 93), DE.slot_arena("cpu", 94)
    own = _Owner()
    with use_slot(94):
        b.carve(1000, own)
    monkeypatch.setattr(DE.torch.cuda, "empty_cache", lambda: None)
    done = threading.Event()
    with b.lock:  # slot 94 is busy carving
        t = threading.Thread(target=lambda: (DE.release_device_memory(keep_arena=a), done.set()))
        t.start()
        t.join(10)
        assert done.is_set(), "release_device_memory blocked on another slot's arena lock"
    assert b.buf is not None  # (skipped, not dropped)
    DE.release_device_memory(keep_arena=a)
    assert b.buf is None


def test_growing_slot_goes_straight_to_the_largest_peer(monkeypatch):
    """Every slot runs every kind of statement: a slot arena that must grow takes the largest
    peer's size at once (one growth per slot instead of a doubling series whose dropped storages
    pile up in the caching allocator's per-stream pools)."""
    monkeypatch.setattr(DE, "_ARENAS", {})
    monkeypatch.setattr(DE, "ARENA_MIN", 4096)
    big, small = DE.slot_arena("cpu", 1), DE.slot_arena("cpu", 2)
    with use_slot(1):
        big.carve(50_000, _Owner())
    assert big.cap == 53_248
    with use_slot(2):
        small.carve(100, _Owner())
    assert small.cap == big.cap


def test_part_pool_presize_fills_one_slab_per_slot(monkeypatch):
    """Warm-up presizing (NativeHiveServer.settle): the partition scratch pool holds one free slab
    per slot at the largest size any statement asked for; smaller free slabs are replaced."""
    pool = DE.PartScratchPool()
    monkeypatch.setattr(pool, "_budget", lambda dev: 1 << 20)
    s1 = pool.acquire("cpu", 100)
    s2 = pool.acquire("cpu", 1000)
    pool.release(s1)
    pool.release(s2)
    assert pool.presize("cpu", 4) == 3
    assert sorted(x.words for x in pool.free) == [1000] * 4
    assert pool.total == 4 * 2 * 1000 * 4
    assert pool.presize("cpu", 4) == 0
    s = pool.acquire("cpu", 500)  # served from the presized slabs
    assert s.words == 1000 and pool.total == 4 * 2 * 1000 * 4


@pytest.mark.gpu
def test_shared_allocation_stream_reuses_dropped_storage():
    """Arena storages and partition slabs come from one allocation stream: a storage dropped by a
    slot on one stream is the next growth's free block on another slot's stream (allocated per slot
    stream, it stayed cached on its own stream until a free-everything retry)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    n = 256 << 20
    with torch.cuda.stream(s1):
        a = DE.shared_empty(n, torch.uint8, dev)
        a.fill_(1)
    r0 = torch.cuda.memory_reserved(dev)
    del a
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(s2):
        b = DE.shared_empty(n, torch.uint8, dev)
        b.fill_(2)
    assert torch.cuda.memory_reserved(dev) == r0
    torch.cuda.synchronize(dev)
    assert int(b[::1 << 20].min()) == 2
