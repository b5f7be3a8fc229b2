"""Segment-batched ("historical") execution across ranks with batch j's merge collectives
overlapping batch j+1's scan (``PreparedQuery._run_pipelined``, ``parallel/merge.start_dense_merge``),
asked for (``segments_per_query``) or chosen by itself on the default path (``AUTO_PIPELINE``: a large
dense state keyed by a leading time bucket).

Ranks hold shards of different sizes, so their batch counts differ: the smaller shard pads with
identity partials after agreeing on the count.  Results must equal the one-merge-after-combine
path (which ``test_distributed.py`` checks against the union oracle), for the one-shot gather and
the bucketed all-reduce merge, and a scan failure in a middle batch must abort every rank."""
import dataclasses
import os
import pickle
import socket
import tempfile

import pytest
import torch.multiprocessing as mp

NAMES = ["TPCH Q1", "TPCH Q7", "Basic Aggregation", "TPCH Q3"]


def _ts_month():
    from spark_druid_olap_amd.query import spec as S

    return S.TimeSeriesQuerySpec("tpch", ["1992-01-01/1999-01-01"], granularity=S.Granularity.parse("month"),
                                 aggregations=[S.FunctionAggregationSpec("longSum", "q", "l_quantity"),
                                               S.FunctionAggregationSpec("count", "n")])


def _gb_week():
    from spark_druid_olap_amd.query import spec as S

    return S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("l_returnflag")],
                              granularity=S.Granularity.parse("week"), intervals=["1992-01-01/1999-01-01"],
                              aggregations=[S.FunctionAggregationSpec("doubleSum", "s", "l_extendedprice")])


# time-leading group keys: each batch merges only its slice of the table (historical interval
# partitioning, engine/executor.py _batch_key_slices)
TIME_LEADING = {"TS month": _ts_month, "GB week x flag": _gb_week}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, device="cpu"):
    try:
        _work(rank, world, port, outdir, device)
    except BaseException:
        import traceback

        with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
            f.write(traceback.format_exc())
        raise


def _work(rank, world, port, outdir, device="cpu"):
    if device == "cuda":
        os.environ["SDO_GLOO_GPU"] = "1"  # ranks share the one card, collectives over gloo
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1",
                      SDO_REF_SPARSE_G="1000")  # Q3's order-key groups come back sparse (hash-like)
    from spark_druid_olap_amd.engine import executor as X
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.models.bench_queries import DRUID_JSON
    from spark_druid_olap_amd.parallel.fault import FAULTS, InjectedFault, RankFailure
    from spark_druid_olap_amd.parallel.world import init_world
    from spark_druid_olap_amd.planner import cost
    from spark_druid_olap_amd.query.spec import query_from_json

    w = init_world(backend="gloo")
    # uneven shards: the last rank keeps the earliest quarter of its rows (fewer segment batches;
    # same dictionaries, so the group-by layouts agree)
    flat = tpch.generate_flat(float(os.environ.get("PM_SF", 0.004 if device == "cpu" else 0.05)), device, rank=rank, world=world)
    if rank == world - 1:
        n = flat.num_rows // 4
        flat = dataclasses.replace(flat, num_rows=n, ship_day=flat.ship_day[:n],
                                   dims={k: (dct, t[:n]) for k, (dct, t) in flat.dims.items()},
                                   nums={k: (t[:n], kind, sc) for k, (t, kind, sc) in flat.nums.items()})
    ds = tpch.to_datasource(flat, profile="bench")
    eng = X.Engine(w, use_native=device == "cuda")
    from spark_druid_olap_amd.session import Session

    Session(engine=eng).register_datasource(ds)  # the cluster-wide time interval (same layouts)
    out = {"nseg": len(ds.segments)}
    for oneshot in (True, False):
        saved = cost.ONESHOT_MAX_BYTES
        if not oneshot:
            cost.ONESHOT_MAX_BYTES = 0  # force the bucketed ring all-reduces
        try:
            for name in NAMES + list(TIME_LEADING):
                q = query_from_json(DRUID_JSON[name]) if name in NAMES else TIME_LEADING[name]()
                X.PIPELINE_MERGE = True
                p = eng.prepare(q, ds, segments_per_query=2)
                a = p.run().sorted_rows()
                X.PIPELINE_MERGE = False
                b = eng.prepare(q, ds, segments_per_query=2).run().sorted_rows()
                out[(name, oneshot)] = (a, b, p._nbatches, len(p.scans), p._pipeline_ok)
                out[(name, oneshot, "slices")] = (p._slices, p.scans[0][1].G if p.scans else 0)
        finally:
            cost.ONESHOT_MAX_BYTES = saved
            X.PIPELINE_MERGE = True
    # the default path (no segments_per_query): a time-leading dense state above the size threshold
    # pipelines by itself, with the batch count agreed across ranks; below it, one merge
    saved_min = X.AUTO_PIPELINE_MIN_BYTES
    X.AUTO_PIPELINE_MIN_BYTES = 512
    X.AUTO_PIPELINE_FORCE = True  # (gloo stages through the host: the cost model would never split)
    try:
        p = eng.prepare(_ts_month(), ds)
        a = p.run().sorted_rows()
        X.AUTO_PIPELINE = False
        q0 = eng.prepare(_ts_month(), ds)
        b = q0.run().sorted_rows()
        out["auto"] = (a, b, p._nbatches, bool(p.segments_per_query), p._pipeline_ok, bool(q0.segments_per_query))
    finally:
        X.AUTO_PIPELINE, X.AUTO_PIPELINE_MIN_BYTES, X.AUTO_PIPELINE_FORCE = True, saved_min, False
    small = eng.prepare(query_from_json(DRUID_JSON["TPCH Q1"]), ds)
    out["auto_small"] = bool(small.segments_per_query)
    # a scan failure in the second batch of rank 0: both ranks abort consistently
    q = query_from_json(DRUID_JSON["TPCH Q1"])
    p = eng.prepare(q, ds, segments_per_query=2)
    p.run()
    calls = {"n": 0}
    orig = p._scan

    def failing(prog, prep):
        calls["n"] += 1
        if rank == 0 and calls["n"] == 2:
            FAULTS.configure(0, "scan", 1)
        return orig(prog, prep)

    p._scan = failing
    try:
        p.run()
        out["fault"] = "none"
    except InjectedFault:
        out["fault"] = "local"
    except RankFailure:
        out["fault"] = "peer"
    FAULTS.clear()
    out["after"] = eng.prepare(q, ds, segments_per_query=2).run().sorted_rows()  # the world still works
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(out, f)
    w.barrier()


def _close(a, b):
    if len(a) != len(b):
        return False
    for ra, rb in zip(a, b):
        for x, y in zip(ra, rb):
            if isinstance(x, float) and isinstance(y, float):
                if x != pytest.approx(y, rel=1e-9, abs=1e-9):
                    return False
            elif x != y:
                return False
    return True


def _run(world, device):
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_worker, args=(world, _free_port(), d, device), nprocs=world, join=False,
                                 start_method="spawn")
        for p in ctx.processes:
            p.join(300)
        errs = [open(os.path.join(d, f)).read() for f in sorted(os.listdir(d)) if f.startswith("err")]
        assert all(p.exitcode == 0 for p in ctx.processes), ([p.exitcode for p in ctx.processes], errs)
        outs = [pickle.load(open(os.path.join(d, f"r{r}.pkl"), "rb")) for r in range(world)]
    _check(outs, device)


@pytest.mark.parametrize("world", [2, 3])
def test_pipelined_merge_matches_combined_merge(world):
    _run(world, "cpu")


@pytest.mark.gpu
def test_pipelined_merge_on_gpu_scans():
    """The HIP scan kernels per segment batch with gloo collectives staged through the host (two
    ranks on the one card of the test box)."""
    _run(2, "cuda")


def _check(outs, device):
    for name in TIME_LEADING:
        for oneshot in (True, False):
            sl = [o[(name, oneshot, "slices")] for o in outs]
            assert len({repr(x) for x in sl}) == 1, sl  # every rank merges the same slices
            slices, G = sl[0]
            assert slices is not None and sum(b - a for a, b in slices) < len(slices) * G, slices
    for name in NAMES + list(TIME_LEADING):
        for oneshot in (True, False):
            per_rank = [o[(name, oneshot)] for o in outs]
            nb = {x[2] for x in per_rank}
            assert len(nb) == 1, (name, nb)  # the agreed batch count
            for a, b, nbatches, nscans, ok in per_rank:
                assert _close(a, b), (name, oneshot)
                if name in ("TPCH Q3", "GB week x flag") and device == "cpu":
                    assert ok is False  # hash partials (> SDO_REF_SPARSE_G groups): one merge after the combine
                else:
                    assert ok is True and nbatches >= nscans
            assert _close(per_rank[0][0], per_rank[-1][0])
    for o in outs:
        a, b, nb, auto, ok, off = o["auto"]
        assert _close(a, b) and auto and ok is True and nb > 1 and not off, o["auto"][2:]
        assert not o["auto_small"]  # Q1's 4-group state: never split
    assert len({o["auto"][2] for o in outs}) == 1
    # the small last shard ran fewer batches than the agreed count (identity padding exercised)
    last = outs[-1][("TPCH Q1", True)]
    assert last[3] < last[2]
    assert outs[0]["fault"] == "local" and all(o["fault"] == "peer" for o in outs[1:])
    assert all(_close(o["after"], outs[0]["after"]) for o in outs)
