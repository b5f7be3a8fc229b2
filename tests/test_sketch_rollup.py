"""Stored sketch metrics with ingest-time rollup (K12 hyperUnique merge, K13 theta, K20 ingest).

A Druid index task rolls rows up and keeps a sketch per rolled-up row
(``src/test/resources/zip_codeAll.json.template:49-59``).  Here the rolled-up index must answer
hyperUnique / thetaSketch aggregations EXACTLY like the raw (non-rolled) index of the same input:
the stored sparse HLL pairs are bit-identical to the query-time updates, and the stored KMV hashes
are the raw rows' hashes."""
import csv

import numpy as np
import pytest
import torch

from spark_druid_olap_amd.engine.columns import materialize
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.query import spec as S
from spark_druid_olap_amd.segment.datasource import DataSource
from spark_druid_olap_amd.segment.ingest import IndexSpec, ingest


def _write(path, n=6000, seed=3):
    rng = np.random.default_rng(seed)
    users = [f"user{i:05d}" for i in range(2500)]
    with open(path, "w", newline="") as f:
        w = csv.writer(f, delimiter="\t")
        for _ in range(n):
            day = f"2016-0{int(rng.integers(1, 4))}-{int(rng.integers(1, 29)):02d}T{int(rng.integers(0, 24)):02d}:00:00"
            w.writerow([day, ["web", "ios", "android"][int(rng.integers(0, 3))],
                        ["US", "DE", "IN", "BR"][int(rng.integers(0, 4))], users[int(rng.integers(0, len(users)))],
                        f"{rng.uniform(1, 100):.2f}"])
    return path


def _spec(data_dir, rollup=True, qgran="day"):
    return {"type": "index", "spec": {
        "dataSchema": {
            "dataSource": "events",
            "parser": {"type": "string", "parseSpec": {
                "format": "tsv", "timestampSpec": {"column": "ts", "format": "iso"},
                "columns": ["ts", "platform", "country", "user", "amount"],
                "dimensionsSpec": {"dimensions": ["platform", "country"]}}},
            "metricsSpec": [{"type": "count", "name": "count"},
                            {"type": "doubleSum", "name": "amount", "fieldName": "amount"},
                            {"type": "hyperUnique", "name": "uniq_users", "fieldName": "user"},
                            {"type": "thetaSketch", "name": "user_sketch", "fieldName": "user", "size": 256}],
            "granularitySpec": {"type": "uniform", "segmentGranularity": "MONTH", "queryGranularity": qgran,
                                "rollup": rollup, "intervals": ["2016-01-01/2016-12-31"]}},
        "ioConfig": {"type": "index", "firehose": {"type": "local", "baseDir": str(data_dir), "filter": "*.tsv"}}}}


@pytest.fixture(scope="module")
def data_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("events")
    _write(str(d / "events.tsv"))
    return d


@pytest.fixture(scope="module")
def pair(data_dir):
    return ingest(_spec(data_dir, rollup=True), block_bytes=1 << 16), ingest(_spec(data_dir, rollup=False))


def _q(agg, dims=("country",), filt=None):
    return S.GroupByQuerySpec("events", [S.DefaultDimensionSpec(d) for d in dims], aggregations=agg,
                              intervals=["2016-01-01/2016-12-31"], filter=filt)


def _run(ds, q):
    r = Engine(use_native=False).execute(q, ds)
    keys = [tuple(materialize(r.data[d]).tolist()[i] for d in ("country", "platform") if d in r.data)
            for i in range(r.num_rows)]
    return {k: tuple(np.asarray(r.data[c])[i] for c in r.columns if c not in ("country", "platform"))
            for i, k in enumerate(keys)}


def test_rollup_compacts_and_keeps_sketches(pair):
    rolled, raw = pair
    assert rolled.rollup and not raw.rollup
    assert rolled.num_rows < raw.num_rows and raw.num_rows == 6000
    assert rolled.metrics["uniq_users"].sketch is not None and rolled.metrics["uniq_users"].sketch.kind == "hll"
    assert rolled.metrics["user_sketch"].sketch.kind == "theta"
    assert raw.metrics["uniq_users"].sketch is None
    # rollup preserves counts and sums
    assert int(rolled.metrics["count"].data[: rolled.num_rows].sum()) == 6000
    assert float(rolled.metrics["amount"].data[: rolled.num_rows].sum()) == pytest.approx(
        float(raw.metrics["amount"].data[: raw.num_rows].sum()))


@pytest.mark.parametrize("dims", [("country",), ("country", "platform"), ()])
def test_hyperunique_rolled_equals_raw(pair, dims):
    rolled, raw = pair
    q = _q([S.HyperUniqueAggregationSpec("u", "uniq_users"), S.FunctionAggregationSpec("longSum", "n", "count")],
           dims)
    a, b = _run(rolled, q), _run(raw, q.copy())
    assert a.keys() == b.keys()
    for k in a:
        assert a[k][0] == b[k][0]  # same registers -> bitwise-equal estimate
        assert a[k][1] == b[k][1]


def test_hyperunique_filtered_and_exactness(pair, data_dir):
    import pandas as pd

    rolled, raw = pair
    df = pd.read_csv(data_dir / "events.tsv", sep="\t", header=None, names=["ts", "platform", "country", "user", "a"])
    filt = S.SelectorFilterSpec("platform", "ios")
    q = _q([S.HyperUniqueAggregationSpec("u", "uniq_users"),
            S.FilteredAggregationSpec(S.SelectorFilterSpec("country", "US"),
                                      S.HyperUniqueAggregationSpec("u_us", "uniq_users"), "u_us")], filt=filt)
    a, b = _run(rolled, q), _run(raw, q.copy())
    assert a == b
    exact = df[df.platform == "ios"].groupby("country").user.nunique()
    for (c,), (u, u_us) in a.items():
        assert u == pytest.approx(exact[c], rel=0.05)
        assert (u_us > 0) == (c == "US")


def test_theta_rolled_equals_raw(pair, data_dir):
    import pandas as pd

    rolled, raw = pair
    q = _q([S.ThetaSketchAggregationSpec("t", "user_sketch", 256)], ("platform",))
    a, b = _run(rolled, q), _run(raw, q.copy())
    assert a == b
    df = pd.read_csv(data_dir / "events.tsv", sep="\t", header=None, names=["ts", "platform", "country", "user", "a"])
    exact = df.groupby("platform").user.nunique()
    for (p_,), (t,) in a.items():
        assert t == pytest.approx(exact[p_], rel=0.2)


def test_sketch_columns_persist(pair, tmp_path):
    rolled, _ = pair
    rolled.save(str(tmp_path / "seg"))
    back = DataSource.load(str(tmp_path / "seg"))
    for nm in ("uniq_users", "user_sketch"):
        a, b = rolled.metrics[nm].sketch, back.metrics[nm].sketch
        assert b is not None and a.kind == b.kind and torch.equal(a.offsets, b.offsets) and torch.equal(a.values, b.values)
    q = _q([S.HyperUniqueAggregationSpec("u", "uniq_users")])
    assert _run(rolled, q) == _run(back, q.copy())


def test_sharded_ingest_partitions_rolled_rows(data_dir):
    whole = ingest(_spec(data_dir))
    shards = [ingest(_spec(data_dir), rank=r, world=2) for r in range(2)]
    assert sum(s.num_rows for s in shards) == whole.num_rows
    assert all(s.global_num_rows == whole.num_rows for s in shards)
    npairs = sum(int(s.metrics["uniq_users"].sketch.values.numel()) for s in shards)
    assert npairs == int(whole.metrics["uniq_users"].sketch.values.numel())


@pytest.mark.gpu
def test_gpu_ingest_and_stored_merge_match_cpu(data_dir):
    """hll_pairs + hll_merge_stored HIP kernels vs the torch path: identical sketches, identical
    registers, identical estimates."""
    cpu = ingest(_spec(data_dir))
    gpu = ingest(_spec(data_dir), device="cuda")
    for nm in ("uniq_users", "user_sketch"):
        a, b = cpu.metrics[nm].sketch, gpu.metrics[nm].sketch
        assert torch.equal(a.offsets, b.offsets.cpu()) and torch.equal(a.values, b.values.cpu())
    q = _q([S.HyperUniqueAggregationSpec("u", "uniq_users"), S.ThetaSketchAggregationSpec("t", "user_sketch", 256)],
           ("country", "platform"))
    rc = _run(cpu, q)
    rg = Engine(use_native=True).execute(q.copy(), gpu)
    keys = list(zip(materialize(rg.data["country"]).tolist(), materialize(rg.data["platform"]).tolist()))
    got = {k: (rg.data["u"][i], rg.data["t"][i]) for i, k in enumerate(keys)}
    assert got == rc


@pytest.mark.gpu
def test_gpu_stored_hll_union_fused_in_the_scan_kernel(pair):
    """K12 fused: the JIT scan unions the selected rows' stored sketches in place (A_HLL_STORED) --
    no post-scan row re-derivation -- and equals query-time HLL over the raw index, also for a
    filtered hyperUnique."""
    from spark_druid_olap_amd.segment.datasource import DataSource  # noqa: F401

    rolled, raw = pair
    gr = rolled.to("cuda")
    q = _q([S.HyperUniqueAggregationSpec("u", "uniq_users"),
            S.FilteredAggregationSpec(S.SelectorFilterSpec("platform", "ios"),
                                      S.HyperUniqueAggregationSpec("u_ios", "uniq_users"), "u_ios")],
           ("country",))
    pq = Engine(use_native=True).prepare(q.copy(), gr)
    preps = [p for _, _, p in pq.scans]
    assert preps and all(getattr(p, "stored_fused", False) for p in preps), "stored sketches not fused"
    got, want = _run_native(gr, q.copy()), _run(raw, q.copy())
    assert got.keys() == want.keys()
    for k in want:  # same registers; the GPU (MFMA) and host estimators differ in the last ulp
        assert got[k] == pytest.approx(want[k], rel=1e-12)


def _run_native(ds, q):
    r = Engine(use_native=True).execute(q, ds)
    keys = [tuple(materialize(r.data[d]).tolist()[i] for d in ("country", "platform") if d in r.data)
            for i in range(r.num_rows)]
    return {k: tuple(np.asarray(r.data[c])[i] for c in r.columns if c not in ("country", "platform"))
            for i, k in enumerate(keys)}


def _split_worker(rank, world, port, data_dir, outdir):
    import os
    import pickle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    from spark_druid_olap_amd.parallel.world import init_world

    w = init_world(backend="gloo")
    ds = ingest(_spec(data_dir), rank=rank, world=world, block_bytes=1 << 14)  # many blocks: split by rank
    out = {"rows": ds.num_rows, "global": ds.global_num_rows, "split": ds.ingest_split,
           "dicts": {d: list(map(str, ds.dims[d].dictionary.values.tolist())) for d in ("platform", "country")},
           "pairs": int(ds.metrics["uniq_users"].sketch.values.numel()),
           "amount": float(ds.metrics["amount"].data[: ds.num_rows].sum()),
           "count": int(ds.metrics["count"].data[: ds.num_rows].sum())}
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(out, f)
    w.barrier()
    import torch.distributed as dist

    dist.destroy_process_group()
    # (Arrow's CSV reader pool can abort interpreter teardown under load: the result is written)
    os._exit(0)


def test_split_ingest_across_ranks_equals_single_ingest(data_dir, tmp_path):
    """Each rank parses only its blocks, dictionaries are unified and raw rows shuffled to their
    partition owner before rollup: the union of the shards equals one whole ingest (gloo, 3 ranks)."""
    import pickle
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 3
    ctx = mp.start_processes(_split_worker, args=(world, port, str(data_dir), str(tmp_path)), nprocs=world,
                             join=False, start_method="spawn")
    for p in ctx.processes:
        p.join(240)
    assert all(p.exitcode == 0 for p in ctx.processes)
    outs = [pickle.load(open(tmp_path / f"r{r}.pkl", "rb")) for r in range(world)]
    whole = ingest(_spec(data_dir))
    assert all(o["split"] for o in outs)
    assert sum(o["rows"] for o in outs) == whole.num_rows
    assert all(o["global"] == whole.num_rows for o in outs)
    for d in ("platform", "country"):
        want = list(map(str, whole.dims[d].dictionary.values.tolist()))
        assert all(o["dicts"][d] == want for o in outs)
    assert sum(o["pairs"] for o in outs) == int(whole.metrics["uniq_users"].sketch.values.numel())
    assert sum(o["count"] for o in outs) == int(whole.metrics["count"].data[: whole.num_rows].sum())
    assert sum(o["amount"] for o in outs) == pytest.approx(float(whole.metrics["amount"].data[: whole.num_rows].sum()))


def test_stored_hll_partitioned_producer_compiles(pair, tmp_path, monkeypatch):
    """The partitioned producer of a rolled-up hyperUnique group-by (CPU compile): each record ends
    with one row-id word per stored sketch (all-ones when the aggregator's filter rejects the row)."""
    from spark_druid_olap_amd.engine.lower import Lowerer
    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.ops import jit

    monkeypatch.setenv("SDO_JIT_CACHE", str(tmp_path))
    rolled, _ = pair
    q = _q([S.HyperUniqueAggregationSpec("u", "uniq_users"),
            S.FilteredAggregationSpec(S.SelectorFilterSpec("platform", "ios"),
                                      S.HyperUniqueAggregationSpec("u_ios", "uniq_users"), "u_ios")],
           ("country", "platform"))
    prog = Engine(use_native=False).prepare(q, rolled).scans[0][1]
    assert len(prog.stored_hll) == 2 and prog.nhll == 0
    assert jit.part_eligible(prog) and jit.part_stored_count(prog) == 2 and jit.part_hll_count(prog) == 2
    prog.packed = {}
    js = jit.JitScan(prog, D.M_PART, 4, False, 1 << prog.hll_p, True, load=False)
    assert "0xffffffffu" in js.src  # the filtered sketch's "no row" word
    fields = jit.part_fields(prog)
    assert sum(w for _, w in fields) + 1 + 2 == 3 + sum(w for _, w in fields)


@pytest.mark.gpu
def test_gpu_stored_hll_partitioned(pair, monkeypatch):
    """A rolled-up hyperUnique group-by through the radix-partitioned path (records carry the row
    id, partition.hip part_agg unions the row's stored pairs per group) gives the same registers
    as the fused dense scan, and through the planner the same estimates as query-time HLL over the
    raw index."""
    from spark_druid_olap_amd.engine import device_exec as DE
    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.planner import cost

    rolled, raw = pair
    gr = rolled.to("cuda")
    aggs = [S.HyperUniqueAggregationSpec("u", "uniq_users"),
            S.FilteredAggregationSpec(S.SelectorFilterSpec("platform", "ios"),
                                      S.HyperUniqueAggregationSpec("u_ios", "uniq_users"), "u_ios"),
            S.FunctionAggregationSpec("longSum", "n", "count")]
    q = _q(aggs, ("country", "platform"))
    prog = Engine(use_native=True).prepare(q.copy(), gr).scans[0][1]
    part = DE.PreparedScan(prog, mode=D.M_PART)
    assert part.mode == D.M_PART and part.stored_fused and part.part["nhll"] == 2, "not partitioned"
    ref = DE.PreparedScan(prog, mode=D.M_DENSE_GLOBAL)
    assert ref.stored_fused
    for _ in range(2):  # re-execution over the same slot buffers
        a = part.run()
    b = ref.run()
    assert a.kind == "dense" and b.kind == "dense" and len(a.hll) == len(b.hll) == 2
    assert torch.equal(a.acc.cpu(), b.acc.cpu())
    for x, y in zip(a.hll, b.hll):
        assert torch.equal(x.cpu(), y.cpu())
    # end to end: the planner partitions it (forced), estimates equal the raw index's query-time HLL
    monkeypatch.setattr(cost, "FORCE_PARTITIONED", True)
    for knob in ("PLAN_LDS_BUDGET", "SHARED_LDS_MAX"):  # (no LDS table plan for the 1,056 groups)
        monkeypatch.setattr(cost, knob, 0)
    qd = S.GroupByQuerySpec("events", [S.DefaultDimensionSpec("country"), S.DefaultDimensionSpec("platform")],
                            aggregations=aggs[:2], intervals=["2016-01-01/2016-12-31"],
                            granularity=S.Granularity.parse("day"))
    pq = Engine(use_native=True).prepare(qd.copy(), gr)
    modes = [getattr(p, "mode", None) for _, _, p in pq.scans]
    assert D.M_PART in modes, modes
    got = Engine(use_native=True).execute(qd.copy(), gr)
    want = Engine(use_native=False).execute(qd.copy(), raw)
    assert got.num_rows == want.num_rows

    def rows(r):
        ts = np.asarray(r.data["timestamp"]).tolist()
        c, p = materialize(r.data["country"]).tolist(), materialize(r.data["platform"]).tolist()
        return {(ts[i], c[i], p[i]): (float(r.data["u"][i]), float(r.data["u_ios"][i])) for i in range(r.num_rows)}

    g, w = rows(got), rows(want)
    assert g.keys() == w.keys()
    for k in w:
        assert g[k] == pytest.approx(w[k], rel=1e-12)
