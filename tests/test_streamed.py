"""Shards larger than HBM: a host-resident shard is streamed through the device in
row windows (double-buffered copies on a side stream); every query must return exactly what the
resident engine returns over the same rows."""
import numpy as np
import pytest
import torch

from spark_druid_olap_amd.engine.columns import materialize
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models.bench_queries import bench_specs
from spark_druid_olap_amd.query import spec as S
from spark_druid_olap_amd.query.granularity import Granularity
from spark_druid_olap_amd.segment.streamed import HostShard, StreamedQuery

EXTRA = [
    ("by month", S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("l_shipmode")], granularity=Granularity.parse("month"),
                                    aggregations=[S.FunctionAggregationSpec("count", "n"),
                                                  S.FunctionAggregationSpec("longMax", "mx", "l_quantity")],
                                    intervals=["1993-01-01/1996-06-01"])),
    ("topN", S.TopNQuerySpec("tpch", S.DefaultDimensionSpec("p_brand"), S.NumericTopNMetricSpec("rev"), 5,
                             aggregations=[S.FunctionAggregationSpec("doubleSum", "rev", "l_extendedprice")],
                             intervals=["1992-01-01/1999-01-01"])),
    ("orders", S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("o_orderkey")],
                                  aggregations=[S.FunctionAggregationSpec("longSum", "q", "l_quantity")],
                                  filter=S.SelectorFilterSpec("c_mktsegment", "BUILDING"),
                                  intervals=["1995-01-01/1995-04-01"])),
]


def _table(res):
    cols = res.columns
    rows = list(zip(*[materialize(res.data[c]).tolist() for c in cols]))
    return sorted(tuple(round(x, 4) if isinstance(x, float) else x for x in r) for r in rows)


@pytest.mark.parametrize("window_rows", [1 << 14, 3 * 4096 + 5])
def test_streamed_equals_resident(ds_small, window_rows):
    eng = Engine(use_native=False)
    shard = HostShard(ds_small, "cpu", window_rows=window_rows, pin=False)
    assert len(shard.windows) > 3
    for name, q in bench_specs() + EXTRA:
        want = _table(eng.execute(q, ds_small))
        got = StreamedQuery(eng, q, shard).run()
        assert _table(got) == want, name
        assert got.stats["windows"] == len(shard.windows)


def test_streamed_copies_only_the_columns_read(ds_small):
    eng = Engine(use_native=False)
    shard = HostShard(ds_small, "cpu", window_rows=1 << 15, pin=False)
    q = dict(bench_specs())["Ship Date Range"]
    sq = StreamedQuery(eng, q, shard)
    dims, mets, _ = sq._cols
    assert len(dims) + len(mets) <= 6 < len(ds_small.dims)
    sq.run()
    per_row = shard.bytes_copied / ds_small.num_rows
    assert per_row < 16, per_row


@pytest.mark.gpu
def test_gpu_streamed_equals_resident(tmp_path):
    """Host shard streamed through the HIP kernels with double-buffered H2D copies vs the same
    shard resident in HBM (the same rows: saved once, loaded on each side)."""
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.segment.datasource import DataSource

    tpch.to_datasource(tpch.generate_flat(0.1, "cpu"), profile="bench").save(str(tmp_path / "s"))
    host = DataSource.load(str(tmp_path / "s"), "cpu")
    dev = DataSource.load(str(tmp_path / "s"), "cuda")
    eng = Engine(use_native=True)
    shard = HostShard(host, "cuda", window_rows=1 << 17)
    assert shard.copy_stream is not None and len(shard.windows) >= 4
    for name, q in bench_specs() + EXTRA:
        want = _table(eng.execute(q, dev))
        got = StreamedQuery(eng, q, shard).run()
        assert _table(got) == want, name


def test_sql_over_a_host_shard(ds_small, df_small):
    """A HostShard registers like any datasource: the SQL planner reads its metadata, aggregate
    queries stream it."""
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.session import Session

    def sess(ds):
        s = Session(engine=Engine(use_native=False))
        s.register_datasource(ds)
        s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
        s.sql(tpch.druid_ddl(with_column_mapping=False))
        return s

    shard = HostShard(ds_small, "cpu", window_rows=1 << 14, pin=False)
    a, b = sess(ds_small), sess(shard)
    for q in ["select l_returnflag, l_linestatus, count(*), sum(l_extendedprice), avg(l_discount) "
              "from orderLineItemPartSupplier group by l_returnflag, l_linestatus",
              "select s_nation, sum(l_quantity) from orderLineItemPartSupplier where s_region = 'EUROPE' "
              "and l_shipdate >= '1995-01-01' group by s_nation"]:
        ra = sorted(a.sql(q).collect())
        rb = sorted(b.sql(q).collect())
        assert len(ra) == len(rb)
        for x, y in zip(ra, rb):
            for u, v in zip(x, y):
                assert (u == pytest.approx(v, rel=1e-9)) if isinstance(u, float) else u == v
