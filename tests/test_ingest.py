"""Ingestion from the reference's own Druid index-task templates, then SQL over the result.

* ``zip_codeAll.json.template`` + ``zipCodes/sample/zip_codes_states.csv`` (the reference's
  QueryExtTest fixture): HLL / theta metrics, a spatial dimension, record_date time column.
* ``tpch_index_task.json.template`` over a synthetic flattened TPC-H file (the real
  ``orderLineItemPartSupplierCustomer.small`` is not in the mirror): schemaless dimensions,
  JavaScript metrics, DAY query granularity with rollup, MONTH segments.
"""
import json
import os

import numpy as np
import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.query import spec as S
from spark_druid_olap_amd.segment.ingest import IndexSpec, ingest
from spark_druid_olap_amd.session import Session

REF = "/root/reference/src/test/resources"
HAVE_REF = os.path.exists(f"{REF}/zip_codeAll.json.template")

ZIP_INFOS = json.dumps([
    {"column": "city", "druidColumn": "city", "hllMetric": "unique_city", "sketchMetric": "city_sketch"},
    {"column": "latitude", "spatialIndex": {"druidColumn": "coordinates", "spatialPosition": 0,
                                            "minValue": -90.0, "maxValue": 90.0}},
    {"column": "longitude", "spatialIndex": {"druidColumn": "coordinates", "spatialPosition": 1,
                                             "minValue": -180.0, "maxValue": 180.0}}])


@pytest.fixture(scope="module")
def zsess():
    if not HAVE_REF:
        pytest.skip("reference checkout not mounted")
    ds = ingest(f"{REF}/zip_codeAll.json.template", data_dir=f"{REF}/zipCodes/sample")
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds)
    s.sql(f"""CREATE TABLE zipCodesBase(record_date string, zip_code string, latitude double, longitude double,
      city string, state string, county string) USING com.databricks.spark.csv
      OPTIONS (path "{REF}/zipCodes/sample/zip_codes_states.csv", header "false", delimiter ",")""")
    s.sql(f"""CREATE TABLE zipCodesFull USING org.sparklinedata.druid OPTIONS (sourceDataframe "default.zipCodesBase",
      timeDimensionColumn "record_date", druidDatasource "zipCodesAll", columnInfos '{ZIP_INFOS}',
      nonAggregateQueryHandling "push_project_and_filters", allowTopNRewrite "true")""")
    return s


def test_zip_ingest_shape(zsess):
    ds = zsess.catalog.cluster.get("zipCodesAll")
    assert ds.num_rows == 1000
    assert ds.spatial == {"coordinates": ["coordinates.0", "coordinates.1"]}
    assert ds.metrics["unique_city"].kind == "hll" and ds.metrics["count"].kind == "long"


def test_zip_hll_metric(zsess):
    d = zsess.sql("select state, approx_count_distinct(city) from zipCodesFull group by state")
    [q] = d.druid_query_specs()
    assert any(isinstance(a, S.HyperUniqueAggregationSpec) and a.fieldName == "unique_city" for a in q.aggregations)
    exact = dict(zsess.sql("select state, count(distinct city) from zipCodesBase group by state").collect())
    for st, v in d.collect():
        assert v == pytest.approx(exact[st], rel=0.08, abs=2)


def test_zip_spatial_filters(zsess):
    for cond in ["latitude >= 40", "latitude > 35 and latitude < 42 and longitude > -72",
                 "longitude <= -71.5 and latitude < 42.5"]:
        d = zsess.sql(f"select state, count(*) from zipCodesFull where {cond} group by state")
        assert "SpatialFilterSpec" in json.dumps(d.druid_query_specs()[0].to_json())
        b = zsess.sql(f"select state, count(*) from zipCodesBase where {cond} group by state")
        assert sorted(d.collect()) == sorted(b.collect())


def test_zip_select(zsess):
    d = zsess.sql("select zip_code, city from zipCodesFull where state = 'RI' and latitude > 41.8")
    assert isinstance(d.druid_query_specs()[0], S.SelectSpec)
    b = zsess.sql("select zip_code, city from zipCodesBase where state = 'RI' and latitude > 41.8")
    assert sorted(d.collect()) == sorted(b.collect())


@pytest.mark.skipif(not HAVE_REF, reason="reference checkout not mounted")
def test_tpch_index_template_rollup(tmp_path, df_small):
    from spark_druid_olap_amd.models import tpch

    cols = [c for c, _ in tpch.FLAT_SCHEMA]
    df = df_small[cols].copy()
    df.to_csv(tmp_path / "part-00000", sep="|", header=False, index=False)
    spec = IndexSpec.parse(f"{REF}/tpch_index_task.json.template", data_dir=str(tmp_path))
    assert "o_orderkey" in spec.dimensions and "count" not in spec.dimensions
    ds = ingest(spec)
    assert ds.rollup and ds.time_unit_ms == 86_400_000
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", df, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(datasource="tpch"))
    inside = df[(df.l_shipdate >= "1993-01-01") & (df.l_shipdate < "1997-12-31")]
    got = dict(s.sql("select l_returnflag, count(*) from orderLineItemPartSupplier group by l_returnflag").collect())
    assert got == inside.groupby("l_returnflag").size().to_dict()  # count(*) -> longSum(count) over rollup
    q = s.sql("select l_returnflag, count(*) from orderLineItemPartSupplier group by l_returnflag").druid_query_specs()[0]
    assert q.aggregations[0].type == "longSum" and q.aggregations[0].fieldName == "count"
    got = dict(s.sql("select s_nation, sum(l_quantity) from orderLineItemPartSupplier group by s_nation").collect())
    exp = inside.groupby("s_nation").l_quantity.sum()
    for k, v in got.items():
        assert v == pytest.approx(exp[k])
    # the JS metric l_discount = sum(l_extendedprice * l_discount) (tpch_index_task.json.template:150-156)
    got = s.sql("select sum(l_discount) from orderLineItemPartSupplier").collect()[0][0]
    assert got == pytest.approx(float((inside.l_extendedprice * inside.l_discount).sum()), rel=1e-9)
