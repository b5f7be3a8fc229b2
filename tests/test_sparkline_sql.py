"""The reference's SparklineSQLTest suite (``tc/SparklineSQLTest.scala:25-305``), case by case:
metadata views, CLEAR DRUID CACHE, the SPL parse error, ON DRUIDDATASOURCE ... EXECUTE QUERY (broker
and historical) and EXPLAIN DRUID REWRITE."""
import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.session import Session
from spark_druid_olap_amd.sql.parser import ParseError

T = "orderLineItemPartSupplier"


@pytest.fixture(scope="module")
def sess(ds_small, df_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table(T + "Base", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    return s


@pytest.mark.parametrize("view,min_rows", [("d$druidrelations", 1), ("d$druidservers", 1),
                                           ("d$druidsegments", 1), ("d$druidserverassignments", 1)])
def test_metadata_views(sess, view, min_rows):
    # tc/SparklineSQLTest.scala:25-43 (druidrelations / druidservers / druidsegments / assignments)
    df = sess.sql(f"select * from `{view}`")
    assert df.count() >= min_rows


@pytest.mark.parametrize("stmt", ["clear druid cache localhost", "clear druid cache"])
def test_clear_cache(sess, stmt):
    # tc/SparklineSQLTest.scala:45-53; queries still answer after the cache is dropped
    sess.sql(stmt)
    assert sess.sql(f"select count(*) from {T}").collect()[0][0] > 0


def test_parse_exception(sess):
    # tc/SparklineSQLTest.scala:55-71: the misspelt command fails to parse and says where
    with pytest.raises(ParseError) as ei:
        sess.sql("clear drud cache")
    msg = str(ei.value)
    assert "drud" in msg


_Q = """{
  "jsonClass" : "GroupByQuerySpec", "queryType" : "groupBy", "dataSource" : "tpch",
  "dimensions" : [ {"jsonClass" : "DefaultDimensionSpec", "type" : "default",
                    "dimension" : "l_returnflag", "outputName" : "l_returnflag"},
                   {"jsonClass" : "DefaultDimensionSpec", "type" : "default",
                    "dimension" : "l_linestatus", "outputName" : "l_linestatus"} ],
  "granularity" : "all",
  "aggregations" : [ {"jsonClass" : "FunctionAggregationSpec", "type" : "count", "name" : "count",
                      "fieldName" : "count"},
                     {"jsonClass" : "FunctionAggregationSpec", "type" : "doubleSum", "name" : "s",
                      "fieldName" : "l_extendedprice"} ],
  "intervals" : [ "1993-01-01T00:00:00.000Z/1997-12-31T00:00:01.000Z" ]
}"""


@pytest.mark.parametrize("historical", [False, True])
def test_exec_query(sess, historical):
    # tc/SparklineSQLTest.scala:73-280 (execQueryHistorical, execQuery1): a hand-written QuerySpec
    # runs as is, through the broker path or per segment batch, with the same answer
    using = "using historical " if historical else ""
    r = sess.sql(f"on druiddatasource {T} {using}execute query {_Q}").to_pandas()
    ref = sess.sql(f"on druiddatasource {T} execute query {_Q}").to_pandas()
    assert len(r) == 4 and set(r["l_returnflag"]) == {"A", "N", "R"}
    key = ["l_returnflag", "l_linestatus"]
    a, b = r.sort_values(key).reset_index(drop=True), ref.sort_values(key).reset_index(drop=True)
    assert (a["count"] == b["count"]).all()
    assert ((a["s"] - b["s"]).abs() <= 1e-6 * b["s"].abs().max()).all()


@pytest.mark.parametrize("sql,pushed", [
    # tc/SparklineSQLTest.scala:282-289
    (f"""SELECT COUNT(DISTINCT CAST(`{T}`.`l_shipdate` AS TIMESTAMP)) AS `ctd_date_string_ok`
        FROM `{T}` HAVING (COUNT(1) > 0)""", True),
    # 291-297
    (f"SELECT p_name, count(*) FROM `{T}` group by p_name", True),
    # 299-305: l_quantity is a metric of this index -- Druid cannot group on a metric, so the
    # rewrite keeps the aggregate in the host plan (the reference test only prints the plan)
    (f"SELECT l_quantity + 1, count(*) FROM `{T}` group by l_quantity + 1", False),
])
def test_explain_druid_rewrite(sess, sql, pushed):
    rows = sess.sql("explain druid rewrite " + sql).collect()
    txt = "\n".join(str(r[0]) for r in rows)
    if pushed:
        assert "DruidQuery" in txt and "QuerySpec" in txt, txt
    else:
        assert "Aggregate" in txt and "Relation" in txt, txt
