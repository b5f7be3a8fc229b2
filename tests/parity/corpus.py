"""Session fixture + runner for the reference SQL corpus (tests/parity/extract.py)."""
import math
import os
import re

def build_session(sf=0.01, device="cpu", use_native=False):
    """Every table the reference's test suites query (TPC-H flat + star, select/datatype variants,
    zip codes).  ``device="cuda"`` + ``use_native=True`` runs the same corpus through the HIP engine."""
    import json

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.segment.ingest import ingest
    from spark_druid_olap_amd.session import Session

    flat = tpch.generate_flat(sf, device)
    ds = tpch.to_datasource(flat, profile="test")
    df = tpch.to_pandas(flat)
    s = Session(engine=Engine(use_native=use_native))
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", df, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl())
    for name, frame in tpch.star_tables(df).items():
        s.register_table(name, frame, schema=tpch.STAR_SCHEMAS[name])
    s.sql(tpch.star_ddl())
    # SelectQueryTest.scala:37-63: push_project_and_filters variants of the flat and star tables
    nah = ', nonAggregateQueryHandling "push_project_and_filters"'
    s.sql(tpch.druid_ddl(table="orderLineItemPartSupplier_select", extra_options=nah,
                         star_schema='{"factTable" : "orderLineItemPartSupplier_select", "relations" : []}'))
    s.sql(tpch.star_ddl(table="lineitem_select", extra_options=nah))
    # DataTypesTest.scala:53-134: the same rows with date / timestamp typed source columns
    import pandas as pd

    dt = df.copy()
    dt["o_orderdate"] = pd.to_datetime(dt["o_orderdate"]).dt.date
    dt["l_commitdate"] = pd.to_datetime(dt["l_commitdate"]).dt.date
    dt["l_receiptdate"] = pd.to_datetime(dt["l_receiptdate"])
    typ = {"o_orderdate": "date", "l_commitdate": "date", "l_receiptdate": "timestamp"}
    schema1 = [(c, typ.get(c, t)) for c, t in tpch.FLAT_SCHEMA]
    s.register_table("orderLineItemPartSupplierDataTypesBase", dt, schema=schema1)
    dt2 = dt.copy()
    dt2["l_shipdate"] = pd.to_datetime(dt2["l_shipdate"])
    s.register_table("orderLineItemPartSupplierDataTypes2Base", dt2,
                     schema=[(c, "timestamp" if c == "l_shipdate" else t) for c, t in schema1])
    for suffix, src in (("datatypes", "orderLineItemPartSupplierDataTypesBase"),
                        ("datatypes2", "orderLineItemPartSupplierDataTypes2Base")):
        tn = f"orderLineItemPartSupplier_{suffix}"
        s.sql(tpch.druid_ddl(table=tn, source=src, star_schema=f'{{"factTable" : "{tn}", "relations" : []}}'))
    import tempfile

    from parity.zipcodes import index_spec, write_csv

    zdir = tempfile.mkdtemp(prefix="sdo_zip_")
    zcsv = write_csv(os.path.join(zdir, "zip_codes_states.csv"))
    for dsn, full in (("zipCodes", False), ("zipCodesAll", True)):
        s.register_datasource(ingest(index_spec(dsn, full, zdir), device=device))
    s.sql(f"""CREATE TABLE zipCodesBase(record_date string, zip_code string, latitude double, longitude double,
      city string, state string, county string) USING com.databricks.spark.csv
      OPTIONS (path "{zcsv}", header "false", delimiter ",")""")
    for full in (False, True):
        infos = json.dumps([
            {"column": "city", **({"druidColumn": "city"} if full else {}), "hllMetric": "unique_city",
             "sketchMetric": "city_sketch"},
            {"column": "latitude", "spatialIndex": {"druidColumn": "coordinates", "spatialPosition": 0,
                                                    "minValue": -90.0, "maxValue": 90.0}},
            {"column": "longitude", "spatialIndex": {"druidColumn": "coordinates", "spatialPosition": 1,
                                                     "minValue": -180.0, "maxValue": 180.0}}])
        s.sql(f"""CREATE TABLE if not exists {'zipCodesFull' if full else 'zipCodes'} USING org.sparklinedata.druid
          OPTIONS (sourceDataframe "default.zipCodesBase", timeDimensionColumn "record_date",
          druidDatasource "{'zipCodesAll' if full else 'zipCodes'}", columnInfos '{infos}',
          nonAggregateQueryHandling "push_project_and_filters", allowTopNRewrite "true")""")
    return s


def norm_rows(rows):
    out = []
    for r in rows:
        t = []
        for v in r:
            if isinstance(v, float):
                v = None if math.isnan(v) else round(v, 1)
            elif hasattr(v, "isoformat"):
                v = str(v)[:19]
            t.append(v)
        out.append(tuple(t))
    # exact cells order first, floats numerically after: a 1-decimal rounding difference must not
    # reorder otherwise-equal result sets
    return sorted(out, key=lambda r: (tuple((x is None, str(x)) for x in r if not isinstance(x, float)),
                                      tuple(-1e300 if x is None else x for x in r if isinstance(x, float))))


def rows_equal(a, b):
    """Cell-by-cell with the reference's 1-decimal rounding tolerance (tc/AbstractTest.scala:184-190)."""
    if len(a) != len(b):
        return False
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            if isinstance(u, float) or isinstance(v, float):
                if u is None or v is None or abs(u - v) > 0.11 + 1e-9 * max(abs(u), abs(v)):
                    return False
            elif u != v:
                return False
    return True


def to_base(sql):
    return re.sub(r"\borderLineItemPartSupplier\b", "orderLineItemPartSupplierBase",
                  re.sub(r"\blineitem\b", "lineitembase", sql))


def run_case(s, case):
    """-> (status, detail) ; status in ok | shape | mismatch | error"""
    fn, name, kind, sql, ndruid, base_sql = case
    try:
        d = s.sql(sql)
        nq = len(d.druid_queries())
        rows = norm_rows(d.collect())
    except Exception as e:  # noqa: BLE001
        return "error", f"{type(e).__name__}: {str(e)[:200]}"
    bsql = base_sql or to_base(sql)
    cmp_status = None
    if bsql != sql:
        try:
            b = norm_rows(s.sql(bsql).collect())
            if not rows_equal(rows, b):
                ordered = "limit" in sql.lower()
                if not (ordered and len(b) == len(rows)):
                    cmp_status = f"rows differ ({len(rows)} vs {len(b)})"
        except Exception as e:  # noqa: BLE001
            cmp_status = f"base failed: {type(e).__name__}: {str(e)[:120]}"
    if cmp_status:
        return "mismatch", cmp_status
    if ndruid is not None and nq != ndruid:
        return "shape", f"druid queries {nq} != {ndruid}"
    return "ok", ""
