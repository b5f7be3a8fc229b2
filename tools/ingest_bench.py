"""Ingest benchmark: the reference's quickstart TPC-H index task over a flattened TPC-H TSV.

``python tools/ingest_bench.py --sf 1 --device cuda [--dir /tmp/tpch_tsv] [--keep]``

1. Writes a synthetic flattened TPC-H SF-``sf`` TSV (``|``-delimited, the 53 columns of
   ``quickstart/tpch_index_task.json.template``'s ``columns`` list) in chunks of 2M rows.
2. Ingests it with the same index spec as the quickstart template (schemaless dimensions,
   count / doubleSum / longSum / javascript metrics, DAY query granularity, MONTH segments,
   interval 1993-01-01/1997-12-31) built programmatically -- the template itself is not on the
   GPU box.
3. Prints one JSON line: rows read, rows after rollup, seconds, input MB/s, plus a check query
   (count and sum(l_quantity) by l_returnflag) against the generator's own numbers.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

METRICS = [
    {"type": "count", "name": "count"},
    {"type": "doubleSum", "name": "o_totalprice", "fieldName": "o_totalprice"},
    {"type": "longSum", "name": "sum_l_quantity", "fieldName": "l_quantity"},
    {"type": "doubleSum", "name": "l_extendedprice", "fieldName": "l_extendedprice"},
    {"type": "javascript", "name": "l_tax", "fieldNames": ["l_extendedprice", "l_discount", "l_tax"],
     "fnAggregate": "function(current, l_extendedprice, l_discount, l_tax) "
                    "{ return current + (l_extendedprice *(1 - l_discount) * l_tax); }",
     "fnCombine": "function(partialA, partialB) { return partialA + partialB; }",
     "fnReset": "function() { return 0; }"},
    {"type": "javascript", "name": "l_discount", "fieldNames": ["l_extendedprice", "l_discount"],
     "fnAggregate": "function(current, l_extendedprice, l_discount) { return current + (l_extendedprice * l_discount); }",
     "fnCombine": "function(partialA, partialB) { return partialA + partialB; }",
     "fnReset": "function() { return 0; }"},
    {"type": "longSum", "name": "sum_ps_availqty", "fieldName": "ps_availqty"},
    {"type": "doubleSum", "name": "ps_supplycost", "fieldName": "ps_supplycost"},
    {"type": "doubleSum", "name": "c_acctbal", "fieldName": "c_acctbal"},
]


def index_spec(data_dir: str) -> dict:
    from spark_druid_olap_amd.models import tpch

    cols = [c for c, _ in tpch.FLAT_SCHEMA]
    return {"type": "index", "spec": {
        "dataSchema": {
            "dataSource": "tpch",
            "parser": {"type": "string", "parseSpec": {
                "format": "tsv", "timestampSpec": {"column": "l_shipdate", "format": "iso"}, "columns": cols,
                "delimiter": "|", "dimensionsSpec": {"dimension": [], "dimensionExclusions": [],
                                                     "spatialDimensions": []}}},
            "metricsSpec": METRICS,
            "granularitySpec": {"type": "uniform", "segmentGranularity": "MONTH", "queryGranularity": "DAY",
                                "intervals": ["1993-01-01/1997-12-31"]}},
        "ioConfig": {"type": "index", "firehose": {"type": "local", "baseDir": data_dir, "filter": "part*"}}}}


def write_tsv(sf: float, out_dir: str, chunk: int = 2_000_000) -> dict:
    import numpy as np
    import pyarrow as pa
    import pyarrow.csv as pacsv
    import torch

    from spark_druid_olap_amd.models import tpch

    os.makedirs(out_dir, exist_ok=True)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    flat = tpch.generate_flat(sf, dev)
    n = flat.num_rows
    ship = flat.ship_day[:n].cpu().numpy()
    qty = flat.nums["l_quantity"]
    qv = qty[0][:n].cpu().numpy().astype(np.float64)
    if qty[1] == "decimal":
        qv = qv / (10.0 ** qty[2])
    rf_d, rf_ids = flat.dims["l_returnflag"]
    rf = rf_d.decode(rf_ids[:n].cpu().numpy().astype(np.int64))
    path = os.path.join(out_dir, "part-00000")
    t0 = time.perf_counter()
    with open(path, "wb") as f:
        for a in range(0, n, chunk):
            df = tpch.to_pandas(flat, a, a + chunk)
            tbl = pa.Table.from_pandas(df, preserve_index=False)
            buf = pa.BufferOutputStream()
            pacsv.write_csv(tbl, buf, pacsv.WriteOptions(include_header=False, delimiter="|", quoting_style="none"))
            f.write(buf.getvalue().to_pybytes())
            print(f"[ingest_bench] wrote {min(n, a + chunk)}/{n} rows", flush=True)
    # expected answer of the check query, straight from the generator (rows shipped in the interval)
    import pandas as pd

    ship_str = pd.Series(tpch.date_strings(tpch.START_DAY, tpch.DATE_DICT_END), dtype=object).to_numpy()[
        ship.astype(np.int64) - tpch.START_DAY]
    inside = (ship_str >= "1993-01-01") & (ship_str < "1997-12-31")
    exp = pd.DataFrame({"rf": rf[inside], "q": qv[inside]}).groupby("rf").agg(n=("q", "size"), q=("q", "sum"))
    return {"rows": n, "bytes": os.path.getsize(path), "write_s": time.perf_counter() - t0,
            "expected": {k: [int(v.n), float(v.q)] for k, v in exp.iterrows()}}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--dir", default="/tmp/sdo_tpch_tsv")
    ap.add_argument("--block-mb", type=int, default=64)
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    import torch

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.query import spec as S
    from spark_druid_olap_amd.segment.ingest import ingest

    gen = write_tsv(a.sf, a.dir)
    print(f"[ingest_bench] TSV {gen['bytes'] / 1e9:.2f} GB written in {gen['write_s']:.1f}s", flush=True)
    if a.device.startswith("cuda"):
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    ds = ingest(index_spec(a.dir), device=a.device, block_bytes=a.block_mb << 20)
    if a.device.startswith("cuda"):
        torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    q = S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("l_returnflag")],
                           aggregations=[S.FunctionAggregationSpec("longSum", "n", "count"),
                                         S.FunctionAggregationSpec("longSum", "q", "sum_l_quantity")],
                           intervals=["1993-01-01/1997-12-31"])
    r = Engine(use_native=a.device.startswith("cuda")).execute(q, ds)
    from spark_druid_olap_amd.engine.columns import materialize

    got = {k: [int(n), float(qq)] for k, n, qq in zip(materialize(r.data["l_returnflag"]).tolist(),
                                                        r.data["n"].tolist(), r.data["q"].tolist())}
    ok = all(got.get(k, [0, 0])[0] == v[0] and abs(got.get(k, [0, 0])[1] - v[1]) < 1e-6 * max(1, v[1])
             for k, v in gen["expected"].items())
    print(json.dumps({"metric": "ingest_seconds", "sf": a.sf, "device": a.device, "input_rows": ds.ingested_rows,
                      "rolled_rows": ds.num_rows, "dims": len(ds.dims), "metrics": len(ds.metrics),
                      "input_gb": round(gen["bytes"] / 1e9, 3), "ingest_s": round(secs, 2),
                      "input_mb_per_s": round(gen["bytes"] / 1e6 / secs, 1), "segments": len(ds.segments),
                      "check_ok": ok}), flush=True)
    if not a.keep:
        shutil.rmtree(a.dir, ignore_errors=True)
    if not ok:
        print("expected", gen["expected"], "got", got)
        sys.exit(1)


if __name__ == "__main__":
    main()
