"""Synthetic stand-in for the reference's zip-code fixture (``src/test/resources/zipCodes/sample``,
1,000 rows of ``record_date,zip_code,lat,long,city,state,county``) and its two index specs
(``zip_code(All).json.template``: a spatial ``coordinates`` dimension over lat/long, a count, a
hyperUnique metric on city and a 16384-entry theta sketch on city; the "All" variant also keeps
lat/long/city as dimensions).

The corpus compares every Druid-backed result with the same SQL over the base table, so any data of
this shape exercises the same paths; the generator keeps the fixture's properties the queries depend
on (two record dates, US-like latitudes/longitudes including a few Caribbean points below 18 degrees,
repeated city names across zip codes, states starting with 'N')."""
import csv
import os

import numpy as np

STATES = ["NY", "NJ", "NC", "ND", "NE", "NH", "NM", "NV", "PR", "MA", "CT", "PA", "CA", "TX", "FL", "OH",
          "VI", "AK", "HI", "WA"]
SYL = ["holt", "ad", "jun", "tas", "ville", "burg", "spring", "field", "lake", "mont", "ridge", "port", "san",
       "ford", "ham", "ton", "dale", "wood", "brook", "haven"]


def _name(rng, k=2):
    return "".join(SYL[i] for i in rng.integers(0, len(SYL), k)).capitalize()


def write_csv(path: str, n: int = 1000, seed: int = 11) -> str:
    rng = np.random.default_rng(seed)
    cities = [_name(rng) for _ in range(420)]
    counties = [_name(rng, 1) for _ in range(150)]
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        for i in range(n):
            st = STATES[int(rng.integers(0, len(STATES)))]
            if st in ("PR", "VI"):
                lat, lon = rng.uniform(17.6, 18.5), rng.uniform(-67.3, -64.5)
            elif st in ("AK",):
                lat, lon = rng.uniform(55, 70), rng.uniform(-165, -135)
            elif st == "HI":
                lat, lon = rng.uniform(18.9, 22.2), rng.uniform(-160, -154.8)
            else:
                lat, lon = rng.uniform(25, 49), rng.uniform(-124, -67)
            date = "2016-01-01" if rng.random() < 0.8 else "2015-06-01"
            w.writerow([date, f"{500 + 7 * i:05d}", f"{lat:.6f}", f"{lon:.6f}",
                        cities[int(rng.integers(0, len(cities)))], st, counties[int(rng.integers(0, len(counties)))]])
    return path


def index_spec(datasource: str, full: bool, data_dir: str) -> dict:
    dims = ["zip_code", "state", "county"] + (["lat", "long", "city"] if full else [])
    return {"type": "index", "spec": {
        "dataSchema": {
            "dataSource": datasource,
            "parser": {"type": "string", "parseSpec": {
                "format": "csv", "timestampSpec": {"column": "record_date", "format": "iso"},
                "columns": ["record_date", "zip_code", "lat", "long", "city", "state", "county"],
                "delimiter": ",",
                "dimensionsSpec": {"dimensions": dims, "dimensionExclusions": [],
                                   "spatialDimensions": [{"dimName": "coordinates", "dims": ["lat", "long"]}]}}},
            "metricsSpec": [{"type": "count", "name": "count"},
                            {"type": "hyperUnique", "name": "unique_city", "fieldName": "city"},
                            {"type": "thetaSketch", "name": "city_sketch", "fieldName": "city", "size": 16384}],
            "granularitySpec": {"type": "uniform", "segmentGranularity": "MONTH", "queryGranularity": "all",
                                "intervals": ["2015-01-01/2016-12-31"]}},
        "ioConfig": {"type": "index", "firehose": {"type": "local", "baseDir": data_dir, "filter": "*.csv"}},
        "tuningConfig": {"type": "index", "partitionsSpec": {"type": "hashed", "targetPartitionSize": 5000000}}}}
