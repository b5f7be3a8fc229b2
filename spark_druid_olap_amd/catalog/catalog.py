"""Session catalog: databases, base tables, views and Druid-backed relations.

Parity:
  * ``DefaultSource.createRelation`` (``sd/DefaultSource.scala:32-194``): required options, JSON
    options (columnMapping, columnInfos, functionalDependencies, starSchema), relation creation.
  * ``DruidRelationInfo`` / ``MappingBuilder.buildMapping`` / ``DruidRelationColumn``
    (``sd/metadata/DruidRelationInfo.scala:39-252``, ``sd/metadata/DruidRelationColumn.scala:36-224``):
    every column of every star-schema table maps to the time dimension, a dimension, a metric, a
    spatial axis, or an HLL / theta-sketch metric.
  * ``DruidMetadataCache`` (``sd/metadata/DruidMetadataCache.scala:176-297``): here the "cluster" is
    the in-process registry of device-resident datasources; ``clear_cache`` backs
    ``CLEAR DRUID CACHE``.
  * Multi-database lookup (``tc/MultiDBTest.scala``): names resolve as ``[db.]table``.
"""
from __future__ import annotations

import json
import os
import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import pandas as pd

from ..sql.types import AnalysisError, base, to_series
from .functional_deps import DependencyGraph, FunctionalDependency
from .options import REQUIRED, DruidRelationOptions
from .star_schema import StarSchema, StarSchemaInfo

DRUID_PROVIDERS = ("org.sparklinedata.druid", "sparklinedata.druid", "druid")
CSV_PROVIDERS = ("com.databricks.spark.csv", "csv", "org.apache.spark.sql.csv")
SUPPORTED_TYPES = ("tinyint", "smallint", "int", "bigint", "float", "double", "decimal", "string", "date",
                   "timestamp", "boolean")


class Table:
    kind = "table"

    def __init__(self, db: str, name: str, schema: List[Tuple[str, str]]):
        self.db = db
        self.name = name
        self.schema = schema

    @property
    def qualified_name(self) -> str:
        return f"{self.db}.{self.name}"

    def column_names(self) -> List[str]:
        return [c for c, _ in self.schema]


class BaseTable(Table):
    """A plain (host-resident) table: a pandas frame, a CSV/Parquet/JSON file set, or a loader."""

    kind = "base"

    def __init__(self, db, name, schema, data: Optional[pd.DataFrame] = None,
                 loader: Optional[Callable[[], pd.DataFrame]] = None, provider: Optional[str] = None,
                 options: Optional[dict] = None):
        super().__init__(db, name, schema)
        self._data = data
        self._loader = loader
        self.provider = provider
        self.options = options or {}
        self.cached = False
        self._lock = threading.Lock()

    @property
    def has_data(self) -> bool:
        return self._data is not None or self._loader is not None

    def frame(self) -> pd.DataFrame:
        with self._lock:
            if self._data is None:
                if self._loader is None:
                    raise AnalysisError(f"table {self.qualified_name} has no data (schema-only registration)")
                raw = self._loader()
                self._data = conform(raw, self.schema)
            return self._data


def conform(df: pd.DataFrame, schema: List[Tuple[str, str]]) -> pd.DataFrame:
    cols = {}
    lower = {c.lower(): c for c in df.columns}
    for c, t in schema:
        src = c if c in df.columns else lower.get(c.lower())
        if src is None:
            raise AnalysisError(f"column {c} missing from data")
        cols[c] = to_series(df[src], t)
    return pd.DataFrame(cols)


def csv_loader(path: str, schema: List[Tuple[str, str]], options: dict) -> Callable[[], pd.DataFrame]:
    def load():
        sep = options.get("delimiter", options.get("sep", ","))
        header = str(options.get("header", "false")).lower() == "true"
        files = []
        if os.path.isdir(path):
            for f in sorted(os.listdir(path)):
                if not f.startswith((".", "_")):
                    files.append(os.path.join(path, f))
        else:
            files = [path]
        frames = []
        for f in files:
            frames.append(pd.read_csv(f, sep=sep, header=0 if header else None, dtype=str, keep_default_na=False,
                                      na_values=[""], usecols=range(len(schema)), names=None if header else
                                      [c for c, _ in schema], engine="c"))
        df = pd.concat(frames, ignore_index=True) if frames else pd.DataFrame(columns=[c for c, _ in schema])
        if header:
            df.columns = [c for c, _ in schema][: len(df.columns)]
        return df

    return load


class ViewTable(Table):
    kind = "view"

    def __init__(self, db, name, query, text: str = "", schema=None):
        super().__init__(db, name, schema or [])
        self.query = query
        self.text = text


# ------------------------------------------------------------------------------------------------
@dataclass
class SpatialIndexInfo:
    druid_column: str
    position: int
    min_value: Optional[float] = None
    max_value: Optional[float] = None


@dataclass
class DruidRelationColumn:
    column: str                      # SQL column
    druid_column: Optional[str]      # direct link (dimension / metric / __time)
    kind: Optional[str]              # time | dimension | metric | None (only indirect links)
    sql_type: str
    spatial: Optional[SpatialIndexInfo] = None
    hll_metric: Optional[str] = None
    sketch_metric: Optional[str] = None
    cardinality: int = 1
    metric_kind: Optional[str] = None  # long | double | decimal | hll

    @property
    def is_dimension(self) -> bool:
        return self.kind in ("dimension", "time")

    @property
    def is_time(self) -> bool:
        return self.kind == "time"

    @property
    def is_metric(self) -> bool:
        return self.kind == "metric"


class DruidRelationInfo:
    def __init__(self, source_name: str, time_dim_col: str, ds_name: str, datasource,
                 column_map: Dict[str, DruidRelationColumn], fds: List[FunctionalDependency],
                 star: StarSchema, options: DruidRelationOptions, raw_options: dict):
        self.source_name = source_name
        self.time_dim_col = time_dim_col
        self.ds_name = ds_name
        self.datasource = datasource
        self.column_map = column_map
        self.fds = fds
        self.star = star
        self.options = options
        self.raw_options = raw_options
        dims = [c.druid_column for c in column_map.values() if c.kind == "dimension"]
        self.dep_graph = DependencyGraph(dims, [FunctionalDependency(self._druid_name(f.col1),
                                                                     self._druid_name(f.col2), f.type) for f in fds])

    def _druid_name(self, col: str) -> str:
        c = self.column_map.get(col.lower())
        return c.druid_column if c is not None and c.druid_column else col

    def column(self, name: str) -> Optional[DruidRelationColumn]:
        return self.column_map.get(name.lower())

    def spatial_indexes(self) -> Dict[str, List[DruidRelationColumn]]:
        out: Dict[str, List[DruidRelationColumn]] = {}
        for c in self.column_map.values():
            if c.spatial is not None:
                out.setdefault(c.spatial.druid_column, []).append(c)
        for v in out.values():
            v.sort(key=lambda c: c.spatial.position)
        return out

    def estimate_cardinality(self, druid_dims: List[str]) -> int:
        ds = self.datasource

        def card(d):
            if d in ds.dims:
                return len(ds.dims[d].dictionary)
            return 1000
        return self.dep_graph.estimate_cardinality(druid_dims, card)


class DruidTable(Table):
    kind = "druid"

    def __init__(self, db, name, schema, info: DruidRelationInfo, options: dict):
        super().__init__(db, name, schema)
        self.info = info
        self.options = options


# ------------------------------------------------------------------------------------------------
class DruidCluster:
    """In-process registry of device-resident datasources (the reference's metadata cache +
    coordinator/broker view, ``sd/metadata/DruidMetadataCache.scala``)."""

    def __init__(self):
        self.datasources: Dict[str, Any] = {}
        self.generation = 0        # datasource registry (plan caches key on it)
        self.meta_generation = 0   # discovery / metadata views
        self._lock = threading.Lock()
        self.discovery = None
        self.server_name = "gpu:0"

    def attach_discovery(self, disc, rank: int = 0, server_info: Optional[dict] = None) -> None:
        """Announce this rank as a historical, announce its segments, and clear the metadata cache
        whenever any server or segment comes or goes (CuratorConnection.scala:77-133)."""
        if self.discovery is disc:
            return
        self.discovery = disc
        self.server_name = f"gpu:{rank}"
        disc.announce_server(self.server_name, server_info or {"type": "historical", "tier": "_default_tier",
                                                               "priority": 0, "rank": rank})
        for name, ds in list(self.datasources.items()):
            self._announce(name, ds)
        disc.watch_membership(lambda ev, path: self.clear_cache())

    def _announce(self, name: str, ds) -> None:
        if self.discovery is None:
            return
        for s in getattr(ds, "segments", []) or []:
            self.discovery.announce_segment(self.server_name, s.identifier, {"dataSource": name})

    def register(self, ds, name: Optional[str] = None) -> None:
        with self._lock:
            self.datasources[name or ds.name] = ds
            self.generation += 1
        self._announce(name or ds.name, ds)

    def get(self, name: str):
        ds = self.datasources.get(name)
        if ds is None:
            raise AnalysisError(f"Druid datasource '{name}' is not loaded (register it or ingest it first)")
        return ds

    def clear_cache(self, host: Optional[str] = None) -> None:
        """Metadata changed (a discovery watch fired, or CLEAR DRUID CACHE): the ``d$*`` views must
        be recomputed.  Only ``meta_generation`` moves: discovery events arrive asynchronously and
        at different moments on different ranks, and plans of every rank must stay in lock-step
        (preparing a pushed query issues collectives), so the registry ``generation`` that keys
        the plan caches moves only with registrations, which every rank performs alike."""
        with self._lock:
            self.meta_generation += 1


class Catalog:
    def __init__(self, cluster: Optional[DruidCluster] = None):
        self.dbs: Dict[str, Dict[str, Table]] = {"default": {}}
        self.current_db = "default"
        self.cluster = cluster or DruidCluster()
        self.temp: Dict[str, Table] = {}
        self._ver = [0]  # shared with session views (plan caches key on it)
        self._lock = threading.RLock()

    @property
    def version(self) -> int:
        return self._ver[0]

    @version.setter
    def version(self, v: int) -> None:
        self._ver[0] = v

    def session_view(self) -> "Catalog":
        """A per-client view (one HiveServer2 session): the databases, tables and Druid cluster are
        shared, the current database and temporary views are the session's own -- Spark's
        SessionCatalog split between the shared external catalog and session state."""
        v = Catalog.__new__(Catalog)
        v.dbs = self.dbs
        v.current_db = "default"
        v.cluster = self.cluster
        v.temp = {}
        v._ver = self._ver
        v._lock = self._lock
        return v

    def _split(self, parts) -> Tuple[Optional[str], str]:
        if isinstance(parts, str):
            parts = tuple(parts.split("."))
        if len(parts) == 1:
            return None, parts[0]
        return parts[-2].lower(), parts[-1]

    def create_database(self, name: str, if_not_exists: bool = False):
        with self._lock:
            if name.lower() in self.dbs:
                if not if_not_exists:
                    raise AnalysisError(f"Database '{name}' already exists")
                return
            self.dbs[name.lower()] = {}
            self.version += 1

    def use(self, name: str):
        if name.lower() not in self.dbs:
            raise AnalysisError(f"Database '{name}' not found")
        self.current_db = name.lower()

    def lookup(self, parts) -> Optional[Table]:
        db, name = self._split(parts)
        with self._lock:
            if db is None and name.lower() in self.temp:
                return self.temp[name.lower()]
            d = self.dbs.get(db or self.current_db)
            if d is None:
                return None
            return d.get(name.lower())

    def get(self, parts) -> Table:
        t = self.lookup(parts)
        if t is None:
            nm = parts if isinstance(parts, str) else ".".join(parts)
            raise AnalysisError(f"Table or view not found: {nm}")
        return t

    def register(self, t: Table, replace: bool = True, temporary: bool = False):
        with self._lock:
            if temporary:
                self.temp[t.name.lower()] = t
            else:
                d = self.dbs.setdefault(t.db, {})
                if not replace and t.name.lower() in d:
                    raise AnalysisError(f"Table {t.qualified_name} already exists")
                d[t.name.lower()] = t
            self.version += 1

    def drop(self, parts, if_exists=False):
        db, name = self._split(parts)
        with self._lock:
            if db is None and name.lower() in self.temp:
                del self.temp[name.lower()]
                self.version += 1
                return
            d = self.dbs.get(db or self.current_db, {})
            if name.lower() not in d:
                if if_exists:
                    return
                raise AnalysisError(f"Table or view not found: {name}")
            del d[name.lower()]
            self.version += 1

    def tables(self, db: Optional[str] = None) -> List[Table]:
        d = self.dbs.get((db or self.current_db).lower(), {})
        return list(d.values()) + (list(self.temp.values()) if db is None else [])

    def druid_tables(self) -> List[DruidTable]:
        out = []
        for d in self.dbs.values():
            out += [t for t in d.values() if isinstance(t, DruidTable)]
        return out

    # ------------------------------------------------------------------------------ DDL helpers
    def create_druid_relation(self, name: Tuple[str, ...], options: Dict[str, str]) -> DruidTable:
        """``DefaultSource.createRelation`` (sd/DefaultSource.scala:32-194)."""
        for r in REQUIRED:
            if r not in options:
                raise AnalysisError(f"{r} must be specified for a Druid datasource")
        src = self.get(options["sourceDataframe"])
        if not isinstance(src, BaseTable):
            raise AnalysisError(f"sourceDataframe {options['sourceDataframe']} must be a table")
        time_col = options["timeDimensionColumn"]
        ds_name = options["druidDatasource"]
        ds = self.cluster.get(ds_name)
        mapping = json.loads(options.get("columnMapping", "{}") or "{}")
        infos = json.loads(options.get("columnInfos", "[]") or "[]")
        fds = FunctionalDependency.parse_list(options.get("functionalDependencies", "[]"))
        db, tname = self._split(name)
        db = db or self.current_db
        if "starSchema" in options:
            ssi = StarSchemaInfo.parse(options["starSchema"])
        else:
            ssi = StarSchemaInfo(f"{db}.{tname}", [])
        src_short = src.name.lower()

        def columns_of(tab: str) -> List[str]:
            if tab.lower() in (src_short, src.qualified_name.lower()):
                return src.column_names()
            return self.get(tab).column_names()

        star = StarSchema.build(src.qualified_name, ssi, columns_of)
        ropts = DruidRelationOptions.from_options(options)
        colmap = build_mapping(self, src, star, mapping, infos, time_col, ds)
        info = DruidRelationInfo(src.qualified_name, time_col, ds_name, ds, colmap, fds, star, ropts, dict(options))
        t = DruidTable(db, tname, list(src.schema), info, dict(options))
        return t


def druid_column_kind(ds, druid_col: str, time_col: str) -> Tuple[Optional[str], Optional[str], int]:
    if druid_col == time_col or druid_col == "__time":
        return "time", None, max(len(getattr(ds, "time_values_host", ())) or 1, 1)
    if druid_col in ds.dims:
        return "dimension", None, len(ds.dims[druid_col].dictionary)
    if druid_col in ds.metrics:
        return "metric", ds.metrics[druid_col].kind, 1
    return None, None, 0


def build_mapping(cat: Catalog, src: BaseTable, star: StarSchema, name_mapping: dict, infos: list,
                  time_col: str, ds) -> Dict[str, DruidRelationColumn]:
    """MappingBuilder.buildMapping (sd/metadata/DruidRelationInfo.scala:221-252)."""
    user = {i["column"].lower(): i for i in infos}
    out: Dict[str, DruidRelationColumn] = {}
    for tname, st in star.table_map.items():
        tbl = src if st.parent is None else cat.get(tname)
        for col, sqlt in tbl.schema:
            if base(sqlt) not in SUPPORTED_TYPES:
                continue
            ci = user.get(col.lower(), {"column": col, "druidColumn": name_mapping.get(col, col)})
            dcol = ci.get("druidColumn")
            kind, mkind, card = (None, None, 0)
            if dcol is not None:
                kind, mkind, card = druid_column_kind(ds, dcol, time_col)
                if dcol == time_col:
                    dcol = "__time"
                if kind is None:
                    dcol = None
            sp = ci.get("spatialIndex")
            spatial = None
            if sp is not None:
                if sp.get("druidColumn") not in ds.dims and sp.get("druidColumn") not in getattr(ds, "spatial", {}):
                    continue
                spatial = SpatialIndexInfo(sp["druidColumn"], int(sp.get("spatialPosition", 0)),
                                           sp.get("minValue"), sp.get("maxValue"))
            hll = ci.get("hllMetric")
            sketch = ci.get("sketchMetric")
            if hll is not None and hll not in ds.metrics:
                hll = None
            if sketch is not None and sketch not in ds.metrics:
                sketch = None
            if kind is None and spatial is None and hll is None and sketch is None:
                continue
            if ci.get("cardinalityEstimate") is not None:
                card = int(ci["cardinalityEstimate"])
            out[col.lower()] = DruidRelationColumn(col, dcol, kind, sqlt, spatial, hll, sketch, card, mkind)
    return out
