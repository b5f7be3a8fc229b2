"""Druid HTTP clients: broker/historical query client, coordinator client, overlord client.

Parity: ``sd/client/DruidClient.scala`` (``DruidClient`` 130-372 with pooled connections 46-74,
``DruidQueryServerClient`` 385-452: query, ``timeBoundary``, ``segmentMetadata``;
``DruidCoordinatorClient`` 454-500) and ``sd/client/DruidOverlordClient.scala:51-129``
(submitTask / getTaskStatus / waitUntilTaskCompletes).  They talk to any Druid-compatible endpoint,
including this framework's own ``server/druid_http.py``.  Errors surface as
``DruidDataSourceException``; idempotent GETs retry with exponential backoff (``utils/retry.py``).
"""
from __future__ import annotations

import json
import threading
from typing import Any, Dict, List, Optional

import requests
from requests.adapters import HTTPAdapter

from ..query import spec as S
from . import smile
from ..utils.errors import DruidDataSourceException
from ..utils.retry import exec_with_backoff, retry_until

_POOLS: Dict[tuple, requests.Session] = {}
_LOCK = threading.Lock()


def _pool(max_total: int = 100, per_route: int = 20) -> requests.Session:
    """Process-wide pooled HTTP connections (ConnectionManager, DruidClient.scala:46-74)."""
    key = (max_total, per_route)
    with _LOCK:
        s = _POOLS.get(key)
        if s is None:
            s = requests.Session()
            ad = HTTPAdapter(pool_connections=max(1, max_total // max(per_route, 1)), pool_maxsize=per_route)
            s.mount("http://", ad)
            s.mount("https://", ad)
            _POOLS[key] = s
        return s


class DruidClient:
    def __init__(self, host: str, port: int, timeout_s: float = 300.0, use_smile: bool = False,
                 max_connections: int = 100, max_per_route: int = 20):
        self.base = f"http://{host}:{port}"
        self.timeout = timeout_s
        self.use_smile = use_smile  # Smile request bodies + responses (DruidClient.scala:183-189, 244-251)
        self.http = _pool(max_connections, max_per_route)

    def _check(self, r: requests.Response):
        if r.status_code >= 300:
            body = r.content
            if smile.is_smile(body):
                body = json.dumps(smile.loads(body)).encode()
            raise DruidDataSourceException(f"{r.request.method} {r.url} -> {r.status_code}: {body[:500]!r}")
        if not r.content:
            return None
        return smile.decode_body(r.content, r.headers.get("Content-Type"))

    def post(self, path: str, obj: Any):
        if self.use_smile:
            data, hdr = smile.dumps(obj), {"Content-Type": smile.MIME, "Accept": smile.MIME}
        else:
            data, hdr = json.dumps(obj), {"Content-Type": "application/json"}
        try:
            r = self.http.post(self.base + path, data=data, headers=hdr, timeout=self.timeout)
        except requests.RequestException as e:
            raise DruidDataSourceException(str(e)) from e
        return self._check(r)

    def get(self, path: str, retry: bool = True):
        def go():
            return self._check(self.http.get(self.base + path, timeout=self.timeout))
        if not retry:
            return go()
        return exec_with_backoff(go, max_attempts=4, start_s=0.05,
                                 retry_on=(requests.RequestException, DruidDataSourceException),
                                 should_retry=lambda e: not (isinstance(e, DruidDataSourceException) and "-> 4" in str(e)))

    def delete(self, path: str):
        try:
            return self._check(self.http.delete(self.base + path, timeout=self.timeout))
        except requests.RequestException as e:
            raise DruidDataSourceException(str(e)) from e


class DruidQueryServerClient(DruidClient):
    """Broker / historical: native queries, timeBoundary, segmentMetadata."""

    def execute_query(self, q) -> List[Dict[str, Any]]:
        body = q.to_json() if isinstance(q, S.QuerySpec) else q
        return self.post("/druid/v2/", body)

    def cancel_query(self, query_id: str):
        return self.delete(f"/druid/v2/{query_id}")

    def time_boundary(self, datasource: str) -> Dict[str, str]:
        r = self.post("/druid/v2/", {"queryType": "timeBoundary", "dataSource": datasource})
        return r[0]["result"]

    def metadata(self, datasource: str, intervals: Optional[List[str]] = None) -> Dict[str, Any]:
        body = {"queryType": "segmentMetadata", "dataSource": datasource, "merge": True,
                "analysisTypes": ["cardinality", "interval"]}
        if intervals:
            body["intervals"] = intervals
        r = self.post("/druid/v2/", body)
        return r[0]

    def datasources(self) -> List[str]:
        return self.get("/druid/v2/datasources")


class DruidCoordinatorClient(DruidClient):
    def leader(self) -> str:
        return self.get("/druid/coordinator/v1/leader")

    def servers_info(self) -> List[Dict[str, Any]]:
        return self.get("/druid/coordinator/v1/servers?full")

    def datasource_info(self, datasource: str) -> Dict[str, Any]:
        return self.get(f"/druid/coordinator/v1/datasources/{datasource}")

    def segments(self, datasource: str, full: bool = True) -> List[Any]:
        return self.get(f"/druid/coordinator/v1/datasources/{datasource}/segments" + ("?full" if full else ""))


class DruidOverlordClient(DruidClient):
    def submit_task(self, task_spec: Dict[str, Any]) -> str:
        return self.post("/druid/indexer/v1/task", task_spec)["task"]

    def task_status(self, task_id: str) -> Dict[str, Any]:
        return self.get(f"/druid/indexer/v1/task/{task_id}/status")["status"]

    def wait_until_task_completes(self, task_id: str, timeout_s: float = 600.0, poll_s: float = 1.0):
        st = retry_until(lambda: self.task_status(task_id), lambda s: s.get("status") in ("SUCCESS", "FAILED"),
                         timeout_s=timeout_s, delay_s=poll_s)
        if st.get("status") != "SUCCESS":
            raise DruidDataSourceException(f"task {task_id} failed: {st}")
        return st


def discover_clients(druid_host: str = "localhost", druid_path: str = "/druid", qualify_names: bool = False,
                     use_smile: bool = False):
    """(broker, coordinator, overlord) clients located through service discovery, the way the
    reference finds them through ZooKeeper (CuratorConnection.scala:203-209)."""
    from .discovery import Discovery, registry_for

    d = Discovery(registry_for(druid_host), druid_path, qualify_names)
    out = []
    for svc, cls in (("broker", DruidQueryServerClient), ("coordinator", DruidCoordinatorClient),
                     ("overlord", DruidOverlordClient)):
        hp = d.get_service(svc)
        if hp is None:
            raise DruidDataSourceException(f"no {svc} registered under {druid_path}/discovery at {druid_host}")
        out.append(cls(hp[0], hp[1], use_smile=use_smile) if cls is DruidQueryServerClient else cls(hp[0], hp[1]))
    return tuple(out)
