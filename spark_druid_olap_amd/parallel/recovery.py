"""Elastic recovery: abort the communicator, rebuild it over the surviving ranks and re-home the
lost shards ("ncclCommAbort plus communicator rebuild on hang; degrade to fewer
GPUs by reassigning that GPU's segments").

The reference survives a dead historical because ZooKeeper drops it from the segment inventory
and Druid's coordinator re-loads its segments elsewhere from deep storage
(``sd/client/CuratorConnection.scala:77-133``, ``sd/metadata/DruidMetadataCache.scala:105-148``).
The MI355X analogue, one process per GPU:

* **Liveness**: every rank heart-beats into the job's rendezvous store (the TCPStore behind the
  default process group -- hosted by rank 0 or by torchrun's agent, which outlives any rank).
* **Detection**: a query's collective fails (the peer's socket closed, or the process-group
  timeout fired) -- the status-word agreement of ``parallel/fault.py`` covers ranks that are alive
  but failed their scan; this module covers ranks that are gone.
* **Agreement**: survivors register in the store under a recovery epoch; once every rank with a
  fresh heartbeat has arrived (or ``settle_s`` passed) the lowest arrived rank publishes the
  membership and everyone adopts it.
* **Rebuild**: the old communicator is aborted/destroyed and the default process group is
  re-initialised over the members on a fresh store prefix (``sdo/pg<epoch>``); ranks renumber.
* **Re-home**: the lost shards are loaded from the segment store (``DataSource.save`` layout,
  ``<store>/<datasource>/rank<r>``) by the member ``failed[i] -> members[i % len(members)]`` and
  concatenated into its shard (``DataSource.concat``), so the next query sees every row again.

``run_with_recovery`` wraps a query: on a collective failure it recovers once and re-runs it.
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .world import World, set_world

log = logging.getLogger("sdo.recovery")

_HB_PREFIX = "sdo/hb/"


class Membership:
    """Heartbeats of every rank in the rendezvous store (a background thread per rank)."""

    def __init__(self, store, rank: int, size: int, interval_s: float = 0.5):
        self.store = store
        self.rank = rank
        self.size = size
        self.interval_s = interval_s
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    def start(self) -> "Membership":
        self._beat()
        self._t = threading.Thread(target=self._loop, name=f"sdo-heartbeat-{self.rank}", daemon=True)
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def _beat(self) -> None:
        self.store.set(f"{_HB_PREFIX}{self.rank}", repr(time.time()))

    def _loop(self) -> None:
        while not self._stop.wait(self.interval_s):
            try:
                self._beat()
            except Exception:  # noqa: BLE001  (store gone: rank 0 died; nothing left to report to)
                return

    def alive(self, ranks: Sequence[int], stale_s: float) -> List[int]:
        now = time.time()
        out = []
        for r in ranks:
            k = f"{_HB_PREFIX}{r}"
            try:
                if self.store.check([k]) and now - float(self.store.get(k).decode()) < stale_s:
                    out.append(r)
            except Exception:  # noqa: BLE001
                pass
        return out


class ElasticState:
    """Per-process recovery state: the base store, the heartbeat, the original rank ids of the
    current members and the recovery epoch."""

    def __init__(self, world: World, store=None, interval_s: float = 0.5, segment_store: Optional[str] = None):
        self.segment_store = segment_store
        self.store = store if store is not None else dist.distributed_c10d._get_default_store()
        self.orig_rank = world.rank           # this process's rank in the ORIGINAL world
        self.members = list(range(world.size))  # original ranks of the current members, by new rank
        self.epoch = 0
        self.backend = world.backend
        self.local_rank = world.local_rank
        self.membership = Membership(self.store, world.rank, world.size, interval_s).start()

    def stop(self) -> None:
        self.membership.stop()


_STATE: Optional[ElasticState] = None


def enable(world: World, interval_s: float = 0.5, segment_store: Optional[str] = None) -> ElasticState:
    """Start heart-beating (call once after ``init_world`` on every rank); ``segment_store`` is
    where lost shards are re-loaded from (``DataSource.save`` layout)."""
    global _STATE
    if _STATE is None and world.distributed:
        _STATE = ElasticState(world, interval_s=interval_s, segment_store=segment_store)
    return _STATE


def state() -> Optional[ElasticState]:
    return _STATE


def agree_members(st: ElasticState, stale_s: float = 3.0, settle_s: float = 20.0) -> List[int]:
    """Original ranks of the survivors, identical on every survivor (see the module doc)."""
    st.epoch += 1
    base = f"sdo/recover{st.epoch}/"
    st.store.set(f"{base}arrived/{st.orig_rank}", "1")
    t0 = time.time()
    while True:
        arrived = [r for r in st.members if st.store.check([f"{base}arrived/{r}"])]
        alive = st.membership.alive(st.members, stale_s)
        if (set(alive) <= set(arrived) and time.time() - t0 > stale_s) or time.time() - t0 > settle_s:
            break
        time.sleep(0.1)
    if min(arrived) == st.orig_rank:
        st.store.set(f"{base}members", ",".join(str(r) for r in sorted(arrived)))
    st.store.wait([f"{base}members"], datetime.timedelta(seconds=settle_s + 30))
    members = [int(x) for x in st.store.get(f"{base}members").decode().split(",")]
    if st.orig_rank not in members:
        raise RuntimeError(f"rank {st.orig_rank} arrived too late for recovery epoch {st.epoch}")
    return members


def rebuild(st: ElasticState, members: List[int], timeout_s: Optional[float] = None) -> World:
    """Abort/destroy the current communicator and initialise a new default process group over
    ``members`` (original rank ids) on a fresh prefix of the base store."""
    if dist.is_initialized():
        try:
            if st.backend == "nccl":
                dist.distributed_c10d._abort_process_group()
            else:
                dist.destroy_process_group()
        except Exception as e:  # noqa: BLE001  (an already-broken communicator)
            log.warning("communicator teardown: %s", e)
    new_rank = members.index(st.orig_rank)
    n = len(members)
    st.members = list(members)
    timeout_s = float(timeout_s or os.environ.get("SDO_COLLECTIVE_TIMEOUT_S", 600))
    if n > 1:
        kw = {}
        if st.backend == "nccl":
            kw["device_id"] = torch.device("cuda", st.local_rank % torch.cuda.device_count())
        dist.init_process_group(backend=st.backend, store=dist.PrefixStore(f"sdo/pg{st.epoch}", st.store),
                                rank=new_rank, world_size=n, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    w = World(new_rank, n, st.local_rank, st.backend if n > 1 else "none", None)
    set_world(w)
    return w


def adopt_shards(session, segment_store: str, failed: Sequence[int], members: Sequence[int],
                 my_orig_rank: int) -> List[Tuple[str, int]]:
    """Load the failed ranks' shards assigned to this member from the segment store and merge them
    into the local shards (re-registered, so plan caches drop the old ones).  Returns the
    (datasource, original rank) pairs adopted here."""
    from ..segment.datasource import DataSource

    mine = [f for i, f in enumerate(sorted(failed)) if members[i % len(members)] == my_orig_rank]
    adopted = []
    cluster = session.catalog.cluster
    for name in list(cluster.datasources):
        ds = cluster.get(name)
        extra = []
        for f in mine:
            path = os.path.join(segment_store, name, f"rank{f}")
            if os.path.exists(os.path.join(path, "manifest.json")):
                extra.append(DataSource.load(path, ds.device))
                adopted.append((name, f))
        if extra:
            merged = DataSource.concat([ds] + extra)
            merged.global_num_rows = ds.global_num_rows
            # the cluster-wide interval is unchanged (registration must not issue a collective:
            # only the adopting members re-register)
            merged.global_interval_ms = getattr(ds, "global_interval_ms", None)
            # cluster-wide derived state (all-reduced FD tables, metric value ranges) is unchanged
            # too: carry it over so the adopting member issues no collective its peers skip
            for k in ("_fd_cache", "_lut_cache"):
                if k in ds.__dict__:
                    merged.__dict__[k] = ds.__dict__[k]
            for mname, m in ds.metrics.items():
                if hasattr(m, "_value_range"):
                    merged.metrics[mname]._value_range = m._value_range
            session.register_datasource(merged, name)
            for t in session.catalog.druid_tables():  # DDL-bound relations follow the new shard
                if t.info.datasource is ds:
                    t.info.datasource = merged
    return adopted


def recover(session, segment_store: Optional[str] = None, stale_s: float = 3.0, settle_s: float = 20.0) -> Dict:
    """Full recovery on this survivor: agree -> rebuild -> re-home.  Every survivor must call it."""
    st = _STATE
    if st is None:
        raise RuntimeError("elastic recovery is not enabled (parallel.recovery.enable)")
    segment_store = segment_store or st.segment_store
    before = list(st.members)
    members = agree_members(st, stale_s, settle_s)
    failed = [r for r in before if r not in members]
    w = rebuild(st, members)
    session.engine.world = w
    session.engine._coalescer = None
    adopted = adopt_shards(session, segment_store, failed, members, st.orig_rank) if segment_store and failed else []
    session._plan_cache.clear()
    log.warning("recovered: failed ranks %s, %d members, this rank %d -> %d, adopted %s", failed, len(members),
                st.orig_rank, w.rank, adopted)
    return {"failed": failed, "members": members, "rank": w.rank, "adopted": adopted, "epoch": st.epoch}


def run_with_recovery(session, fn: Callable[[], object], segment_store: Optional[str] = None, retries: int = 1):
    """Run ``fn`` (a query); if a collective fails because a rank is gone, recover and re-run."""
    for attempt in range(retries + 1):
        try:
            return fn()
        except Exception as e:  # noqa: BLE001
            if attempt == retries or _STATE is None or not _is_comm_failure(e):
                raise
            log.warning("query failed in a collective (%s): recovering", e)
            recover(session, segment_store)


def is_comm_failure(e: BaseException) -> bool:
    return _STATE is not None and _is_comm_failure(e)


def _is_comm_failure(e: BaseException) -> bool:
    from .fault import RankFailure

    if isinstance(e, RankFailure):
        return False  # a live rank failed its scan: the ranks already agreed, nothing to rebuild
    names = {type(x).__name__ for x in (e, e.__cause__, e.__context__) if x is not None}
    if names & {"DistBackendError", "DistNetworkError", "DistStoreError"}:
        return True
    msg = str(e)
    if not any(s in msg for s in ("Connection closed", "Connection reset", "Timed out", "timed out", "Broken pipe",
                                  "NCCL", "RCCL", "Socket", "peer")):
        return False
    # a transport-sounding message alone (e.g. a socket timeout inside one statement on one rank)
    # is not evidence of a dead peer: recovery starts only once some member's heartbeat went stale,
    # otherwise this rank would publish a membership of itself and its live peers would be stranded
    return _member_went_stale()


def _member_went_stale(stale_s: float = 3.0, wait_s: Optional[float] = None) -> bool:
    st = _STATE
    if st is None:
        return False
    deadline = time.time() + (stale_s + 1.5 if wait_s is None else wait_s)
    while True:
        others = [r for r in st.members if r != st.orig_rank]
        if len(st.membership.alive(others, stale_s)) < len(others):
            return True
        if time.time() >= deadline:
            return False
        time.sleep(0.1)
