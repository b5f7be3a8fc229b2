"""Service discovery + membership watching: the ZooKeeper/Curator layer of the reference.

The reference finds the Druid broker and coordinator through Curator service discovery under
``<zkDruidPath>/discovery`` and watches ``<zkDruidPath>/announcements`` (servers) and
``<zkDruidPath>/segments`` (per-server segment inventory); any child added or removed clears the
metadata cache (``sd/client/CuratorConnection.scala:41-235``: listener -> ``cache.clearCache``
77-88, per-server segment caches 90-133, ``getService`` 181-201, ``getBroker/getCoordinator``
203-209).

There is no ZooKeeper here and no external cluster: the "servers" are the GPUs of the process
group and the services are this framework's own endpoints (Druid HTTP API, Thrift server).  The
registry keeps the same znode *layout* and the same watch semantics with two backends:

* ``memory``: in-process (one controller per node; the default for ``druidHost 'localhost'``);
* ``file``: a directory tree (``druidHost 'file:///dev/shm/sdo-zk'``), one file per ephemeral
  node, so separate processes on a host (torchrun ranks, a Thrift server and its clients) see each
  other.  Ephemeral nodes carry the owner pid and vanish when it exits (session expiry).

Watchers are polled by one daemon thread per registry (Curator's PathChildrenCache does the same
with ZK watches); callbacks get ``(event, path)`` with event ``CHILD_ADDED`` / ``CHILD_REMOVED`` /
``CHILD_UPDATED``.
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

CHILD_ADDED, CHILD_REMOVED, CHILD_UPDATED = "CHILD_ADDED", "CHILD_REMOVED", "CHILD_UPDATED"

Listener = Callable[[str, str], None]


def _norm(path: str) -> str:
    p = "/" + "/".join(x for x in path.split("/") if x)
    return p


class Registry:
    """Hierarchical node store with child watches (ZooKeeper subset)."""

    poll_s = 0.05

    def __init__(self):
        self._watches: List[Tuple[str, Listener]] = []
        self._snap: Dict[str, Dict[str, bytes]] = {}
        self._lock = threading.RLock()
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()

    # -- backend primitives ------------------------------------------------------------------
    def create(self, path: str, data: bytes = b"", ephemeral: bool = True) -> None:
        raise NotImplementedError

    def delete(self, path: str) -> None:
        raise NotImplementedError

    def get(self, path: str) -> Optional[bytes]:
        raise NotImplementedError

    def children(self, path: str) -> Dict[str, bytes]:
        raise NotImplementedError

    # -- watches -------------------------------------------------------------------------------
    def watch_children(self, path: str, fn: Listener) -> None:
        path = _norm(path)
        with self._lock:
            self._watches.append((path, fn))
            self._snap.setdefault(path, dict(self.children(path)))
        self._ensure_thread()

    def _ensure_thread(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, daemon=True, name="sdo-discovery")
            self._thread.start()

    def poll(self) -> int:
        """Diff every watched path against its last snapshot and fire listeners; returns #events."""
        n = 0
        with self._lock:
            paths = {p for p, _ in self._watches}
            for p in paths:
                cur = dict(self.children(p))
                old = self._snap.get(p, {})
                events = [(CHILD_ADDED, k) for k in cur if k not in old]
                events += [(CHILD_REMOVED, k) for k in old if k not in cur]
                events += [(CHILD_UPDATED, k) for k in cur if k in old and cur[k] != old[k]]
                self._snap[p] = cur
                for ev, k in events:
                    for wp, fn in self._watches:
                        if wp == p:
                            try:
                                fn(ev, f"{p}/{k}")
                            except Exception:  # noqa: BLE001  (a listener must not kill the watcher)
                                pass
                    n += 1
        return n

    def _loop(self):
        while not self._stop.wait(self.poll_s):
            self.poll()

    def close(self):
        self._stop.set()


class MemoryRegistry(Registry):
    def __init__(self):
        super().__init__()
        self._nodes: Dict[str, bytes] = {}

    def create(self, path, data=b"", ephemeral=True):
        with self._lock:
            self._nodes[_norm(path)] = bytes(data)

    def delete(self, path):
        with self._lock:
            self._nodes.pop(_norm(path), None)

    def get(self, path):
        return self._nodes.get(_norm(path))

    def children(self, path):
        p = _norm(path) + "/"
        out = {}
        with self._lock:
            for k, v in self._nodes.items():
                if k.startswith(p):
                    rest = k[len(p):]
                    if "/" not in rest:
                        out[rest] = v
        return out


class FileRegistry(Registry):
    """Nodes are files under ``root``; ephemeral nodes record their owner pid."""

    def __init__(self, root: str):
        super().__init__()
        self.root = root
        os.makedirs(root, exist_ok=True)

    def _fs(self, path: str) -> str:
        return os.path.join(self.root, _norm(path).lstrip("/"))

    def create(self, path, data=b"", ephemeral=True):
        f = self._fs(path)
        os.makedirs(os.path.dirname(f), exist_ok=True)
        tmp = f"{f}.tmp{os.getpid()}"
        with open(tmp, "wb") as fh:
            fh.write(json.dumps({"owner": os.getpid() if ephemeral else None}).encode() + b"\n" + bytes(data))
        os.replace(tmp, f)

    def delete(self, path):
        try:
            os.remove(self._fs(path))
        except FileNotFoundError:
            pass

    @staticmethod
    def _alive(pid: Optional[int]) -> bool:
        if pid is None:
            return True
        try:
            os.kill(pid, 0)
            return True
        except ProcessLookupError:
            return False
        except PermissionError:
            return True

    def _read(self, f: str) -> Optional[bytes]:
        try:
            with open(f, "rb") as fh:
                raw = fh.read()
        except (FileNotFoundError, IsADirectoryError):
            return None
        head, _, data = raw.partition(b"\n")
        try:
            owner = json.loads(head).get("owner")
        except ValueError:
            return None
        if not self._alive(owner):
            try:  # expired session: the ephemeral node goes away
                os.remove(f)
            except OSError:
                pass
            return None
        return data

    def get(self, path):
        return self._read(self._fs(path))

    def children(self, path):
        d = self._fs(path)
        out = {}
        try:
            names = os.listdir(d)
        except (FileNotFoundError, NotADirectoryError):
            return out
        for n in names:
            if ".tmp" in n:
                continue
            f = os.path.join(d, n)
            if os.path.isfile(f):
                v = self._read(f)
                if v is not None:
                    out[n] = v
        return out


_REGISTRIES: Dict[str, Registry] = {}
_RLOCK = threading.Lock()


def registry_for(druid_host: str) -> Registry:
    """``druidHost`` option (the ZK connect string) -> registry (shared per connect string)."""
    key = druid_host or "localhost"
    with _RLOCK:
        r = _REGISTRIES.get(key)
        if r is None:
            if key.startswith("file://"):
                r = FileRegistry(key[len("file://"):])
            else:
                r = MemoryRegistry()
            _REGISTRIES[key] = r
        return r


class Discovery:
    """Curator-style service discovery + server/segment announcements for one ``zkDruidPath``."""

    def __init__(self, registry: Registry, druid_path: str = "/druid", qualify_names: bool = False):
        self.reg = registry
        self.base = _norm(druid_path)
        self.qualify = qualify_names

    def _svc(self, name: str) -> str:
        # zkQualifyDiscoveryNames: services are registered as "druid:broker" (DefaultSource.scala:286-287)
        return f"druid:{name}" if self.qualify and not name.startswith("druid:") else name

    # -- services --------------------------------------------------------------------------------
    def announce_service(self, name: str, host: str, port: int, instance: Optional[str] = None) -> str:
        inst = instance or f"{host}:{port}"
        payload = {"name": self._svc(name), "id": inst, "address": host, "port": int(port),
                   "registrationTimeUTC": int(time.time() * 1000), "serviceType": "DYNAMIC"}
        path = f"{self.base}/discovery/{self._svc(name)}/{inst}"
        self.reg.create(path, json.dumps(payload).encode())
        return path

    def get_service(self, name: str) -> Optional[Tuple[str, int]]:
        """First live instance of a service (CuratorConnection.getService, 181-201)."""
        kids = self.reg.children(f"{self.base}/discovery/{self._svc(name)}")
        for _, v in sorted(kids.items()):
            d = json.loads(v)
            return d["address"], int(d["port"])
        return None

    def get_broker(self) -> Optional[Tuple[str, int]]:
        return self.get_service("broker")

    def get_coordinator(self) -> Optional[Tuple[str, int]]:
        return self.get_service("coordinator")

    def get_overlord(self) -> Optional[Tuple[str, int]]:
        return self.get_service("overlord")

    # -- servers and segments ---------------------------------------------------------------------
    def announce_server(self, host: str, info: dict) -> None:
        self.reg.create(f"{self.base}/announcements/{host}", json.dumps(info).encode())

    def announce_segment(self, host: str, segment_id: str, info: Optional[dict] = None) -> None:
        node = segment_id.replace("/", "_")  # znode names cannot nest (interval "a/b" in ids)
        self.reg.create(f"{self.base}/segments/{host}/{node}", json.dumps(info or {}).encode())

    def unannounce(self, path: str) -> None:
        self.reg.delete(path)

    def servers(self) -> Dict[str, dict]:
        return {k: json.loads(v) for k, v in self.reg.children(f"{self.base}/announcements").items()}

    def segments(self, host: str) -> List[str]:
        return sorted(self.reg.children(f"{self.base}/segments/{host}"))

    def watch_membership(self, on_change: Callable[[str, str], None]) -> None:
        """Any server or segment added/removed -> on_change (the reference clears its metadata
        cache, CuratorConnection.scala:77-88).  Segment watches are installed per announced
        server as servers appear."""
        watched = set()

        def on_server(ev, path):
            host = path.rsplit("/", 1)[-1]
            if ev == CHILD_ADDED and host not in watched:
                watched.add(host)
                self.reg.watch_children(f"{self.base}/segments/{host}", on_change)
            on_change(ev, path)

        self.reg.watch_children(f"{self.base}/announcements", on_server)
        for host in self.servers():
            if host not in watched:
                watched.add(host)
                self.reg.watch_children(f"{self.base}/segments/{host}", on_change)
