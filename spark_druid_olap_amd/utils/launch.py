"""One process per GPU on one node, without torchrun (the deployment piece the reference's EMR
spin-up tool covers for its cluster, ``tools/spinup-tool/spinup.sh``).

``spawn_ranks(n, cmd)`` starts ``n`` copies of ``cmd`` with the torchrun environment (RANK,
LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and waits for them; a rank that dies
takes the others down (they would block in their next collective).  The parent imports nothing
GPU-related -- it must never initialise the GPU, since it only starts the ranks that do.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, n: int, port: str, base: Optional[dict] = None) -> dict:
    env = dict(base if base is not None else os.environ)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def spawn_ranks(n: int, cmd: Sequence[str], quiet_peers: bool = True, env: Optional[dict] = None) -> int:
    """Run ``cmd`` as ``n`` ranks; returns the first non-zero exit code (0 if all succeeded).
    Rank 0 inherits stdout; the other ranks' stdout is discarded when ``quiet_peers``."""
    port = (env or os.environ).get("MASTER_PORT") or str(free_port())
    procs: List[subprocess.Popen] = []
    for r in range(n):
        procs.append(subprocess.Popen(list(cmd), env=rank_env(r, n, port, env),
                                      stdout=None if (r == 0 or not quiet_peers) else subprocess.DEVNULL))

    def _forward(sig, _frame):
        # rank 0 shuts down cleanly and tells its peers (server/spmd.py); a second signal hits all
        if procs[0].poll() is None and not getattr(_forward, "sent", False):
            _forward.sent = True
            procs[0].send_signal(sig)
            return
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
    old = {s: signal.signal(s, _forward) for s in (signal.SIGINT, signal.SIGTERM)}
    rc = 0
    live = list(procs)
    try:
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in live:
                        q.terminate()
            time.sleep(0.1)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc


def main(argv=None) -> None:
    """``python -m spark_druid_olap_amd.utils.launch --nproc 8 -- python -m <module> [args]``"""
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing command")
    sys.exit(spawn_ranks(a.nproc, cmd))


if __name__ == "__main__":
    main()
