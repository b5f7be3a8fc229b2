#!/usr/bin/env python3
"""Multi-rank rehearsal on one GPU: the 8 headline queries on 2 ranks sharing the card (gloo
between them, P2P merge on and off) and on 1 rank at the same per-rank scale factor, each with the
per-phase split (scan / merge / finalize / post) of ``PreparedQuery.run`` -- what the second rank
costs, phase by phase.  Writes ``<out>_2rank.json`` and ``<out>_1rank.json``.

  python tools/rehearsal.py --sf 10 --out gpurun_out/rehearsal
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10.0, help="scale factor per rank")
    ap.add_argument("--out", default="gpurun_out/rehearsal")
    a = ap.parse_args()
    from spark_druid_olap_amd.utils.launch import spawn_ranks

    env = dict(os.environ, SDO_GLOO_GPU="1", MASTER_ADDR="127.0.0.1")
    rc = 0
    for n in (2, 1):
        path = f"{a.out}_{n}rank.json"
        rc = spawn_ranks(n, [sys.executable, os.path.join(ROOT, "tools", "p2p_check.py"), "--out", path,
                             "--sf", str(a.sf)], env=env)
        if rc:
            print(f"[rehearsal] {n} rank(s) failed: exit {rc}", flush=True)
            return rc
        r = json.load(open(path))
        print(f"== {n} rank(s), SF{a.sf:g} per rank", flush=True)
        for q, modes in r.get("phases", {}).items():
            print(f"  {q[:45]:45s} " + "  ".join(
                f"{m}: {v['ms']:.3f} ms (" + " ".join(f"{k[:-3]}={x:.3f}" for k, x in v.items() if k != "ms") + ")"
                for m, v in modes.items()), flush=True)
        for m, v in (r.get("auto_pipeline") or {}).items():
            print(f"  auto-pipelined day x shipmode ({m}): " + " ".join(
                f"{k}={x:.3f}" if isinstance(x, float) else f"{k}={x}" for k, x in v.items()), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
