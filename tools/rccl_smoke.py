#!/usr/bin/env python3
"""One-rank RCCL smoke: every distributed code path through a REAL ``nccl`` (RCCL) process group.

A one-GPU box cannot hold two RCCL ranks (RCCL refuses two ranks on one device), and the
multi-rank rehearsals on one card run over gloo (``SDO_GLOO_GPU=1``) -- so without this, no RCCL
collective of the engine would ever execute before an 8-GPU node does.  Here a process group of
ONE rank is created with the ``nccl`` backend and the world is told to run its collectives anyway
(``SDO_FORCE_COLLECTIVES=1``, ``parallel/world.py``): every merge, shuffle, gather and agreement
takes the multi-rank path and RCCL executes it (a one-rank all-gather / all-to-all / all-reduce is
still a real RCCL kernel on the group's stream).

Checks (rank 0 writes a JSON report to ``--out``):

1. primitives: ``all_gather_into_tensor``, ``all_to_all_single`` with split sizes (the varlen
   exchange), ``all_reduce`` sum / max / min, ``barrier(device_ids=...)``, object broadcast /
   all-gather, the root-only varlen gather -- each against its known one-rank answer;
2. the 8 headline SQL queries (TPC-H Q3 among them, its sparse groups through the all-to-all
   shuffle) and a few TPC-H 22 queries (partitioned / hashed / HAVING paths), each with the results
   gathered to the root and to every rank, equal to the same session without a process group.

Launch: ``python -c "from spark_druid_olap_amd.utils.launch import spawn_ranks; ..."`` with one rank
(tests/test_gpu_rccl.py), which sets MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def primitives(w, dev):
    import torch

    out = {}
    t = torch.arange(10, dtype=torch.int64, device=dev)
    g = w.all_gather_tensor(t)
    out["all_gather"] = tuple(g.shape) == (1, 10) and bool(torch.equal(g[0], t))
    f = torch.rand(33, dtype=torch.float64, device=dev)
    out["all_reduce_sum"] = bool(torch.equal(w.all_reduce(f.clone(), "sum"), f))
    out["all_reduce_max"] = bool(torch.equal(w.all_reduce(t.clone(), "max"), t))
    out["all_reduce_min"] = bool(torch.equal(w.all_reduce(t.clone(), "min"), t))
    rows = torch.randint(0, 1 << 40, (37, 3), dtype=torch.int64, device=dev)
    recv, rc, sts = w.all_to_all_varlen(rows, torch.tensor([37], dtype=torch.int64, device=dev), status=0)
    out["all_to_all_varlen"] = bool(torch.equal(recv, rows)) and rc.tolist() == [37] and sts == [0]
    got, sts = w.gather_varlen(rows, root=0, status=0)
    out["gather_varlen"] = len(got) == 1 and bool(torch.equal(got[0], rows)) and sts == [0]
    ag, sts = w.all_gather_varlen(rows[:5], status=0)
    out["all_gather_varlen"] = len(ag) == 1 and bool(torch.equal(ag[0], rows[:5])) and sts == [0]
    # a failed status word travels with the count exchange and skips the payload
    _, _, sts = w.all_to_all_varlen(rows, torch.tensor([37], dtype=torch.int64, device=dev), status=1)
    out["status_word"] = sts == [1]
    w.barrier()
    out["barrier"] = True
    out["broadcast_object"] = w.broadcast_object({"k": 7}) == {"k": 7}
    out["all_gather_object"] = w.all_gather_object(("r", 0)) == [("r", 0)]
    out["max_float"] = w.max_float(2.5) == 2.5
    torch.cuda.synchronize()
    return out


def _rows(b):
    return sorted(tuple(round(x, 6) if isinstance(x, float) else x for x in r)
                  for r in b.to_pandas().itertuples(index=False, name=None))


def engine(w, dev, sf, out):
    import torch

    from spark_druid_olap_amd.engine.executor import Engine, results_on_root
    from spark_druid_olap_amd.models import tpch, tpch22
    from spark_druid_olap_amd.parallel import p2p
    from spark_druid_olap_amd.parallel.world import World
    from spark_druid_olap_amd.session import Session

    p2p.ENABLED = False  # (the RCCL path: the P2P mailboxes have their own tests)
    ds = tpch.to_datasource(tpch.generate_flat(sf, dev), profile="bench")
    sessions = {}
    for name, world in (("rccl", w), ("local", World())):
        s = Session(engine=Engine(world))
        s.register_datasource(ds)
        s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
        s.sql(tpch.druid_ddl(with_column_mapping=False))
        sessions[name] = s
    qs = list(tpch.BENCH_QUERIES) + [(n, q) for n, q in tpch22.QUERIES if n in ("Q1", "Q3", "Q10", "Q13", "Q16", "Q18")]
    eq, ms, ran = {}, {}, {}
    for name, q in qs:
        want = _rows(sessions["local"].sql(q))
        res = {}
        for root in (True, False):
            with results_on_root(root):
                d = sessions["rccl"].sql(q)
                b = d.run()
                torch.cuda.synchronize()
                t = time.perf_counter()
                b = d.run()
                torch.cuda.synchronize()
                ms[f"{name}{' (root)' if root else ''}"] = round((time.perf_counter() - t) * 1e3, 3)
                res[root] = _rows(b)
        eq[name] = res[True] == want and res[False] == want
        if not eq[name]:  # what differs: row counts and a few rows only one side has
            diag = out.setdefault("mismatch", {})
            for root in (True, False):
                a, b_ = set(res[root]), set(want)
                diag[f"{name}{' (root)' if root else ''}"] = {
                    "rows": len(res[root]), "want_rows": len(want),
                    "only_rccl": [list(map(str, r)) for r in sorted(a - b_)[:3]],
                    "only_local": [list(map(str, r)) for r in sorted(b_ - a)[:3]]}
        ran[name] = len(want)
    out["engine_equal"] = eq
    out["engine_rows"] = ran
    out["engine_ms"] = ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--sf", type=float, default=0.2)
    a = ap.parse_args()
    os.environ["SDO_FORCE_COLLECTIVES"] = "1"
    import torch
    import torch.distributed as dist

    from spark_druid_olap_amd.parallel.world import init_world, shutdown

    w = init_world(backend="nccl")
    assert w.distributed and w.backend == "nccl" and w.size == 1, w
    dev = w.device()
    out = {"backend": dist.get_backend(), "world": w.size, "forced": w.force_collectives,
           "rccl_version": str(getattr(torch.cuda, "nccl", None) and torch.cuda.nccl.version())}
    out["primitives"] = primitives(w, dev)
    engine(w, dev, a.sf, out)
    with open(a.out, "w") as f:
        json.dump(out, f)
    print(json.dumps(out)[:4000], flush=True)
    shutdown()


if __name__ == "__main__":
    main()
