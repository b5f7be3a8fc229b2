#!/usr/bin/env python3
"""Where a forced one-rank collective merge diverges from the local answer (tools/rccl_smoke.py
found TPC-H Q3 / Q18 rows whose values belong to the next key at SF1): wraps
parallel/merge.py merge_partials and checks, per call, that the merged groups (key -> slot values)
equal the input's -- with one rank every merge is an identity -- and reports the plan taken.

  spawn_ranks(1, [python, tools/merge_probe.py, --out, F, --sf, 1])   (tools/gpu/merge_probe.sh)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _mapping(p):
    sp = p.compact()
    k = sp.keys.to("cpu").tolist()
    a = sp.acc.to("cpu").tolist()
    return dict(zip(k, map(tuple, a)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--query", default="TPCH Q3")
    a = ap.parse_args()
    os.environ["SDO_FORCE_COLLECTIVES"] = "1"
    import torch

    from spark_druid_olap_amd.engine.executor import Engine, results_on_root
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.parallel import merge as M
    from spark_druid_olap_amd.parallel import p2p
    from spark_druid_olap_amd.parallel.world import init_world, shutdown
    from spark_druid_olap_amd.session import Session

    w = init_world(backend=os.environ.get("PROBE_BACKEND", "nccl"))
    p2p.ENABLED = False
    dev = w.device()
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(engine=Engine(w))
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    calls = []
    orig = M.merge_partials

    def wrapped(world, prog, part, *args, **kw):
        rec = {"kind": part.kind, "rows": part.rows, "plan": M.merge_plan_for(world, part, kw.get("disjoint_keys",
                                                                                                 bool(args and args[0]))).kind,
               "args": [str(x) for x in args], "kw": {k: str(v) for k, v in kw.items()}}
        before = _mapping(part)
        out = orig(world, prog, part, *args, **kw)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        after = _mapping(out) if out.rows else {}
        rec["groups_in"], rec["groups_out"] = len(before), len(after)
        bad = [k for k in before if after.get(k) != before[k]][:5]
        rec["mismatched_keys"] = len([k for k in before if after.get(k) != before[k]])
        rec["examples"] = [(k, before[k], after.get(k)) for k in bad[:3]]
        calls.append(rec)
        return out

    M.merge_partials = wrapped
    orig_g = M.gather_groups

    def wrapped_g(world, sp, *args, **kw):
        before = _mapping(sp)
        out = orig_g(world, sp, *args, **kw)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        after = _mapping(out) if out.rows else {}
        bad = [k for k in before if after.get(k) != before[k]]
        calls.append({"gather_groups": True, "rows_in": sp.rows, "rows_out": out.rows,
                      "keys_contiguous_out": bool(out.keys.is_contiguous()),
                      "acc_contiguous_out": bool(out.acc.is_contiguous()),
                      "mismatched_keys": len(bad), "examples": [(k, before[k], after.get(k)) for k in bad[:3]]})
        return out

    M.gather_groups = wrapped_g
    import spark_druid_olap_amd.engine.executor as EX

    if getattr(EX, "merge_partials", None) is orig:
        EX.merge_partials = wrapped
    q = dict(tpch.BENCH_QUERIES)[a.query]
    with results_on_root(True):
        s.sql(q).run()
    res = {"calls": calls}
    with open(a.out, "w") as f:
        json.dump(res, f, default=str)
    print(json.dumps(res, default=str)[:3000], flush=True)
    shutdown()


if __name__ == "__main__":
    main()
