#!/usr/bin/env python3
"""Which Python line launches each torch op of a BI template's repeat run: torch.profiler (CPU
activity, with stacks) around the third run of one binding; prints the ops by total CPU time with
their innermost repo frame.

  python tools/op_trace.py --sf 100 --template TopVolume [--binding 0] [--top 25]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--template", default="TopVolume")
    ap.add_argument("--binding", type=int, default=0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import bi, tpch
    from spark_druid_olap_amd.session import Session

    dev = torch.device("cuda", 0)
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(engine=Engine(use_native=True))
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    bi.register(s)
    t = [t for t in bi.templates() if t["name"].startswith(a.template)][0]
    q = bi.render(t["sql"], bi.binding(a.binding, "years"))
    for _ in range(2):
        s.sql(q).to_pandas()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        s.sql(q).to_pandas()
        torch.cuda.synchronize()
    rows = []
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            continue
        frame = next((f for f in (ev.stack or []) if "spark_druid_olap_amd" in f), "?")
        rows.append((ev.name, frame.split("spark_druid_olap_amd/")[-1], ev.cpu_time_total))
    agg = {}
    for n, f, us in rows:
        k = (n, f)
        c, tot = agg.get(k, (0, 0.0))
        agg[k] = (c + 1, tot + us)
    for (n, f), (c, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{tot / 1e3:8.3f} ms  x{c:<4d} {n:36s} {f}")
    print("scatter/gather ops:")
    for (n, f), (c, tot) in agg.items():
        if "scatter" in n or "gather" in n:
            print(f"   {n} x{c} at {f}")


if __name__ == "__main__":
    main()
