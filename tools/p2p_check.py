#!/usr/bin/env python3
"""One rank of the peer-to-peer merge check (parallel/p2p.py), run as N processes on the GPU(s):

  python -c "from spark_druid_olap_amd.utils.launch import spawn_ranks; ..."   (tests/test_gpu_p2p.py)

Ranks talk over gloo with their shards on the GPU (``SDO_GLOO_GPU=1``: several ranks may share one
card -- IPC mappings work within a device as across xGMI).  Checks, on every rank:

1. synthetic dense partials (int sum / f64 sum / min / max slots, HLL register bytes) merged by the
   P2P kernel equal the RCCL/gloo one-shot all-gather merge, over several epochs (both mailbox
   slots), and a failed rank's status word reaches every peer;
2. the 8 headline SQL queries (Q1 / Q5 / Q7 among them) with the P2P merge on and off give the same
   answers, with the per-phase times (scan / merge / finalize / post, ``PreparedQuery.run`` stats)
   of both for the rehearsal breakdown.

Run as ONE process it times the same queries on one rank at the same per-rank scale factor (the
baseline the 2-rank phases compare against; tools/rehearsal.py runs both).

Per-phase times are GPU-event times (``SDO_PHASE_EVENTS``: HIP events recorded on the compute
stream at the scan / merge / gather / finalize boundaries, ``gpu_*_ms``) next to the host stamps
(``*_ms``).  The non-P2P mode is labelled with the process group's backend (``gloo`` in the
one-card rehearsal, ``nccl`` = RCCL across GPUs).

Fail-safe scenarios (``--scenario``, tests/test_gpu_p2p.py):

* ``selftest_fail`` (with ``SDO_P2P_SELFTEST_FAIL=<rank>``): the exchange's known-value self-test
  fails on one rank, so no rank uses P2P and every statement completes over the collective path;
* ``delay`` (with ``SDO_P2P_DELAY=rank=1,s=1.5,times=1``): one rank launches a merge after the
  peers' soft wait expired; every rank abandons that epoch together and the statement re-runs over
  the collective path with the same answer;
* ``late`` (with ``SDO_P2P_DELAY=rank=1,s=3,times=1`` and ``SDO_P2P_HARD_TIMEOUT_S=1``): one rank,
  alive, arrives after the peers' HARD deadline.  The early rank aborts the epoch (its final word),
  so EVERY rank -- the late one too -- reports the timeout, fails that statement and disables its
  exchange; the next statements run over the collective path with the unchanged answers.

Rank 0 writes a JSON report to ``--out``."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Prog:
    def __init__(self, slots):
        self.slots = slots
        self.nslots = len(slots)


def synthetic(world, dev, out):
    import torch

    from spark_druid_olap_amd.engine.partials import Partials
    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.parallel import p2p
    from spark_druid_olap_amd.parallel.merge import start_dense_merge

    slots = [(D.S_SUM_I, 0), (D.S_SUM_F, 0), (D.S_MIN_I, 1 << 62), (D.S_MAX_I, -(1 << 62))]
    prog = _Prog(slots)
    ex = p2p.exchange_for(world)
    out["exchange"] = ex is not None
    if ex is None:
        return
    ok = True
    for epoch in range(5):
        g = torch.Generator().manual_seed(1000 * epoch + world.rank)
        R = 37 + epoch
        acc = torch.randint(-10 ** 6, 10 ** 6, (R, 4), generator=g, dtype=torch.int64)
        acc[:, 1] = torch.rand(R, generator=g, dtype=torch.float64).view(torch.int64)
        hll = [torch.randint(0, 40, (R, 128), generator=g, dtype=torch.int64).to(torch.uint8)]
        part = Partials("dense", acc.to(dev), None, [h.to(dev) for h in hll])
        status = 1 if (epoch == 3 and world.rank == world.size - 1) else 0
        m = ex.merge(prog, part, status)
        ref, sts_ref = start_dense_merge(world, prog, part, status, "oneshot-allgather").wait()
        sts = m.status_dev.tolist()
        if epoch == 3:
            out["failed_status_seen"] = sts == [0] * (world.size - 1) + [1]
        same = torch.equal(m.acc[:, [0, 2, 3]].cpu(), ref.acc[:, [0, 2, 3]].cpu()) and \
            torch.allclose(m.acc[:, 1].cpu().view(torch.float64), ref.acc[:, 1].cpu().view(torch.float64),
                           rtol=1e-12, atol=1e-12) and \
            all(torch.equal(a.cpu(), b.cpu()) for a, b in zip(m.hll, ref.hll)) and sts == list(sts_ref)
        ok = ok and same
    out["synthetic_equal"] = ok
    # timing: P2P vs all-gather merge of a Q1-sized state (6 groups, 8 slots, one HLL block)
    acc = torch.zeros((6, 4), dtype=torch.int64, device=dev)
    part = Partials("dense", acc, None, [torch.zeros((6, 2048), dtype=torch.uint8, device=dev)])
    for name, fn in (("p2p", lambda: ex.merge(prog, part, 0).status_dev.tolist()),
                     ("allgather", lambda: start_dense_merge(world, prog, part, 0, "oneshot-allgather").wait())):
        ts = []
        for i in range(30):
            world.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e6)
        out[f"merge_us_{name}"] = statistics.median(ts[5:])


def engine(world, dev, sf, out):
    import torch

    from spark_druid_olap_amd.engine.executor import Engine, results_on_root
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.parallel import p2p
    from spark_druid_olap_amd.session import Session

    ds = tpch.to_datasource(tpch.generate_flat(sf, dev, rank=world.rank, world=world.size), profile="bench")
    sess = Session(engine=Engine(world), conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    sess.register_datasource(ds)
    sess.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    sess.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    res, phases = {}, {}
    other = "gloo" if world.backend == "gloo" else "rccl"
    modes = ("p2p", other) if world.size > 1 else ("local",)
    retries = {}
    for mode in modes:
        p2p.ENABLED = mode == "p2p"
        sess._plan_cache.clear()
        with results_on_root():
            for name, q in tpch.BENCH_QUERIES:
                df = sess.sql(q)
                for _ in range(2):
                    df.run()
                    for st in df.last_stats.get("druid", []):
                        if (st.get("stats") or {}).get("p2p_retry"):
                            retries[name] = retries.get(name, 0) + 1
                ts, ph = [], {}
                for _ in range(10):
                    world.barrier()
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    b = df.run()
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t) * 1e3)
                    for st in df.last_stats.get("druid", []):
                        for k, v in (st.get("stats") or {}).items():
                            if k.endswith("_ms"):
                                ph.setdefault(k, []).append(v)
                            if k == "p2p_retry":
                                retries[name] = retries.get(name, 0) + 1
                rows = sorted(tuple(round(x, 6) if isinstance(x, float) else x for x in r)
                              for r in b.to_pandas().itertuples(index=False, name=None))
                res.setdefault(name, {})[mode] = rows
                phases.setdefault(name, {})[mode] = {"ms": statistics.median(ts),
                                                    **{k: round(statistics.median(v), 4) for k, v in ph.items()}}
    p2p.ENABLED = True
    # the default path's automatic pipelining (engine/executor.py AUTO_PIPELINE): a groupBy keyed
    # by day x ship mode holds a 280 KB dense state, so every rank splits its scan into batches and
    # merges each batch's day slice while the next batch scans; timed against the same query with
    # the pipelining off (one scan, then one merge of the whole table)
    if world.size > 1:
        from spark_druid_olap_amd.engine import executor as X
        from spark_druid_olap_amd.query import spec as S

        spec = S.GroupByQuerySpec("tpch", [S.DefaultDimensionSpec("l_shipmode")], granularity=S.Granularity.parse("day"),
                                  intervals=["1992-01-01/1999-01-01"],
                                  aggregations=[S.FunctionAggregationSpec("doubleSum", "s", "l_extendedprice"),
                                                S.FunctionAggregationSpec("count", "n")])
        pipe = {}
        for auto in (True, False):
            X.AUTO_PIPELINE = auto
            pq = sess.engine.prepare(spec.copy(), ds)
            with results_on_root():
                for _ in range(2):
                    pq.run()
                ts, ph = [], {}
                for _ in range(10):
                    world.barrier()
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    r = pq.run()
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t) * 1e3)
                    for k, v in (r.stats or {}).items():
                        if k.endswith("_ms"):
                            ph.setdefault(k, []).append(v)
            pipe["auto" if auto else "one_merge"] = {
                "ms": statistics.median(ts), "batches": pq._nbatches, "pipelined": bool(pq._pipeline_ok),
                "rows": r.num_rows, **{k: round(statistics.median(v), 4) for k, v in ph.items()}}
        X.AUTO_PIPELINE = True
        out["auto_pipeline"] = pipe
    out["p2p_stats"] = p2p.stats(world)
    out["retried_statements"] = retries
    if world.rank == 0:
        if world.size > 1:
            out["engine_equal"] = {n: r["p2p"] == r[other] for n, r in res.items()}
        out["engine_rows"] = {n: len(next(iter(r.values()))) for n, r in res.items()}
        out["phases"] = phases


def late(world, dev, sf, out):
    """A live peer later than the hard deadline: every rank must see the same outcome."""
    from spark_druid_olap_amd.engine.executor import Engine, results_on_root
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.parallel import p2p
    from spark_druid_olap_amd.session import Session

    ds = tpch.to_datasource(tpch.generate_flat(sf, dev, rank=world.rank, world=world.size), profile="bench")
    sess = Session(engine=Engine(world))
    sess.register_datasource(ds)
    sess.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    sess.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    q = dict(tpch.BENCH_QUERIES)["TPCH Q1"]
    rows = lambda b: sorted(tuple(round(x, 6) if isinstance(x, float) else x for x in r)  # noqa: E731
                            for r in b.to_pandas().itertuples(index=False, name=None))
    with results_on_root():
        p2p.ENABLED = False
        sess._plan_cache.clear()
        want = rows(sess.sql(q).run())
        p2p.ENABLED = True
        sess._plan_cache.clear()
        df = sess.sql(q)
        try:
            df.run()
            outcome = "ok"
        except Exception as e:  # noqa: BLE001
            outcome = type(e).__name__
        outcomes = world.all_gather_object(outcome)
        enabled = world.all_gather_object(bool(p2p.stats(world).get("enabled")))
        after = rows(df.run())
    out["late_outcomes"] = outcomes
    out["late_enabled_after"] = enabled
    same = world.all_gather_object(after == want if world.rank == 0 else True)
    out["late_answer_equal"] = all(same)
    out["p2p_stats"] = p2p.stats(world)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--sf", type=float, default=1.0, help="scale factor per rank")
    ap.add_argument("--skip-engine", action="store_true")
    ap.add_argument("--scenario", default="normal", choices=["normal", "selftest_fail", "delay", "late"])
    a = ap.parse_args()
    os.environ.setdefault("SDO_PHASE_EVENTS", "1")
    import torch

    from spark_druid_olap_amd.parallel.world import init_world, shutdown

    world = init_world(backend="gloo")
    dev = world.device() if world.size > 1 else torch.device("cuda", 0)
    assert dev.type == "cuda", "run with SDO_GLOO_GPU=1 on a GPU box"
    torch.cuda.set_device(dev)
    out = {"world": world.size, "rank": world.rank, "sf_per_rank": a.sf}
    out["scenario"] = a.scenario
    if world.size > 1 and a.scenario == "normal":
        synthetic(world, dev, out)
    if a.scenario == "late":
        late(world, dev, a.sf, out)
    elif not a.skip_engine and (out.get("exchange") or world.size == 1 or a.scenario != "normal"):
        engine(world, dev, a.sf, out)  # (one rank: the same-SF baseline of the per-phase split)
    world.barrier()
    if world.rank == 0:
        with open(a.out, "w") as f:
            json.dump(out, f)
    shutdown()


if __name__ == "__main__":
    main()
