#!/usr/bin/env python3
"""BASELINE config 5: the HiveServer2 Thrift endpoint under many concurrent JDBC-style clients.

The reference's BI benchmark drives its Thrift server with JMeter threads over JDBC
(``docs/bi-benchmark/snap-sales-demo.jmx:87-101``: 5 threads x 5 loops, fair scheduler pool); it
publishes no results.  Here:

* the server (``server/hive_server.py``) runs in this process with a synthetic TPC-H datasource
  resident on the GPU (``--sf``) and the reference's DDL;
* ``--clients`` concurrent clients (spread over ``--procs`` client processes, each with its own
  Thrift connection and session) issue the 8 benchmark queries round-robin -- TPC-H Q3 with its
  standard ``ORDER BY ... LIMIT 10`` so a dashboard client does not pull a million rows;
* open loop at a fixed aggregate rate ``--qps`` (each client sends on its own schedule; latency is
  measured from the *scheduled* send time, so queueing delay counts -- no coordinated omission),
  or closed loop (``--qps 0``: every client sends its next query when the previous one returns);
* prints one JSON line: achieved QPS, p50/p90/p99/max latency overall and per query.

  python tools/concurrency_bench.py --sf 100 --clients 64 --qps 400 --duration 30
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


WORKLOAD = "fixed"


def queries():
    """The statements the clients cycle through: the 8 benchmark queries (``fixed``), or
    ``varied``: ~2,000 distinct parameterizations of the same 8 shapes -- random ship / order date
    windows, nations, regions, market segments, part types -- so no two clients share a text by
    construction and every execution is a real scan (identical-statement sharing cannot help)."""
    from spark_druid_olap_amd.models import tpch

    if WORKLOAD == "varied":
        return varied_queries()
    if WORKLOAD == "jmx":
        from spark_druid_olap_amd.models import bi

        return [(n, q) for n, _, q in bi.statements(25, BIND)]
    out = []
    for name, q in tpch.BENCH_QUERIES:
        if name == "TPCH Q3":
            q = q.rstrip() + " order by price desc, o_orderdate limit 10"
        out.append((name, " ".join(q.split())))
    return out


def varied_queries(n: int = 2000, seed: int = 7):
    import random

    from spark_druid_olap_amd.models import tpch

    T = tpch.T
    rnd = random.Random(seed)
    nations = ["ALGERIA", "ARGENTINA", "BRAZIL", "CANADA", "EGYPT", "ETHIOPIA", "FRANCE", "GERMANY", "INDIA",
               "INDONESIA", "IRAN", "IRAQ", "JAPAN", "JORDAN", "KENYA", "MOROCCO", "MOZAMBIQUE", "PERU", "CHINA",
               "ROMANIA", "SAUDI ARABIA", "VIETNAM", "RUSSIA", "UNITED KINGDOM", "UNITED STATES"]
    regions = ["AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"]
    segs = ["AUTOMOBILE", "BUILDING", "FURNITURE", "HOUSEHOLD", "MACHINERY"]
    types = [f"{a} {b} {c}" for a in ("ECONOMY", "PROMO", "STANDARD") for b in ("ANODIZED", "BRUSHED", "PLATED")
             for c in ("STEEL", "BRASS", "COPPER")]

    def day(lo=1992, hi=1998):
        return f"{rnd.randint(lo, hi)}-{rnd.randint(1, 12):02d}-{rnd.randint(1, 28):02d}"

    shapes = [
        ("ShipDate", lambda: f"select l_returnflag, l_linestatus, count(*) from {T} where l_shipdate >= '{day(1992, 1995)}' "
                             f"and l_shipdate < '{day(1996, 1998)}' group by l_returnflag, l_linestatus"),
        ("Q1-window", lambda: f"select l_returnflag, l_linestatus, count(*), sum(l_extendedprice), max(ps_supplycost), "
                              f"avg(ps_availqty) from {T} where l_shipdate <= '{day(1996, 1998)}' "
                              f"group by l_returnflag, l_linestatus"),
        ("Q3", lambda: f"select o_orderkey, sum(l_extendedprice) as price, o_orderdate, o_shippriority from {T} "
                       f"where c_mktsegment = '{rnd.choice(segs)}' and o_orderdate < '{day(1994, 1996)}' "
                       f"and l_shipdate > '{day(1994, 1996)}' group by o_orderkey, o_orderdate, o_shippriority "
                       f"order by price desc, o_orderdate limit 10"),
        ("Q5", lambda: f"select s_nation, sum(l_extendedprice) from {T} where s_region = '{rnd.choice(regions)}' "
                       f"and o_orderdate >= '{day(1993, 1995)}' and o_orderdate < '{day(1996, 1997)}' group by s_nation"),
        ("Q7", lambda: (lambda a, b: f"select s_nation, c_nation, year(dateTime(`l_shipdate`)) as y, sum(l_extendedprice) "
                                     f"from {T} where ((s_nation = '{a}' and c_nation = '{b}') or "
                                     f"(c_nation = '{a}' and s_nation = '{b}')) group by s_nation, c_nation, "
                                     f"year(dateTime(`l_shipdate`))")(*rnd.sample(nations, 2))),
        ("Q8", lambda: f"select year(dateTime(`o_orderdate`)) as y, sum(l_extendedprice) from {T} "
                       f"where c_region = '{rnd.choice(regions)}' and p_type = '{rnd.choice(types)}' "
                       f"and o_orderdate >= '{day(1993, 1994)}' and o_orderdate <= '{day(1995, 1997)}' "
                       f"group by year(dateTime(`o_orderdate`))"),
        ("Nation-mix", lambda: f"select c_nation, count(*), sum(l_quantity) from {T} where s_nation = "
                               f"'{rnd.choice(nations)}' and l_shipdate >= '{day()}' group by c_nation"),
        ("Segment", lambda: f"select c_mktsegment, count(*), sum(l_extendedprice) from {T} where "
                            f"p_type = '{rnd.choice(types)}' and o_orderdate < '{day()}' group by c_mktsegment"),
    ]
    out, seen = [], set()
    while len(out) < n:
        name, f = shapes[len(out) % len(shapes)]
        q = " ".join(f().split())
        if q not in seen:
            seen.add(q)
            out.append((name, q))
    return out


def _client_proc(pid, nthreads, nclients, start_q, out_q, workload="fixed", bind="years"):
    import threading

    from spark_druid_olap_amd.server.hive_client import connect

    global NCLIENTS, WORKLOAD, BIND
    NCLIENTS = nclients
    WORKLOAD = workload
    BIND = bind
    port, t_start, duration, interval = start_q.get()

    qs = queries()
    res = []
    lock = threading.Lock()

    def worker(k):
        cid = pid * nthreads + k
        conn = connect(port=port)
        i = cid
        sched_it = None
        if WORKLOAD == "jmx":
            # the JMeter plan: this client belongs to one thread group and walks its templates in
            # random order per iteration, the shared CSV cursors giving each iteration's parameters
            from spark_druid_olap_amd.models import bi

            sched_it = bi.client_schedule(cid, NCLIENTS, BIND)
        # stagger the open-loop schedules so the aggregate arrival rate is uniform
        nxt = t_start + (cid * interval / max(1, NCLIENTS)) if interval else t_start
        while True:
            now = time.time()
            if interval:
                if nxt > t_start + duration:
                    break
                if nxt > now:
                    time.sleep(nxt - now)
                sched = nxt
                nxt += interval
            else:
                if now > t_start + duration:
                    break
                sched = now
            if sched_it is not None:
                name, sql = next(sched_it)
            else:
                name, sql = qs[(i * 7919) % len(qs)] if WORKLOAD == "varied" else qs[i % len(qs)]
            i += NCLIENTS if WORKLOAD == "varied" else 1
            err = None
            try:
                cur = conn.cursor().execute(sql)
                rows = cur.fetchall()
                cur.close()
                n = len(rows)
            except Exception as e:  # noqa: BLE001
                err, n = f"{type(e).__name__}: {e}", 0
            done = time.time()
            with lock:
                res.append((name, sched, done, n, err))
        conn.close()

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    out_q.put(res)


NCLIENTS = 1
BIND = "years"


def pct(xs, p):
    if not xs:
        return None
    xs = sorted(xs)
    k = min(len(xs) - 1, max(0, int(round(p / 100.0 * (len(xs) - 1)))))
    return xs[k]


def main():
    global NCLIENTS
    from spark_druid_olap_amd.utils.memory import serving_allocator_conf

    serving_allocator_conf()  # the server's allocator settings (server/hive_server.py main)
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--qps", type=float, default=200.0, help="aggregate target rate; 0 = closed loop")
    ap.add_argument("--duration", type=float, default=20.0)
    ap.add_argument("--warmup", type=float, default=3.0)
    ap.add_argument("--server", default="native", choices=["native", "python"],
                    help="native C++ gateway (server/csrc/hs2_gateway.cpp) or the pure-Python server")
    ap.add_argument("--sample", default=None, help="write a sampling profile of the server threads here")
    ap.add_argument("--include-warmup", action="store_true",
                    help="--timeline / --sample also cover the closed loop's warm-up seconds (the cold burst)")
    ap.add_argument("--workload", default="fixed", choices=["fixed", "varied", "jmx"],
                    help="fixed: the 8 benchmark texts; varied: ~2,000 distinct parameterizations; jmx: the "
                         "reference's BI plan (docs/bi-benchmark/snap-sales-demo.jmx, models/bi)")
    ap.add_argument("--bind", default="years", choices=["years", "jmeter"],
                    help="jmx workload: CSV binding (models/bi: 'jmeter' reproduces the plan's ccode overwrite)")
    ap.add_argument("--coalesce", default="on", choices=["on", "off"],
                    help="off: every statement executes (identical queued statements are not shared)")
    ap.add_argument("--timeline", default=None,
                    help="native server: record every execution's phases (admission queue, prepare, slot wait, "
                         "run, encode) and write them here; the JSON line gets per-phase percentiles")
    ap.add_argument("--prewarm", type=int, default=0,
                    help="varied workload: plan + compile this many distinct texts before the clock starts")
    ap.add_argument("--wait", default="spin", choices=["blocking", "spin"],
                    help="HIP's wait mode for the server's threads (utils/hipsync.py): spin (HIP's default; the "
                         "engine's own waits still sleep after 2 ms, ops/csrc/bindings.cpp wait_stream) or "
                         "blocking (every wait sleeps on the interrupt: least CPU, ~40%% less capacity at 400 QPS, "
                         "profiles/r6/thrift_jmx_q400_blocking_wait.json)")
    ap.add_argument("--settle", action="store_true",
                    help="after the warm-up: wait for its background compiles and size the slots' device "
                         "memory for the largest statement (a server's warm-up step)")
    a = ap.parse_args()
    global WORKLOAD, BIND
    WORKLOAD = a.workload
    BIND = a.bind
    os.environ["SDO_COALESCE"] = "1" if a.coalesce == "on" else "0"
    NCLIENTS = a.clients
    nthreads = max(1, a.clients // a.procs)
    nproc = max(1, a.clients // nthreads)
    # client processes start BEFORE this process touches the GPU (no fork/exec of a GPU process)
    ctx = mp.get_context("spawn")
    res_q = ctx.Queue()
    start_q = ctx.Queue()
    ps = [ctx.Process(target=_client_proc, args=(i, nthreads, a.clients, start_q, res_q, a.workload, a.bind))
          for i in range(nproc)]
    for p in ps:
        p.start()
    # before anything touches the GPU (the flag only takes before the device is initialised)
    from spark_druid_olap_amd.utils.hipsync import set_wait_mode

    wait_set = set_wait_mode(a.wait, int(os.environ.get("LOCAL_RANK", "0"))) if a.wait != "spin" else False
    import torch

    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.server.hive_client import connect
    from spark_druid_olap_amd.server.hive_server import HiveThriftServer
    from spark_druid_olap_amd.session import Session

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    t0 = time.time()
    ds = tpch.to_datasource(tpch.generate_flat(a.sf, dev), profile="bench")
    s = Session(conf={"spark.sparklinedata.druid.approxCountDistinct": "true"})
    s.register_datasource(ds)
    s.register_table("orderLineItemPartSupplierBase", schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(source="orderLineItemPartSupplierBase", datasource="tpch", with_column_mapping=False))
    if a.workload == "jmx":
        from spark_druid_olap_amd.models import bi

        bi.register(s)  # sales_demo_source (a shared view: every client session sees it)
    exec_cost = []  # (thread CPU s, wall s) of every server-side execution
    if a.server == "native":
        from spark_druid_olap_amd.server.gateway import NativeHiveServer

        srv = NativeHiveServer(s, port=0)
        real = srv._execute

        def timed(bid, sid, stmt, *rec):
            c0, w0 = time.thread_time(), time.perf_counter()
            try:
                return real(bid, sid, stmt, *rec)
            finally:
                exec_cost.append((time.thread_time() - c0, time.perf_counter() - w0))

        srv._execute = timed
        srv.start()
    else:
        srv = HiveThriftServer(s, port=0).start()
    print(f"[conc] server up on {srv.port}: SF{a.sf:g} {ds.num_rows} rows on {dev} in {time.time() - t0:.1f}s",
          file=sys.stderr, flush=True)
    # warm every query's plan + kernel once through the server (varied: the kernel shapes, and
    # --prewarm texts; the rest are planned on first sight, inside the measured window)
    with connect(port=srv.port) as c:
        qs = queries()
        if a.workload == "jmx":
            # one text per template (the shapes' kernels), like the varied workload's 8
            seen_t, warm = set(), []
            for n, q in qs:
                if n not in seen_t:
                    seen_t.add(n)
                    warm.append((n, q))
            warm += qs[len(warm):max(len(warm), a.prewarm)]
        else:
            warm = qs if a.workload == "fixed" else qs[:max(len(qs) and 8, a.prewarm)]
        for i, (name, sql) in enumerate(warm):
            tw = time.time()
            c.cursor().execute(sql).fetchall()
            # (progress on stderr: a long warm-up -- first-seen shapes compile -- stays visibly alive)
            print(f"[conc] warm {i + 1}/{len(warm)} {name[:40]} {time.time() - tw:.2f}s", file=sys.stderr, flush=True)
    if a.settle and a.server == "native":
        # the warm-up's background compiles finish, their statements re-prepare once, then the
        # slots' device memory is sized for the largest statement seen (NativeHiveServer.settle)
        from spark_druid_olap_amd.engine.device_exec import wait_background_compiles

        if wait_background_compiles():
            with connect(port=srv.port) as c:
                for name, sql in warm:
                    c.cursor().execute(sql).fetchall()
        print(f"[conc] settled: {srv.settle()}", file=sys.stderr, flush=True)
    interval = (a.clients / a.qps) if a.qps > 0 else 0.0
    if a.timeline and a.server == "native":
        # (from the open loop's start: its warm-up seconds -- negative times -- included)
        from spark_druid_olap_amd.utils.metrics import log_events

        log_events(True)
        srv.stalls = []
        if a.include_warmup:
            srv.timeline = []
    t_start = time.time() + 1.0 + a.warmup
    for _ in ps:
        start_q.put((srv.port, t_start - a.warmup, a.duration + a.warmup, interval))
    # server-side counters over the measured window: process CPU (GIL-bound if ~1 core), number of
    # executions vs statements (identical-statement batching), stream-slot waits
    co = s.engine.coalescer()

    def counters():
        if a.server == "native":
            st = srv.stats()
            return st["coalesced"], st["batches"]
        return co.stats["coalesced"], co.stats["executions"]

    sampler = None
    if a.sample and a.include_warmup:
        from spark_druid_olap_amd.utils.sampler import Sampler

        sampler = Sampler().start()
    time.sleep(max(0.0, t_start - time.time()))
    if sampler is not None:  # (--include-warmup: the profile covers the warm-up seconds only)
        sampler.stop()
        with open(a.sample, "w") as f:
            f.write(sampler.report(60))
        sampler = None
    if a.timeline and a.server == "native" and not a.include_warmup:
        srv.timeline = []
    cpu0 = time.process_time()
    co0, ex0 = counters()
    if a.sample and not a.include_warmup:
        from spark_druid_olap_amd.utils.sampler import Sampler

        sampler = Sampler().start()
    t_end = time.time() + a.duration
    while time.time() < t_end:
        time.sleep(min(15.0, max(0.0, t_end - time.time())))
        print(f"[conc] measuring, {max(0.0, t_end - time.time()):.0f}s left", file=sys.stderr, flush=True)
    if sampler is not None:
        sampler.stop()
        with open(a.sample, "w") as f:
            f.write(sampler.report(60))
    cpu1 = time.process_time()
    co1, ex1 = counters()
    ncost = len(exec_cost)
    res = []
    import faulthandler

    # a client that never gets its answer: every server thread's stack, every 60 s, to stderr
    faulthandler.dump_traceback_later(60, repeat=True, file=sys.stderr)
    for i, _ in enumerate(ps):
        res.extend(res_q.get())
        print(f"[conc] client process {i + 1}/{len(ps)} done", file=sys.stderr, flush=True)
    faulthandler.cancel_dump_traceback_later()
    for p in ps:
        p.join()
    srv.stop()
    res = [r for r in res if r[1] >= t_start]  # drop the warm-up window
    errs = [r for r in res if r[4]]
    lat = [(r[2] - r[1]) * 1e3 for r in res if not r[4]]
    span = max((r[2] for r in res), default=t_start) - t_start
    per = {}
    for name in dict(queries()):
        xs = [(r[2] - r[1]) * 1e3 for r in res if r[0] == name and not r[4]]
        per[name] = {"n": len(xs), "p50_ms": pct(xs, 50), "p99_ms": pct(xs, 99)}
    out = {"metric": "thrift_concurrent_latency", "clients": nproc * nthreads, "target_qps": a.qps,
           "workload": a.workload, "coalesce": a.coalesce, "distinct_texts": len(qs),
           "bind": a.bind if a.workload == "jmx" else None,
           "executions_per_s": round((ex1 - ex0) / a.duration, 2),
           "achieved_qps": round(len(lat) / span, 2) if span > 0 else None, "queries": len(res),
           "errors": len(errs), "p50_ms": pct(lat, 50), "p90_ms": pct(lat, 90), "p99_ms": pct(lat, 99),
           "max_ms": max(lat) if lat else None, "sf": a.sf, "device": dev, "per_query": per,
           "first_error": errs[0][4] if errs else None,
           "server": {"kind": a.server, "cpu_cores": round((cpu1 - cpu0) / a.duration, 2), "executions": ex1 - ex0,
                      "exec_thread_cpu_ms": round(1e3 * sum(c for c, _ in exec_cost[:ncost]) / max(1, ncost), 3),
                      "exec_wall_ms": round(1e3 * sum(w for _, w in exec_cost[:ncost]) / max(1, ncost), 3),
                      "executors": getattr(srv, "nexec", None),
                      "coalesced": co1 - co0, "slots": co.scheduler.nslots,
                      "slot_wait_ms_total": round(co.scheduler.stats["wait_ms"], 1),
                      "gpu_wait": a.wait if wait_set or a.wait == "spin" else "spin (flag refused)"},
           "device_memory": _mem_report()}
    if a.timeline and a.server == "native" and srv.timeline is not None:
        out["timeline"] = timeline_summary(srv.timeline, a.timeline)
        t0 = min((r["t"] for r in srv.timeline), default=0.0)
        ev = log_events(False)
        out["stalls"] = [dict(s, t=round(s["t"] - t0, 3),
                              events=[(round(e[0] - t0, 3),) + tuple(e[1:]) for e in ev
                                      if s["t"] - s["idle_ms"] / 1e3 - 0.2 <= e[0] <= s["t"]][:40])
                         for s in (srv.stalls or [])]
        evc = {}
        for e in ev:
            evc[e[1]] = evc.get(e[1], 0) + 1
        out["timeline"]["events"] = evc
        with open(a.timeline + ".events.json", "w") as f:
            json.dump([(round(e[0] - t0, 4),) + tuple(e[1:]) for e in ev], f)
    print(json.dumps(out), flush=True)


def timeline_summary(tl, path):
    """Per-phase percentiles of the server's executions, the phase split of the slowest 1%, and
    the worst 100 ms windows (executions that started in them and their slowest phase) -- a stall
    that hits every slot at once shows up as one window with many slow runs."""
    import math

    tl = list(tl)
    with open(path, "w") as f:
        json.dump(tl, f)
    phases = ("queue_ms", "sql_ms", "prepare_ms", "slot_wait_ms", "run_ms", "encode_ms")
    retried = [r for r in tl if r.get("alloc_retries")]
    tot = lambda r: sum(r.get(k, 0.0) for k in phases)  # noqa: E731
    summ = {k: {"p50": pct([r.get(k, 0.0) for r in tl], 50), "p99": pct([r.get(k, 0.0) for r in tl], 99),
                "max": max((r.get(k, 0.0) for r in tl), default=None)} for k in phases}
    slow = sorted(tl, key=tot, reverse=True)[:max(1, len(tl) // 100)]
    summ["slowest_1pct_mean"] = {k: round(sum(r.get(k, 0.0) for r in slow) / len(slow), 2) for k in phases} \
        if slow else {}
    t0 = min((r["t"] for r in tl), default=0.0)
    win = {}
    for r in tl:
        w = int(math.floor((r["t"] - t0) / 0.1))
        win.setdefault(w, []).append(r)
    worst = sorted(win.items(), key=lambda kv: max(tot(r) for r in kv[1]), reverse=True)[:5]
    summ["worst_windows"] = [{"t_s": round(w * 0.1, 1), "n": len(rs), "max_total_ms": round(max(tot(r) for r in rs), 1),
                              "mean": {k: round(sum(r.get(k, 0.0) for r in rs) / len(rs), 1) for k in phases}}
                             for w, rs in worst]
    summ["n"] = len(tl)
    # statements during which the caching allocator freed every cached block and retried
    summ["alloc_retry_statements"] = [{"t_s": round(r["t"] - t0, 3), "retries": r["alloc_retries"],
                                       "run_ms": round(r.get("run_ms", 0.0), 1), "stmt": r["stmt"][:80]}
                                      for r in sorted(retried, key=lambda r: r["t"])[:20]]
    return summ


def _mem_report():
    try:
        from spark_druid_olap_amd.engine.device_exec import device_memory_report

        return device_memory_report()
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)}


if __name__ == "__main__":
    main()
