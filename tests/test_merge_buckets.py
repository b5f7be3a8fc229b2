"""Two-rank (gloo) test of the large-dense partial merge (parallel/merge.py): the bucketed
collectives (int sums + status, float sums, max + NOT(min)) must equal a plain per-slot reduction
of both ranks' partials, including INT64 extremes in min/max slots, and a failing rank must make
every rank raise after the same collective sequence."""
import json
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

SLOTS = [(0, 0), (1, 0), (2, 2 ** 63 - 1), (3, -2 ** 63), (0, 0), (2, 2 ** 63 - 1), (3, -2 ** 63), (1, 0)]


class _Prog:
    slots = SLOTS


def _partial(rank: int, R: int = 300):
    g = torch.Generator().manual_seed(1234 + rank)
    acc = torch.randint(-10 ** 12, 10 ** 12, (R, len(SLOTS)), generator=g, dtype=torch.int64)
    for s, (op, _) in enumerate(SLOTS):
        if op == 1:
            acc[:, s] = (torch.rand(R, generator=g, dtype=torch.float64) * 1e6).view(torch.int64)
    acc[0, 2] = -2 ** 63       # INT64_MIN in a min slot (negation would overflow)
    acc[1, 3] = 2 ** 63 - 1    # INT64_MAX in a max slot
    hll = [torch.randint(0, 30, (R, 64), generator=g, dtype=torch.int32)]
    return acc, hll


def _expected(world: int):
    parts = [_partial(r) for r in range(world)]
    accs = torch.stack([p[0] for p in parts])
    out = torch.empty_like(accs[0])
    for s, (op, _) in enumerate(SLOTS):
        col = accs[:, :, s]
        if op == 0:
            out[:, s] = col.sum(0)
        elif op == 1:
            out[:, s] = col.contiguous().view(torch.float64).sum(0).view(torch.int64)
        elif op == 2:
            out[:, s] = col.amin(0)
        else:
            out[:, s] = col.amax(0)
    hll = torch.stack([p[1][0] for p in parts]).amax(0)
    return out, hll


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from spark_druid_olap_amd.engine.partials import Partials
    from spark_druid_olap_amd.parallel import merge
    from spark_druid_olap_amd.parallel.fault import RankFailure
    from spark_druid_olap_amd.parallel.world import init_world, shutdown

    w = init_world(backend="gloo")
    merge.ONE_SHOT_BYTES = 0          # force the large-state (bucketed all-reduce) path
    acc, hll = _partial(rank)
    m = merge.merge_partials(w, _Prog(), Partials("dense", acc, None, hll))
    exp_acc, exp_hll = _expected(world)
    log = {"ok": bool(torch.equal(m.acc, exp_acc)) and bool(torch.equal(m.hll[0], exp_hll))}
    err = RuntimeError("boom") if rank == 1 else None
    try:
        merge.merge_partials(w, _Prog(), Partials("dense", acc, None, hll), local_error=err)
        log["fault"] = "none"
    except RankFailure:
        log["fault"] = "peer-failed"
    except RuntimeError:
        log["fault"] = "own"
    m2 = merge.merge_partials(w, _Prog(), Partials("dense", acc, None, hll))   # still in lock-step
    log["after"] = bool(torch.equal(m2.acc, exp_acc))
    with open(os.path.join(outdir, f"m{rank}.json"), "w") as f:
        json.dump(log, f)
    w.barrier()
    shutdown()


@pytest.mark.timeout(240)
def test_bucketed_dense_merge_two_ranks():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        ctx = mp.get_context("spawn")
        port = _free_port()
        ps = [ctx.Process(target=_worker, args=(r, world, port, td)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(200)
            assert p.exitcode == 0, f"rank failed with {p.exitcode}"
        logs = [json.load(open(os.path.join(td, f"m{r}.json"))) for r in range(world)]
    assert all(lg["ok"] for lg in logs), logs
    assert logs[0]["fault"] == "peer-failed" and logs[1]["fault"] == "own"
    assert all(lg["after"] for lg in logs)
