"""Multi-rank (gloo, 2 / 3 / 4 ranks) tests of the partial merges (parallel/merge.py).

* The bucketed dense merge (int sums + per-rank status words, float sums, max + NOT(min)) must equal a
  plain per-slot reduction of every rank's partials, including INT64 extremes in min/max slots
  (int / min / max / HLL slots exactly; f64 sums to a relative tolerance, since a ring all-reduce of
  more than two ranks adds in a different order), and a failing rank must make every rank raise after
  the same collective sequence, naming the rank that failed.
* The sparse hash-partitioned all-to-all shuffle must equal a single-process merge of the union, and
  each rank must receive only about 1/N of the partial rows.
"""
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
    hll = [torch.randint(0, 30, (R, 64), generator=g, dtype=torch.int32).to(torch.uint8)]
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


def _same(got: torch.Tensor, exp: torch.Tensor) -> bool:
    for s, (op, _) in enumerate(SLOTS):
        if op == 1:
            if not torch.allclose(got[:, s].view(torch.float64), exp[:, s].view(torch.float64), rtol=1e-12):
                return False
        elif not torch.equal(got[:, s], exp[:, s]):
            return False
    return True


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

    from spark_druid_olap_amd.planner import cost

    w = init_world(backend="gloo")
    cost.ONESHOT_MAX_BYTES = 0        # the one-shot gather is infeasible -> bucketed all-reduce path
    assert merge.merge_plan_for(w, Partials("dense", *_partial(rank))).kind == "bucketed-allreduce"
    acc, hll = _partial(rank)
    m = merge.merge_partials(w, _Prog(), Partials("dense", acc, None, hll))
    exp_acc, exp_hll = _expected(world)
    log = {"ok": _same(m.acc, exp_acc) and bool(torch.equal(m.hll[0], exp_hll))}
    err = RuntimeError("boom") if rank == 1 else None
    try:
        merge.merge_partials(w, _Prog(), Partials("dense", acc, None, hll), local_error=err)
        log["fault"] = "none"
    except RankFailure as e:
        log["fault"] = "peer-failed"
        log["msg"] = str(e)
    except RuntimeError:
        log["fault"] = "own"
    m2 = merge.merge_partials(w, _Prog(), Partials("dense", acc, None, hll))   # still in lock-step
    log["after"] = _same(m2.acc, exp_acc)
    with open(os.path.join(outdir, f"m{rank}.json"), "w") as f:
        json.dump(log, f)
    w.barrier()
    shutdown()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 3, 4])
def test_bucketed_dense_merge(world):
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
    assert logs[1]["fault"] == "own"
    for r in [0] + list(range(2, world)):
        assert logs[r]["fault"] == "peer-failed" and "[1]" in logs[r]["msg"], logs[r]
    assert all(lg["after"] for lg in logs)


# ------------------------------------------------------------------------------ sparse shuffle
SPARSE_SLOTS = [(0, 0), (1, 0), (2, 2 ** 63 - 1), (3, -2 ** 63)]


class _SProg:
    slots = SPARSE_SLOTS


def _sparse_partial(rank: int, n: int = 4000):
    g = torch.Generator().manual_seed(77 + rank)
    keys = torch.randperm(12000, generator=g)[:n].to(torch.int64) * 7919  # overlapping key sets
    acc = torch.randint(0, 10 ** 9, (n, len(SPARSE_SLOTS)), generator=g, dtype=torch.int64)
    acc[:, 1] = (torch.rand(n, generator=g, dtype=torch.float64) * 1e3).view(torch.int64)
    hll = [torch.randint(0, 20, (n, 16), generator=g, dtype=torch.int32).to(torch.uint8)]
    return keys, acc, hll


def _shuffle_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from spark_druid_olap_amd.engine.partials import Partials, merge_sparse
    from spark_druid_olap_amd.parallel import merge
    from spark_druid_olap_amd.parallel.world import init_world, shutdown

    w = init_world(backend="gloo")
    keys, acc, hll = _sparse_partial(rank)
    recv = {}
    orig = w.all_to_all_varlen

    def spy(t, counts, status=None):
        out = orig(t, counts, status)
        if t.dim() == 2 and t.dtype == torch.uint8 and t.shape[1] == 8 * (1 + len(SPARSE_SLOTS)) + 16:
            recv["rows"] = int(out[0].shape[0])
        return out
    w.all_to_all_varlen = spy
    m = merge.merge_partials(w, _SProg(), Partials("sparse", acc, keys, hll))
    parts = []
    for r in range(world):
        k, a, h = _sparse_partial(r)
        parts.append(Partials("sparse", a, k, h))
    exp = merge_sparse(parts, SPARSE_SLOTS)
    o = torch.argsort(m.keys)
    ok = torch.equal(m.keys[o], exp.keys)
    for s, (op, _) in enumerate(SPARSE_SLOTS):
        if op == 1:
            ok &= torch.allclose(m.acc[o, s].view(torch.float64), exp.acc[:, s].view(torch.float64), rtol=1e-12)
        else:
            ok &= torch.equal(m.acc[o, s], exp.acc[:, s])
    ok &= torch.equal(m.hll[0][o], exp.hll[0])
    with open(os.path.join(outdir, f"s{rank}.json"), "w") as f:
        json.dump({"ok": bool(ok), "recv": recv.get("rows", -1), "sent": int(keys.numel())}, f)
    w.barrier()
    shutdown()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 4])
def test_sparse_shuffle_merge(world):
    with tempfile.TemporaryDirectory() as td:
        ctx = mp.get_context("spawn")
        port = _free_port()
        ps = [ctx.Process(target=_shuffle_worker, args=(r, world, port, td)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(200)
            assert p.exitcode == 0, f"rank failed with {p.exitcode}"
        logs = [json.load(open(os.path.join(td, f"s{r}.json"))) for r in range(world)]
    assert all(lg["ok"] for lg in logs), logs
    total = sum(lg["sent"] for lg in logs)
    for lg in logs:  # each rank receives ~total/N partial rows (hash partitioning), not the total
        assert 0.6 * total / world < lg["recv"] < 1.4 * total / world, logs


def test_unpacked_rows_are_contiguous():
    """parallel/merge.py unpack_rows: the exchanged key / accumulator columns go to native kernels
    that take raw pointers, so they must not be strided views of the packed rows."""
    import torch

    from spark_druid_olap_amd.engine.partials import Partials
    from spark_druid_olap_amd.parallel.merge import pack_rows, unpack_rows

    keys = torch.tensor([3, 7, 11], dtype=torch.int64)
    acc = torch.tensor([[1, 10], [2, 20], [3, 30]], dtype=torch.int64)
    out = unpack_rows(pack_rows(Partials("sparse", acc, keys, [])), 2, [])
    assert out.keys.is_contiguous() and out.acc.is_contiguous()
    assert out.keys.tolist() == [3, 7, 11] and out.acc.tolist() == acc.tolist()
