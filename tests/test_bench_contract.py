"""The driver's bench contract (bench.py): ``--gpus N`` without torchrun must start N ranks itself
(one process per GPU; here gloo on CPU), report ``n_gpus == N`` and the process-group size, and print
exactly one JSON line with the required keys."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_spawns_ranks(gpus):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--sf", "0.002",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True, timeout=540, env=env,
                       cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == gpus and out["config"]["world"]["size"] == gpus
    assert out["steps"] == 1 and out["warmup"] == 0 and out["value"] > 0


@pytest.mark.timeout(600)
def test_bench_total_sf_strong_scaling():
    """``--total-sf``: the fixed-total-SF (strong scaling) curve -- 2 ranks each hold half of SF 0.02
    and the JSON line says so (scaling "strong", the total and per-GPU scale factors in config)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--total-sf", "0.02",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True, timeout=540, env=env,
                       cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["scaling"] == "strong" and out["n_gpus"] == 2
    assert out["config"]["scale_factor_total"] == pytest.approx(0.02)
    assert out["config"]["scale_factor_per_gpu"] == pytest.approx(0.01)
    assert "SF0.02 total" in out["config"]["model"]
