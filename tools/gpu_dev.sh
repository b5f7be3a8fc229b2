#!/bin/bash
# GPU box: focused GPU tests (-k filter) + headline bench + stage probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_dev.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_dev.log | tail -20; tail -40 gpurun_out/pytest_dev.log; exit 1; }
tail -2 gpurun_out/pytest_dev.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_dev.json 2> gpurun_out/bench_dev.err || { tail -30 gpurun_out/bench_dev.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_dev.json')); print(d['value'], d['per_query_ms'])"
timeout -k 10 300 python tools/stage_probe.py --sf 100 --reps 20 > gpurun_out/stage_dev.txt 2>&1 || { tail -20 gpurun_out/stage_dev.txt; exit 1; }
cat gpurun_out/stage_dev.txt
