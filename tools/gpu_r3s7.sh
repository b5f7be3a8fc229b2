#!/bin/bash
# GPU box: HIP-graph replay of small dense executions -- tests, headline bench graphs on/off, stage probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_kernels.py tests/test_gpu_tpch22.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_graphs.log 2>&1 || { tail -40 gpurun_out/t_graphs.log; exit 1; }
tail -2 gpurun_out/t_graphs.log
SDO_GRAPHS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/h_nograph.json 2> gpurun_out/h_nograph.err || { tail -30 gpurun_out/h_nograph.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/h_graph.json 2> gpurun_out/h_graph.err || { tail -30 gpurun_out/h_graph.err; exit 1; }
grep "\[bench\]" gpurun_out/h_nograph.err | cut -c1-100; cat gpurun_out/h_nograph.json | cut -c1-200
grep "\[bench\]" gpurun_out/h_graph.err | cut -c1-100; cat gpurun_out/h_graph.json | cut -c1-200
timeout -k 10 200 python tools/stage_probe.py --sf 100 --reps 40 > gpurun_out/stage_probe_graph.txt 2>&1 || { tail -30 gpurun_out/stage_probe_graph.txt; exit 1; }
grep -v Warn gpurun_out/stage_probe_graph.txt | tail -9
