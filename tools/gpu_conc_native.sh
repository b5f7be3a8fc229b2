#!/bin/bash
# GPU box: BASELINE config 5 with the native gateway -- 64 clients, closed loop + fixed rates; plus
# the HIP-engine run of the reference corpus
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for QPS in ${QPS_LIST:-0 1500}; do
  timeout -k 10 200 python tools/concurrency_bench.py --sf ${SF:-100} --clients 64 --procs 16 --qps $QPS --duration ${DUR:-10} --warmup 2 \
    --server native > gpurun_out/connat_qps$QPS.json 2> gpurun_out/connat_qps$QPS.log || { tail -20 gpurun_out/connat_qps$QPS.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/connat_qps$QPS.json')); print($QPS, d['achieved_qps'], d['p50_ms'], d['p99_ms'], d['errors'], d['server'], d['first_error'])"
done
timeout -k 10 600 python -u -m pytest tests/test_reference_corpus.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/corpus_gpu.log 2>&1 || { tail -40 gpurun_out/corpus_gpu.log; exit 1; }
tail -3 gpurun_out/corpus_gpu.log
