#!/bin/bash
# GPU box: 2-rank root-only rehearsal (gloo, one card) after the peer-stub fix, then the
# concurrency benchmark on a varied workload (2,000 distinct parameterized texts) at SF100 with
# identical-statement sharing off and on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SDO_GLOO_GPU=1 SDO_RESULTS_ON_ROOT=1 timeout -k 10 400 python bench.py --gpus 2 --sf 20 --steps 5 --warmup 2 --verbose > gpurun_out/bench2_gloo_root1b.json 2> gpurun_out/bench2_gloo_root1b.err || { tail -30 gpurun_out/bench2_gloo_root1b.err; exit 1; }
tail -1 gpurun_out/bench2_gloo_root1b.json
for C in off on; do
timeout -k 10 300 python tools/concurrency_bench.py --sf 100 --clients 64 --procs 8 --qps 0 --duration 20 --warmup 3 --workload varied --coalesce $C > gpurun_out/conc_varied_$C.json 2> gpurun_out/conc_varied_$C.err || { tail -30 gpurun_out/conc_varied_$C.err; exit 1; }
cut -c1-400 gpurun_out/conc_varied_$C.json
done
