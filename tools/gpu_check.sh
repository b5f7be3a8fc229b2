#!/bin/bash
# One GPU-box session: build, kernel tests, bench at two scales, rocprof stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "== build"; timeout -k 10 300 python __graft_entry__.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for SF in ${BENCH_SFS:-10 100}; do
  for MODE in ${BENCH_MODES:-sql}; do
    echo "== bench sf$SF $MODE"; timeout -k 10 500 python bench.py --mode $MODE --sf $SF --steps 5 --warmup 2 --verbose > gpurun_out/bench_sf${SF}_$MODE.log 2>&1 || { tail -30 gpurun_out/bench_sf${SF}_$MODE.log; exit 1; }
    tail -12 gpurun_out/bench_sf${SF}_$MODE.log
  done
done
if [ -n "$PROFILE_SF" ]; then
  echo "== rocprof sf$PROFILE_SF"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode ${PROFILE_MODE:-sql} --sf $PROFILE_SF --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
  find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head
fi
echo "== done"
