#!/bin/bash
# GPU box: kernel trace of the headline bench's timed steps (per-kernel totals + one step's timeline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out
rm -rf gpurun_out/profh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$R/gpurun_out/profh" -o run -- python3 "$R/bench.py" --steps ${STEPS:-10} --warmup 3 \
  > "$R/gpurun_out/profh.log" 2>&1 || { tail -20 "$R/gpurun_out/profh.log"; exit 1; }
cd "$R"
DB=$(find gpurun_out/profh -name "*.db" | head -1)
python tools/rocpd_summary.py "$DB" --tail-ms ${TAIL:-100} --top 40 --timeline-ms ${TL:-12} > gpurun_out/profh_summary.txt
head -50 gpurun_out/profh_summary.txt
