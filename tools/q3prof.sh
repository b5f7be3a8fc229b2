set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/host_profile.py --sf 100 --mode sql --steps 3 --query "Q3" > gpurun_out/hp_q3.log 2>&1 || { tail -20 gpurun_out/hp_q3.log; exit 1; }
head -12 gpurun_out/hp_q3.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/profq3" -o run -- python3 "$GRAFT_REPO_ROOT/tools/host_profile.py" --sf 100 --mode sql --steps 1 --query "Q3" > "$GRAFT_REPO_ROOT/gpurun_out/profq3.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/profq3.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/profq3" -name "*kernel_stats*" -exec head -20 {} \;
