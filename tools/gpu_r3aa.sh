#!/bin/bash
# GPU box: headline bench + per-stage probe after the lazy result columns
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/h_lazy.json 2> gpurun_out/h_lazy.err || { tail -30 gpurun_out/h_lazy.err; exit 1; }
cat gpurun_out/h_lazy.json
export SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
W=spark_druid_olap_amd.engine.device_exec:PreparedScan.run,spark_druid_olap_amd.engine.partials:finalize,spark_druid_olap_amd.sql.execute:Executor._DruidQuery,spark_druid_olap_amd.engine.executor:PreparedQuery.run,spark_druid_olap_amd.sql.execute:Executor._Project,spark_druid_olap_amd.engine.executor:PreparedQuery.run_partials,spark_druid_olap_amd.engine.partials:_fetch_small
timeout -k 10 170 python tools/stage_probe.py --sf 100 --reps 40 > gpurun_out/stage_probe2.txt 2>&1 || { tail -30 gpurun_out/stage_probe2.txt; exit 1; }
timeout -k 10 170 python tools/stage_probe.py --sf 100 --reps 40 --wrap $W > gpurun_out/stage_probe_wrap2.txt 2>&1 || { tail -30 gpurun_out/stage_probe_wrap2.txt; exit 1; }
grep -v "^$" gpurun_out/stage_probe2.txt | grep -v Warn | tail -9
