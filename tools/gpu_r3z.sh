#!/bin/bash
# GPU box: per-stage host / GPU latency of the headline queries, with per-function timers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 SDO_JIT_SPECIALIZE=sync SDO_JIT_SPECIALIZE_AFTER=1
W=spark_druid_olap_amd.engine.device_exec:PreparedScan.run,spark_druid_olap_amd.engine.partials:finalize,spark_druid_olap_amd.engine.executor:PreparedQuery._post,spark_druid_olap_amd.sql.execute:Executor._DruidQuery,spark_druid_olap_amd.session:Session.run_druid,spark_druid_olap_amd.engine.executor:PreparedQuery.run,spark_druid_olap_amd.sql.execute:Executor._Project,spark_druid_olap_amd.engine.executor:PreparedQuery.run_partials
timeout -k 10 170 python tools/stage_probe.py --sf 100 --reps 40 > gpurun_out/stage_probe.txt 2>&1 || { tail -30 gpurun_out/stage_probe.txt; exit 1; }
timeout -k 10 170 python tools/stage_probe.py --sf 100 --reps 40 --wrap $W > gpurun_out/stage_probe_wrap.txt 2>&1 || { tail -30 gpurun_out/stage_probe_wrap.txt; exit 1; }
cat gpurun_out/stage_probe.txt | tail -9
grep -v "^$" gpurun_out/stage_probe_wrap.txt | tail -80
