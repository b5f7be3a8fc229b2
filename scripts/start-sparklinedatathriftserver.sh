#!/bin/bash
# Start the HiveServer2-compatible endpoint (scripts/start-sparklinedatathriftserver.sh in the
# reference launched HiveThriftServer2 via spark-daemon.sh).  Extra args go to the server:
#   --port 10000 --host 0.0.0.0 --tpch-sf 1 --init-sql ddl.sql
# One node, all GPUs (one rank per GPU, RCCL over xGMI), data from an index task, persisted so a
# restart resumes from the segment store:
#   --gpus 8 --ingest tpch_index_task.json@/data/tpch --segments /data/sdo_store --init-sql ddl.sql
#   (restart: --gpus 8 --segments /data/sdo_store --init-sql ddl.sql)
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
PIDFILE="${SDO_PID_DIR:-/tmp}/sdo-thriftserver.pid"
LOG="${SDO_LOG_DIR:-/tmp}/sdo-thriftserver.log"
if [ -f "$PIDFILE" ] && kill -0 "$(cat "$PIDFILE")" 2>/dev/null; then
  echo "thrift server already running as process $(cat "$PIDFILE")"; exit 1
fi
cd "$ROOT"
nohup python3 -m spark_druid_olap_amd.server.hive_server "$@" > "$LOG" 2>&1 &
echo $! > "$PIDFILE"
echo "started thrift server (pid $(cat "$PIDFILE")), log: $LOG"
