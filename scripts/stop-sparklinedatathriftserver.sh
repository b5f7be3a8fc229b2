#!/bin/bash
# Stop the server started by start-sparklinedatathriftserver.sh (by its recorded PID only).
PIDFILE="${SDO_PID_DIR:-/tmp}/sdo-thriftserver.pid"
if [ ! -f "$PIDFILE" ]; then echo "no pid file $PIDFILE"; exit 1; fi
PID="$(cat "$PIDFILE")"
if kill -0 "$PID" 2>/dev/null; then kill "$PID"; echo "stopped $PID"; else echo "process $PID not running"; fi
rm -f "$PIDFILE"
