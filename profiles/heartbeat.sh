#!/bin/bash
# Run a command with a progress line every 60 s on stdout (long GPU profiling
# runs whose tools only write at the end), then exit with its status.
#   bash profiles/heartbeat.sh <command...>
( while sleep 60; do echo "[heartbeat] $(date +%T) still running: $1 $2 $3"; done ) &
HB=$!
"$@"
rc=$?
kill $HB 2>/dev/null
wait $HB 2>/dev/null
exit $rc
