#!/bin/bash
# Run one gpurun call, re-submitting it only while gpurun answers 3 (no box or
# slot free: nothing ran, nothing charged).  Any other exit code -- a run that
# started, failed or was refused -- ends the loop.
# usage: tools/gpurun_retry.sh <log> <timeout-s> <command>
LOG=$1; TMO=$2; CMD=$3
for i in $(seq 1 ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep ${PAUSE:-150}
done
echo "rc=$rc tries=$i" >> "$LOG"
