#!/bin/bash
# Submit one gpurun command, re-submitting only while the pool reports that
# nothing ran (no box free, or the infrastructure back-off): at most TRIES
# submissions, WAIT seconds apart.  A command that ran -- whatever its exit
# status -- is never re-submitted.  Usage: gpurun_when_free.sh LOG TIMEOUT 'CMD'
LOG=$1; LIM=$2; CMD=$3
TRIES=${TRIES:-12}; WAIT=${WAIT:-150}
for i in $(seq 1 $TRIES); do
  timeout $((LIM + 900)) /usr/local/graft/bin/gpurun --timeout "$LIM" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG"; then
    w=$(grep -oE "retry in [0-9]+s" "$LOG" | grep -oE "[0-9]+" | tail -1)
    w=$(( ${w:-0} + 15 > WAIT ? ${w:-0} + 15 : WAIT ))
    echo "[when_free] attempt $i: no box ($(date +%T)); waiting $w s" >> "$LOG.tries"
    sleep "$w"
    continue
  fi
  echo "[when_free] attempt $i ran, rc=$rc" >> "$LOG.tries"
  exit $rc
done
exit 3
