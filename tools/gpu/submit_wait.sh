#!/bin/bash
# Submit one gpurun command, resubmitting only while no GPU slot or box is free (gpurun exit
# code 3: nothing ran, nothing charged), every 3 minutes, at most 12 times.  Any other outcome
# (the command ran, failed, or was refused) ends it.
#   tools/gpu/submit_wait.sh LOG TIMEOUT 'command'
LOG=$1; TMO=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -eq 0 ] && exit 0
  grep -q "slot(s) on this pod are busy\|no box\|no free box\|retry in a few minutes" "$LOG" || exit $rc
  sleep 180
done
exit 3
