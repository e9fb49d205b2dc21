#!/bin/bash
# Submit one command to the GPU box with gpurun, re-submitting only while no box is free
# (gpurun exit status 3: nothing ran, nothing charged).  Any other status is final.
#   tools/gpu/submit.sh TIMEOUT_S 'command'
T=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3
