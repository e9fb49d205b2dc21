#!/bin/bash
# team vs one-lane Miller loop at full occupancy (64,512-set call): per-kernel ms
set -o pipefail
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
timeout -k 10 200 python tools/gpu/roof_call.py > gpurun_out/r02/roof_lane.json 2>&1 || { tail -5 gpurun_out/r02/roof_lane.json; exit 1; }
cat gpurun_out/r02/roof_lane.json
BGV_TEAM_MILLER_MAX=1000000 timeout -k 10 200 python tools/gpu/roof_call.py > gpurun_out/r02/roof_team.json 2>&1 || { tail -5 gpurun_out/r02/roof_team.json; exit 1; }
cat gpurun_out/r02/roof_team.json
