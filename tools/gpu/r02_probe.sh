#!/bin/bash
# Round-2 probe: the driver's bench command under several super-batch geometries
# (steady-state question of VERDICT r01 item 2), plus a kernel trace of the default run.
set -o pipefail
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-block-import"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 $B > gpurun_out/probe/$name.json 2> gpurun_out/probe/$name.err || { echo "$name failed rc=$?"; tail -5 gpurun_out/probe/$name.err; exit 1; }
  python tools/gpu/summarize.py gpurun_out/probe/$name.json
}
run base BGV_TRACE=1
run s40k BGV_TRACE=1 BGV_MAX_BATCH_SLOTS=40960
run s16k_d8 BGV_TRACE=1 BGV_MAX_BATCH_SLOTS=16384 BGV_DISPATCHERS=8 GPU_MAX_HW_QUEUES=16
run s8k_d16 BGV_TRACE=1 BGV_MAX_BATCH_SLOTS=8192 BGV_DISPATCHERS=16 GPU_MAX_HW_QUEUES=16
timeout -k 10 200 python bench.py --steps 64 --warmup 16 --no-cpu-baseline --no-block-import > gpurun_out/probe/long.json 2> gpurun_out/probe/long.err || exit 1
python tools/gpu/summarize.py gpurun_out/probe/long.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/probe/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-block-import > gpurun_out/probe/trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/probe/trace.log; exit 1; }
echo done
