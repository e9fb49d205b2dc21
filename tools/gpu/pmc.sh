#!/bin/bash
# PMC passes (one counter group per run, rocprofv3 --pmc only, no tracing) over one
# unloaded 131072-set verify call: HBM traffic and instruction mix per kernel.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--nsets 131072 --inflight 1 --steps 1 --warmup 0 --no-cpu-baseline"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok: $grp"
done
find gpurun_out/pmc -name "*counter_collection*" | head
