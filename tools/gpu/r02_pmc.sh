#!/bin/bash
# PMC passes (one counter group per run, --pmc only) over the bench's isolated roofline call.
set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d gpurun_out/pmc2/p$i -o run --output-format csv -- python3 tools/gpu/roof_call.py > gpurun_out/pmc2/p$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 gpurun_out/pmc2/p$i.log; exit 1; }
  echo "pass $i ok: $grp"
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc2/trace -o run --output-format csv -- python3 tools/gpu/roof_call.py > gpurun_out/pmc2/trace.log 2>&1 || { echo trace failed; tail -5 gpurun_out/pmc2/trace.log; exit 1; }
tail -1 gpurun_out/pmc2/trace.log
