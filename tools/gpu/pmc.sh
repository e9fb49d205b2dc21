#!/bin/bash
# PMC passes (one counter group per run, --pmc only) and a kernel trace over the bench's
# isolated roofline call.  Outputs under gpurun_out/s3/<TAG>_pmc.
set -o pipefail
TAG=${TAG:-roof}
D=gpurun_out/${TAG}/pmc
mkdir -p $D
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $D/p$i -o run --output-format csv -- python3 tools/gpu/roof_call.py > $D/p$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 $D/p$i.log; exit 1; }
  echo "pass $i ok: $grp"
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python3 tools/gpu/roof_call.py > $D/trace.log 2>&1 || { echo trace failed; tail -5 $D/trace.log; exit 1; }
tail -1 $D/trace.log
python tools/gpu/pmc_summary.py $D > $D/summary.json && python -c "
import json; d=json.load(open('$D/summary.json'))['per_dispatch']
for k in ('k_prep','k_miller','k_final'):
    c=d.get(k,{}); 
    if not c: continue
    w=c.get('SQ_WAVES',1); cyc=c.get('SQ_WAVE_CYCLES',1)
    print(k, 'GB', round((c.get('FETCH_SIZE',0)*2+c.get('WRITE_SIZE',0))*1024/1e9,2), 'valu/wave', int(c.get('SQ_INSTS_VALU',0)/w), 'vmem_wr/wave', int(c.get('SQ_INSTS_VMEM_WR',0)/w), 'valu_active', round(c.get('SQ_ACTIVE_INST_VALU',0)/max(1,c.get('SQ_BUSY_CYCLES',1)),3), 'wait_any/cyc', round(c.get('SQ_WAIT_ANY',0)/cyc,3), 'active_valu/cyc', round(c.get('SQ_ACTIVE_INST_VALU',0)/cyc,3))
"
