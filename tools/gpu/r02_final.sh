#!/bin/bash
# Round-2 measurement snapshot: the driver's default bench (with the CPU baseline), the
# rocprofv3 kernel-trace summary of the same command, and the PMC traffic passes of the
# isolated roofline call.  Everything under gpurun_out/final_$TAG.
set -o pipefail
TAG=${TAG:-a}
D=gpurun_out/final_$TAG
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
python tools/gpu/summarize.py $D/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_traced.json 2> $D/bench_traced.err || { tail -5 $D/bench_traced.err; exit 1; }
f=$(find $D/trace -name "*kernel_stats.csv" | head -1); cp $f $D/kernel_stats.csv
f=$(find $D/trace -name "*kernel_trace.csv" | head -1); python tools/gpu/trace_summary.py $f $D/trace_summary.json > /dev/null
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $D/pmc$i -o run --output-format csv -- python3 tools/gpu/roof_call.py > $D/pmc$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 $D/pmc$i.log; exit 1; }
  echo "pmc pass $i ok: $grp"
done
