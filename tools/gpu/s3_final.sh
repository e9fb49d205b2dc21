#!/bin/bash
# Measurement snapshot: the driver's default bench (with the CPU baseline and the N=1
# extras), the rocprofv3 kernel-trace summary of the driver's 20/5 bench command, and the
# PMC passes + kernel trace of the bench's isolated roofline call (tools/gpu/s3_pmc.sh).
# Everything under gpurun_out/s3/<TAG>_final.
set -o pipefail
TAG=${TAG:-a}
D=gpurun_out/s3/${TAG}_final
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -5 $D/bench_default.err; exit 1; }
python tools/gpu/summarize.py $D/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_traced.json 2> $D/bench_traced.err || { tail -5 $D/bench_traced.err; exit 1; }
f=$(find $D/trace -name "*kernel_stats.csv" | head -1); cp $f $D/bench_kernel_stats.csv
f=$(find $D/trace -name "*kernel_trace.csv" | head -1); python tools/gpu/trace_summary.py $f $D/bench_trace_summary.json > /dev/null
rm -rf $D/trace
TAG=$TAG bash tools/gpu/s3_pmc.sh
