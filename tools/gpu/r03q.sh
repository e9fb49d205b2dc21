set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
BGV_TRACE=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep > $O/trace.json 2> $O/trace.err || exit 1
grep "round" $O/trace.err | tail -9
