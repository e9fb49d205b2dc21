set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
BGV_TRACE=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep > $O/trace_cur.json 2> $O/trace_cur.err || exit 1
grep -c "pattern unit" $O/trace_cur.err
