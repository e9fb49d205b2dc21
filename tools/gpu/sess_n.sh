# Round-4 session n: latency-path point programs (projective G2 chains, G1 r * pk programs,
# 2-round doublings / 3-round additions): GPU suite, config-3 latency, kernel trace, Node gossip.
#   bash tools/gpu/sess_n.sh OUTDIR
set -o pipefail
O=$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; echo suite failed; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat.jsonl 2>>$O/err.txt || { echo lat failed; exit 1; }
done
cat $O/lat.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o run --output-format csv \
  -- python3 tools/gpu/latency_probe.py 30 > $O/lat_traced.json 2>> $O/err.txt || { echo trace failed; exit 1; }
cat $O/lat_trace/run_kernel_stats.csv
timeout -k 10 200 node tests/node/gossip_bench.js 5 64 "63:1" > $O/gossip.jsonl 2> $O/gossip.err || { echo gossip failed; exit 1; }
cat $O/gossip.jsonl
