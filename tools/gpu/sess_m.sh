# Round-4 session m: k_final_fold with the lean squaring operands (BGV_FOLD_LEAN, default on)
# against the select-based forms: GPU suite, config-3 latency interleaved, kernel trace of the
# latency probe, Node gossip.
#   bash tools/gpu/sess_m.sh OUTDIR
set -o pipefail
O=$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; echo suite failed; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat_lean.jsonl 2>>$O/err.txt || { echo lat failed; exit 1; }
  BGV_FOLD_LEAN=0 timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat_sel.jsonl 2>>$O/err.txt || { echo lat_sel failed; exit 1; }
done
cat $O/lat_lean.jsonl $O/lat_sel.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o run --output-format csv \
  -- python3 tools/gpu/latency_probe.py 30 > $O/lat_traced.json 2>> $O/err.txt || { echo trace failed; exit 1; }
cat $O/lat_trace/run_kernel_stats.csv
timeout -k 10 200 node tests/node/gossip_bench.js 5 64 "63:1" > $O/gossip.jsonl 2> $O/gossip.err || { echo gossip failed; exit 1; }
cat $O/gossip.jsonl
