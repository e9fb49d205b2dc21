# Round-4 session o: k_final_fold with register part sums (tm_wide8_dpp_ops, default) against
# the LDS part sums (BGV_FOLD_LEAN=1): GPU suite, config-3 latency interleaved, kernel trace,
# Node gossip, then the headline window twice (the retry rounds' team Miller loops now run the
# projective programs).
#   bash tools/gpu/sess_o.sh OUTDIR
set -o pipefail
O=$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; echo suite failed; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat.jsonl 2>>$O/err.txt || { echo lat failed; exit 1; }
  BGV_FOLD_LEAN=1 timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat_lds.jsonl 2>>$O/err.txt || { echo lat_lds failed; exit 1; }
done
cat $O/lat.jsonl $O/lat_lds.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o run --output-format csv \
  -- python3 tools/gpu/latency_probe.py 30 > $O/lat_traced.json 2>> $O/err.txt || { echo trace failed; exit 1; }
cat $O/lat_trace/run_kernel_stats.csv
timeout -k 10 200 node tests/node/gossip_bench.js 5 64 "63:1" > $O/gossip.jsonl 2> $O/gossip.err || { echo gossip failed; exit 1; }
cat $O/gossip.jsonl
Q="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep"
for i in 1 2; do
  timeout -k 10 200 $Q >> $O/quick.jsonl 2>>$O/err.txt || { echo quick failed; exit 1; }
done
python tools/gpu/summarize.py $O/quick.jsonl
