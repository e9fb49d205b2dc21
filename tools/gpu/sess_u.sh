# Round-4 session u: the idle coalescing window (BGV_IDLE_COALESCE_US, default 50) at 50 / 10 / 0 on
# the config-3 latency and the Node 64-caller gossip rate.
#   bash tools/gpu/sess_u.sh OUTDIR
set -o pipefail
O=$1; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for w in 50 10 0; do
    BGV_IDLE_COALESCE_US=$w timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat_w$w.jsonl 2>>$O/err.txt || { echo lat failed; exit 1; }
  done
done
for w in 50 10 0; do
  BGV_IDLE_COALESCE_US=$w timeout -k 10 100 node tests/node/gossip_bench.js 5 64 "63:1" >> $O/gossip_w$w.jsonl 2>> $O/gossip.err || { echo gossip failed; exit 1; }
done
for w in 50 10 0; do echo "w=$w"; cat $O/lat_w$w.jsonl | python -c "import sys,json; print([round(json.loads(l)['p50_latency_ms'],3) for l in sys.stdin])"; cat $O/gossip_w$w.jsonl; done
