# device-side coalescing windows for small calls: config-3 p50 and the Node gossip bench
set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
for w in 200 50 0; do
  BGV_IDLE_COALESCE_US=$w timeout -k 10 120 python tools/gpu/latency_probe.py 40 > $O/lat_idle$w.json 2>>$O/err || exit 1
  echo "idle $w: $(cat $O/lat_idle$w.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["p50_latency_ms"], d["p90_latency_ms"])')"
done
for cw in "2000 200" "500 50" "200 20"; do
  set -- $cw
  BGV_COALESCE_US=$1 BGV_IDLE_COALESCE_US=$2 timeout -k 10 120 node tests/node/gossip_bench.js 5 64 "16:1,64:1" > $O/gossip_$1_$2.jsonl 2>>$O/err || exit 1
  echo "coalesce $1/$2: $(python -c "
import json
for l in open('$O/gossip_$1_$2.jsonl'): d=json.loads(l); print(round(d['sets_per_s']), d['latency_ms']['p50'], end='; ')
")"
done
