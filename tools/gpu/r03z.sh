# Node gossip callers: dispatcher count x JS buffer size after the setImmediate dispatch
set -o pipefail
O=gpurun_out/r03z3; mkdir -p $O
for d in 2; do
  BGV_DISPATCHERS=$d timeout -k 10 150 node tests/node/gossip_bench.js 4 64 "0:1,31:1,63:1" > $O/gossip_d$d.jsonl 2>>$O/err || exit 1
  echo "dispatchers $d: $(python -c "
import json
for l in open('$O/gossip_d$d.jsonl'): d=json.loads(l); print(d['maxBufferedSigs'], round(d['sets_per_s']), d['latency_ms']['p50'], end='; ')
")"
done
