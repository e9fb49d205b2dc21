# Node gossip 64 callers: idle coalescing window 50 us (default) vs 0, interleaved
set -o pipefail
O=gpurun_out/r03s2; mkdir -p $O
for rep in 1 2; do
  for w in 50 0; do
    BGV_IDLE_COALESCE_US=$w timeout -k 10 60 node tests/node/gossip_bench.js 4 64 "63:1" > $O/g_${w}_$rep.jsonl 2>>$O/err || exit 1
    echo "idle $w rep $rep: $(cat $O/g_${w}_$rep.jsonl)"
  done
done
