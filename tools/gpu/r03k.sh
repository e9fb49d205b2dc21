# Node gossip bench (64 concurrent one-set callers through BlsGpuVerifier) + config-3 p50
set -o pipefail
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 200 node tests/node/gossip_bench.js 6 64 "32:100,1024:20,64:5,32:2,64:1,16:1" > $O/gossip.jsonl 2> $O/gossip.err || { echo gossip failed; tail $O/gossip.err; exit 1; }
cat $O/gossip.jsonl
