#!/bin/bash
# Round-2 GPU pass 2: full -m gpu suite, Node-level gossip throughput, default bench with the
# CPU baseline (host report + config-1 single-core row).
set -o pipefail
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
TAG=${TAG:-b}
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r02/pytest_$TAG.log; tail -4 gpurun_out/r02/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 node tests/node/gossip_bench.js 8 64 "32:100,1024:20,64:5,32:2,16:1" > gpurun_out/r02/gossip_$TAG.jsonl 2> gpurun_out/r02/gossip_$TAG.err || { tail -5 gpurun_out/r02/gossip_$TAG.err; exit 1; }
cat gpurun_out/r02/gossip_$TAG.jsonl
timeout -k 10 300 python bench.py > gpurun_out/r02/bench_default_$TAG.json 2> gpurun_out/r02/bench_default_$TAG.err || { tail -5 gpurun_out/r02/bench_default_$TAG.err; exit 1; }
python tools/gpu/summarize.py gpurun_out/r02/bench_default_$TAG.json
