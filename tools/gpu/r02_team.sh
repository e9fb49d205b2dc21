#!/bin/bash
# team Miller loop: GPU parity suite, config-3 latency trace, default bench
set -o pipefail
mkdir -p gpurun_out/r02 gpurun_out/lat
export TMPDIR=/tmp
TAG=${TAG:-t9}
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r02/pytest_$TAG.log; tail -4 gpurun_out/r02/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
TAG=$TAG bash tools/gpu/r02_latency.sh || exit 1
timeout -k 10 150 node tests/node/gossip_bench.js 6 64 "32:2,16:1,64:1" > gpurun_out/r02/gossip_$TAG.jsonl 2> gpurun_out/r02/gossip_$TAG.err || { tail -5 gpurun_out/r02/gossip_$TAG.err; exit 1; }
cat gpurun_out/r02/gossip_$TAG.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r02/bench_$TAG.json 2> gpurun_out/r02/bench_$TAG.err || { tail -5 gpurun_out/r02/bench_$TAG.err; exit 1; }
python tools/gpu/summarize.py gpurun_out/r02/bench_$TAG.json
