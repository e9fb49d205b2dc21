#!/bin/bash
# Round-2 GPU check: parity tests, then the driver's bench command and a longer one.
set -o pipefail
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
TAG=${TAG:-a}
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r02/pytest_$TAG.log; tail -4 gpurun_out/r02/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02/bench20_$TAG.json 2> gpurun_out/r02/bench20_$TAG.err || { tail -5 gpurun_out/r02/bench20_$TAG.err; exit 1; }
python tools/gpu/summarize.py gpurun_out/r02/bench20_$TAG.json
timeout -k 10 200 python bench.py --steps 64 --warmup 16 --no-cpu-baseline --no-block-import > gpurun_out/r02/bench64_$TAG.json 2> gpurun_out/r02/bench64_$TAG.err || { tail -5 gpurun_out/r02/bench64_$TAG.err; exit 1; }
python tools/gpu/summarize.py gpurun_out/r02/bench64_$TAG.json
