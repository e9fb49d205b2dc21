#!/bin/bash
# Session-3 GPU check: parity tests, the isolated roofline call (per-kernel times), the
# driver's default bench command.  Outputs under gpurun_out/s3/<TAG>_*.
set -o pipefail
D=gpurun_out/s3
mkdir -p $D
export TMPDIR=/tmp
TAG=${TAG:-a}
if [ -z "$NOTEST" ]; then
  timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $D/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $D/${TAG}_pytest.log; tail -3 $D/${TAG}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python tools/gpu/roof_call.py > $D/${TAG}_roof.json 2> $D/${TAG}_roof.err || { tail -5 $D/${TAG}_roof.err; exit 1; }
cat $D/${TAG}_roof.json | head -c 1500; echo
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/${TAG}_bench20.json 2> $D/${TAG}_bench20.err || { tail -5 $D/${TAG}_bench20.err; exit 1; }
python tools/gpu/summarize.py $D/${TAG}_bench20.json
