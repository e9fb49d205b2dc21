#!/bin/bash
# k_final on 12-lane teams (k_final12, default) vs 16-lane teams (BGV_FINAL12=0): GPU suite on the default,
# then the default bench interleaved.
set -o pipefail
D=gpurun_out/s3/final12
mkdir -p $D
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -20 $D/pytest_gpu.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $D/pytest_gpu.log
for round in ${ROUNDS:-1 2 3}; do
  for v in 1 0; do
    BGV_FINAL12=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-block-import > $D/f12_${v}_$round.json 2> $D/f12_${v}_$round.err || { tail -3 $D/f12_${v}_$round.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value']), round(d['call_device_ms'],1), {k: round(v,3) for k,v in r.get('kernel_ms_isolated', {}).items()} if isinstance(r, dict) else '')" $D/f12_${v}_$round.json f12=$v
  done
done
