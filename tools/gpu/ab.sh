#!/bin/bash
# GPU suite, then an interleaved A/B of library builds on the bench's headline window and
# isolated roofline call.  Stops at the first GPU fault, abort, crash or time limit (pytest
# exit 1 = failing tests only, the A/B still runs).
#   tools/gpu/ab.sh OUTDIR ROUNDS LIB...
OUT=$1; N=$2; shift 2
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for i in $(seq 1 "$N"); do
  for L in "$@"; do
    tag=$(basename "$L" .so)
    BLSGPU_LIB=$L timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep \
      >> "$OUT/ab_$tag.jsonl" 2>> "$OUT/ab.err" || { echo "bench $tag rc=$?: stopping"; exit 1; }
  done
done
echo "pytest rc=$rc"
