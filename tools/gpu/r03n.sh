# dispatchers x streams per dispatcher on the headline window
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep"
for i in 1 2; do
  timeout -k 10 150 $B >> $O/d2s2.jsonl 2>>$O/err || exit 1
  BGV_STREAMS=1 timeout -k 10 150 $B >> $O/d2s1.jsonl 2>>$O/err || exit 1
  BGV_STREAMS=1 BGV_DISPATCHERS=3 timeout -k 10 150 $B >> $O/d3s1.jsonl 2>>$O/err || exit 1
done
BGV_STREAMS=1 BGV_DISPATCHERS=3 BGV_TRACE=1 timeout -k 10 150 $B > $O/trace.json 2> $O/trace.err || exit 1
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r03n/*.jsonl')):
    v=[json.loads(l) for l in open(f) if l.startswith('{')]
    print(f, [round(x['value']/1e6,3) for x in v])
PY
grep "calls 16" gpurun_out/r03n/trace.err | tail -4
