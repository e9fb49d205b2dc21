# pipeline headroom: headline window with and without corrupted sets
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep"
for i in 1 2; do
  timeout -k 10 150 $B --corrupt 0 >> $O/c0.jsonl 2>>$O/err || exit 1
  timeout -k 10 150 $B >> $O/c1.jsonl 2>>$O/err || exit 1
done
BGV_TRACE=1 timeout -k 10 150 $B --corrupt 0 > $O/trace_c0.json 2> $O/trace_c0.err || exit 1
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r03m/*.jsonl')):
    v=[json.loads(l) for l in open(f) if l.startswith('{')]
    print(f, [round(x['value']/1e6,3) for x in v])
PY
grep "calls 16" gpurun_out/r03m/trace_c0.err | tail -4
