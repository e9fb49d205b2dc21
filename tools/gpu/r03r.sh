set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep"
for i in 1 2 3; do
  timeout -k 10 150 $B >> $O/team.jsonl 2>>$O/err || exit 1
  BGV_RETRY_LANE_PAIRS=1024 timeout -k 10 150 $B >> $O/lane1024.jsonl 2>>$O/err || exit 1
  BGV_RETRY_LANE_PAIRS=128 timeout -k 10 150 $B >> $O/lane128.jsonl 2>>$O/err || exit 1
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r03r/*.jsonl')):
    v=[json.loads(l) for l in open(f) if l.startswith('{')]
    print(f, [round(x['value']/1e6,3) for x in v])
PY
