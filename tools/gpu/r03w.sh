# retry rounds: Exec pool size, one-lane group pairs with a larger pool
set -o pipefail
O=gpurun_out/r03w; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep"
for i in 1 2; do
  timeout -k 10 150 $B >> $O/e4.jsonl 2>>$O/err || exit 1
  BGV_EXECS=8 timeout -k 10 150 $B >> $O/e8.jsonl 2>>$O/err || exit 1
  BGV_EXECS=8 BGV_RETRY_LANE_PAIRS=1024 timeout -k 10 150 $B >> $O/e8_lane.jsonl 2>>$O/err || exit 1
  BGV_EXECS=12 BGV_RETRY_LANE_PAIRS=1024 timeout -k 10 150 $B >> $O/e12_lane.jsonl 2>>$O/err || exit 1
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r03w/*.jsonl')):
    v=[json.loads(l) for l in open(f) if l.startswith('{')]
    print(f, [round(x['value']/1e6,3) for x in v])
PY
