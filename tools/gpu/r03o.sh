# retry pairs + compacted closing products: GPU suite, headline A/B against the previous build
set -o pipefail
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep"
for i in 1 2 3; do
  timeout -k 10 150 $B >> $O/cur.jsonl 2>>$O/err || exit 1
  BLSGPU_LIB=$PWD/lodestar_amd/libblsgpu_prev.so timeout -k 10 150 $B >> $O/prev.jsonl 2>>$O/err || exit 1
done
BGV_TRACE=1 timeout -k 10 150 $B > $O/trace.json 2> $O/trace.err || exit 1
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r03p/*.jsonl')):
    v=[json.loads(l) for l in open(f) if l.startswith('{')]
    print(f, [round(x['value']/1e6,3) for x in v], [x['device_groups_per_step'] for x in v])
PY
grep "\[bgv\] dev" gpurun_out/r03p/trace.err | tail -3
