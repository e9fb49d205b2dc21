set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_retry.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BGV_TRACE=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep > $O/trace_cur.json 2> $O/trace_cur.err || exit 1
for i in 1 2; do timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep >> $O/bench.jsonl 2>>$O/bench.err || exit 1; done
python -c "
import json
for l in open('$O/bench.jsonl'): d=json.loads(l); print(round(d['value']/1e6,3), d['device_groups_per_step'], d['retries_per_step'])
"
