# GLV additions without the doubling branch: hostsim-independent GPU parity + isolated k_prep A/B
set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 120 python tools/gpu/roof_call.py >> $O/cur.jsonl 2>>$O/err || exit 1
  BLSGPU_LIB=$PWD/lodestar_amd/libblsgpu_prev.so timeout -k 10 120 python tools/gpu/roof_call.py >> $O/prev.jsonl 2>>$O/err || exit 1
done
python - <<'PY'
import json
for t in ('cur','prev'):
    for l in open('gpurun_out/r03t/%s.jsonl'%t):
        d=json.loads(l); print(t, {k:round(v,2) for k,v in d['kernel_ms_isolated'].items()}, round(d['frac'],3))
PY
