# wide final exponentiation in k_final_fold: GPU suite, config-3 latency trace, node gossip
set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/lat -o run --output-format csv -- python3 tools/gpu/latency_probe.py 30 > $O/lat.log 2>&1 || { echo lat failed; tail $O/lat.log; exit 1; }
grep p50 $O/lat.log
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r03x/lat/run_kernel_stats.csv')): print(r['Name'][:30], r['Calls'], round(float(r['AverageNs'])/1e6,3))
PY
