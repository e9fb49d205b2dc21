# A/B: NRVO fix (current) vs previous build; 3 dispatchers; config-3 latency kernel trace.
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep"
for i in 1 2; do
  timeout -k 10 150 $B >> $O/cur.jsonl 2>>$O/err || exit 1
  BLSGPU_LIB=$PWD/lodestar_amd/libblsgpu_prev.so timeout -k 10 150 $B >> $O/prev.jsonl 2>>$O/err || exit 1
  BGV_DISPATCHERS=3 timeout -k 10 150 $B >> $O/disp3.jsonl 2>>$O/err || exit 1
done
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/lat -o run --output-format csv -- python3 tools/gpu/latency_probe.py 30 > $O/lat.log 2>&1 || { echo lat failed; tail $O/lat.log; exit 1; }
tail -1 $O/lat.log
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r03f/*.jsonl')):
    v=[json.loads(l) for l in open(f) if l.startswith('{')]
    print(f, [round(x['value']/1e6,3) for x in v], [ {k:round(t,2) for k,t in x['roofline']['kernel_ms_isolated'].items()} for x in v])
PY
