# A/B of the current library against two earlier builds on the headline window, then one
# traced run of the current library (per-super-batch phase times on stderr).
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
for i in 1 2; do
  for L in lodestar_amd/libblsgpu.so lodestar_amd/libblsgpu_c88.so lodestar_amd/libblsgpu_c3a.so; do
    tag=$(basename $L .so)
    BLSGPU_LIB=$PWD/$L timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep \
      >> $O/ab_$tag.jsonl 2>> $O/ab.err || { echo "bench $tag rc=$?"; exit 1; }
  done
done
BGV_TRACE=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep > $O/trace_cur.json 2> $O/trace_cur.err || exit 1
BGV_TRACE=1 BLSGPU_LIB=$PWD/lodestar_amd/libblsgpu_c88.so timeout -k 10 150 python bench.py --no-cpu-baseline --no-block-import --no-epoch-sweep > $O/trace_c88.json 2> $O/trace_c88.err || exit 1
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r03b/ab_*.jsonl')):
    v=[json.loads(l) for l in open(f) if l.startswith('{')]
    print(f, [round(x['value']/1e6,3) for x in v], [x.get('device_groups_per_step') for x in v], [round(x['roofline']['kernel_ms_isolated']['k_miller'],2) for x in v])
PY
