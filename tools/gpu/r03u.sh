# k_prep tasks at two waves per SIMD (BGV_PREP_W2 bits: 2 = sig, 4 = pk) on the isolated call
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
for i in 1 2; do
  for m in 0 4 2 6; do
    BGV_PREP_W2=$m timeout -k 10 120 python tools/gpu/roof_call.py >> $O/w2_$m.jsonl 2>>$O/err || exit 1
  done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r03u/w2_*.jsonl')):
    print(f, [round(json.loads(l)['kernel_ms']['k_prep'],2) for l in open(f)])
PY
