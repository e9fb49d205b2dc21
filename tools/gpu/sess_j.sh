# Round-4 session j: GPU suite, then config-3 latency of the default library and of an A/B
# library given as $2 (interleaved, 2 rounds each), then the default bench under a kernel trace.
#   bash tools/gpu/sess_j.sh OUTDIR ABLIB
set -o pipefail
O=$1; L=$2; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu/record.sh $O suite || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat_default.jsonl 2>>$O/err.txt || { echo lat failed; exit 1; }
  BLSGPU_LIB=$L timeout -k 10 120 python tools/gpu/latency_probe.py 30 >> $O/lat_ab.jsonl 2>>$O/err.txt || { echo lat ab failed; exit 1; }
done
cat $O/lat_default.jsonl $O/lat_ab.jsonl
