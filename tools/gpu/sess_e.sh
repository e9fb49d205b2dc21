set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu/record.sh $O suite; rc=$?
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu/record.sh $O pmc
