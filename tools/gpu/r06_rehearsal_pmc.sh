set -o pipefail; O=gpurun_out/r06s3; mkdir -p $O; export TMPDIR=/tmp
BGV_BENCH_DEVICE=0 timeout -k 10 900 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_2ranks_1gpu.json 2> $O/bench_2ranks.err || { echo "2-rank rc=$?"; tail -30 $O/bench_2ranks.err; exit 1; }
python tools/gpu/summarize.py $O/bench_2ranks_1gpu.json
bash tools/gpu/record.sh $O roof || exit 1
TAG=r06s3 bash tools/gpu/pmc.sh || exit 1
